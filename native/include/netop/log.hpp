// klog-compatible leveled logging for the node agent.
//
// The reference agent logs through klog with per-NIC detail at V(3)
// (reference cmd/discover/network.go:175-213) and exposes klog's flag set
// (cmd/discover/main.go:273-276).  This is a small, lock-protected
// re-implementation of the klog header format:
//     Lmmdd hh:mm:ss.uuuuuu threadid file:line] msg
// plus an optional JSON-lines format (--logging-format=json) for log shippers.
#pragma once

#include <cstdarg>
#include <string>

namespace netop::log {

enum class Format { Text, Json };

void set_verbosity(int v);
int verbosity();
void set_format(Format f);
void set_skip_headers(bool s);
// Redirect output to a file in addition to / instead of stderr ("" = stderr only).
void set_log_file(const std::string& path);
// Capture sink for unit tests: when non-null, every rendered line is appended.
void set_capture(std::string* sink);

void emit(char severity, const char* file, int line, const char* fmt, ...) __attribute__((format(printf, 4, 5)));

}  // namespace netop::log

#define NLOG_I(...) ::netop::log::emit('I', __FILE__, __LINE__, __VA_ARGS__)
#define NLOG_W(...) ::netop::log::emit('W', __FILE__, __LINE__, __VA_ARGS__)
#define NLOG_E(...) ::netop::log::emit('E', __FILE__, __LINE__, __VA_ARGS__)
#define NLOG_V(level, ...)                                                          \
    do {                                                                            \
        if (::netop::log::verbosity() >= (level)) ::netop::log::emit('I', __FILE__, __LINE__, __VA_ARGS__); \
    } while (0)

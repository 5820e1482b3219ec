#include "netop/log.hpp"

#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <cstring>
#include <mutex>

#include "netop/common.hpp"

namespace netop::log {
namespace {
std::atomic<int> g_verbosity{0};
std::atomic<Format> g_format{Format::Text};
std::atomic<bool> g_skip_headers{false};
std::mutex g_mu;
FILE* g_file = nullptr;
std::string* g_capture = nullptr;

std::string json_escape(const std::string& s) {
    std::string o;
    o.reserve(s.size() + 8);
    for (unsigned char c : s) {
        switch (c) {
            case '"': o += "\\\""; break;
            case '\\': o += "\\\\"; break;
            case '\n': o += "\\n"; break;
            case '\r': o += "\\r"; break;
            case '\t': o += "\\t"; break;
            default:
                if (c < 0x20)
                    o += strfmt("\\u%04x", c);
                else
                    o += char(c);
        }
    }
    return o;
}
}  // namespace

void set_verbosity(int v) { g_verbosity = v; }
int verbosity() { return g_verbosity; }
void set_format(Format f) { g_format = f; }
void set_skip_headers(bool s) { g_skip_headers = s; }

void set_log_file(const std::string& path) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_file) {
        std::fclose(g_file);
        g_file = nullptr;
    }
    if (!path.empty()) g_file = std::fopen(path.c_str(), "a");
}

void set_capture(std::string* sink) {
    std::lock_guard<std::mutex> lk(g_mu);
    g_capture = sink;
}

void emit(char severity, const char* file, int line, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    char msgbuf[2048];
    std::vsnprintf(msgbuf, sizeof msgbuf, fmt, ap);
    va_end(ap);
    std::string msg(msgbuf);
    while (!msg.empty() && msg.back() == '\n') msg.pop_back();

    const char* base = std::strrchr(file, '/');
    base = base ? base + 1 : file;

    timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);
    struct tm tm;
    localtime_r(&ts.tv_sec, &tm);
    long tid = long(::syscall(SYS_gettid));

    std::string out;
    if (g_format == Format::Json) {
        char tbuf[64];
        gmtime_r(&ts.tv_sec, &tm);
        std::strftime(tbuf, sizeof tbuf, "%Y-%m-%dT%H:%M:%S", &tm);
        const char* lvl = severity == 'E' ? "error" : severity == 'W' ? "warning" : "info";
        out = strfmt("{\"ts\":\"%s.%06ldZ\",\"level\":\"%s\",\"caller\":\"%s:%d\",\"msg\":\"%s\"}\n", tbuf,
                     ts.tv_nsec / 1000, lvl, base, line, json_escape(msg).c_str());
    } else if (g_skip_headers) {
        out = msg + "\n";
    } else {
        out = strfmt("%c%02d%02d %02d:%02d:%02d.%06ld %7ld %s:%d] %s\n", severity, tm.tm_mon + 1, tm.tm_mday,
                     tm.tm_hour, tm.tm_min, tm.tm_sec, ts.tv_nsec / 1000, tid, base, line, msg.c_str());
    }

    std::lock_guard<std::mutex> lk(g_mu);
    if (g_capture) {
        g_capture->append(out);
        return;
    }
    std::fwrite(out.data(), 1, out.size(), stderr);
    if (g_file) {
        std::fwrite(out.data(), 1, out.size(), g_file);
        std::fflush(g_file);
    }
}

}  // namespace netop::log

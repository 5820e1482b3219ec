// Helpers shared by the agent's translation units (agent.cpp, agent_ownership.cpp,
// agent_links.cpp, agent_monitor.cpp); not part of the public interface.
#pragma once

#include <poll.h>

#include <cstdint>
#include <string>

#include "netop/common.hpp"

namespace netop::agent::detail {

// Non-blocking: is `fd` readable now (the stop pipe, a wake-up fd)?  false for fd < 0.
inline bool fd_readable(int fd) {
    if (fd < 0) return false;
    pollfd p{fd, POLLIN, 0};
    return ::poll(&p, 1, 0) > 0;
}

// 400000 Mb/s -> "400".
inline std::string format_gbps(int64_t mbps) { return strfmt("%g", double(mbps) / 1000.0); }

// Longest a --verify-peers re-probe may hold the monitor loop (see Agent::monitor).
constexpr int64_t kMonitorVerifyNs = 250LL * 1000000;

}  // namespace netop::agent::detail

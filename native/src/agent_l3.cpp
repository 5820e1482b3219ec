// Agent: L3 configuration of one NIC from its LLDP-derived /30 -- the address, the kernel /30
// and the /16 via the switch (reference cmd/discover/network.go:311-469), and the per-rail
// source-routing tables (--rail-table-base).
#include "netop/agent.hpp"

#include <errno.h>
#include <linux/if.h>
#include <poll.h>
#include <sys/epoll.h>
#include <sys/resource.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include <cstddef>

#include <algorithm>
#include <cstring>
#include <ctime>
#include <sched.h>
#include <sys/syscall.h>
#include <mutex>
#include <regex>
#include <set>
#include <system_error>

#include "agent_internal.hpp"
#include "netop/log.hpp"

namespace netop::agent {

using detail::fd_readable;

void Agent::add_route(NicState& n, int mask) {
    nl::RouteSpec r;
    r.ifindex = n.link.index;
    if (!n.addr) throw AgentError("interface '" + n.ifname + "' has no local address");
    r.dst = Ipv4Prefix{n.addr->local, mask}.masked();
    std::string desc = r.dst.str();
    if (mask == l3::kRoutedNetworkMask) {
        r.gateway = n.addr->peer;  // protocol left at the netlink library default (boot)
        desc += " gateway " + n.addr->peer.str();
    } else {
        r.protocol = RTPROT_KERNEL;  // identical to the route the kernel adds with the address
        r.scope = RT_SCOPE_LINK;
        r.prefsrc = n.addr->local;
    }
    try {
        ops_.route_append(r);
        NLOG_V(3, "Configured route %s for interface '%s'", desc.c_str(), n.ifname.c_str());
    } catch (const SysError& e) {
        if (e.code() == EEXIST) {
            NLOG_V(3, "Route %s already exists for interface '%s'", desc.c_str(), n.ifname.c_str());
            return;
        }
        NLOG_W("Could not add route %s for interface '%s': %s", desc.c_str(), n.ifname.c_str(), e.what());
        throw;
    }
}

uint32_t Agent::rail_table(const NicState& n) const { return uint32_t(cfg_.rail_table_base + n.rail_index); }

void Agent::assign_rail_indices() {
    // GPU-paired NICs keep their GPU index; the others (extra --interfaces, a GPU without a NIC
    // in reach) follow the highest GPU index, so no two NICs ever share a table.
    int next = -1;
    std::set<int> used;
    for (auto& n : nics_)
        if (n.gpu_index >= 0 && used.insert(n.gpu_index).second) {
            n.rail_index = n.gpu_index;
            next = std::max(next, n.gpu_index);
        } else {
            n.rail_index = -1;
        }
    for (auto& n : nics_)
        if (n.rail_index < 0) n.rail_index = ++next;
}

void Agent::add_rail_routing(NicState& n) {
    const uint32_t t = rail_table(n);
    // Routes carry an 8-bit table id here, and 253..255 are the kernel's default / main / local.
    if (t == 0 || t >= RT_TABLE_DEFAULT)
        throw AgentError(strfmt("rail table %u of '%s' is outside 1..252 (lower --rail-table-base)", t, n.ifname.c_str()));
    nl::RuleSpec rule{Ipv4Prefix{n.addr->local, 32}, t, t, kRailProtocol};
    // What this agent installed for an earlier address of this rail (Port Description change).
    if (n.rail_rule && !(*n.rail_rule == rule)) remove_rail_routing(n);
    // Leftovers of an earlier agent run (crash, restart with another NIC set): only rules and
    // routes tagged with our protocol, and only for this rail's table / priority.
    for (const auto& r : ops_.rule_list())
        if (r.protocol == kRailProtocol && (r.table == t || r.priority == t) && !(r == rule)) {
            try {
                ops_.rule_del(r);
            } catch (const SysError& e) {
                if (e.code() != ENOENT) throw;
            }
        }
    nl::RouteSpec p2p;
    p2p.ifindex = n.link.index;
    p2p.dst = n.addr->local_prefix().masked();
    p2p.scope = RT_SCOPE_LINK;
    p2p.prefsrc = n.addr->local;
    p2p.table = uint8_t(t);
    p2p.protocol = kRailProtocol;
    nl::RouteSpec routed;
    routed.ifindex = n.link.index;
    routed.dst = Ipv4Prefix{n.addr->local, l3::kRoutedNetworkMask}.masked();
    routed.gateway = n.addr->peer;
    routed.prefsrc = n.addr->local;
    routed.table = uint8_t(t);
    routed.protocol = kRailProtocol;
    auto same = [](const nl::RouteSpec& a, const nl::RouteSpec& b) {
        return a.dst.masked() == b.dst.masked() && a.gateway == b.gateway && a.ifindex == b.ifindex;
    };
    for (const auto& r : ops_.route_list(uint32_t(t))) {
        if (r.protocol != kRailProtocol || same(r, p2p) || same(r, routed)) continue;
        try {
            ops_.route_del(r);
        } catch (const SysError&) {
        }
    }
    n.rail_routes.clear();
    for (const auto& r : {p2p, routed}) {
        try {
            ops_.route_append(r);
        } catch (const SysError& e) {
            if (e.code() != EEXIST) throw;
        }
        n.rail_routes.push_back(r);
    }
    try {
        ops_.rule_add(rule);
    } catch (const SysError& e) {
        if (e.code() != EEXIST) throw;
    }
    n.rail_rule = rule;
    NLOG_V(3, "Rail routing for '%s': table %u, rule %s", n.ifname.c_str(), t, rule.str().c_str());
}

void Agent::remove_rail_routing(NicState& n) {
    if (n.rail_rule) {
        try {
            ops_.rule_del(*n.rail_rule);
        } catch (const SysError& e) {
            if (e.code() != ENOENT) NLOG_W("Could not remove the rail rule of '%s': %s", n.ifname.c_str(), e.what());
        }
        n.rail_rule.reset();
    }
    for (const auto& r : n.rail_routes) {
        try {
            ops_.route_del(r);
        } catch (...) {  // already gone with the address / link
        }
    }
    n.rail_routes.clear();
}

void Agent::remove_rail_routing() {
    for (auto& n : nics_) remove_rail_routing(n);
}

bool Agent::configure_interface(NicState& n) {
    if (!n.addr || n.configured) return n.configured;
    // Two switch ports describing the same /30 (a copy-pasted port description, two cables on
    // one link): the kernel would take the address twice and ARP and routing would pick either
    // NIC.  The first NIC keeps it; this one stays unconfigured, and the error says why.
    const Ipv4Prefix net = n.addr->local_prefix().masked();
    for (const auto& m : nics_) {
        if (&m == &n || !m.addr || !(m.addr->local_prefix().masked() == net)) continue;
        if (!m.configured && &m > &n) continue;  // neither configured yet: the earlier NIC wins
        n.config_error = strfmt("its switch port describes %s, the link of %s too (two ports, one /30: check the "
                                "switch's Port Descriptions and the cabling)",
                                n.addr->local_prefix().str().c_str(), m.ifname.c_str());
        NLOG_W("Interface '%s' not configured: %s", n.ifname.c_str(), n.config_error.c_str());
        return false;
    }
    // The 802.3 Maximum Frame Size counts the whole frame: MTU + 14 (header) + 4 (FCS), + 4 more
    // for an 802.1Q tag on a VLAN NIC -- the same count the agent advertises (make_node_frame).
    const int need = max_frame_for_mtu(cfg_.mtu, n.link.kind == "vlan");
    if (cfg_.check_peer_mtu && n.peer_max_frame > 0 && n.peer_max_frame < need) {
        n.config_error = strfmt("its switch port accepts frames up to %d bytes, but MTU %d needs %d%s: jumbo RoCE "
                                "frames would be dropped (raise the switch port's MTU, or lower the policy's mtu)",
                                n.peer_max_frame, cfg_.mtu, need, n.link.kind == "vlan" ? " (802.1Q tagged)" : "");
        NLOG_W("Interface '%s' not configured: %s", n.ifname.c_str(), n.config_error.c_str());
        return false;
    }
    if (std::string why = check_link_speed(n); !why.empty() || !(why = check_pcie(n)).empty()) {
        n.config_error = why;
        NLOG_W("Interface '%s' not configured: %s", n.ifname.c_str(), n.config_error.c_str());
        return false;
    }
    if (!cfg_.rail_switch_pattern.empty() && n.gpu_index >= 0) {
        std::string want = cfg_.rail_switch_pattern;
        for (size_t at; (at = want.find("{rail}")) != std::string::npos;) want.replace(at, 6, std::to_string(n.gpu_index));
        const auto ok = ecmascript_full_match(want, n.peer_system_name);
        if (!ok) {  // (run() checked the pattern for every rail index; kept as a guard)
            n.config_error = "invalid --rail-switch-pattern '" + cfg_.rail_switch_pattern + "' for rail " +
                             std::to_string(n.gpu_index) + ": " + ecmascript_regex_error(want);
            NLOG_W("Interface '%s' not configured: %s", n.ifname.c_str(), n.config_error.c_str());
            return false;
        }
        if (!*ok) {
            n.config_error = strfmt("rail %d is cabled to switch '%s' port '%s', not to one matching '%s' (a NIC on "
                                    "another rail's leaf crosses the spine: check the cabling)",
                                    n.gpu_index, n.peer_system_name.c_str(), n.peer_port_id.c_str(), want.c_str());
            NLOG_W("Interface '%s' not configured: %s", n.ifname.c_str(), n.config_error.c_str());
            return false;
        }
    }
    std::vector<nl::AddrInfo> addrs;
    try {
        addrs = ops_.addr_list(n.link.index, AF_INET);
    } catch (const std::exception& e) {
        n.config_error = e.what();
        NLOG_W("Could not get addresses for link '%s': %s", n.ifname.c_str(), e.what());
        return false;
    }
    bool existing = std::any_of(addrs.begin(), addrs.end(), [&](const nl::AddrInfo& a) { return a.local == n.addr->local; });
    try {
        if (!existing) {
            // The kernel adds the /30 connected route along with the address (and the RDMA core
            // a RoCE GID for it, in a slot of its choosing: the index is looked up again).
            ops_.addr_add(n.link.index, n.addr->local_prefix());
            n.gid_index.reset();
            NLOG_I("Configured address and route %s for interface '%s'", n.addr->local_prefix().str().c_str(), n.ifname.c_str());
        } else {
            NLOG_I("Interface '%s' already configured with address %s", n.ifname.c_str(), n.addr->local_prefix().str().c_str());
            add_route(n, l3::kPointToPointMask);
        }
        add_route(n, l3::kRoutedNetworkMask);
        if (cfg_.rail_table_base > 0) add_rail_routing(n);
    } catch (const std::exception& e) {
        n.config_error = e.what();
        if (!existing) NLOG_W("Could not configure address %s for interface '%s': %s", n.addr->local.str().c_str(), n.ifname.c_str(), e.what());
        return false;
    }
    n.configured = true;
    n.config_error.clear();
    n.t_configured = mono_ns();
    return true;
}

int Agent::configure_all() {
    NLOG_I("Configuring interfaces...");
    int c = 0;
    for (auto& n : nics_)
        if (configure_interface(n)) ++c;
    return c;
}

}  // namespace netop::agent

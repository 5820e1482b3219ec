// Agent: who owns which NIC.  The node-wide locks (one per label file, one per NIC) and the
// node's own interfaces that no agent configures: default-route NICs (directly or under a bond
// or VLAN), bond / bridge / team ports, NICs with addresses or routes the agent never installs.
#include "netop/agent.hpp"

#include <errno.h>
#include <linux/rtnetlink.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include <algorithm>
#include <cstddef>
#include <cstring>
#include <thread>

#include "agent_internal.hpp"
#include "netop/log.hpp"

namespace netop::agent {

int Agent::take_lock(const std::string& name, int64_t deadline, int stop_fd, const std::string& waiting,
                     const std::string& busy) {
    sockaddr_un sa{};
    sa.sun_family = AF_UNIX;
    const size_t n = std::min(name.size(), sizeof sa.sun_path - 1);
    std::memcpy(sa.sun_path + 1, name.data(), n);  // abstract: sun_path[0] == 0
    const socklen_t len = socklen_t(offsetof(sockaddr_un, sun_path) + 1 + n);
    bool waited = false;
    for (;;) {
        int fd = ::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
        if (fd < 0) throw AgentError("lock " + name + ": socket: " + std::strerror(errno));
        if (::bind(fd, reinterpret_cast<sockaddr*>(&sa), len) == 0) {
            if (waited) NLOG_I("Lock '%s' acquired", name.c_str());
            return fd;
        }
        const int err = errno;
        ::close(fd);
        if (err != EADDRINUSE) throw AgentError("lock " + name + ": bind: " + std::strerror(err));
        if (!waited) NLOG_I("%s: waiting", waiting.c_str());
        waited = true;
        if (mono_ns() >= deadline) throw AgentError(busy);
        if (stop_fd >= 0) {
            pollfd p{stop_fd, POLLIN, 0};
            if (::poll(&p, 1, 100) > 0) throw AgentError("Interrupted while waiting for lock " + name);
        } else {
            ::usleep(100000);
        }
    }
}

void Agent::acquire_node_lock(int stop_fd) {
    if (cfg_.node_lock.empty() || node_lock_fd_ >= 0) return;
    node_lock_fd_ = take_lock("netop-agent:" + cfg_.node_lock, mono_ns() + cfg_.node_lock_wait_ns, stop_fd,
                              "Node lock '" + cfg_.node_lock + "' is held by another agent on this node",
                              "Another agent (or its cleanup) holds the node lock '" + cfg_.node_lock +
                                  "': two policies of one configuration type select this node, or the previous agent "
                                  "is still exiting");
}

void Agent::acquire_nic_locks(int stop_fd) {
    if (!cfg_.nic_locks || !nic_lock_fds_.empty()) return;
    // Name order: two agents wanting overlapping NIC sets can never wait on each other in a cycle.
    std::vector<std::string> names;
    for (const auto& n : nics_) names.push_back(n.ifname);
    std::sort(names.begin(), names.end());
    const int64_t deadline = mono_ns() + cfg_.node_lock_wait_ns;
    for (const auto& name : names)
        nic_lock_fds_.push_back(take_lock(
            "netop-nic:" + name, deadline, stop_fd, "NIC '" + name + "' is held by another agent on this node",
            "Another agent holds NIC '" + name +
                "' (its NIC lock): an amd-so and a host-nic policy, or two host-nic policies, select this NIC, or the "
                "previous agent is still exiting.  Every NIC has one owner: select it in one policy only"));
}

Agent::~Agent() {
    if (node_lock_fd_ >= 0) ::close(node_lock_fd_);
    for (int fd : nic_lock_fds_) ::close(fd);
    // Both socket sets wait for an RCU grace period when closed: overlap the two waits, so
    // --verify-peers adds nothing to SIGTERM -> exit.
    std::thread closing;
    if (arp_) closing = arp_->close_async();
    lldp_.reset();
    if (closing.joinable()) closing.join();
}

const std::vector<int>& Agent::uplinks() {
    if (!uplinks_read_) {
        try {
            uplinks_ = ops_.default_route_links();
        } catch (const std::exception& e) {
            // Not knowing which NIC is the node's uplink is no reason to guess: touch nothing.
            throw AgentError(std::string("Cannot read the node's routes (needed to leave its own uplinks alone): ") +
                             e.what());
        }
        uplinks_read_ = true;
    }
    return uplinks_;
}

namespace {
std::string protocol_name(uint8_t p) {
    switch (p) {
        case RTPROT_KERNEL: return "kernel";
        case RTPROT_BOOT: return "boot";
        case RTPROT_STATIC: return "static";
        case RTPROT_RA: return "ra";
        case RTPROT_DHCP: return "dhcp";
    }
    return std::to_string(int(p));
}
}  // namespace

std::vector<nl::LinkInfo> Agent::stacked_on(const nl::LinkInfo& l) {
    // Its master from rtnetlink (IFLA_MASTER: bond, bridge, team, VRF), and whatever sysfs lists
    // as an upper device (VLANs and macvlans too).  Unreadable ones are skipped.
    std::vector<nl::LinkInfo> out;
    auto add = [&](std::optional<nl::LinkInfo> u) {
        if (u && u->index != l.index &&
            std::none_of(out.begin(), out.end(), [&](const nl::LinkInfo& x) { return x.index == u->index; }))
            out.push_back(std::move(*u));
    };
    if (l.master != 0) {
        try {
            add(ops_.link_by_ifindex(l.master));
        } catch (const std::exception&) {
        }
    }
    const std::string root = cfg_.sysfs_root.empty() ? topo::sysfs_root() : cfg_.sysfs_root;
    for (const auto& u : topo::netdev_uppers(root, l.name)) {
        try {
            add(ops_.link_by_name(u));
        } catch (const std::exception&) {
        }
    }
    return out;
}

std::optional<std::string> Agent::uplink_path(const nl::LinkInfo& l, int depth) {
    const auto& up = uplinks();
    if (std::find(up.begin(), up.end(), l.index) != up.end()) return std::string();
    if (depth >= 4) return std::nullopt;  // bond on VLAN on bond on ...: deeper stacks are not built
    for (const auto& u : stacked_on(l))
        if (auto via = uplink_path(u, depth + 1)) return " via " + u.name + *via;
    return std::nullopt;
}

std::string Agent::node_owned_reason(const nl::LinkInfo& l, int depth) {
    if (auto via = uplink_path(l)) return "carries the node's default route" + *via;
    const auto uppers = stacked_on(l);
    if (l.master != 0) {
        // A bond / bridge / team port, or a NIC in a VRF: the master device is configured, never
        // its ports.
        std::string master = "ifindex " + std::to_string(l.master);
        for (const auto& u : uppers)
            if (u.index == l.master) master = u.name;
        return "is a port of " + master + " (a bond, bridge, team or VRF: the node configures the master, not its ports)";
    }
    // The agent only ever assigns /30s (the LLDP point-to-point links): anything else on the NIC
    // was put there by the node (DHCP, netplan, a static management address).
    const auto addrs = ops_.addr_list(l.index, AF_INET);
    for (const auto& a : addrs)
        if (a.prefixlen != l3::kPointToPointMask)
            return "holds " + a.prefix().str() + ", an address the agent never assigns (it only uses /30s)";
    // The agent never assigns IPv6 either: a global or ULA address (a storage or management
    // network) is the node's.  Link-local ones come with every up interface.
    try {
        for (const auto& a : ops_.addr_list(l.index, AF_INET6))
            if (a.family == AF_INET6 && a.ifindex == l.index && a.scope < RT_SCOPE_LINK && !a.address6.empty())
                return "holds " + a.address6 + "/" + std::to_string(a.prefixlen) +
                       ", an IPv6 address the agent never assigns";
    } catch (const SysError& e) {
        if (e.code() != EAFNOSUPPORT) throw;  // a kernel without IPv6
    }
    // Routes through it that the agent does not install: its /30 (kernel), the /16 via the switch
    // end of a /30 of this NIC (boot), and its rail tables (kRailProtocol).
    auto agents = [&](const nl::RouteSpec& r) {
        if (r.protocol == kRailProtocol) return true;
        if (r.protocol == RTPROT_KERNEL && r.dst.len == l3::kPointToPointMask) return true;
        if (r.protocol == RTPROT_BOOT && r.dst.len == l3::kRoutedNetworkMask && r.gateway)
            for (const auto& a : addrs)
                if (a.prefix().contains(*r.gateway)) return true;
        return false;
    };
    for (const auto& r : ops_.route_list(0)) {
        if (r.table == RT_TABLE_LOCAL || r.type != RTN_UNICAST) continue;
        if (r.ifindex != l.index && std::find(r.nexthops.begin(), r.nexthops.end(), l.index) == r.nexthops.end()) continue;
        if (!agents(r))
            return strfmt("has the route %s (protocol %s) that the agent does not install", r.dst.masked().str().c_str(),
                          protocol_name(r.protocol).c_str());
    }
    // VLANs / macvlans on it that the node uses (a management VLAN on a RoCE port).
    if (depth < 4)
        for (const auto& u : uppers) {
            std::string why;
            try {
                why = node_owned_reason(u, depth + 1);
            } catch (const AgentError&) {
                throw;
            } catch (const std::exception&) {
                continue;
            }
            if (!why.empty()) return "carries " + u.name + ", which " + why;
        }
    return "";
}

void Agent::refuse_uplinks() {
    // Flushing the addresses of, or re-MTUing, the NIC the node reaches its gateway through can
    // cut the kubelet off the cluster: never, in any mode, whoever named the NIC.
    // A NIC under the uplink (a bond port, the parent of a VLAN) counts: changing its MTU or
    // bouncing it moves the device on top.
    std::vector<std::string> bad;   // refused NICs
    std::vector<std::string> why;   // per refused NIC: what it carries ("the node's default route via bond0")
    for (const auto& n : nics_) {
        if (auto via = uplink_path(n.link)) {
            bad.push_back(n.ifname);
            why.push_back("the node's default route" + *via);
        }
    }
    const size_t uplinks = bad.size();
    // A default route in a per-NIC policy-routing table ("from <its subnet> lookup 101") is the
    // site's source routing for that NIC, not the node's way out through the main table.  But a
    // NIC that routes that way *and* holds the node's own address -- one the agent never installs
    // (not a /30), or the source the rule selects -- is how the node reaches some network (a
    // source-routed management or storage NIC): flushing it can cut the node off just as well
    // (ADVICE r5).  Refused like an uplink, unless --allow-policy-routed; a rail whose policy
    // table only serves the agent's own /30 is configured, with a warning.
    std::vector<std::pair<int, uint32_t>> policy;
    try {
        policy = ops_.policy_default_routes();
    } catch (const std::exception&) {
    }
    std::vector<nl::RuleSpec> rules;
    if (!policy.empty()) {
        try {
            rules = ops_.rule_list();
        } catch (const std::exception&) {
        }
    }
    for (const auto& [ifindex, table] : policy) {
        for (const auto& n : nics_) {
            if (n.link.index != ifindex || std::find(bad.begin(), bad.end(), n.ifname) != bad.end()) continue;
            std::string owned;
            std::vector<nl::AddrInfo> addrs;
            try {
                addrs = ops_.addr_list(ifindex, AF_INET);
            } catch (const std::exception&) {
            }
            for (const auto& a : addrs) {
                for (const auto& r : rules)
                    if (r.table == table && r.selective && r.src.len > 0 && r.src.contains(a.local)) {
                        owned = strfmt("%s, the source its rule 'from %s lookup %u' selects", a.prefix().str().c_str(),
                                       r.src.masked().str().c_str(), table);
                        break;
                    }
                if (owned.empty() && a.prefixlen != 30)
                    owned = a.prefix().str() + ", an address the agent never installs (not a /30)";
                if (!owned.empty()) break;
            }
            if (owned.empty() || cfg_.allow_policy_routed) {
                NLOG_W("Interface '%s' has a default route in routing table %u, which only selective rules reach "
                       "(policy routing): not the node's uplink; it depends on the addresses the agent replaces%s",
                       n.ifname.c_str(), table, owned.empty() ? "" : (" (--allow-policy-routed; it holds " + owned + ")").c_str());
                continue;
            }
            bad.push_back(n.ifname);
            why.push_back(strfmt("a default route in policy-routing table %u and the node's address %s", table, owned.c_str()));
        }
    }
    if (bad.empty()) return;
    // Uplinks keep the reference-era wording ("ens0 via bond0: the node's default route leaves
    // through it"); policy-routed NICs say what they hold.
    std::vector<std::string> up_named, pol_named;
    for (size_t i = 0; i < bad.size(); ++i) {
        if (i < uplinks)
            up_named.push_back(bad[i] + why[i].substr(std::string("the node's default route").size()));
        else
            pol_named.push_back(bad[i] + " (" + why[i] + ")");
    }
    std::string what;
    if (!up_named.empty()) what = join(up_named, ", ") + ": the node's default route leaves through it";
    if (!pol_named.empty())
        what += (what.empty() ? "" : "; ") + join(pol_named, ", ") + ": the node reaches a network through it";
    if (cfg_.dry_run) {
        NLOG_W("dry run: would refuse to configure %s", what.c_str());
        for (size_t i = 0; i < bad.size(); ++i) excluded_.emplace_back(bad[i], "carries " + why[i] + " (refused)");
        return;
    }
    throw AgentError("Refusing to configure " + what +
                     " (flushing its addresses or changing its MTU could cut the node off the network).  Select only "
                     "scale-out / host RDMA NICs in the policy" +
                     (pol_named.empty() ? std::string()
                                        : std::string(" (a NIC whose policy-routing table is only its own rail's: "
                                                      "allowPolicyRouted in the policy, --allow-policy-routed)")));
}

}  // namespace netop::agent

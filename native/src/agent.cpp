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

void sanitize(Config& c) {
    if (c.mtu < 1500) {
        NLOG_I("Forcing MTU value 1500 (old %d)", c.mtu);
        c.mtu = 1500;
    } else if (c.mtu > 9000) {
        NLOG_I("Limiting MTU value 9000 (old %d)", c.mtu);
        c.mtu = 9000;
    }
    std::string m = to_upper(c.mode);
    if (m != "L2" && m != "L3") throw AgentError("Invalid mode '" + c.mode + "'");
    c.mode = m;
}

// ---------------------------------------------------------------------------
// LLDP source over AF_PACKET
// ---------------------------------------------------------------------------
namespace {
class PacketSource final : public LldpSource {
   public:
    explicit PacketSource(bool promisc) : promisc_(promisc) {}
    void add(const std::string& ifname, int ifindex, const MacAddr& own) override {
        listener_.add(ifname, ifindex, own, promisc_);
    }
    pkt::ListenResult run(int64_t deadline, const std::function<bool(const std::string&, const lldp::Frame&)>& cb,
                          int stop_fd) override {
        auto r = listener_.run(deadline, cb, stop_fd);
        auto& s = listener_.stats();
        NLOG_V(2, "LLDP listener: %llu frames, %llu own, %llu malformed, %llu wakeups", (unsigned long long)s.frames,
               (unsigned long long)s.own, (unsigned long long)s.malformed, (unsigned long long)s.wakeups);
        return r;
    }
    void announce(const std::string& ifname, const std::vector<uint8_t>& frame) override {
        listener_.send(ifname, frame);
    }
    pkt::ListenerStats stats() const override { return listener_.stats(); }
    std::optional<pkt::ListenerStats> stats_for(const std::string& ifname) const override {
        return listener_.stats_for(ifname);
    }

   private:
    bool promisc_;
    pkt::LldpListener listener_;
};
}  // namespace

std::unique_ptr<LldpSource> make_packet_source(bool promisc) { return std::make_unique<PacketSource>(promisc); }

int max_frame_for_mtu(int mtu, bool vlan_tagged) { return mtu + 18 + (vlan_tagged ? 4 : 0); }

lldp::Frame make_node_frame(const std::string& node_name, const std::string& ifname, const MacAddr& mac,
                            const std::string& gpu_bdf, uint16_t ttl, int mtu) {
    lldp::Frame f;
    f.dst = lldp::kNearestBridge;
    f.src = mac;
    f.chassis_subtype = lldp::kChassisLocal;
    f.chassis_id = node_name.empty() ? mac.str() : node_name;
    f.port_subtype = lldp::kPortIfName;
    f.port_id = ifname;
    f.ttl = ttl;
    f.port_description = gpu_bdf.empty() ? "scale-out NIC" : "scale-out NIC of GPU " + gpu_bdf;
    f.system_name = node_name;
    f.system_description = "AMD Instinct MI355X node (amd-network-operator link discovery)";
    f.capabilities = std::make_pair(uint16_t(0x0080), uint16_t(0x0080));  // station only
    if (mtu > 0 && ttl > 0) f.set_max_frame_size(uint16_t(std::min(max_frame_for_mtu(mtu, false), 0xffff)));
    return f;
}

// ---------------------------------------------------------------------------
// Agent
// ---------------------------------------------------------------------------
Agent::Agent(Config cfg, nl::NetOps& ops, std::unique_ptr<LldpSource> lldp, NmFactory nm_factory)
    : cfg_(std::move(cfg)), ops_(ops), lldp_(std::move(lldp)), nm_factory_(std::move(nm_factory)) {
    arp_probe = [this](std::vector<arp::Probe>& ps, int64_t timeout_ns, int64_t retry_ns, int stop_fd) {
        if (!arp_) arp_ = std::make_unique<arp::Prober>();
        return arp_->probe(ps, timeout_ns, retry_ns, stop_fd);
    };
}

void Agent::mark(const std::string& phase) {
    int64_t now = mono_ns();
    phases_[phase] = now - t_last_;
    t_last_ = now;
}

void Agent::pre_cleanups() {
    // Stale label from a previous (crashed) run: the node is not ready until we say so.
    if (path_exists(cfg_.labels.path())) {
        NLOG_I("NFD label file already exists, removing it...");
        if (!artifacts::remove_labels(cfg_.labels)) NLOG_W("Failed to remove NFD label file: %s", std::strerror(errno));
    }
    if (!cfg_.networkd.empty()) {
        try {
            mkdir_p(cfg_.networkd);
        } catch (const std::exception& e) {
            throw AgentError(std::string("Failed to pre-cleanup: Cannot create systemd-networkd directory: ") + e.what());
        }
        NLOG_I("Created systemd-networkd directory %s", cfg_.networkd.c_str());
    }
}

void Agent::disable_fw_lldp() {
    std::vector<ethtool::FlagRule> rules;
    try {
        rules = ethtool::parse_rules(cfg_.fw_lldp_flags);
    } catch (const std::exception& e) {
        throw AgentError(std::string("Invalid --fw-lldp-priv-flag: ") + e.what());
    }
    if (!ethtool_) {
        try {
            ethtool_ = ethtool::make_ioctl_ops();
        } catch (const std::exception& e) {
            NLOG_W("ethtool unavailable, firmware LLDP agents left alone: %s", e.what());
            return;
        }
    }
    // An earlier agent of this node (--keep-config) may have changed them already: its record
    // holds the real originals, which this run must neither lose nor take for "already set".
    // (Read without --keep-config too: an agent that failed left them changed, or the policy just
    // dropped keepConfigOnRestart; this agent then restores the true originals on a clean exit.)
    std::map<std::string, ethtool::FwLldpResult> earlier;
    if (!cfg_.fw_lldp_state.empty())
        if (auto t = read_file(cfg_.fw_lldp_state))
            for (auto& e : ethtool::decode_state(*t)) earlier[e.ifname] = e;
    for (auto& n : nics_) {
        auto r = ethtool::disable_fw_lldp(*ethtool_, n.ifname, rules, true, cfg_.fw_lldp_dcbx_host);
        n.fw_lldp = r.summary();
        if (r.dcbx) n.dcbx = ethtool::dcbx_str(*r.dcbx);
        n.dcbx_embedded = r.dcbx && ethtool::dcbx_embedded(*r.dcbx) && !r.dcbx_changed;
        if (!r.error.empty()) NLOG_W("%s: firmware LLDP: %s", n.ifname.c_str(), r.error.c_str());
        NLOG_V(2, "%s: driver %s, firmware LLDP: %s", n.ifname.c_str(), r.driver.c_str(), n.fw_lldp.c_str());
        if (auto it = earlier.find(n.ifname); it != earlier.end()) {
            if (it->second.changed) {
                r.changed = true;
                r.original_bits = it->second.original_bits;
            }
            if (it->second.dcbx_changed) {
                r.dcbx_changed = true;
                r.dcbx = it->second.dcbx;
            }
            earlier.erase(it);
        }
        fw_lldp_.push_back(std::move(r));
    }
    // What is left of the record belongs to NICs this agent does not select any more: they are
    // not ours now, so their originals go back at once; one that cannot be reached (renamed,
    // gone) stays in the record for --cleanup.
    for (auto& [name, r] : earlier) {
        NLOG_I("%s: no longer selected; restoring its firmware LLDP settings", name.c_str());
        if (!ethtool::restore(*ethtool_, r)) fw_lldp_carried_.push_back(r);
    }
    save_fw_lldp_state();
}

void Agent::save_fw_lldp_state(bool with_current) {
    if (cfg_.fw_lldp_state.empty()) return;  // also without --keep-config: an agent that fails leaves them changed
    try {
        std::vector<ethtool::FwLldpResult> all;
        if (with_current) all = fw_lldp_;
        all.insert(all.end(), fw_lldp_carried_.begin(), fw_lldp_carried_.end());
        const std::string text = ethtool::encode_state(all);
        if (!text.empty())
            write_file_atomic(cfg_.fw_lldp_state, text);
        else if (::unlink(cfg_.fw_lldp_state.c_str()) != 0 && errno != ENOENT)
            NLOG_W("Could not remove %s: %s", cfg_.fw_lldp_state.c_str(), std::strerror(errno));
    } catch (const std::exception& e) {
        NLOG_W("Could not record the firmware LLDP originals in %s: %s", cfg_.fw_lldp_state.c_str(), e.what());
    }
}

void Agent::restore_fw_lldp_from_state() {
    // --cleanup: what --keep-config agents changed on this node's NICs, from their record.
    if (cfg_.fw_lldp_state.empty()) return;
    auto t = read_file(cfg_.fw_lldp_state);
    if (!t) return;
    auto recs = ethtool::decode_state(*t);
    if (!recs.empty() && !ethtool_) ethtool_ = ethtool::make_ioctl_ops();
    for (const auto& r : recs) {
        NLOG_I("%s: restoring the NIC's firmware LLDP settings%s%s", r.ifname.c_str(),
               r.changed ? strfmt(" (private flags 0x%x)", r.original_bits).c_str() : "",
               r.dcbx_changed ? (" (DCBX " + ethtool::dcbx_str(*r.dcbx) + ")").c_str() : "");
        ethtool::restore(*ethtool_, r);
    }
    if (::unlink(cfg_.fw_lldp_state.c_str()) != 0 && errno != ENOENT)
        NLOG_W("Could not remove %s: %s", cfg_.fw_lldp_state.c_str(), std::strerror(errno));
}

void Agent::post_cleanups() {
    NLOG_I("Clean up before exiting...");
    if (ethtool_ && !persist_fw_lldp()) {  // kept on the node for the next agent / --cleanup otherwise
        for (const auto& r : fw_lldp_) ethtool::restore(*ethtool_, r);
        if (!fw_lldp_.empty()) save_fw_lldp_state(false);  // only what could not be reached stays (normally: none)
    }
    if (cfg_.lldp_announce && cfg_.mode == "L3" && !cfg_.keep_config) {
        // Shutdown LLDPDU (TTL 0): the switch drops us from its neighbour table right away.
        for (auto& n : nics_) {
            if (!n.link.up()) continue;
            try {
                lldp_->announce(n.ifname, lldp::encode(make_node_frame(cfg_.node_name, n.ifname, n.link.mac, n.gpu_bdf, 0)));
            } catch (...) {
            }
        }
    }
    if (!artifacts::remove_labels(cfg_.labels)) NLOG_W("Failed to remove NFD label file: %s", std::strerror(errno));
    if (cfg_.keep_config) {
        // The next agent adopts addresses, routes and rail rules; jobs keep their links meanwhile.
        NLOG_I("Keeping addresses, routes and links for the next agent (--keep-config)");
        return;
    }
    NLOG_I("Restoring interfaces to original state...");
    remove_rail_routing();
    try {
        remove_existing_ips();
    } catch (const std::exception& e) {
        NLOG_W("Failed to remove any existing IPs from interfaces: %s", e.what());
    }
    if (cfg_.restore_mtu) restore_mtus();
    try {
        interfaces_restore_down();
    } catch (const std::exception& e) {
        NLOG_W("Failed to restore interfaces to original state: %s", e.what());
    }
    restore_network_manager();
}

namespace {
std::map<std::string, int> read_mtu_state(const std::string& path) {
    std::map<std::string, int> out;
    auto t = read_file(path);
    if (!t) return out;
    for (const auto& line : split(*t, '\n')) {
        auto f = split(trim(line), ' ');
        if (f.size() != 2 || f[0].empty() || f[0].size() > 15) continue;
        try {
            const int mtu = std::stoi(f[1]);
            if (mtu >= 68 && mtu <= 65535) out[f[0]] = mtu;
        } catch (const std::exception&) {
        }
    }
    return out;
}

void write_mtu_state(const std::string& path, const std::map<std::string, int>& m) {
    if (m.empty()) {
        if (::unlink(path.c_str()) != 0 && errno != ENOENT)
            NLOG_W("Could not remove %s: %s", path.c_str(), std::strerror(errno));
        return;
    }
    std::string t;
    for (const auto& [n, mtu] : m) t += n + " " + std::to_string(mtu) + "\n";
    write_file_atomic(path, t);
}
}  // namespace

void Agent::load_mtu_state() {
    // The first agent's view of each NIC is the original; a later (--keep-config) agent finds the
    // MTU it set itself, so the recorded value wins.
    if (!cfg_.restore_mtu || cfg_.mtu_state.empty()) return;
    auto m = read_mtu_state(cfg_.mtu_state);
    for (auto& n : nics_) {
        auto it = m.find(n.ifname);
        if (it == m.end())
            m[n.ifname] = n.orig_mtu;
        else
            n.orig_mtu = it->second;
    }
    try {
        write_mtu_state(cfg_.mtu_state, m);
    } catch (const std::exception& e) {
        NLOG_W("Could not record the NICs' MTUs in %s: %s", cfg_.mtu_state.c_str(), e.what());
    }
}

void Agent::restore_mtus() {
    // Host NICs are the node's general-purpose interfaces: the MTU they had goes back with the
    // agent (the reference, and amd-so, leave the scale-out rails at the policy's MTU).
    std::map<std::string, int> left = cfg_.mtu_state.empty() ? std::map<std::string, int>{}
                                                              : read_mtu_state(cfg_.mtu_state);
    for (auto& n : nics_) {
        if (n.orig_mtu <= 0) continue;
        bool ok = n.link.mtu == n.orig_mtu;
        if (!ok) {
            try {
                ops_.link_set_mtu(n.link.index, n.orig_mtu);
                NLOG_I("Setting MTU of '%s' back to %d", n.ifname.c_str(), n.orig_mtu);
                n.link.mtu = n.orig_mtu;
                ok = true;
            } catch (const std::exception& e) {
                NLOG_W("Cannot set MTU of '%s' back to %d: %s", n.ifname.c_str(), n.orig_mtu, e.what());
            }
        }
        if (ok) left.erase(n.ifname);
    }
    if (!cfg_.mtu_state.empty()) {
        try {
            write_mtu_state(cfg_.mtu_state, left);  // what could not be put back stays for --cleanup
        } catch (const std::exception& e) {
            NLOG_W("Could not update %s: %s", cfg_.mtu_state.c_str(), e.what());
        }
    }
}

void Agent::restore_mtu_state() {
    if (!cfg_.restore_mtu || cfg_.mtu_state.empty()) return;
    auto m = read_mtu_state(cfg_.mtu_state);
    std::map<std::string, int> left;
    for (const auto& [name, mtu] : m) {
        try {
            auto l = ops_.link_by_name(name);
            if (l.mtu != mtu) {
                ops_.link_set_mtu(l.index, mtu);
                NLOG_I("Setting MTU of '%s' back to %d", name.c_str(), mtu);
            }
        } catch (const std::exception& e) {
            NLOG_W("Cannot set MTU of '%s' back to %d: %s", name.c_str(), mtu, e.what());
            left[name] = mtu;
        }
    }
    write_mtu_state(cfg_.mtu_state, left);
}

void Agent::restore_network_manager() {
    // Only with --nm-restore: the reference leaves its runtime Managed=false behind, and this
    // agent's keyfile keeps the NICs unmanaged across agent restarts and reboots (Config::nm_restore).
    if (!cfg_.nm_restore) return;
    if (nm_keyfile_written_ && nm::remove_keyfile(cfg_.nm_keyfile_dir, nm::keyfile_name(cfg_.labels.file))) {
        NLOG_I("Removed NetworkManager keyfile from %s", cfg_.nm_keyfile_dir.c_str());
        nm_keyfile_written_ = false;
    }
    if (nm_unmanaged_.empty()) return;
    try {
        auto nmapi = nm_factory_();
        nm::restore_for_interfaces(*nmapi, nm_unmanaged_);
        nm_unmanaged_.clear();
    } catch (const std::exception& e) {
        NLOG_W("Could not hand the interfaces back to NetworkManager: %s", e.what());
    }
}

std::vector<std::string> Agent::collect_interfaces(bool quiet) {
    std::string root = cfg_.sysfs_root.empty() ? topo::sysfs_root() : cfg_.sysfs_root;
    disc_ = topo::discover(cfg_.discovery, root);
    excluded_ = disc_.excluded;
    if (!quiet)
        for (const auto& [name, why] : disc_.excluded) NLOG_I("Leaving '%s' alone: %s", name.c_str(), why.c_str());
    if (cfg_.discovery.mode == topo::DiscoveryMode::Rdma) {
        // Host RDMA NICs: never the node's own management / frontend NICs.  A NIC --interfaces
        // names explicitly is the operator's choice (below), except for the default route.
        std::vector<std::string> kept;
        for (const auto& name : disc_.ifnames) {
            std::string why;
            try {
                why = node_owned_reason(ops_.link_by_name(name));
            } catch (const AgentError&) {
                throw;
            } catch (const std::exception&) {  // not in this namespace: reported as missing later
            }
            if (why.empty()) {
                kept.push_back(name);
                continue;
            }
            if (!quiet) NLOG_I("Leaving '%s' alone: it %s", name.c_str(), why.c_str());
            excluded_.emplace_back(name, "the node's own NIC: it " + why);
        }
        disc_.ifnames = kept;
    }
    std::vector<std::string> names = disc_.ifnames;
    for (auto& p : disc_.pairs) {
        if (quiet) break;
        const auto& g = disc_.gpus[size_t(p.gpu)];
        const auto& n = disc_.nics[size_t(p.nic)];
        NLOG_I("GPU %d (%s) <-> NIC %s (%s, %s, path %s)", g.index, g.pci.bdf.c_str(), n.ifname.c_str(), n.pci.bdf.c_str(),
               n.rdma_dev.empty() ? "no rdma" : n.rdma_dev.c_str(), topo::to_string(p.path));
    }
    if (!cfg_.interfaces.empty()) {
        for (auto& i : split(cfg_.interfaces, ',')) {
            auto t = trim(i);
            if (t.empty()) continue;
            if (std::find(names.begin(), names.end(), t) == names.end()) names.push_back(t);  // dedupe
        }
    }
    return names;
}

void Agent::get_network_configs(const std::vector<std::string>& names) {
    nics_.clear();
    for (auto& name : names) {
        NicState n;
        n.ifname = name;
        try {
            n.link = ops_.link_by_name(name);
        } catch (const std::exception& e) {
            NLOG_W("Link '%s' not found: %s", name.c_str(), e.what());
            continue;
        }
        n.orig_flags = n.link.flags;
        n.orig_mtu = n.link.mtu;
        for (auto& p : disc_.pairs) {
            const auto& nic = disc_.nics[size_t(p.nic)];
            if (nic.ifname != name) continue;
            n.gpu_index = disc_.gpus[size_t(p.gpu)].index;
            n.gpu_bdf = disc_.gpus[size_t(p.gpu)].pci.bdf;
            n.rdma_dev = nic.rdma_dev;
            n.rdma_port = nic.rdma_port;
            n.numa_node = disc_.gpus[size_t(p.gpu)].pci.numa;
            n.pcie_path = topo::to_string(p.path);
        }
        if (n.rdma_dev.empty())  // host NICs (rdma discovery): no GPU, but still an RDMA device
            for (auto& nic : disc_.nics)
                if (nic.ifname == name) {
                    n.rdma_dev = nic.rdma_dev;
                    n.rdma_port = nic.rdma_port;
                    n.numa_node = nic.pci.numa;
                }
        nics_.push_back(std::move(n));
    }
    assign_rail_indices();
}

void Agent::interfaces_up() {
    auto watcher = ops_.subscribe_links();
    for (auto& n : nics_) {
        n.expect_response = false;
        if (n.link.up()) continue;
        try {
            ops_.link_set_up(n.link.index);
            n.expect_response = true;
        } catch (const std::exception& e) {
            NLOG_W("Cannot set link '%s' up: %s", n.ifname.c_str(), e.what());
        }
    }
    // Wait for the RTM_NEWLINK echoes (network.go:242-257); a timeout is not fatal.
    int64_t deadline = mono_ns() + cfg_.link_wait_ns;
    auto pending = [&] {
        return std::any_of(nics_.begin(), nics_.end(), [](const NicState& n) { return n.expect_response; });
    };
    while (pending()) {
        auto evs = watcher->wait(deadline);
        if (evs.empty() && mono_ns() >= deadline) break;
        for (auto& ev : evs) {
            if (ev.deleted) continue;
            for (auto& n : nics_) {
                if (n.link.index == ev.link.index && n.expect_response) {
                    n.link.flags = ev.link.flags;
                    n.link.operstate = ev.link.operstate;
                    if (n.link.up()) n.expect_response = false;
                }
            }
        }
    }
    for (auto& n : nics_) {
        if (!n.expect_response) continue;
        NLOG_W("timeout waiting for netlink reply for '%s'", n.ifname.c_str());
        try {  // re-read: the echo may have been lost in an overrun
            auto l = ops_.link_by_name(n.ifname);
            n.link.flags = l.flags;
        } catch (...) {
        }
        n.expect_response = false;
    }
}

void Agent::interfaces_restore_down() {
    std::unique_ptr<nl::LinkWatcher> watcher;
    std::string subscribe_err;
    try {
        watcher = ops_.subscribe_links();
    } catch (const std::exception& e) {
        subscribe_err = e.what();
    }
    for (auto& n : nics_) {
        n.expect_response = false;
        if (!(n.orig_flags & IFF_UP) && n.link.up()) {
            try {
                ops_.link_set_down(n.link.index);
                NLOG_I("Setting link '%s' back down", n.ifname.c_str());
                n.expect_response = true;
            } catch (const std::exception& e) {
                NLOG_W("Cannot set link '%s' back down: %s", n.ifname.c_str(), e.what());
            }
        }
    }
    if (!subscribe_err.empty()) throw AgentError(subscribe_err);
    int64_t deadline = mono_ns() + cfg_.link_wait_ns;
    while (std::any_of(nics_.begin(), nics_.end(), [](const NicState& n) { return n.expect_response; })) {
        auto evs = watcher->wait(deadline);
        if (evs.empty() && mono_ns() >= deadline) break;
        for (auto& ev : evs)
            for (auto& n : nics_)
                if (n.link.index == ev.link.index && n.expect_response && !(ev.link.flags & IFF_UP)) {
                    n.link.flags = ev.link.flags;
                    n.expect_response = false;
                }
    }
    for (auto& n : nics_) {
        if (n.expect_response) n.link.flags &= ~unsigned(IFF_UP);
        n.expect_response = false;
    }
}

void Agent::interfaces_set_mtu() {
    for (auto& n : nics_) {
        if (n.link.mtu == cfg_.mtu) continue;  // already right: skip the netlink round trip
        try {
            ops_.link_set_mtu(n.link.index, cfg_.mtu);
            n.link.mtu = cfg_.mtu;
        } catch (const std::exception& e) {
            NLOG_W("Could not set MTU %d for interface '%s': %s", cfg_.mtu, n.ifname.c_str(), e.what());
        }
    }
}

void Agent::remove_existing_ips(const std::map<std::string, Ipv4Prefix>& keep) {
    for (auto& n : nics_) {
        auto k = keep.find(n.ifname);
        auto addrs = ops_.addr_list(n.link.index, AF_INET);
        for (auto& a : addrs) {
            if (k != keep.end() && a.local == k->second.addr && a.prefixlen == k->second.len) {
                NLOG_I("Interface '%s': keeping %s from the previous agent (--keep-config)", n.ifname.c_str(),
                       a.prefix().str().c_str());
                continue;
            }
            ops_.addr_del(a);
        }
    }
}

std::map<std::string, Ipv4Prefix> Agent::cached_addresses() const {
    // The same validity rules as apply_lldp_cache: this NIC (name and MAC), not too old, parses.
    std::map<std::string, Ipv4Prefix> out;
    if (cfg_.lldp_cache.empty()) return out;
    const int64_t now = int64_t(::time(nullptr));
    for (const auto& e : artifacts::read_lldp_cache(cfg_.lldp_cache)) {
        for (const auto& n : nics_) {
            if (e.ifname != n.ifname || e.nic_mac != n.link.mac.str()) continue;
            if (now - e.unix_s > cfg_.lldp_cache_max_age_ns / 1000000000 || e.unix_s > now + 60) continue;
            if (auto addr = l3::parse_port_description(e.port_description, cfg_.token_policy, nullptr))
                out[n.ifname] = addr->local_prefix();
        }
    }
    return out;
}

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
    if (std::string why = check_link_speed(n); !why.empty()) {
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
            // The kernel adds the /30 connected route along with the address.
            ops_.addr_add(n.link.index, n.addr->local_prefix());
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

void Agent::write_l2_artifacts() {
    std::string root = cfg_.sysfs_root.empty() ? topo::sysfs_root() : cfg_.sysfs_root;
    for (auto& n : nics_) n.configured = n.link.up() && !n.no_carrier && n.config_error.empty();
    const int64_t deadline = mono_ns() + cfg_.gid_wait_ns;
    for (;;) {
        bool missing = false;
        for (auto& n : nics_) {
            if (n.rdma_dev.empty() || !n.configured || n.gid_index) continue;
            n.gid_index = topo::find_rocev2_linklocal_gid_index(root, n.rdma_dev, n.rdma_port);
            missing |= !n.gid_index;
        }
        if (!missing || mono_ns() >= deadline) break;
        ::usleep(2000);
    }
    write_rccl_env_file();
}

void Agent::dry_run_report() {
    if (cfg_.mode == "L3" && cfg_.disable_fw_lldp) {
        // What --disable-fw-lldp would change (read-only: private flags, DCBX mode).
        std::vector<ethtool::FlagRule> rules;
        try {
            rules = ethtool::parse_rules(cfg_.fw_lldp_flags);
            if (!ethtool_) ethtool_ = ethtool::make_ioctl_ops();
            for (auto& n : nics_) {
                auto r = ethtool::disable_fw_lldp(*ethtool_, n.ifname, rules, false, cfg_.fw_lldp_dcbx_host);
                n.fw_lldp = r.summary();
                if (r.dcbx) {
                    n.dcbx = ethtool::dcbx_str(*r.dcbx);
                    n.dcbx_embedded = ethtool::dcbx_embedded(*r.dcbx);
                }
                NLOG_I("dry run: %s (%s): firmware LLDP: %s", n.ifname.c_str(), r.driver.empty() ? "?" : r.driver.c_str(),
                       n.fw_lldp.c_str());
            }
        } catch (const std::exception& e) {
            NLOG_W("dry run: firmware LLDP not inspected: %s", e.what());
        }
    }
    // NICs refuse_uplinks() recorded: a real start would fail on them, and touch nothing.
    std::set<std::string> refused;
    for (const auto& [name, why] : excluded_)
        if (why.size() >= 9 && why.compare(why.size() - 9, 9, "(refused)") == 0) refused.insert(name);
    for (const auto& n : nics_) {
        NLOG_I("dry run: %s (%s, mtu %d -> %d, %s): GPU %d %s, RDMA %s, path %s%s", n.ifname.c_str(),
               n.link.up() ? "up" : "down", n.link.mtu, cfg_.mtu, n.link.mac.str().c_str(), n.gpu_index,
               n.gpu_bdf.empty() ? "-" : n.gpu_bdf.c_str(), n.rdma_dev.empty() ? "-" : n.rdma_dev.c_str(),
               n.pcie_path.empty() ? "-" : n.pcie_path.c_str(), refused.count(n.ifname) ? " -- REFUSED" : "");
    }
    if (!cfg_.rccl_topo.empty()) {
        start_topo();
        const std::string env = write_topo();
        mark("rccl_topo");
        NLOG_I("dry run: NCCL_TOPO_FILE %s (%zu bytes)%s", cfg_.rccl_topo.c_str(), topo_xml().size(),
               env.empty() ? " not written" : "");
    }
    if (!cfg_.rccl_env.empty()) {
        // The intra-node part of rccl.env: NCCL_TOPO_FILE and the site settings.  Nothing was
        // configured, so no HCA, GID or socket interface is named (a job on this node could not
        // use them yet); bench.py and validate.py apply exactly this file to their RCCL runs.
        write_rccl_env_file();
        NLOG_I("dry run: RCCL environment file %s", cfg_.rccl_env.c_str());
    }
    write_status();
    if (!refused.empty())
        NLOG_W("dry run: a real start would fail: refusing %s (the node's default route); nothing was changed",
               join(std::vector<std::string>(refused.begin(), refused.end()), ", ").c_str());
    else
        NLOG_I("dry run: %zu interface(s) would be configured in %s mode; nothing was changed", nics_.size(),
               cfg_.mode.c_str());
}

namespace {
// Everything the file is generated from that can change without a reboot: the generator, the
// GPUs and the NICs (name, PCI function, RDMA device).  The PCIe tree above them is fixed until
// the next boot, hence the boot id.
std::string topo_fingerprint(const topo::DiscoveryResult& disc, const std::vector<std::string>& names,
                             const std::string& root) {
    std::string fp = strfmt("netop-rccl-topo v%d\n", artifacts::kRcclTopoXmlVersion);
    auto boot = read_file("/proc/sys/kernel/random/boot_id");
    fp += "boot " + (boot ? trim(*boot) : std::string("?")) + "\nroot " + root + "\n";
    for (const auto& g : disc.gpus) fp += "gpu " + g.pci.path + "\n";
    for (const auto& n : names) {
        std::string where = "-";
        for (const auto& d : disc.nics)
            if (d.ifname == n) where = d.pci.path + " " + d.rdma_dev + ":" + std::to_string(d.rdma_port);
        fp += "nic " + n + " " + where + "\n";
    }
    return fp;
}

// The interface names the agent works on: discovery's, then --interfaces (collect_interfaces).
std::vector<std::string> topo_names(const topo::DiscoveryResult& disc, const std::string& interfaces) {
    std::vector<std::string> names = disc.ifnames;
    for (auto& i : split(interfaces, ',')) {
        auto t = trim(i);
        if (!t.empty() && std::find(names.begin(), names.end(), t) == names.end()) names.push_back(t);
    }
    return names;
}

// The whole job of the topology worker: the file a previous run of this boot left (same inputs),
// or a fresh sysfs walk above the discovered GPUs and NICs.
Agent::TopoResult make_topology(const topo::DiscoveryResult& disc, const std::string& interfaces,
                                const std::string& root, const std::string& path) {
    Agent::TopoResult r;
    r.names = topo_names(disc, interfaces);
    r.fp = topo_fingerprint(disc, r.names, root);
    auto key = read_file(path + ".key");
    if (key && *key == r.fp) {
        if (auto xml = read_file(path); xml && !xml->empty()) {
            r.xml = *xml;
            r.reused = true;
            return r;
        }
    }
    r.xml = artifacts::generate_rccl_topo(disc.gpus, artifacts::topo_nics(disc, r.names, root), topo::cpu_identity(),
                                          root);
    return r;
}
}  // namespace

void Agent::start_topo() {
    if (cfg_.rccl_topo.empty() || topo_future_.valid() || topo_) return;
    std::string root = cfg_.sysfs_root.empty() ? topo::sysfs_root() : cfg_.sysfs_root;
    // Inputs are copied: the worker shares nothing with the agent thread.
    const int main_cpu = ::sched_getcpu();
    auto work = [disc = disc_, interfaces = cfg_.interfaces, root = std::move(root), path = cfg_.rccl_topo,
                 main_cpu](bool background) {
        if (!background) return make_topology(disc, interfaces, root, path);  // on the agent thread
        // Off the agent thread's CPU: at low priority on the same CPU it would only run when the
        // agent thread blocks (measured: the join then waited ~4 ms in L3).
        cpu_set_t set;
        if (main_cpu >= 0 && ::sched_getaffinity(0, sizeof set, &set) == 0 && CPU_COUNT(&set) > 1) {
            CPU_CLR(main_cpu, &set);
            (void)::sched_setaffinity(0, sizeof set, &set);
        }
        // Background priority: on a busy or CPU-limited node the critical path (discovery,
        // link-up, LLDP) runs first and this fills its gaps instead of competing with it.
        // nice 19 under SCHED_OTHER, not SCHED_IDLE: the agent never has to raise it again
        // (leaving SCHED_IDLE or lowering a nice value needs CAP_SYS_NICE, which the DaemonSet
        // does not grant), and when the agent thread blocks on the result this thread gets the
        // whole CPU quota of the container anyway.  Measured in the netns harness, 8 NICs, L3:
        // total_ready +5.6 ms over no topology file at normal priority, +1 ms at idle priority.
        if (::setpriority(PRIO_PROCESS, pid_t(::syscall(SYS_gettid)), 19) != 0)
            NLOG_V(2, "topology worker: setpriority(19): %s", std::strerror(errno));
        return make_topology(disc, interfaces, root, path);
    };
    try {
        topo_future_ = std::async(std::launch::async, work, true);
    } catch (const std::system_error& e) {  // no thread to spare: generate it when it is needed
        NLOG_V(2, "topology worker thread unavailable (%s): generating on demand", e.what());
        topo_future_ = std::async(std::launch::deferred, work, false);
    }
}

const std::string& Agent::topo_xml() {
    if (!topo_) {
        if (!topo_future_.valid()) start_topo();
        try {
            topo_ = topo_future_.get();
            // The worker's interface list is the agent's (same discovery); kept as a guard.
            std::vector<std::string> mine = topo_names(disc_, cfg_.interfaces);
            if (topo_->names != mine) {
                NLOG_I("Interfaces changed while the topology file was generated: generating it again");
                std::string root = cfg_.sysfs_root.empty() ? topo::sysfs_root() : cfg_.sysfs_root;
                topo_->names = mine;
                topo_->fp = topo_fingerprint(disc_, mine, root);
                topo_->xml = artifacts::generate_rccl_topo(disc_.gpus, artifacts::topo_nics(disc_, mine, root),
                                                           topo::cpu_identity(), root);
                topo_->reused = false;
            } else if (topo_->reused) {
                NLOG_V(2, "RCCL topology file %s is current (same boot and devices): reused", cfg_.rccl_topo.c_str());
            }
        } catch (const std::exception& e) {
            NLOG_E("Error generating the RCCL topology file: %s", e.what());
            topo_ = TopoResult{};
        }
    }
    return topo_->xml;
}

std::string Agent::write_topo() {
    if (cfg_.rccl_topo.empty()) return "";
    const std::string& xml = topo_xml();
    if (xml.empty()) return "";  // rccl.env then names no topology
    if (!topo_->reused) {
        try {
            ::unlink((cfg_.rccl_topo + ".key").c_str());  // never a key next to a file it does not describe
            write_file_atomic(cfg_.rccl_topo, xml, 0644);
            if (!topo_->fp.empty()) write_file_atomic(cfg_.rccl_topo + ".key", topo_->fp, 0644);
        } catch (const std::exception& e) {
            NLOG_E("Error writing RCCL topology file: %s", e.what());
            return "";
        }
        topo_->reused = true;  // written: later refreshes (re-addressing) keep it
    }
    return cfg_.rccl_topo_env_path.empty() ? cfg_.rccl_topo : cfg_.rccl_topo_env_path;
}

std::vector<std::string> Agent::socket_ifnames() const {
    const std::string& s = cfg_.socket_ifname;
    if (s.empty() || s == "none") return {};
    if (s != "auto") {
        std::vector<std::string> out;
        for (auto& i : split(s, ','))
            if (!trim(i).empty()) out.push_back(trim(i));
        return out;
    }
    if (cfg_.mode != "L3") return {};
    std::vector<const NicState*> v;
    for (const auto& n : nics_)
        if (n.configured && n.addr) v.push_back(&n);
    std::stable_sort(v.begin(), v.end(), [](const NicState* a, const NicState* b) {
        int ga = a->gpu_index < 0 ? 1 << 30 : a->gpu_index, gb = b->gpu_index < 0 ? 1 << 30 : b->gpu_index;
        return ga != gb ? ga < gb : a->ifname < b->ifname;
    });
    std::vector<std::string> out;
    for (const NicState* n : v) out.push_back(n->ifname);
    return out;
}

void Agent::write_rccl_env_file() {
    const std::string topo_env = write_topo();
    if (cfg_.rccl_env.empty()) return;
    try {
        artifacts::write_rccl_env(cfg_.rccl_env, nics_, topo_env, rccl_env_extra_, socket_ifnames(), cfg_.mode != "L3");
    } catch (const std::exception& e) {
        NLOG_E("Error writing RCCL env: %s", e.what());
    }
}

void Agent::write_artifacts() {
    std::string root = cfg_.sysfs_root.empty() ? topo::sysfs_root() : cfg_.sysfs_root;
    // Poll all configured RDMA NICs together until each has its RoCE v2 GID or the wait ends.
    const int64_t gid_deadline = mono_ns() + cfg_.gid_wait_ns;
    for (;;) {
        bool missing = false;
        for (auto& n : nics_) {
            if (n.rdma_dev.empty() || !n.addr || !n.configured || n.gid_index) continue;
            n.gid_index = topo::find_rocev2_gid_index(root, n.rdma_dev, n.rdma_port, n.addr->local);
            missing |= !n.gid_index;
        }
        if (!missing || mono_ns() >= gid_deadline) break;
        ::usleep(2000);
    }
    for (auto& n : nics_)
        if (!n.rdma_dev.empty() && n.addr && n.configured && !n.gid_index)
            NLOG_W("%s (%s): no RoCE v2 GID for %s after %s; rccl.env gets no NCCL_IB_GID_INDEX for it",
                   n.ifname.c_str(), n.rdma_dev.c_str(), n.addr->local.str().c_str(),
                   format_go_duration(cfg_.gid_wait_ns).c_str());
    if (!cfg_.rccl_net.empty()) {
        try {
            artifacts::write_rccl_net(cfg_.rccl_net, nics_);
        } catch (const std::exception& e) {
            NLOG_E("Error: %s", e.what());  // not fatal (main.go:220-224)
        }
    }
    write_rccl_env_file();
}

void Agent::write_host_config() {
    // What the node needs after a reboot or an agent restart, not what a job needs now: written
    // after the readiness label, off the node-ready critical path.
    save_lldp_cache();
    if (!cfg_.networkd.empty()) {
        try {
            artifacts::write_networkd(cfg_.networkd, nics_);
        } catch (const std::exception& e) {
            throw AgentError(std::string("Could not create systemd-networkd configuration files: ") + e.what());
        }
    }
}

void Agent::check_xgmi() {
    if (cfg_.xgmi_expect_links < 0) return;
    std::string root = cfg_.sysfs_root.empty() ? topo::sysfs_root() : cfg_.sysfs_root;
    xgmi_ = topo::read_xgmi(root);
    int expect = cfg_.xgmi_expect_links == 0 ? xgmi_.pairs_expected : cfg_.xgmi_expect_links;
    NLOG_I("xGMI: %zu GPUs, %d/%d GPU pairs linked, %llu MB/s per GPU advertised", xgmi_.gpus.size(), xgmi_.pairs_connected,
           xgmi_.pairs_expected, (unsigned long long)xgmi_.per_gpu_bw_mbs());
    for (auto& [a, b] : xgmi_.missing) NLOG_W("xGMI: no link between %s and %s", a.c_str(), b.c_str());
    if (xgmi_.pairs_connected < expect)
        throw AgentError(strfmt("xGMI mesh incomplete: %d of %d GPU pairs linked", xgmi_.pairs_connected, expect));
}

std::map<std::string, std::string> Agent::status_node() const {
    std::map<std::string, std::string> m;
    if (!cfg_.node_name.empty()) m["node"] = cfg_.node_name;
    if (!gdr_.kernel.empty()) {
        m["gpudirect_rdma"] = gdr_.mode();
        m["kernel"] = gdr_.kernel;
    }
    if (cfg_.xgmi_expect_links >= 0)
        m["xgmi_pairs"] = std::to_string(xgmi_.pairs_connected) + "/" + std::to_string(xgmi_.pairs_expected);
    if (cpu_ms_at_ready_ >= 0) m["cpu_ms_at_ready"] = strfmt("%.3f", cpu_ms_at_ready_);
    if (!excluded_.empty()) {
        std::vector<std::string> parts;
        for (const auto& [n, why] : excluded_) parts.push_back(n + ": " + why);
        m["excluded"] = join(parts, "; ");
    }
    if (cfg_.dry_run) {
        m["dry_run"] = "true";
        if (!dry_run_missing_.empty()) m["not_in_netns"] = join(dry_run_missing_, ",");
    }
    return m;
}

void Agent::check_gdr() {
    std::string root = cfg_.sysfs_root.empty() ? topo::sysfs_root() : cfg_.sysfs_root;
    gdr_ = topo::detect_gdr(root);
    NLOG_I("GPUDirect RDMA: %s (peer-memory %s, ib_uverbs %s, kernel %s)", gdr_.mode().c_str(),
           gdr_.peer_mem ? gdr_.peer_mem_version.c_str() : "absent", gdr_.ib_uverbs ? "loaded" : "absent",
           gdr_.kernel.c_str());
    const std::string& want = cfg_.require_gdr;
    if (want.empty()) return;
    bool ok = want == "any" ? gdr_.mode() != "none" : want == "peermem" ? gdr_.peer_mem : want == "dmabuf" ? gdr_.dmabuf : false;
    if (want != "any" && want != "peermem" && want != "dmabuf") throw AgentError("Invalid --require-gdr '" + want + "'");
    if (!ok)
        throw AgentError("GPUDirect RDMA unavailable (" + gdr_.mode() + ", required: " + want +
                         "): RCCL would stage inter-node traffic through host memory");
}

void Agent::log_results() {
    for (auto& n : nics_) {
        NLOG_V(3, "Interface '%s' %s:", n.ifname.c_str(), n.link.flags_str().c_str());
        std::string s = "\tConfigured addresses: ";
        std::vector<nl::AddrInfo> addrs;
        try {
            addrs = ops_.addr_list(n.link.index, AF_UNSPEC);
        } catch (...) {
        }
        if (addrs.empty()) s += "no addresses";
        for (auto& a : addrs) {
            s += a.prefix().str();
            if (n.addr && a.local == n.addr->local) s += "(matches lldp)";
            s += " ";
        }
        NLOG_V(3, "%s", s.c_str());
        if (cfg_.mode == "L3") {
            NLOG_V(3, "\tPeer MAC address: %s", n.peer_mac ? n.peer_mac->str().c_str() : "none");
            NLOG_V(3, "\tPeer LLDP address: %s", n.addr ? n.addr->peer.str().c_str() : "none");
            NLOG_V(3, "\tLocal /30 LLDP address: %s", n.addr ? n.addr->local.str().c_str() : "none");
        }
    }
}

int Agent::metrics_port() const { return httpd_ ? httpd_->port() : 0; }

std::string Agent::render_metrics() const {
    std::string o;
    auto metric = [&](const char* name, const char* type, const char* help) {
        o += strfmt("# HELP %s %s\n# TYPE %s %s\n", name, help, name, type);
    };
    metric("netop_agent_ready", "gauge", "1 while the scale-out readiness label is published");
    o += strfmt("netop_agent_ready{mode=\"%s\"} %d\n", cfg_.mode.c_str(), ready_ ? 1 : 0);
    metric("netop_agent_nic_configured", "gauge", "1 when the NIC carries its LLDP-derived /30 and routes (L3) / is up (L2)");
    for (auto& n : nics_)
        o += strfmt("netop_agent_nic_configured{nic=\"%s\",gpu=\"%s\",rdma=\"%s\"} %d\n",
                    httpd::escape_label(n.ifname).c_str(), n.gpu_bdf.c_str(), n.rdma_dev.c_str(),
                    (n.configured && (cfg_.mode == "L3" || n.link.up())) ? 1 : 0);
    if (!excluded_.empty()) {
        // Discovered but left alone (the node's own NICs, another agent's rails): one series per
        // NIC with the kind of reason, so a fleet view shows which nodes hold back which NICs.
        metric("netop_agent_nic_left_alone", "gauge", "1 for a discovered NIC this agent does not configure, by reason");
        for (const auto& [nic, why] : excluded_) {
            const char* kind = why.find("scale-out rail") != std::string::npos    ? "gpu_rail"
                               : why.find("default route") != std::string::npos   ? "default_route"
                               : why.find("is a port of") != std::string::npos    ? "bond_or_bridge_port"
                               : why.find(", which ") != std::string::npos        ? "stacked_device"
                               : why.find("IPv6 address") != std::string::npos    ? "ipv6_address"
                               : why.find("an address the agent") != std::string::npos ? "address"
                               : why.find("has the route") != std::string::npos   ? "route"
                                                                                  : "other";
            o += strfmt("netop_agent_nic_left_alone{nic=\"%s\",reason=\"%s\"} 1\n", httpd::escape_label(nic).c_str(), kind);
        }
    }
    metric("netop_agent_nic_degraded", "gauge", "1 while the NIC has lost link after readiness");
    for (auto& n : nics_)
        o += strfmt("netop_agent_nic_degraded{nic=\"%s\"} %d\n", httpd::escape_label(n.ifname).c_str(), n.degraded ? 1 : 0);
    if (cfg_.mode == "L2") {
        metric("netop_agent_nic_carrier", "gauge",
               "L2: the NIC's carrier state -- 1 up, 0.5 still training within --carrier-wait, 0 no carrier after it");
        for (auto& n : nics_)
            o += strfmt("netop_agent_nic_carrier{nic=\"%s\"} %s\n", httpd::escape_label(n.ifname).c_str(),
                        n.awaiting_carrier ? "0.5" : (n.no_carrier || !n.link.lower_up()) ? "0" : "1");
    }
    if (cfg_.min_link_speed_mbps > 0) {
        metric("netop_agent_nic_speed_mbps", "gauge", "Negotiated link speed of the NIC (checked against --min-link-speed-gbps)");
        for (const auto& n : nics_)
            if (n.speed_mbps >= 0)
                o += strfmt("netop_agent_nic_speed_mbps{nic=\"%s\"} %lld\n", httpd::escape_label(n.ifname).c_str(),
                            (long long)n.speed_mbps);
    }
    metric("netop_agent_link_flaps_total", "counter", "link losses observed after readiness");
    o += strfmt("netop_agent_link_flaps_total %d\n", flaps_);
    metric("netop_agent_reconfigurations_total", "counter", "NIC re-addressings after a Port Description change");
    o += strfmt("netop_agent_reconfigurations_total %d\n", reconfigs_);
    if (cfg_.mode == "L3") {
        metric("netop_agent_lldp_silent", "gauge",
               "1 when the LLDP wait expired without a frame on the NIC (driver: its PCI driver)");
        for (auto& n : nics_)
            o += strfmt("netop_agent_lldp_silent{nic=\"%s\",driver=\"%s\"} %d\n", httpd::escape_label(n.ifname).c_str(),
                        httpd::escape_label(n.driver).c_str(), n.lldp_silent.empty() ? 0 : 1);
        bool any_dcbx = false;
        for (auto& n : nics_) any_dcbx |= !n.dcbx.empty();
        if (any_dcbx) {
            metric("netop_agent_dcbx_embedded", "gauge",
                   "1 when an agent embedded in the NIC runs DCBX (and LLDP) on it; NICs whose DCBX mode was read");
            for (auto& n : nics_)
                if (!n.dcbx.empty())
                    o += strfmt("netop_agent_dcbx_embedded{nic=\"%s\"} %d\n", httpd::escape_label(n.ifname).c_str(),
                                n.dcbx_embedded ? 1 : 0);
        }
    }
    auto st = lldp_ ? lldp_->stats() : pkt::ListenerStats{};
    metric("netop_agent_lldp_frames_total", "counter", "LLDP frames received, by outcome");
    o += strfmt("netop_agent_lldp_frames_total{outcome=\"accepted\"} %llu\n", (unsigned long long)st.frames);
    o += strfmt("netop_agent_lldp_frames_total{outcome=\"own\"} %llu\n", (unsigned long long)st.own);
    o += strfmt("netop_agent_lldp_frames_total{outcome=\"malformed\"} %llu\n", (unsigned long long)st.malformed);
    metric("netop_agent_phase_seconds", "gauge", "duration of each bring-up phase");
    for (auto& [k, v] : phases_) o += strfmt("netop_agent_phase_seconds{phase=\"%s\"} %.9f\n", k.c_str(), double(v) / 1e9);
    if (!gdr_.kernel.empty()) {
        metric("netop_agent_gpudirect_rdma", "gauge", "GPUDirect RDMA mechanism available to RCCL (1 = this one)");
        for (const char* m : {"peermem", "dmabuf", "none"})
            o += strfmt("netop_agent_gpudirect_rdma{mode=\"%s\"} %d\n", m, gdr_.mode() == m ? 1 : 0);
    }
    if (cfg_.mode == "L3" && cfg_.verify_peers_ns > 0) {
        metric("netop_agent_peer_verified", "gauge", "1 when the NIC's switch-side /30 address answered ARP (--verify-peers)");
        for (auto& n : nics_)
            o += strfmt("netop_agent_peer_verified{nic=\"%s\"} %d\n", httpd::escape_label(n.ifname).c_str(),
                        n.peer_verified ? 1 : 0);
        metric("netop_agent_peer_arp_rtt_seconds", "gauge", "ARP round trip to the peer: last request to its answer");
        for (auto& n : nics_)
            if (n.peer_verified)
                o += strfmt("netop_agent_peer_arp_rtt_seconds{nic=\"%s\"} %.9f\n", httpd::escape_label(n.ifname).c_str(),
                            double(n.peer_rtt_ns) / 1e9);
        metric("netop_agent_peer_verify_seconds", "gauge", "time to verify the peer: first ARP request to its answer");
        for (auto& n : nics_)
            if (n.peer_verified)
                o += strfmt("netop_agent_peer_verify_seconds{nic=\"%s\"} %.9f\n", httpd::escape_label(n.ifname).c_str(),
                            double(n.peer_verify_ns) / 1e9);
        metric("netop_agent_peer_mac_mismatch", "gauge",
               "1 when the peer answered ARP from another MAC than its LLDP ChassisID/PortID MAC");
        for (auto& n : nics_)
            if (n.peer_verified)
                o += strfmt("netop_agent_peer_mac_mismatch{nic=\"%s\"} %d\n", httpd::escape_label(n.ifname).c_str(),
                            n.peer_mac_mismatch ? 1 : 0);
    }
    if (cfg_.xgmi_expect_links >= 0) {
        metric("netop_agent_xgmi_pairs", "gauge", "GPU pairs with an xGMI link (KFD topology)");
        o += strfmt("netop_agent_xgmi_pairs{state=\"connected\"} %d\n", xgmi_.pairs_connected);
        o += strfmt("netop_agent_xgmi_pairs{state=\"expected\"} %d\n", xgmi_.pairs_expected);
    }
    return o;
}

void Agent::write_status() {
    if (httpd_) {
        httpd_->set_metrics(render_metrics());
        httpd_->set_ready(ready_);
    }
    if (cfg_.status_file.empty()) return;
    try {
        write_file_atomic(cfg_.status_file, artifacts::generate_status(nics_, phases_, t0_, cfg_.mode, ready_, status_node()) + "\n");
        // Beside it, one line for the readiness probe to print while the node is not ready: the
        // kubelet records probe output in the Pod's events ("Readiness probe failed: ...").
        const std::string why = ready_ ? "" : not_ready_reason();
        if (why.empty())
            ::unlink(reason_path(cfg_.status_file).c_str());
        else
            write_file_atomic(reason_path(cfg_.status_file), why + "\n");
    } catch (const std::exception& e) {
        NLOG_W("Could not write status file: %s", e.what());
    }
}

std::string reason_path(const std::string& status_file) { return status_file + ".not-ready"; }

std::string Agent::not_ready_reason() const {
    if (!config_error_.empty()) return config_error_;
    std::vector<std::string> parts;
    for (const auto& n : nics_) {
        std::string why;
        if (n.degraded)
            why = "link down";
        else if (n.awaiting_carrier)
            why = "waiting for carrier";
        else if (n.no_carrier)
            why = "no carrier (check the cable, the switch port and the optic)";
        else if (!n.lldp_silent.empty())
            why = n.lldp_silent;
        else if (!n.config_error.empty())
            why = n.config_error;
        else if (!n.addr_error.empty() && !n.configured)
            why = n.addr_error;
        else if (n.cache_stale)
            why = "the switch has not confirmed the cached Port Description";
        else if (!n.peer_error.empty())
            why = n.peer_error;
        else if (cfg_.mode == "L3" && !n.configured)
            why = n.lldp_seen                           ? "not configured yet"
                  : n.link.up() && !n.link.lower_up() ? "waiting for carrier"  // no frame can come yet
                                                        : "waiting for LLDP";
        if (!why.empty()) parts.push_back(n.ifname + ": " + why);
    }
    return join(parts, "; ");
}

void Agent::run(int stop_fd) {
    t0_ = t_last_ = mono_ns();
    sanitize(cfg_);
    set_durable_writes(cfg_.fsync_artifacts);
    try {
        rccl_env_extra_ = artifacts::parse_env_extra(cfg_.rccl_env_extra);
    } catch (const std::exception& e) {
        throw AgentError(std::string("Invalid --rccl-env-extra: ") + e.what());
    }
    if (!cfg_.rail_switch_pattern.empty() && !cfg_.cleanup) {
        if (std::string why = rail_pattern_error(cfg_.rail_switch_pattern); !why.empty()) {
            // Admission checks the same grammar (webhook.validate_rail_switch_pattern); a policy
            // that bypassed it (webhooks off) gets one clear reason and an agent that touches
            // nothing and waits, not a crash loop on every selected node.
            config_error_ = "invalid railSwitchPattern '" + cfg_.rail_switch_pattern + "': " + why +
                            " (an ECMAScript regular expression, {rail} = the GPU index); nothing configured";
            NLOG_E("%s", config_error_.c_str());
            if (cfg_.dry_run || !cfg_.keep_running) throw AgentError(config_error_);
            // Our own stale label goes; but only the node lock's holder touches the label file:
            // when another agent of this configuration type holds it (a second policy selecting
            // this node), the label is that agent's, and it stays.  One attempt, no wait.
            bool owner = cfg_.node_lock.empty();
            if (!owner) {
                try {
                    node_lock_fd_ = take_lock("netop-agent:" + cfg_.node_lock, mono_ns(), -1, "Node lock '" + cfg_.node_lock + "'",
                                              "node lock held by another agent");
                    owner = true;
                } catch (const AgentError&) {
                    NLOG_I("Node lock '%s' is held by another agent: its label stays", cfg_.node_lock.c_str());
                }
            }
            if (owner && !artifacts::remove_labels(cfg_.labels))
                NLOG_W("Failed to remove NFD label file: %s", std::strerror(errno));
            write_status();
            idle(stop_fd);
            return;
        }
    }
    if (!cfg_.metrics_addr.empty() && !httpd_) {
        try {
            httpd_ = std::make_unique<httpd::Server>(cfg_.metrics_addr);
            NLOG_I("Serving metrics on %s (port %d)", cfg_.metrics_addr.c_str(), httpd_->port());
        } catch (const std::exception& e) {
            NLOG_W("metrics endpoint disabled: %s", e.what());
        }
        write_status();
    }
    if (!cfg_.dry_run) {
        acquire_node_lock(stop_fd);
        mark("node_lock");
        pre_cleanups();
    }

    auto names = collect_interfaces();
    if (names.empty() && !cfg_.dry_run && !cfg_.cleanup && cfg_.configure && cfg_.keep_running &&
        cfg_.discovery.mode == topo::DiscoveryMode::Rdma && !excluded_.empty()) {
        // host-nic: every RDMA NIC here is the node's own (default route, its addresses) or a GPU's
        // scale-out rail that an amd-so agent owns.  A steady state, not a fault: configure
        // nothing, publish no label, say so once (status file, readiness probe) and wait, instead
        // of the reference's exit for "no interfaces" (cmd/discover/main.go:171-179) and a crash
        // loop on every such node.  (amd-so / accel discovery keep failing: no NIC there is a fault.)
        std::vector<std::string> parts;
        for (const auto& [n, why] : excluded_) parts.push_back(n + ": " + why);
        config_error_ = "no host NIC of its own (left alone: " + join(parts, "; ") + ")";
        NLOG_W("Nothing to configure: %s", config_error_.c_str());
        mark("discover");
        write_status();
        if (idle_until_own_nic(stop_fd))
            NLOG_I("Exiting so that the restarted agent configures it");  // restartPolicy Always
        return;
    }
    if (names.empty()) {
        // A dry run still describes the GPUs and their xGMI mesh (the intra-node topology file a
        // job on a node without scale-out NICs uses); configuring needs NICs.
        if (!cfg_.dry_run || disc_.gpus.empty()) {
            std::vector<std::string> parts;
            for (const auto& [n, why] : excluded_) parts.push_back(n + ": " + why);
            throw AgentError("No interfaces found" + (parts.empty() ? "" : " (left alone: " + join(parts, "; ") + ")"));
        }
        NLOG_W("dry run: no scale-out interfaces found; describing the %zu GPU(s) and the xGMI mesh only",
               disc_.gpus.size());
    }
    get_network_configs(names);
    if (nics_.size() < names.size()) {
        if (!cfg_.dry_run) throw AgentError("Not all interfaces were found in the system");
        NLOG_W("dry run: %zu of %zu discovered interfaces are not in this network namespace", names.size() - nics_.size(),
               names.size());
        for (const auto& i : names)
            if (std::none_of(nics_.begin(), nics_.end(), [&](const NicState& n) { return n.ifname == i; }))
                dry_run_missing_.push_back(i);
    }
    refuse_uplinks();
    mark("discover");
    if (!cfg_.dry_run) {
        acquire_nic_locks(stop_fd);
        mark("nic_locks");
    }
    if (cfg_.cleanup) {
        cleanup_node();
        return;
    }
    // From the agent's discovery, at background priority on another CPU: overlaps the checks,
    // link-up and the LLDP wait.
    start_topo();
    // The xGMI mesh does not depend on LLDP: verify it up front, so a broken mesh fails in
    // milliseconds instead of after the LLDP wait, and nothing is left for the critical path.
    check_xgmi();
    mark("xgmi");
    if (cfg_.mode == "L3" || !cfg_.require_gdr.empty()) {
        check_gdr();
        mark("gdr");
    }
    if (cfg_.dry_run) {
        dry_run_report();
        return;
    }

    if (cfg_.disable_nm) {
        if (!cfg_.nm_keyfile_dir.empty()) {
            try {
                auto p = nm::write_keyfile(cfg_.nm_keyfile_dir, names, nm::keyfile_name(cfg_.labels.file));
                if (!p.empty()) {
                    NLOG_I("Wrote NetworkManager keyfile %s", p.c_str());
                    nm_keyfile_written_ = true;
                }
            } catch (const std::exception& e) {
                NLOG_W("Could not write NetworkManager keyfile: %s", e.what());
            }
        }
        std::unique_ptr<nm::NetworkManagerIf> nmapi;
        try {
            nmapi = nm_factory_();
        } catch (const std::exception& e) {
            throw AgentError(std::string("Failed to create NetworkManager: ") + e.what());
        }
        try {
            nm_unmanaged_ = nm::disable_for_interfaces(*nmapi, names);
        } catch (const std::exception& e) {
            throw AgentError(std::string("Failed to disable interfaces in NetworkManager: ") + e.what());
        }
        mark("networkmanager");
    }

    if (cfg_.mode == "L3" && cfg_.disable_fw_lldp) {
        disable_fw_lldp();  // before link-up: some drivers reset the port when the flag flips
        mark("fw_lldp");
    }
    interfaces_up();
    mark("link_up");
    load_mtu_state();
    interfaces_set_mtu();
    mark("mtu");
    try {
        remove_existing_ips(cfg_.keep_config && cfg_.mode == "L3" ? cached_addresses()
                                                                   : std::map<std::string, Ipv4Prefix>{});
    } catch (const std::exception& e) {
        throw AgentError(std::string("Failed to remove any existing IPs from interfaces: ") + e.what());
    }
    mark("flush");

    if (cfg_.mode == "L2" && cfg_.configure) {
        if (!wait_carrier(stop_fd)) {
            NLOG_I("Interrupted while waiting for carrier");
            post_cleanups();
            return;
        }
        mark("carrier");
        std::vector<std::string> dark;
        for (const auto& n : nics_)
            if (!n.configured) dark.push_back(n.ifname);
        if (!dark.empty() && !(cfg_.keep_running && cfg_.monitor)) {
            // Without the monitor nothing would ever notice the carrier coming: fail, named, and
            // let the kubelet's restart look again.
            write_status();
            throw AgentError(strfmt("Not all interfaces have a link (%zu/%zu). No carrier: ", nics_.size() - dark.size(),
                                    nics_.size()) +
                             join(dark, ", ") + " (check the cable, the switch port and the optic)");
        }
    }

    if (cfg_.mode == "L2" && cfg_.configure && cfg_.min_link_speed_mbps > 0) {
        // L3 checks each NIC as it configures it; L2 has no per-NIC step, so all at once here --
        // for the NICs with a link (a dark NIC is checked when its carrier comes, in monitor()).
        std::vector<std::string> slow;
        for (auto& n : nics_)
            if (n.configured && !(n.configured = l2_link_ok(n))) slow.push_back(n.ifname + ": " + n.config_error);
        if (!slow.empty() && !(cfg_.keep_running && cfg_.monitor)) {
            write_status();
            throw AgentError(strfmt("%zu NIC(s) below the required link speed: ", slow.size()) + join(slow, "; "));
        }
    }
    if (cfg_.mode == "L3") {
        detect_lldp(stop_fd);
        mark("lldp");
        if (aborted_) {
            NLOG_I("Interrupted while waiting for LLDP");
            post_cleanups();
            return;
        }
        bool found = std::any_of(nics_.begin(), nics_.end(), [](const NicState& n) { return bool(n.addr); });
        if (cfg_.configure && found) {
            int configured = configure_all();  // pipelined NICs are already done; this is a no-op for them
            int total = int(nics_.size());
            mark("configure");
            if (configured < total) {
                write_status();
                const std::string why = silent_summary();
                throw AgentError(strfmt("Not all interfaces were configured (%d/%d).", configured, total) +
                                 (why.empty() ? "" : " " + why));
            }
            NLOG_I("Configured %d of %d interfaces", configured, total);
            if (cfg_.verify_peers_ns > 0) {
                std::vector<NicState*> all;
                for (auto& n : nics_) all.push_back(&n);
                const int bad = verify_peers(all, cfg_.verify_peers_ns, stop_fd);
                mark("verify_peers");
                if (bad < 0) {
                    NLOG_I("Interrupted while verifying the switch-side peers");
                    post_cleanups();
                    return;
                }
                if (bad > 0) {
                    write_status();
                    auto first = std::find_if(nics_.begin(), nics_.end(), [](const NicState& n) { return !n.peer_error.empty(); });
                    throw AgentError(strfmt("%d of %d switch-side peers did not answer ARP (%s: %s)", bad, total,
                                            first->ifname.c_str(), first->peer_error.c_str()));
                }
            }
        } else if (cfg_.configure && !found && !cfg_.label_without_peers) {
            write_status();
            const std::string why = silent_summary();
            throw AgentError("No LLDP peers with a /30 Port Description were found" + (why.empty() ? "" : ". " + why));
        }
        write_artifacts();
        mark("artifacts");
    } else if (cfg_.configure && (!cfg_.rccl_env.empty() || !cfg_.rccl_topo.empty())) {
        // L2 (MI355X addition): RCCL still has to know which HCAs are the scale-out ones and which
        // GID to use; without IPv4 that is the RoCE v2 GID of the IPv6 link-local address.
        write_l2_artifacts();
        mark("artifacts");
    }

    log_results();

    if (!cfg_.configure) {
        if (cfg_.mode == "L3") write_host_config();
        interfaces_restore_down();
        write_status();
        return;
    }
    if (!cfg_.keep_running) {
        if (cfg_.mode == "L3") write_host_config();
        write_status();
        return;
    }
    int nconf = int(std::count_if(nics_.begin(), nics_.end(), [](const NicState& n) { return n.configured; }));
    labels_extra_[cfg_.labels.key + ".mode"] = cfg_.mode;
    labels_extra_[cfg_.labels.key + ".nics"] =
        std::to_string(cfg_.mode == "L3" ? nconf : int(nics_.size()));
    if (cfg_.xgmi_expect_links >= 0)
        labels_extra_["amd.feature.node.kubernetes.io/gpu-xgmi.pairs"] = std::to_string(xgmi_.pairs_connected);
    if (!gdr_.kernel.empty()) labels_extra_[cfg_.labels.key + ".gdr"] = gdr_.mode();
    const bool linked = cfg_.mode != "L2" ||
                        std::all_of(nics_.begin(), nics_.end(), [](const NicState& n) { return n.configured; });
    if (!linked) {
        // L2 with the monitor: stay up unlabelled; the carrier on the last dark NIC (at the
        // required speed) publishes the label (monitor()).
        NLOG_W("Not ready: %s; the label follows once every NIC has a link", not_ready_reason().c_str());
        write_status();
        NLOG_I("Monitoring...");
        monitor(stop_fd);
        post_cleanups();
        return;
    }
    try {
        if (publish_label()) NLOG_I("Published readiness label %s", cfg_.labels.path().c_str());
    } catch (const std::exception& e) {
        throw AgentError(std::string("Failed to write NFD label to indicate scale-out readiness: ") + e.what());
    }
    ready_ = true;
    phases_["total_ready"] = mono_ns() - t0_;
    {  // CPU the bring-up used, all threads (the DaemonSet's limit is a CFS quota per 100 ms period)
        rusage ru{};
        if (::getrusage(RUSAGE_SELF, &ru) == 0)
            cpu_ms_at_ready_ = double(ru.ru_utime.tv_sec + ru.ru_stime.tv_sec) * 1e3 +
                               double(ru.ru_utime.tv_usec + ru.ru_stime.tv_usec) / 1e3;
    }
    if (cfg_.mode == "L3") write_host_config();
    write_status();
    NLOG_I("Configurations done. %s...", cfg_.monitor ? "Monitoring" : "Idling");

    if (cfg_.monitor) {
        monitor(stop_fd);
    } else {
        idle(stop_fd);  // reference behaviour
    }
    post_cleanups();
}

bool Agent::idle_until_own_nic(int stop_fd) {
    if (cfg_.rediscover_ns <= 0) {
        idle(stop_fd);
        return false;
    }
    for (;;) {
        for (int64_t until = mono_ns() + cfg_.rediscover_ns; mono_ns() < until;) {
            if (fd_readable(stop_fd)) return false;
            const int64_t left_ms = std::max<int64_t>(1, (until - mono_ns()) / 1000000);
            if (stop_fd >= 0) {
                pollfd p{stop_fd, POLLIN, 0};
                ::poll(&p, 1, int(std::min<int64_t>(left_ms, 1000)));
            } else {
                ::usleep(useconds_t(std::min<int64_t>(left_ms, 1000) * 1000));
            }
        }
        uplinks_read_ = false;  // the node's routes may have changed too
        std::vector<std::string> names;
        try {
            names = collect_interfaces(true);
        } catch (const std::exception& e) {
            NLOG_V(2, "re-discovery failed: %s", e.what());
            continue;
        }
        if (!names.empty()) {
            NLOG_I("Interface(s) of its own appeared: %s", join(names, ", ").c_str());
            return true;
        }
        std::vector<std::string> parts;
        for (const auto& [n, why] : excluded_) parts.push_back(n + ": " + why);
        const std::string why = "no host NIC of its own (left alone: " + join(parts, "; ") + ")";
        if (why != config_error_) {  // what the node holds changed: the probe's reason follows
            config_error_ = why;
            write_status();
        }
    }
}

void Agent::idle(int stop_fd) {
    // Until SIGTERM / SIGINT.
    while (!fd_readable(stop_fd)) {
        if (stop_fd < 0) {
            ::pause();
            continue;
        }
        pollfd p{stop_fd, POLLIN, 0};
        ::poll(&p, 1, -1);
    }
}

std::string ecmascript_regex_error(const std::string& pattern) {
    try {
        std::regex(pattern, std::regex::ECMAScript);
    } catch (const std::regex_error& e) {
        return e.what();
    }
    return "";
}

std::optional<bool> ecmascript_full_match(const std::string& pattern, const std::string& text) {
    try {
        return std::regex_match(text, std::regex(pattern, std::regex::ECMAScript));
    } catch (const std::regex_error&) {
        return std::nullopt;
    }
}

std::string rail_pattern_error(const std::string& pattern) {
    // Every rail index a node can have: "{rail}" changes the pattern ("a{{rail},3}" is fine for
    // rail 0 and a reversed range for rail 5).
    for (int k = 0; k < kMaxRails; ++k) {
        std::string p = pattern;
        for (size_t at; (at = p.find("{rail}")) != std::string::npos;) p.replace(at, 6, std::to_string(k));
        if (std::string e = ecmascript_regex_error(p); !e.empty())
            return k == 0 ? e : e + strfmt(" (with {rail} = %d)", k);
    }
    return "";
}

bool Agent::publish_label() { return artifacts::write_labels(cfg_.labels, labels_extra_); }

void Agent::cleanup_node() {
    // What agents running with --keep-config left behind, once the policy is gone.  Nothing here
    // depends on a previous run's memory: addresses of the discovered NICs, rules and routes
    // carrying the agent's protocol tag, and the agent's own files.
    NLOG_I("Cleaning up the node (--cleanup): %zu interface(s)", nics_.size());
    if (!artifacts::remove_labels(cfg_.labels)) NLOG_W("Failed to remove NFD label file: %s", std::strerror(errno));
    int errors = 0;
    try {
        remove_existing_ips();
    } catch (const std::exception& e) {
        NLOG_W("Failed to remove IPv4 addresses: %s", e.what());
        ++errors;
    }
    try {
        for (const auto& r : ops_.rule_list())
            if (r.protocol == kRailProtocol) ops_.rule_del(r);
        for (const auto& r : ops_.route_list(0))
            if (r.protocol == kRailProtocol) {
                try {
                    ops_.route_del(r);
                } catch (const SysError&) {  // gone with its address
                }
            }
    } catch (const std::exception& e) {
        NLOG_W("Failed to remove the rail rules / routes: %s", e.what());
        ++errors;
    }
    for (const std::string& f : {cfg_.rccl_env, cfg_.rccl_net, cfg_.lldp_cache, cfg_.rccl_topo,
                                 cfg_.rccl_topo.empty() ? std::string() : cfg_.rccl_topo + ".key"})
        if (!f.empty() && ::unlink(f.c_str()) != 0 && errno != ENOENT) {
            NLOG_W("Could not remove %s: %s", f.c_str(), std::strerror(errno));
            ++errors;
        }
    if (!cfg_.networkd.empty()) {
        std::vector<std::string> names;
        for (const auto& n : nics_) names.push_back(n.ifname);
        try {
            artifacts::delete_networkd(cfg_.networkd, names);
        } catch (const std::exception& e) {
            NLOG_W("Could not remove systemd-networkd files: %s", e.what());
            ++errors;
        }
    }
    try {
        restore_fw_lldp_from_state();
    } catch (const std::exception& e) {
        NLOG_W("Could not restore the NICs' firmware LLDP settings: %s", e.what());
        ++errors;
    }
    try {
        restore_mtu_state();
    } catch (const std::exception& e) {
        NLOG_W("Could not restore the NICs' MTUs: %s", e.what());
        ++errors;
    }
    if (cfg_.disable_nm) {
        nm_keyfile_written_ = true;  // a file of ours from an earlier run (remove_keyfile checks it)
        nm_unmanaged_.clear();
        for (const auto& n : nics_) nm_unmanaged_.push_back(n.ifname);
        restore_network_manager();
    }
    mark("cleanup");
    write_status();
    if (errors) throw AgentError(strfmt("Node cleanup incomplete (%d error(s))", errors));
    NLOG_I("Node cleanup done");
}

}  // namespace netop::agent

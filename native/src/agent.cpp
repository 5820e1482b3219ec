// Agent: the run state machine (reference cmd/discover/main.go cmdRun, :161-259) -- sanitising
// the flags, discovery, link-up / MTU / flush, the L2 carrier wait, LLDP and configuration, the
// label, then monitoring or idling until SIGTERM -- plus the --cleanup mode.  The concerns it
// drives live beside it: agent_host.cpp, agent_l3.cpp, agent_artifacts.cpp, agent_status.cpp,
// agent_links.cpp, agent_ownership.cpp, agent_monitor.cpp.
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
#include <tuple>
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
    start_prefetch();
}

void Agent::start_prefetch() {
    // What the start needs from sysfs beyond discovery, read beside link-up and the LLDP wait,
    // each on a thread of its own: the KFD topology (joined right after link-up), the rails' PCIe
    // links (first NIC configured), the GPUs' gpu_metrics (before the label; one thread per GPU).
    // On the box these are ~1.1, ~0.5 and ~1.65 ms of reads (profiles/r5_box_read_costs.json).
    // Every join waits until prefetch_deadline_ at most (Config::sysfs_read_timeout_ns).
    std::vector<std::pair<std::string, std::string>> fns;  // (NIC name, its GPU's BDF)
    for (const auto& n : nics_) fns.emplace_back(n.ifname, n.gpu_bdf);
    std::vector<std::string> gpus;
    for (const auto& g : disc_.gpus) gpus.push_back(g.pci.bdf);
    const bool xgmi = cfg_.xgmi_expect_links >= 0;
    const std::string root = cfg_.sysfs_root.empty() ? topo::sysfs_root() : cfg_.sysfs_root;
    const int main_cpu = ::sched_getcpu();
    auto off_main_cpu = [main_cpu] {  // the agent thread brings the links up meanwhile
        cpu_set_t set;
        if (main_cpu >= 0 && ::sched_getaffinity(0, sizeof set, &set) == 0 && CPU_COUNT(&set) > 1) {
            CPU_CLR(main_cpu, &set);
            (void)::sched_setaffinity(0, sizeof set, &set);
        }
    };
    const int64_t timeout = cfg_.sysfs_read_timeout_ns;
    prefetch_deadline_ = mono_ns() + timeout;
    if (xgmi)
        xgmi_call_ = bounded::Call<topo::XgmiReport>("", [root, off_main_cpu] {
            off_main_cpu();
            return topo::read_xgmi(root);
        });
    pcie_call_ = bounded::Call<std::vector<std::pair<topo::PcieLink, topo::PcieLink>>>("", [root, fns, off_main_cpu] {
        off_main_cpu();
        std::vector<std::pair<topo::PcieLink, topo::PcieLink>> links;
        for (const auto& [ifname, gpu] : fns) {
            topo::PcieLink nic, g;
            if (auto d = topo::netdev_pci(root, ifname)) nic = topo::read_pcie_link(root, d->bdf);
            if (!gpu.empty()) g = topo::read_pcie_link(root, gpu);
            links.emplace_back(nic, g);
        }
        return links;
    });
    pcie_joined_ = false;
    if (xgmi)
        xgmi_health_call_ = bounded::Call<std::vector<topo::XgmiLinkHealth>>("", [root, gpus, timeout, off_main_cpu] {
            off_main_cpu();
            // The amdgpu PCI functions discovery found: KFD lists a GPU the container cannot
            // open with its properties filtered (no BDF), while its PCI device (and gpu_metrics)
            // is still readable.  Without discovered GPUs, KFD's own list.
            std::vector<std::string> bdfs = gpus;
            if (bdfs.empty())
                for (const auto& g : topo::read_xgmi(root).gpus)
                    if (g.is_gpu()) bdfs.push_back(g.bdf());
            return topo::read_xgmi_health(root, bdfs, timeout);
        });
}

void Agent::ensure_pcie() {
    if (pcie_joined_ || !pcie_call_.valid()) return;
    pcie_joined_ = true;
    auto got = pcie_call_.wait(prefetch_deadline_);
    if (!got) {
        pcie_late_ = true;
        ++late_reads_["pcie"];
        NLOG_W("The PCIe link state of the scale-out NICs did not answer in %s: not checked%s",
               format_go_duration(cfg_.sysfs_read_timeout_ns).c_str(),
               cfg_.require_full_pcie ? " (--require-full-pcie: the NICs wait for it)" : "");
        return;
    }
    const auto& links = *got;
    for (size_t i = 0; i < links.size() && i < nics_.size(); ++i) {
        NicState& n = nics_[i];
        std::tie(n.pcie, n.gpu_pcie) = links[i];
        if (n.pcie.degraded()) NLOG_W("Interface '%s': PCIe link trained at %s", n.ifname.c_str(), n.pcie.str().c_str());
        if (n.gpu_pcie.degraded())
            NLOG_W("Interface '%s': the PCIe link of its GPU %s trained at %s", n.ifname.c_str(), n.gpu_bdf.c_str(),
                   n.gpu_pcie.str().c_str());
    }
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
    forget_link_state();
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


void Agent::check_xgmi() {  // dry run: everything in line
    join_xgmi();
    finish_xgmi_health();
}

void Agent::join_xgmi() {
    if (!xgmi_call_.valid()) return;
    auto x = xgmi_call_.wait(prefetch_deadline_);
    xgmi_call_ = {};
    if (!x) {
        ++late_reads_["kfd"];
        const std::string why = "the KFD topology (" + path_join(cfg_.sysfs_root.empty() ? topo::sysfs_root() : cfg_.sysfs_root,
                                                                 "class/kfd") +
                                ") did not answer in " + format_go_duration(cfg_.sysfs_read_timeout_ns);
        if (!cfg_.dry_run) throw AgentError("xGMI: " + why);
        NLOG_W("dry run: a real start would fail: xGMI: %s", why.c_str());
        xgmi_error_ = why;
        return;
    }
    xgmi_ = std::move(*x);
    evaluate_xgmi();
}

void Agent::evaluate_xgmi() {
    int expect = cfg_.xgmi_expect_links == 0 ? xgmi_.pairs_expected : cfg_.xgmi_expect_links;
    NLOG_I("xGMI: %zu GPUs, %d/%d GPU pairs linked, %llu MB/s per GPU advertised", xgmi_.gpus.size(), xgmi_.pairs_connected,
           xgmi_.pairs_expected, (unsigned long long)xgmi_.per_gpu_bw_mbs());
    for (auto& [a, b] : xgmi_.missing) NLOG_W("xGMI: no link between %s and %s", a.c_str(), b.c_str());
    // A dry run reports what a real start would fail on (status.json, the log) and goes on.
    auto fail = [&](const std::string& why) {
        if (!cfg_.dry_run) throw AgentError(why);
        NLOG_W("dry run: a real start would fail: %s", why.c_str());
    };
    if (xgmi_.pairs_connected < expect)
        fail(strfmt("xGMI mesh incomplete: %d of %d GPU pairs linked", xgmi_.pairs_connected, expect));
}

std::vector<std::string> Agent::xgmi_health_bdfs() const {
    // The amdgpu PCI functions discovery found: KFD lists a GPU the container cannot open with
    // its properties filtered (no BDF), while its PCI device (and gpu_metrics) is still readable.
    std::vector<std::string> bdfs;
    for (const auto& g : disc_.gpus) bdfs.push_back(g.pci.bdf);
    if (bdfs.empty())
        for (const auto& g : xgmi_.gpus)
            if (g.is_gpu()) bdfs.push_back(g.bdf());
    return bdfs;
}

void Agent::finish_xgmi_health() {
    if (xgmi_health_call_.valid()) {
        // The reader bounds each GPU's read itself; this deadline only covers the reader thread
        // (and, without discovered GPUs, its KFD read) being late as a whole.
        auto h = xgmi_health_call_.wait(prefetch_deadline_ + cfg_.sysfs_read_timeout_ns);
        xgmi_health_call_ = {};
        if (h) {
            xgmi_health_ = std::move(*h);
        } else {
            xgmi_health_.clear();
            for (const auto& bdf : xgmi_health_bdfs()) {
                topo::XgmiLinkHealth l;
                l.bdf = bdf;
                l.late = true;
                l.error = "gpu_metrics did not answer in " + format_go_duration(cfg_.sysfs_read_timeout_ns);
                xgmi_health_.push_back(std::move(l));
            }
        }
        for (const auto& l : xgmi_health_) late_reads_["gpu_metrics"] += l.late ? 1 : 0;
        note_xgmi_sample();
        const std::string kfd_error = xgmi_error_;  // a late KFD read (dry run) stays reported
        xgmi_error_ = xgmi_health_problem();
        if (!kfd_error.empty()) xgmi_error_ = xgmi_error_.empty() ? kfd_error : kfd_error + "; " + xgmi_error_;
    }
    int gpus = 0, up = 0;
    for (const auto& h : xgmi_health_) {  // one line on the critical path; the details at -v=1
        if (h.known) {
            ++gpus;
            up += h.links_up();
            NLOG_V(1, "xGMI %s: %d link(s) up, %d down, x%d at %d Gb/s (gpu_metrics %s)", h.bdf.c_str(), h.links_up(),
                   h.links_down(), h.width, h.speed_gbps, h.revision.c_str());
        } else {
            NLOG_V(1, "xGMI %s: %s", h.bdf.c_str(), h.error.c_str());
        }
    }
    if (gpus) NLOG_I("xGMI links: %d up on %d GPU(s) (gpu_metrics)", up, gpus);
    xgmi_unread_.clear();
    if (!gpus && !xgmi_health_.empty() &&
        std::none_of(xgmi_health_.begin(), xgmi_health_.end(), [](const topo::XgmiLinkHealth& h) { return h.late; })) {
        // No GPU's gpu_metrics layout is one this agent decodes (other firmware): the links'
        // trained state is not checked, and not watched (said once, at warning level,
        // and in status.json, instead of only at -v=1).  The KFD mesh check still runs.
        std::set<std::string> why;
        for (const auto& h : xgmi_health_) why.insert(h.error);
        xgmi_unread_ = join(std::vector<std::string>(why.begin(), why.end()), "; ");
        NLOG_W("xGMI link state not checked on any of the %zu GPU(s): %s", xgmi_health_.size(), xgmi_unread_.c_str());
    }
    if (xgmi_error_.empty()) return;
    if (cfg_.dry_run) {
        NLOG_W("dry run: a real start would fail: xGMI: %s", xgmi_error_.c_str());
        return;
    }
    if (cfg_.keep_running && cfg_.monitor && cfg_.xgmi_health_interval_ns > 0) {
        // A link can come back (retraining, a reset of the GPU): the NICs are configured, the node
        // stays unlabelled, and the monitor labels it when gpu_metrics shows the link up again.
        NLOG_W("xGMI: %s; the readiness label waits for the link(s)", xgmi_error_.c_str());
        return;
    }
    write_status();
    throw AgentError("xGMI: " + xgmi_error_);
}

void Agent::note_xgmi_sample() {
    for (const auto& h : xgmi_health_) {
        if (!h.known) continue;  // a late or unreadable sample says nothing about the links
        auto& streak = xgmi_down_streak_[h.bdf];
        streak.resize(h.status.size(), 0);
        for (size_t i = 0; i < h.status.size(); ++i) streak[i] = h.status[i] == 0 ? streak[i] + 1 : 0;
    }
}

std::string Agent::xgmi_health_problem(int min_down) const {
    std::vector<std::string> parts;
    for (const auto& h : xgmi_health_) {
        if (h.late) {
            parts.push_back(strfmt("gpu_metrics of %s did not answer in %s", h.bdf.c_str(),
                                   format_go_duration(cfg_.sysfs_read_timeout_ns).c_str()));
            continue;
        }
        if (!h.known) continue;
        auto streak = xgmi_down_streak_.find(h.bdf);
        std::vector<std::string> down;
        for (size_t i = 0; i < h.status.size(); ++i)
            if (h.status[i] == 0 && (streak == xgmi_down_streak_.end() || i >= streak->second.size() ||
                                     streak->second[i] >= min_down))
                down.push_back(std::to_string(i));
        if (!down.empty())
            parts.push_back(strfmt("GPU %s: link%s %s down", h.bdf.c_str(), down.size() > 1 ? "s" : "", join(down, ", ").c_str()));
        else if (cfg_.xgmi_min_link_width > 0 && h.links_up() > 0 && h.width < cfg_.xgmi_min_link_width)
            parts.push_back(strfmt("GPU %s: links trained at x%d, below the required x%d", h.bdf.c_str(), h.width,
                                   cfg_.xgmi_min_link_width));
    }
    return join(parts, "; ");
}


void Agent::check_rdma() {
    no_rdma_.clear();
    for (const auto& p : disc_.pairs) {
        const auto& nic = disc_.nics[size_t(p.nic)];
        if (nic.rdma_dev.empty()) no_rdma_.push_back(nic.ifname);
    }
    if (no_rdma_.empty()) return;
    const std::string why = "scale-out NIC(s) without an RDMA device: " + join(no_rdma_, ", ") +
                            " (RCCL could only use them over TCP sockets: load the NIC's RDMA driver, e.g. ionic_rdma, "
                            "mlx5_ib, bnxt_re)";
    if (cfg_.require_rdma) {
        // Not a crash loop: the NICs are configured, and the label follows the devices (a driver
        // container loading the module while this agent runs).  See rdma_missing().
        if (cfg_.dry_run)
            NLOG_W("dry run: a real start would wait for RDMA devices on %zu rail%s: %s", no_rdma_.size(),
                   no_rdma_.size() == 1 ? "" : "s", why.c_str());
        else
            NLOG_W("%s; the readiness label waits for them", why.c_str());
        return;
    }
    if (cfg_.require_gdr.empty() || cfg_.dry_run) {
        NLOG_W("%s%s", cfg_.require_gdr.empty() ? "" : "dry run: a real start would fail: ", why.c_str());
        return;
    }
    throw AgentError("GPUDirect RDMA required, but " + why);
}

std::vector<std::string> Agent::rdma_missing() const {
    std::vector<std::string> out;
    if (!cfg_.require_rdma) return out;
    for (const auto& n : nics_)
        if (n.rdma_dev.empty()) out.push_back(n.ifname);
    return out;
}

std::string Agent::rdma_reason() const {
    // Start-up only before the node was ever ready: a device that goes away under a labelled node
    // (a driver unloaded) is a fault at once.
    const bool starting = !phases_.count("total_ready") && mono_ns() - t0_ < cfg_.rdma_wait_ns;
    return starting ? "waiting for RDMA device" : "no RDMA device (load its RDMA driver)";
}

bool Agent::refresh_rdma() {
    if (!cfg_.require_rdma) return false;
    const std::string root = cfg_.sysfs_root.empty() ? topo::sysfs_root() : cfg_.sysfs_root;
    bool changed = false;
    for (auto& n : nics_) {
        std::string dev = topo::netdev_rdma_device(root, n.ifname);
        if (dev == n.rdma_dev) continue;
        if (dev.empty())  // the RDMA driver was unloaded (or is reloading): RCCL loses the rail
            NLOG_W("Interface '%s': its RDMA device %s went away", n.ifname.c_str(), n.rdma_dev.c_str());
        else if (n.rdma_dev.empty())
            NLOG_I("Interface '%s': RDMA device %s appeared", n.ifname.c_str(), dev.c_str());
        else  // a driver reload may number the devices anew
            NLOG_I("Interface '%s': RDMA device is %s now (was %s)", n.ifname.c_str(), dev.c_str(), n.rdma_dev.c_str());
        n.rdma_dev = dev;
        n.gid_index.reset();
        for (auto& d : disc_.nics)
            if (d.ifname == n.ifname) d.rdma_dev = dev;
        no_rdma_.erase(std::remove(no_rdma_.begin(), no_rdma_.end(), n.ifname), no_rdma_.end());
        if (dev.empty()) no_rdma_.push_back(n.ifname);
        changed = true;
    }
    if (changed) {  // the topology file names each rail's HCA: generate it again
        topo_call_ = {};
        topo_.reset();
        topo_late_ = false;
    }
    return changed;
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
    // The xGMI mesh does not depend on LLDP: its KFD topology is read beside link-up (~1 ms on
    // the box) and checked right after it, so a broken mesh still fails before any address is
    // touched or the LLDP wait begins.  A dry run reads it in line.
    if (cfg_.dry_run) {
        check_xgmi();
        mark("xgmi");
    }
    check_rdma();
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
    load_link_state();
    interfaces_up();
    mark("link_up");
    join_xgmi();
    mark("xgmi");
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

    if (cfg_.mode == "L2" && cfg_.configure && (cfg_.min_link_speed_mbps > 0 || cfg_.require_full_pcie)) {
        // L3 checks each NIC as it configures it; L2 has no per-NIC step, so all at once here --
        // for the NICs with a link (a dark NIC is checked when its carrier comes, in monitor()).
        std::vector<std::string> slow;
        for (auto& n : nics_)
            if (n.configured && !(n.configured = l2_link_ok(n))) slow.push_back(n.ifname + ": " + n.config_error);
        if (!slow.empty() && !(cfg_.keep_running && cfg_.monitor)) {
            write_status();
            throw AgentError(strfmt("%zu NIC(s) below the required link speed%s: ", slow.size(),
                                    cfg_.require_full_pcie ? " or PCIe link" : "") + join(slow, "; "));
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
    ensure_pcie();         // (reported in the status even where no check needed it)
    finish_xgmi_health();  // the start's gpu_metrics read, beside link-up and LLDP
    mark("xgmi_health");

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
    if (refresh_rdma() && (!cfg_.rccl_env.empty() || !cfg_.rccl_topo.empty())) {
        // A driver loaded during the bring-up, after the artifacts were written without its
        // devices (rccl.env held back): write them again with the HCAs before the label.
        if (cfg_.mode == "L3")
            write_artifacts();
        else
            write_l2_artifacts();
    }
    const std::vector<std::string> no_rdma = rdma_missing();
    const bool linked = xgmi_error_.empty() && no_rdma.empty() &&
                        (cfg_.mode != "L2" ||
                         std::all_of(nics_.begin(), nics_.end(), [](const NicState& n) { return n.configured; }));
    if (!linked && !no_rdma.empty() && !cfg_.monitor) {
        // Nothing would look for the devices again: fail, named, and let the restart look.
        write_status();
        throw AgentError("No RDMA device on " + join(no_rdma, ", ") + " (load the NIC's RDMA driver, e.g. ionic_rdma, "
                         "mlx5_ib, bnxt_re): RCCL could only use these rails over TCP sockets");
    }
    if (!linked) {
        // With the monitor: stay up unlabelled; the carrier on the last dark NIC (L2, at the
        // required speed) or the xGMI link coming back publishes the label (monitor()).
        NLOG_W("Not ready: %s; the label follows once that is resolved", not_ready_reason().c_str());
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
    try {
        restore_link_state();
    } catch (const std::exception& e) {
        NLOG_W("Could not restore the NICs' link states: %s", e.what());
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

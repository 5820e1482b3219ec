// Agent: what it writes for the collective library and the node -- the RCCL topology file
// (built off the critical path), rccl.env, rccl-net.json (the reference's gaudinet.json role,
// cmd/discover/gaudinet.go), systemd-networkd files, and the dry-run report.
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
#include <thread>

#include "agent_internal.hpp"
#include "netop/log.hpp"

namespace netop::agent {

using detail::fd_readable;

bool Agent::gids_missing() const {
    return std::any_of(nics_.begin(), nics_.end(), [&](const NicState& n) {
        return !n.rdma_dev.empty() && n.configured && (cfg_.mode != "L3" || n.addr) && !n.gid_index;
    });
}

bool Agent::look_up_gids() {
    // L3: the RoCE v2 GID of the NIC's /30 address; L2: of its IPv6 link-local address.
    const std::string root = cfg_.sysfs_root.empty() ? topo::sysfs_root() : cfg_.sysfs_root;
    bool found = false;
    for (auto& n : nics_) {
        if (n.rdma_dev.empty() || !n.configured || n.gid_index) continue;
        if (cfg_.mode == "L3") {
            if (!n.addr) continue;
            n.gid_index = topo::find_rocev2_gid_index(root, n.rdma_dev, n.rdma_port, n.addr->local);
        } else {
            n.gid_index = topo::find_rocev2_linklocal_gid_index(root, n.rdma_dev, n.rdma_port);
        }
        found |= bool(n.gid_index);
    }
    return found;
}

void Agent::write_l2_artifacts(int64_t gid_wait_ns) {
    for (auto& n : nics_) n.configured = n.link.up() && !n.no_carrier && n.config_error.empty();
    const int64_t deadline = mono_ns() + (gid_wait_ns < 0 ? cfg_.gid_wait_ns : gid_wait_ns);
    for (;;) {
        look_up_gids();
        if (!gids_missing() || mono_ns() >= deadline) break;
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
    if (cfg_.rccl_topo.empty() || topo_call_.valid() || topo_) return;
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
    // A detached worker (netop/bounded.hpp): the walk reads every bridge's PCI attributes, and a
    // function in error recovery can stall such a read; the join below is bounded, and nothing
    // waits for a stalled worker when the agent exits.  Without a thread, it runs here.
    topo_call_ = bounded::Call<TopoResult>("", [work, agent_thread = std::this_thread::get_id()] {
        return work(std::this_thread::get_id() != agent_thread);  // in line: no affinity or nice change
    });
}

const std::string& Agent::topo_xml() {
    static const std::string none;
    if (!topo_) {
        if (!topo_call_.valid()) start_topo();
        // Bounded like every sysfs read of the start; once late, later artifact writes only look.
        // In the monitor (the file generated again for a renumbered RDMA device) the loop waits
        // 20 ms at most (the walk takes 1-3 ms on the box): a late file is written when the
        // worker answers (monitor(), topo_late_).
        const int64_t wait = monitoring_ ? std::min<int64_t>(cfg_.sysfs_read_timeout_ns, 20000000) : cfg_.sysfs_read_timeout_ns;
        const int64_t deadline = topo_late_ ? mono_ns() : mono_ns() + wait;
        try {
            auto r = topo_call_.wait(deadline);
            if (!r) {
                if (!topo_late_ && monitoring_)  // (not a stall yet: the loop only does not wait for it)
                    NLOG_V(1, "RCCL topology file still being generated: rccl.env names it when it is ready");
                else if (!topo_late_) {
                    ++late_reads_["topology"];
                    NLOG_W("The RCCL topology file was not generated within %s (a PCI attribute read stalled?): "
                           "rccl.env names no NCCL_TOPO_FILE until it is (RCCL then reads the topology itself)",
                           format_go_duration(cfg_.sysfs_read_timeout_ns).c_str());
                }
                topo_late_ = true;
                return none;
            }
            topo_ = std::move(*r);
            if (topo_late_) NLOG_I("The RCCL topology file was generated late: rccl.env names it now");
            topo_late_ = false;
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
            topo_late_ = false;  // answered (with an error): the monitor has nothing left to wait for
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
    if (!cfg_.dry_run && !rdma_missing().empty()) {
        // --require-rdma: no rccl.env that leaves a rail to TCP sockets.  One from an earlier run
        // named HCAs that are gone now: it goes too (written again once the devices are back).
        if (::unlink(cfg_.rccl_env.c_str()) == 0) NLOG_I("Removed %s until every rail has its RDMA device", cfg_.rccl_env.c_str());
        return;
    }
    try {
        artifacts::write_rccl_env(cfg_.rccl_env, nics_, topo_env, rccl_env_extra_, socket_ifnames(), cfg_.mode != "L3");
    } catch (const std::exception& e) {
        NLOG_E("Error writing RCCL env: %s", e.what());
    }
}

void Agent::write_artifacts(int64_t gid_wait_ns) {
    // Poll all configured RDMA NICs together until each has its RoCE v2 GID or the wait ends.
    const int64_t gid_deadline = mono_ns() + (gid_wait_ns < 0 ? cfg_.gid_wait_ns : gid_wait_ns);
    for (;;) {
        look_up_gids();
        if (!gids_missing() || mono_ns() >= gid_deadline) break;
        ::usleep(2000);
    }
    if (gid_wait_ns != 0)  // (the monitor's one look is followed by more: it warns when they end)
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

}  // namespace netop::agent

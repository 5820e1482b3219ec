// Agent: after readiness.  Periodic LLDP announcements, switch-side ARP verification, and the
// monitor loop that withdraws and republishes the readiness label as links and switch ports change.
#include "netop/agent.hpp"

#include <errno.h>
#include <linux/if.h>
#include <linux/rtnetlink.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <map>

#include "agent_internal.hpp"
#include "netop/log.hpp"

namespace netop::agent {

using detail::fd_readable;
using detail::kMonitorVerifyNs;

void Agent::announce_all(uint16_t ttl) {
    if (!cfg_.lldp_announce || cfg_.mode != "L3") return;
    for (auto& n : nics_) {
        if (!n.link.up()) continue;
        try {
            lldp_->announce(n.ifname,
                            lldp::encode(make_node_frame(cfg_.node_name, n.ifname, n.link.mac, n.gpu_bdf, ttl, cfg_.mtu)));
        } catch (const std::exception& e) {
            NLOG_V(2, "LLDP announce on %s failed: %s", n.ifname.c_str(), e.what());
        }
    }
}

int Agent::verify_peers(const std::vector<NicState*>& which, int64_t timeout_ns, int stop_fd) {
    std::vector<arp::Probe> probes;
    std::vector<NicState*> owners;
    for (NicState* n : which) {
        if (!n->addr || !n->configured) continue;
        arp::Probe p;
        p.ifname = n->ifname;
        p.ifindex = n->link.index;
        p.mac = n->link.mac;
        p.local = n->addr->local;
        p.peer = n->addr->peer;
        probes.push_back(p);
        owners.push_back(n);
    }
    if (probes.empty()) return 0;
    bool finished = false;
    try {
        finished = arp_probe(probes, timeout_ns, std::min(cfg_.verify_peers_retry_ns, timeout_ns), stop_fd);
    } catch (const std::exception& e) {
        for (NicState* n : owners) {
            n->peer_verified = false;
            n->peer_error = e.what();
        }
        NLOG_W("Could not verify the switch-side peers: %s", e.what());
        return int(owners.size());
    }
    if (!finished) return -1;
    int failed = 0;
    for (size_t i = 0; i < probes.size(); ++i) {
        const arp::Probe& p = probes[i];
        NicState& n = *owners[i];
        n.peer_verified = p.answered;
        if (p.answered) {
            n.peer_rtt_ns = p.rtt_ns;
            n.peer_verify_ns = p.verify_ns;
            n.peer_arp_mac = p.peer_mac;
            n.peer_error.clear();
            NLOG_V(1, "interface '%s': peer %s (%s) answered ARP: rtt %.3f ms, verified after %.3f ms", n.ifname.c_str(),
                   p.peer.str().c_str(), p.peer_mac.str().c_str(), double(p.rtt_ns) / 1e6, double(p.verify_ns) / 1e6);
            // The LLDP peer MAC (PortID MAC over ChassisID MAC, reference pkg/lldp/client.go:114-129)
            // is the switch port; an ARP answer from elsewhere deserves a look, not a failure.
            const bool mismatch = n.peer_mac && !(*n.peer_mac == p.peer_mac);
            if (mismatch && !n.peer_mac_mismatch)
                NLOG_W("interface '%s': peer %s answered ARP from %s, but its LLDP MAC is %s (proxy ARP or a "
                       "misaddressed port?)", n.ifname.c_str(), p.peer.str().c_str(), p.peer_mac.str().c_str(),
                       n.peer_mac->str().c_str());
            n.peer_mac_mismatch = mismatch;
            continue;
        }
        ++failed;
        n.peer_error = !p.error.empty() ? p.error
                                        : strfmt("peer %s did not answer ARP within %s (%d requests): is the switch port "
                                                 "addressed as its Port Description says?",
                                                 p.peer.str().c_str(), format_go_duration(timeout_ns).c_str(),
                                                 p.requests);
        NLOG_W("interface '%s': %s", n.ifname.c_str(), n.peer_error.c_str());
    }
    return failed;
}

bool Agent::nic_healthy(const NicState& n) const {
    if (!n.link.up() || n.degraded || n.cache_stale || n.no_carrier || !n.config_error.empty() || !n.pcie_error.empty())
        return false;
    if (cfg_.mode == "L3" && cfg_.verify_peers_ns > 0 && !n.peer_verified) return false;
    if (cfg_.require_rdma && n.rdma_dev.empty()) return false;
    return cfg_.mode != "L3" || n.configured;
}

bool Agent::apply_health(const HealthSample& s) {
    bool changed = false;
    for (const auto& h : s.xgmi) late_reads_["gpu_metrics"] += h.late ? 1 : 0;
    for (bool l : s.pcie_late) late_reads_["pcie"] += l ? 1 : 0;
    if (s.xgmi_read) {
        const std::string before = xgmi_error_;
        xgmi_health_ = s.xgmi;
        note_xgmi_sample();
        // A link counts as down only after xgmi_down_samples samples in a row (a status read in
        // the middle of a GPU reset is not a flap); a GPU that did not answer counts at once.
        xgmi_error_ = xgmi_health_problem(std::max(1, cfg_.xgmi_down_samples));
        if (xgmi_error_ != before) {
            if (xgmi_error_.empty())
                NLOG_I("xGMI links healthy again");
            else
                NLOG_W("xGMI: %s", xgmi_error_.c_str());
            changed = true;
        }
    }
    if (s.pcie_read) {
        const std::string late = "its PCIe link state did not answer in " + format_go_duration(cfg_.sysfs_read_timeout_ns);
        for (size_t i = 0; i < nics_.size() && i < s.pcie.size(); ++i) {
            NicState& n = nics_[i];
            // What kept an unconfigured NIC back at start, with the reading it was refused on.
            const std::string was = n.configured ? n.pcie_error : check_pcie(n);
            std::tie(n.pcie, n.gpu_pcie) = s.pcie[i];
            const std::string why = s.pcie_late[i] ? late : check_pcie(n);
            if (!n.configured) {
                // Left unconfigured only for its PCIe link: configured once the link
                // retrains at full speed and width, instead of waiting for a restart that, with the
                // monitor on, never comes.
                if (was.empty() || n.config_error != was || why == was) continue;
                changed = true;
                if (!why.empty()) {
                    n.config_error = why;
                    continue;
                }
                NLOG_I("Interface '%s': PCIe link now at %s: configuring it", n.ifname.c_str(), n.pcie.str().c_str());
                if (cfg_.mode == "L2") {
                    n.configured = l2_link_ok(n);
                } else if (n.addr) {
                    n.config_error.clear();
                    configure_interface(n);
                }
                continue;
            }
            if (why == n.pcie_error) continue;
            if (why.empty())
                NLOG_I("Interface '%s': PCIe link back at %s", n.ifname.c_str(), n.pcie.str().c_str());
            else
                NLOG_W("Interface '%s': %s", n.ifname.c_str(), why.c_str());
            n.pcie_error = why;
            changed = true;
        }
    }
    return changed;
}

namespace {
// An eventfd the health worker signals through; shared with the worker so that a worker finishing
// after the monitor has returned never writes to a closed (or reused) descriptor.
struct SharedFd {
    int fd;
    explicit SharedFd(int f) : fd(f) {}
    ~SharedFd() {
        if (fd >= 0) ::close(fd);
    }
};
}  // namespace

void Agent::monitor(int stop_fd) {
    monitoring_ = true;
    std::unique_ptr<nl::LinkWatcher> watcher;
    try {
        watcher = ops_.subscribe_links();
    } catch (const std::exception& e) {
        NLOG_W("link monitoring disabled: %s", e.what());
    }
    // Carrier baseline: only a 1 -> 0 transition of IFF_LOWER_UP counts as a failure (a NIC
    // whose carrier was never reported up — e.g. a driver without carrier reporting — is not
    // flagged), IFF_UP going away always does.
    std::map<int, bool> carrier;
    for (auto& n : nics_) carrier[n.link.index] = n.link.lower_up();
    int64_t next_tx = mono_ns() + cfg_.lldp_tx_interval_ns;
    int64_t next_verify = 0;
    // The GPUs' xGMI links (gpu_metrics): only when the xGMI check runs and the layout is known
    // (or the start's read did not answer: it is asked again).
    const bool xgmi_watch = cfg_.xgmi_expect_links >= 0 && cfg_.xgmi_health_interval_ns > 0 &&
                            std::any_of(xgmi_health_.begin(), xgmi_health_.end(),
                                        [](const topo::XgmiLinkHealth& h) { return h.known || h.late; });
    const bool pcie_watch = cfg_.require_full_pcie && cfg_.xgmi_health_interval_ns > 0;
    int64_t next_health = mono_ns() + cfg_.xgmi_health_interval_ns;
    // Those reads (an SMU query per GPU, PCIe config space) run on a worker thread, never on this
    // loop: a stalled read must not hold back link events and LLDP re-addressing.  The worker
    // signals `done` (in the epoll set below) when its sample is ready.
    auto done = std::make_shared<SharedFd>(::eventfd(0, EFD_CLOEXEC | EFD_NONBLOCK));
    bounded::Call<HealthSample> poll;
    const std::string root = cfg_.sysfs_root.empty() ? topo::sysfs_root() : cfg_.sysfs_root;
    int64_t next_rdma = cfg_.require_rdma ? mono_ns() : 0;
    int64_t next_gid_look = 0;
    constexpr int64_t kGidLookNs = 100LL * 1000000;
    std::string rdma_said = rdma_reason();
    bool labelled = ready_;  // false: L2 came up with a NIC still without carrier
    // One pollable fd for "stop, link event or health sample": the LLDP wait returns as soon as
    // any fires, so a link failure is acted on in about a millisecond, not at the next tick.
    int wake = ::epoll_create1(EPOLL_CLOEXEC);
    SharedFd wake_guard(wake);
    for (int f : {stop_fd, watcher ? watcher->fd() : -1, done->fd}) {
        if (f < 0 || wake < 0) continue;
        epoll_event ev{};
        ev.events = EPOLLIN;
        ev.data.fd = f;
        ::epoll_ctl(wake, EPOLL_CTL_ADD, f, &ev);
    }
    int wait_fd = wake >= 0 ? wake : stop_fd;
    for (int tick = 0;; ++tick) {
        if (on_monitor_tick) on_monitor_tick(tick);
        if (fd_readable(stop_fd)) return;
        int64_t now = mono_ns();
        if (now >= next_tx) {
            announce_all(120);  // keep our neighbour entry alive on the switch (TTL 120 s)
            next_tx = now + cfg_.lldp_tx_interval_ns;
        }
        if ((xgmi_watch || pcie_watch) && !poll.valid() && now >= next_health) {
            std::vector<std::string> bdfs = xgmi_watch ? xgmi_health_bdfs() : std::vector<std::string>{};
            std::vector<std::pair<std::string, std::string>> fns;  // (NIC, its GPU)
            if (pcie_watch)
                for (const auto& n : nics_) fns.emplace_back(n.ifname, n.gpu_bdf);
            const int64_t timeout = cfg_.sysfs_read_timeout_ns;
            poll = bounded::Call<HealthSample>("", [root, bdfs, fns, timeout, xgmi_watch, pcie_watch] {
                HealthSample s;
                if (xgmi_watch) {
                    s.xgmi = topo::read_xgmi_health(root, bdfs, timeout);
                    s.xgmi_read = true;
                }
                if (pcie_watch) {
                    // One bounded call per NIC, all started first: a stalled function costs one wait.
                    std::vector<bounded::Call<std::pair<topo::PcieLink, topo::PcieLink>>> calls;
                    for (const auto& [ifname, gpu] : fns)
                        calls.emplace_back("pcie:" + ifname, [root, ifname = ifname, gpu = gpu] {
                            topo::PcieLink nic, g;
                            if (auto d = topo::netdev_pci(root, ifname)) nic = topo::read_pcie_link(root, d->bdf);
                            if (!gpu.empty()) g = topo::read_pcie_link(root, gpu);
                            return std::make_pair(nic, g);
                        });
                    const int64_t deadline = mono_ns() + timeout;
                    for (auto& c : calls) {
                        auto r = c.wait(deadline);
                        s.pcie.push_back(r ? *r : std::make_pair(topo::PcieLink{}, topo::PcieLink{}));
                        s.pcie_late.push_back(!r);
                    }
                    s.pcie_read = true;
                }
                return s;
            }, [done] {
                const uint64_t one = 1;
                (void)!::write(done->fd, &one, sizeof one);
            });
        }
        // LLDP: a changed Port Description means the switch port was re-addressed.
        bool changed = false;
        auto on_frame = [&](const std::string& ifname, const lldp::Frame& f) -> bool {
            if (f.ttl == 0) return false;
            for (auto& n : nics_)
                if (n.ifname == ifname && refresh_from_frame(n, f)) changed = true;
            return false;
        };
        int64_t until = std::min(next_tx, mono_ns() + cfg_.monitor_tick_ns);
        if (holddown_until_ > 0) until = std::min(until, holddown_until_);
        if (next_rdma > 0) until = std::min(until, next_rdma);
        if (gid_retry_until_ > 0) until = std::min(until, std::max(next_gid_look, mono_ns()));
        lldp_->run(until, on_frame, wait_fd);
        if (fd_readable(stop_fd)) return;
        for (auto& n : nics_) {  // a cached Port Description the switch never confirmed
            if (!n.lldp_from_cache || n.cache_stale || mono_ns() - n.t_cache_applied < cfg_.lldp_cache_confirm_ns) continue;
            NLOG_W("interface '%s': no LLDP frame confirmed the cached Port Description within %s",
                   n.ifname.c_str(), format_go_duration(cfg_.lldp_cache_confirm_ns).c_str());
            n.cache_stale = true;
            changed = true;
        }
        // Link state.
        std::string removed;
        if (watcher) {
            for (auto& ev : watcher->wait(mono_ns())) {
                for (auto& n : nics_) {
                    if (n.link.index != ev.link.index) continue;
                    if (ev.deleted) {  // driver reload, hot-unplug: the NIC will come back as a new ifindex
                        removed = n.ifname;
                        continue;
                    }
                    bool was_up = n.link.up(), had_carrier = carrier[n.link.index];
                    n.link.flags = ev.link.flags;
                    n.link.operstate = ev.link.operstate;
                    bool up = n.link.up(), lower = n.link.lower_up();
                    if (n.no_carrier) {  // never had a link since the start (L2)
                        if (up && lower) {
                            NLOG_I("Interface '%s' has carrier now", n.ifname.c_str());
                            n.no_carrier = false;
                            n.configured = l2_link_ok(n);  // --min-link-speed-gbps: checked now it has a speed
                            changed = true;
                        }
                        if (lower) carrier[n.link.index] = true;
                        continue;
                    }
                    if ((was_up && !up) || (had_carrier && !lower)) {
                        if (!n.degraded) {
                            NLOG_W("Interface '%s' lost link (%s)", n.ifname.c_str(), n.link.flags_str().c_str());
                            n.degraded = true;
                            ++n.flaps;
                            ++flaps_;
                            changed = true;
                        }
                    } else if (n.degraded && up && (lower || !had_carrier)) {
                        NLOG_I("Interface '%s' recovered", n.ifname.c_str());
                        n.degraded = false;
                        // The RDMA core drops a netdev's IP GIDs when it goes down and adds them
                        // again when it comes up, in whatever GID slots are free then: look the
                        // index up again before rccl.env is written for the republished label.
                        n.gid_index.reset();
                        // Administrative down flushes the routes: ensure address and routes again.
                        if (cfg_.mode == "L3" && n.addr) {
                            n.configured = false;
                            n.peer_verified = false;  // the switch port may have come back different
                            configure_interface(n);
                        } else if (cfg_.mode == "L2") {
                            n.configured = l2_link_ok(n);  // a port may renegotiate down when it comes back
                        }
                        changed = true;
                    }
                    if (lower) carrier[n.link.index] = true;
                }
            }
        }
        if (!removed.empty()) {
            // Everything this agent knows about the NIC (ifindex, LLDP socket, RDMA device, GID) is
            // gone with it.  Tear down and exit: the kubelet restarts the container, and the new agent
            // discovers the node again once the NIC is back (until then it fails to start and
            // retries; the node stays unlabelled).  Monitoring on would otherwise stay degraded for good.
            NLOG_W("Interface '%s' was removed: cleaning up and exiting so that a restarted agent discovers the node again",
                   removed.c_str());
            // Its rail rule is not tied to the link and would outlive it (its routes went with the
            // link): remove what was installed for it before forgetting the NIC.
            for (auto& n : nics_)
                if (n.ifname == removed) remove_rail_routing(n);
            nics_.erase(std::remove_if(nics_.begin(), nics_.end(), [&](const NicState& n) { return n.ifname == removed; }),
                        nics_.end());
            ready_ = false;
            post_cleanups();
            write_status();
            throw AgentError("Interface '" + removed + "' was removed");
        }
        if (poll.valid() && poll.done()) {
            uint64_t n = 0;
            (void)!::read(done->fd, &n, sizeof n);
            const uint64_t late_before = late_reads_total();
            if (auto s = poll.wait(0)) changed |= apply_health(*s);
            if (!changed && late_reads_total() != late_before) write_status();  // the late-read counter, at once
            poll = {};
            next_health = mono_ns() + cfg_.xgmi_health_interval_ns;
        }
        if (topo_late_ && labelled && topo_call_.done())
            write_rccl_env_file();  // the topology worker answered after the start's deadline after all
        if (gid_retry_until_ > 0 && mono_ns() >= next_gid_look) {
            // GIDs the RDMA core had not (re)added when the artifacts were written: looked up again
            // every 100 ms until --gid-wait has passed, never by blocking this loop.  Meanwhile
            // rccl.env names no NCCL_IB_GID_INDEX (RCCL picks each HCA's RoCE v2 GID itself).
            next_gid_look = mono_ns() + kGidLookNs;
            if (look_up_gids() && labelled) {  // every artifact that names a GID index: rccl.env, L3's rccl-net.json
                if (cfg_.mode == "L3")
                    write_artifacts(0);
                else
                    write_l2_artifacts(0);
            }
            if (!gids_missing() || !labelled) {
                gid_retry_until_ = 0;
            } else if (mono_ns() >= gid_retry_until_) {
                for (const auto& n : nics_)
                    if (!n.rdma_dev.empty() && n.configured && !n.gid_index)
                        NLOG_W("%s (%s): no RoCE v2 GID after %s; rccl.env gets no NCCL_IB_GID_INDEX for it", n.ifname.c_str(),
                               n.rdma_dev.c_str(), format_go_duration(cfg_.gid_wait_ns).c_str());
                gid_retry_until_ = 0;
            }
        }
        bool rdma_changed = false;
        if (next_rdma > 0 && mono_ns() >= next_rdma) {
            // --require-rdma: a driver container (or the node) loading the NICs' RDMA driver, and
            // after readiness a driver unloaded or reloaded under a labelled node.
            rdma_changed = refresh_rdma();
            if (rdma_changed) changed = true;
            if (!rdma_missing().empty() && rdma_reason() != rdma_said) changed = true;  // the wait ran out
            rdma_said = rdma_reason();
            // Quickly while a device is missing; at the health interval once every rail has one.
            const int64_t every = rdma_missing().empty() ? cfg_.xgmi_health_interval_ns : cfg_.rdma_poll_ns;
            next_rdma = every > 0 ? mono_ns() + every : 0;
        }
        if (cfg_.mode == "L3" && cfg_.verify_peers_ns > 0 && mono_ns() >= next_verify) {
            // NICs whose peer has not answered (yet): a recovered link, a new /30, or a switch
            // port still without its address.  Failed NICs are asked again a second later.  The
            // probe blocks this loop, so it is capped well below the start-up timeout: a switch
            // answers ARP in microseconds, and a port that is still coming up gets the next round
            // instead of delaying the other NICs' link and LLDP events by the whole --verify-peers.
            std::vector<NicState*> todo;
            for (auto& n : nics_)
                if (n.configured && !n.peer_verified && n.link.up() && !n.degraded) todo.push_back(&n);
            if (!todo.empty()) {
                const int bad = verify_peers(todo, std::min(cfg_.verify_peers_ns, kMonitorVerifyNs), stop_fd);
                if (bad < 0) return;
                changed = true;
                next_verify = bad > 0 ? mono_ns() + 1000000000LL : 0;
            }
        }
        const bool holddown_due = holddown_until_ > 0 && mono_ns() >= holddown_until_;
        if (changed || holddown_due) {
            bool healthy = xgmi_error_.empty() &&
                           std::all_of(nics_.begin(), nics_.end(), [&](const NicState& n) { return nic_healthy(n); });
            if (healthy && !labelled) {
                // After a withdrawal: republish only once the node has stayed healthy for the
                // hold-down (the first publication is not delayed).
                const bool hold = label_withdrawals_ > 0 && cfg_.label_holddown_ns > 0 &&
                                  (holddown_until_ == 0 || mono_ns() < holddown_until_);
                if (hold && holddown_until_ == 0) {
                    holddown_until_ = mono_ns() + cfg_.label_holddown_ns;
                    NLOG_I("Scale-out healthy again: the readiness label follows after %s without a flap (--label-holddown)",
                           format_go_duration(cfg_.label_holddown_ns).c_str());
                }
                if (!hold) {
                    holddown_until_ = 0;
                    if (cfg_.mode == "L3")
                        write_artifacts(0);
                    else if (!cfg_.rccl_env.empty() || !cfg_.rccl_topo.empty())
                        write_l2_artifacts(0);  // a NIC that got its carrier (or RDMA device) only now has its GID now
                    gid_retry_until_ = gids_missing() ? mono_ns() + cfg_.gid_wait_ns : 0;
                    labelled = publish_label();
                    if (labelled && !phases_.count("total_ready")) phases_["total_ready"] = mono_ns() - t0_;
                    if (labelled) NLOG_I("All scale-out interfaces healthy again: readiness label republished");
                    if (cfg_.mode == "L3") write_host_config();
                    announce_all(120);
                }
            } else if (!healthy) {
                if (holddown_until_ > 0) {  // flapped again within the hold-down: the clock starts over
                    holddown_until_ = 0;
                    ++label_suppressed_;
                }
                if (labelled) {
                    ready_ = false;
                    write_status();  // the probe's reason first, then the label (see write_status)
                    artifacts::remove_labels(cfg_.labels);
                    labelled = false;
                    ++label_withdrawals_;
                    NLOG_W("Scale-out degraded: readiness label withdrawn");
                }
                if (rdma_changed && !rdma_missing().empty() && !cfg_.rccl_env.empty())
                    write_rccl_env_file();  // it names an HCA that is gone: removed until the devices are back
            } else if (healthy && labelled && cfg_.mode == "L3") {
                write_artifacts(0);  // re-addressed NIC (or a renumbered RDMA device): refresh the RCCL artifacts
                gid_retry_until_ = gids_missing() ? mono_ns() + cfg_.gid_wait_ns : 0;
                write_host_config();
            } else if (healthy && labelled && rdma_changed && (!cfg_.rccl_env.empty() || !cfg_.rccl_topo.empty())) {
                write_l2_artifacts(0);  // L2: a renumbered RDMA device, its link-local GID
                gid_retry_until_ = gids_missing() ? mono_ns() + cfg_.gid_wait_ns : 0;
            }
            ready_ = labelled;
            write_status();
        }
    }
}

}  // namespace netop::agent

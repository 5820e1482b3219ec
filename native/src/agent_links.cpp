// Agent: what each NIC's link says before it is configured.  LLDP detection (fan-out over all
// NICs, the Port Description cache, the silent-NIC diagnosis), link speed and L2 carrier.
#include "netop/agent.hpp"

#include <errno.h>
#include <linux/if.h>
#include <linux/rtnetlink.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <map>
#include <set>

#include "agent_internal.hpp"
#include "netop/log.hpp"

namespace netop::agent {

using detail::fd_readable;
using detail::format_gbps;

void Agent::on_lldp(NicState& n, const lldp::Frame& f) {
    n.lldp_seen = true;
    n.t_lldp = mono_ns();
    n.port_description = f.port_description.value_or("");
    n.peer_mac = f.peer_mac();
    n.peer_system_name = f.system_name.value_or("");
    n.peer_port_id = f.port_id_str();
    n.peer_max_frame = f.max_frame_size() ? int(*f.max_frame_size()) : -1;
    std::string err;
    n.addr = l3::parse_port_description(n.port_description, cfg_.token_policy, &err);
    if (!n.addr) {
        n.addr_error = err;
        NLOG_W("interface '%s': %s", n.ifname.c_str(), err.c_str());
    } else {
        n.addr_error.clear();
    }
}

bool Agent::refresh_from_frame(NicState& n, const lldp::Frame& f) {
    std::string desc = f.port_description.value_or("");
    n.peer_max_frame = f.max_frame_size() ? int(*f.max_frame_size()) : -1;  // checked at the next (re)configuration
    bool changed = false;
    if (n.lldp_from_cache) {
        n.lldp_from_cache = false;
        changed = true;  // status: lldp_source and, if it was flagged, cache_unconfirmed
        n.cache_stale = false;
        if (desc == n.port_description) {
            NLOG_I("interface '%s': the switch confirmed the cached Port Description", n.ifname.c_str());
            n.peer_mac = f.peer_mac();
            n.peer_system_name = f.system_name.value_or("");
            n.peer_port_id = f.port_id_str();
            save_lldp_cache();
            return changed;
        }
    }
    if (desc == n.port_description) return changed;
    NLOG_I("Port Description of '%s' changed: '%s' -> '%s'", n.ifname.c_str(), n.port_description.c_str(), desc.c_str());
    auto old = n.addr;
    on_lldp(n, f);
    if (n.addr && old && n.addr->local == old->local) return changed;
    // drop the old address (its /30 and /16 routes go with it) and the rail rule and routes
    // installed for it, then configure the new one
    remove_rail_routing(n);
    try {
        for (auto& a : ops_.addr_list(n.link.index, AF_INET)) ops_.addr_del(a);
    } catch (const std::exception& e) {
        NLOG_W("could not remove old address of '%s': %s", n.ifname.c_str(), e.what());
    }
    n.configured = false;
    n.peer_verified = false;  // a new /30: a new peer to ask
    n.gid_index.reset();  // the GID follows the address
    if (n.addr) configure_interface(n);
    ++reconfigs_;
    save_lldp_cache();
    return true;
}

int Agent::apply_lldp_cache(const std::set<int>& listening) {
    if (cfg_.lldp_cache.empty() || !cfg_.keep_running || !cfg_.monitor) return 0;
    const auto entries = artifacts::read_lldp_cache(cfg_.lldp_cache);
    const int64_t now = int64_t(::time(nullptr));
    int applied = 0;
    for (auto& n : nics_) {
        // Only NICs with an LLDP socket: nothing else could ever confirm the entry.
        if (!listening.count(n.link.index) || n.lldp_seen) continue;
        for (const auto& e : entries) {
            if (e.ifname != n.ifname || e.nic_mac != n.link.mac.str()) continue;  // another NIC now
            if (now - e.unix_s > cfg_.lldp_cache_max_age_ns / 1000000000 || e.unix_s > now + 60) break;
            std::string err;
            auto addr = l3::parse_port_description(e.port_description, cfg_.token_policy, &err);
            if (!addr) break;
            n.lldp_seen = true;
            n.lldp_from_cache = true;
            n.t_lldp = n.t_cache_applied = mono_ns();
            n.port_description = e.port_description;
            n.peer_mac = MacAddr::parse(e.peer_mac);
            n.peer_system_name = e.system_name;
            n.peer_port_id = e.port_id;
            n.addr = addr;
            n.addr_error.clear();
            NLOG_I("interface '%s': Port Description '%s' from the LLDP cache (%llds old), awaiting confirmation",
                   n.ifname.c_str(), e.port_description.c_str(), (long long)(now - e.unix_s));
            if (cfg_.pipeline && cfg_.configure) configure_interface(n);
            ++applied;
            break;
        }
    }
    return applied;
}

void Agent::save_lldp_cache() {
    if (cfg_.lldp_cache.empty()) return;
    const auto old = artifacts::read_lldp_cache(cfg_.lldp_cache);
    std::vector<artifacts::LldpCacheEntry> out;
    const int64_t now = int64_t(::time(nullptr));
    for (const auto& n : nics_) {
        if (!n.lldp_seen || !n.addr) continue;
        if (n.lldp_from_cache) {  // not confirmed yet: keep the entry (and its age) as it was
            for (const auto& e : old)
                if (e.ifname == n.ifname && e.nic_mac == n.link.mac.str()) out.push_back(e);
            continue;
        }
        out.push_back({n.link.mac.str(), n.ifname, now, n.peer_mac ? n.peer_mac->str() : "", n.peer_system_name,
                       n.peer_port_id, n.port_description});
    }
    try {
        artifacts::write_lldp_cache(cfg_.lldp_cache, out);
    } catch (const std::exception& e) {
        NLOG_W("Could not write the LLDP cache: %s", e.what());
    }
}

void Agent::detect_lldp(int stop_fd) {
    int listening = 0;
    std::set<int> listened;
    for (auto& n : nics_) {
        if (!n.link.up()) {
            NLOG_I("Link '%s' %s, cannot start LLDP", n.ifname.c_str(), n.link.operstate_str().c_str());
            continue;
        }
        try {
            lldp_->add(n.ifname, n.link.index, n.link.mac);
            ++listening;
            listened.insert(n.link.index);
            NLOG_I("Started LLDP discovery for '%s'...", n.ifname.c_str());
        } catch (const std::exception& e) {
            NLOG_I("Cannot start LLDP client: %s", e.what());
        }
    }
    if (!listening) return;
    for (auto& n : nics_) {  // what each NIC hears while we wait: the diagnosis of a silent one
        if (!listened.count(n.link.index)) continue;
        try {
            if (auto s = ops_.link_stats(n.link.index)) n.rx_at_listen = s->rx_packets;
        } catch (const std::exception&) {  // diagnostics only
        }
    }
    int remaining = listening - apply_lldp_cache(listened);
    if (remaining <= 0) {
        NLOG_I("Every listening interface was configured from the LLDP cache; the switch confirms it while monitoring");
        // Still introduce ourselves as a new neighbour, so a fast-start switch confirms now rather
        // than at its next periodic frame.
        if (cfg_.announce_shutdown_first) announce_all(0);
        announce_all(120);
        return;
    }
    auto cb = [&](const std::string& ifname, const lldp::Frame& f) -> bool {
        if (f.ttl == 0) return false;  // shutdown LLDPDU: the neighbour is going away
        for (auto& n : nics_) {
            if (n.ifname != ifname) continue;
            if (n.lldp_from_cache) {  // configured from the cache: confirm it, or readdress now
                refresh_from_frame(n, f);
                continue;
            }
            if (n.lldp_seen) continue;  // first frame per NIC wins (client.go:141-142)
            on_lldp(n, f);
            if (cfg_.pipeline && cfg_.configure && n.addr) configure_interface(n);
            --remaining;
        }
        return remaining == 0;
    };
    const int64_t deadline = mono_ns() + cfg_.wait_ns;
    std::map<int, int> announces;  // ifindex -> LLDPDUs sent
    auto announce_nic = [&](NicState& n, bool retry) {
        try {
            // After a crash the switch still holds our old neighbour entry and would not treat us
            // as new (no fast start).  A shutdown LLDPDU first deletes that entry (802.1AB-2009
            // 9.2.7.7.1), so the next LLDPDU is a new neighbour again.  Retries do the same: if
            // the switch heard us but its immediate answer was lost (its port was not
            // transmitting yet), only a "new" neighbour makes it answer again before its next
            // fast-transmit tick.
            if ((announces[n.link.index] == 0 || retry) && cfg_.announce_shutdown_first)
                lldp_->announce(n.ifname, lldp::encode(make_node_frame(cfg_.node_name, n.ifname, n.link.mac, n.gpu_bdf, 0)));
            lldp_->announce(n.ifname,
                            lldp::encode(make_node_frame(cfg_.node_name, n.ifname, n.link.mac, n.gpu_bdf, 120, cfg_.mtu)));
        } catch (const std::exception& e) {
            NLOG_V(2, "LLDP announce on %s failed: %s", n.ifname.c_str(), e.what());
        }
        ++announces[n.link.index];
    };
    // A frame sent before the kernel can transmit on the link is dropped without an error:
    // admin-up is not enough, the device is usable once linkwatch has attached its qdisc and
    // set operstate UP — and linkwatch batches that work up to a second apart.  So each NIC is
    // announced the moment its own RTM_NEWLINK says it is operational, not all at link-up.
    std::unique_ptr<nl::LinkWatcher> watcher;
    if (cfg_.lldp_announce) {
        try {
            watcher = ops_.subscribe_links();
        } catch (const std::exception& e) {
            NLOG_V(2, "link events unavailable, announcing on admin-up links: %s", e.what());
        }
        if (watcher && watcher->fd() < 0) watcher.reset();  // no pollable events: announce right away
        if (watcher) {
            for (auto& n : nics_) {  // state after subscribing: no transition can be missed
                try {
                    auto l = ops_.link_by_name(n.ifname);
                    n.link.flags = l.flags;
                    n.link.operstate = l.operstate;
                } catch (const std::exception&) {
                }
            }
        }
    }
    auto can_tx = [&](const NicState& n) {
        if (!watcher) return n.link.up();
        return n.link.up() && (n.link.operstate == IF_OPER_UP || (n.link.operstate == IF_OPER_UNKNOWN && n.link.lower_up()));
    };
    int wake = -1;  // stop_fd or link events
    if (watcher) {
        wake = ::epoll_create1(EPOLL_CLOEXEC);
        for (int f : {stop_fd, watcher->fd()}) {
            if (f < 0 || wake < 0) continue;
            epoll_event ev{};
            ev.events = EPOLLIN;
            ev.data.fd = f;
            ::epoll_ctl(wake, EPOLL_CTL_ADD, f, &ev);
        }
    }
    struct CloseFd {
        int fd;
        ~CloseFd() {
            if (fd >= 0) ::close(fd);
        }
    } wake_guard{wake};
    const int wait_fd = wake >= 0 ? wake : stop_fd;
    int rounds = 0;
    int64_t next_round = mono_ns();
    pkt::ListenResult r = pkt::ListenResult::Deadline;
    // The probe's per-NIC reason ("waiting for carrier" / "waiting for LLDP") once the wait has
    // lasted 100 ms: a fast-start switch answers within a few ms, and writing the status then
    // would sit on the node-ready critical path (~2 ms); the kubelet probes every 5 s anyway.
    bool status_written = false;
    const int64_t status_at = mono_ns() + 100LL * 1000000;
    for (;;) {
        if (cfg_.lldp_announce && rounds < cfg_.announce_count && mono_ns() >= next_round) {
            // Round 0: every NIC that can transmit.  Later rounds (1 s apart): every NIC still
            // silent, operational or not — a lost frame or a driver without operstate.
            for (auto& n : nics_)
                if (n.link.up() && !n.lldp_seen && (rounds > 0 || can_tx(n))) announce_nic(n, rounds > 0);
            ++rounds;
            // Retry early, then back off (25 ms, 100 ms, 300 ms, then the interval): a lost
            // frame or answer costs tens of milliseconds, not a full interval.
            const int64_t step = rounds == 1   ? cfg_.announce_interval_ns / 40
                                 : rounds == 2 ? cfg_.announce_interval_ns / 10
                                 : rounds == 3 ? cfg_.announce_interval_ns * 3 / 10
                                               : cfg_.announce_interval_ns;
            next_round = mono_ns() + step;
        }
        if (!status_written && mono_ns() >= status_at) {
            status_written = true;
            write_status();
        }
        int64_t slice_end = cfg_.lldp_announce && rounds < cfg_.announce_count ? std::min(deadline, next_round) : deadline;
        if (!status_written) slice_end = std::min(slice_end, status_at);
        r = lldp_->run(slice_end, cb, wait_fd);
        if (r == pkt::ListenResult::Interrupted && watcher && !fd_readable(stop_fd)) {
            for (auto& ev : watcher->wait(mono_ns())) {  // link events: announce on newly operational NICs
                for (auto& n : nics_) {
                    if (n.link.index != ev.link.index || ev.deleted) continue;
                    const bool had_carrier = n.link.lower_up();
                    n.link.flags = ev.link.flags;
                    n.link.operstate = ev.link.operstate;
                    if (!n.lldp_seen && announces[n.link.index] == 0 && can_tx(n)) announce_nic(n, false);
                    // "waiting for carrier" -> "waiting for LLDP" (or back) in the probe's reason
                    if (status_written && !n.lldp_seen && had_carrier != n.link.lower_up()) write_status();
                }
            }
            if (mono_ns() >= deadline) {
                r = pkt::ListenResult::Deadline;
                break;
            }
            continue;
        }
        if (r != pkt::ListenResult::Deadline || mono_ns() >= deadline) break;
    }
    if (r == pkt::ListenResult::Interrupted) aborted_ = true;
    if (r == pkt::ListenResult::Deadline) {
        NLOG_I("LLDP wait of %s expired with %d interface(s) silent", format_go_duration(cfg_.wait_ns).c_str(), remaining);
        diagnose_silent();
    }
}

void Agent::diagnose_silent() {
    // The reference's barrier times out without saying why (cmd/discover/main.go:84-122).  On
    // RoCE NICs the usual cause is the NIC firmware's own LLDP/DCBX agent consuming the
    // switch's LLDPDUs; tell that apart from a dead link or an undecodable
    // frame with what the NIC did hear while we waited.
    std::string root = cfg_.sysfs_root.empty() ? topo::sysfs_root() : cfg_.sysfs_root;
    const std::string waited = format_go_duration(cfg_.wait_ns);
    for (auto& n : nics_) {
        if (n.lldp_seen || n.lldp_from_cache) continue;
        try {
            if (auto d = topo::netdev_pci(root, n.ifname)) n.driver = d->driver;
            if (n.driver.empty() && ethtool_) n.driver = ethtool_->driver(n.ifname);
        } catch (const std::exception&) {
        }
        const std::string drv = n.driver.empty() ? "unknown driver" : n.driver;
        if (!n.link.up()) {
            n.lldp_silent = drv + ": link down, nothing listened";
            NLOG_W("%s: %s", n.ifname.c_str(), n.lldp_silent.c_str());
            continue;
        }
        // Admin-up without a carrier for the whole wait: no frame could come, whoever runs LLDP.
        bool carrier = n.link.lower_up();
        try {
            carrier = ops_.link_by_name(n.ifname).lower_up();
        } catch (const std::exception&) {
        }
        if (!carrier) {
            n.lldp_silent = strfmt("%s: no carrier in %s (check the cable, the switch port and the optic)", drv.c_str(),
                                   waited.c_str());
            NLOG_W("%s: %s", n.ifname.c_str(), n.lldp_silent.c_str());
            continue;
        }
        std::optional<uint64_t> rx;
        try {
            if (n.rx_at_listen)
                if (auto s = ops_.link_stats(n.link.index))
                    rx = s->rx_packets >= *n.rx_at_listen ? s->rx_packets - *n.rx_at_listen : 0;
        } catch (const std::exception&) {
        }
        auto ls = lldp_->stats_for(n.ifname);
        std::string heard = rx ? strfmt("%llu frame(s) arrived meanwhile", (unsigned long long)*rx)
                               : std::string("receive counters unavailable");
        // Who runs DCBX (and so LLDP) on this port: the host, or an agent embedded in the NIC?
        // Read-only, unprivileged (DCB netlink); --disable-fw-lldp has read it already.
        if (n.dcbx.empty()) {
            try {
                if (!ethtool_) ethtool_ = ethtool::make_ioctl_ops();
                if (auto m = ethtool_->dcbx_get(n.ifname)) {
                    n.dcbx = ethtool::dcbx_str(*m);
                    n.dcbx_embedded = ethtool::dcbx_embedded(*m);
                }
            } catch (const std::exception& e) {
                NLOG_V(2, "%s: DCBX mode unreadable: %s", n.ifname.c_str(), e.what());
            }
        }
        std::string why;
        if (ls && ls->malformed) {
            why = strfmt("%llu LLDPDU(s) did not decode", (unsigned long long)ls->malformed);
        } else if (rx && *rx == 0) {
            why = "the link received nothing: check the cable, the switch port and its LLDP transmit setting";
        } else if (n.dcbx_embedded) {
            why = "the NIC's embedded agent runs DCBX and LLDP on this port (DCBX " + n.dcbx + ")" +
                  (cfg_.disable_fw_lldp && cfg_.fw_lldp_dcbx_host
                       ? " although --disable-fw-lldp ran (" + n.fw_lldp + ")"
                       : ": run with --disable-fw-lldp --fw-lldp-dcbx-host to hand DCBX to the host (the host must "
                         "then run DCBX for PFC/ETS itself)");
        } else if (n.driver == "i40e" || n.driver == "ice") {
            why = cfg_.disable_fw_lldp ? "NIC-firmware LLDP agent suspected although --disable-fw-lldp ran (" + n.fw_lldp + ")"
                                       : "NIC-firmware LLDP agent suspected: run with --disable-fw-lldp";
        } else if (!n.dcbx.empty()) {
            why = "DCBX is host-managed (" + n.dcbx + "), so no NIC-firmware DCBX agent holds the port: check that the "
                  "switch port transmits LLDP to the nearest-bridge address 01:80:c2:00:00:0e";
        } else {
            why = "NIC-firmware LLDP agent suspected (no verified switch for this driver; see the user guide, "
                  "\"Silent LLDP\")";
        }
        n.lldp_silent = strfmt("%s: no LLDPDU in %s, %s; %s", drv.c_str(), waited.c_str(), heard.c_str(), why.c_str());
        NLOG_W("%s: %s", n.ifname.c_str(), n.lldp_silent.c_str());
    }
}

std::string Agent::check_link_speed(NicState& n) {
    if (cfg_.min_link_speed_mbps <= 0) return "";
    const std::string root = cfg_.sysfs_root.empty() ? topo::sysfs_root() : cfg_.sysfs_root;
    n.speed_mbps = topo::netdev_speed_mbps(root, n.ifname);
    if (n.speed_mbps < 0) {
        NLOG_W("Interface '%s': the driver reports no link speed; --min-link-speed-gbps not checked", n.ifname.c_str());
        return "";
    }
    if (n.speed_mbps >= cfg_.min_link_speed_mbps) return "";
    return strfmt("link negotiated at %s Gb/s, below the required %s Gb/s (a marginal cable or optic, or a port "
                  "renegotiated down: reseat or replace it)",
                  format_gbps(n.speed_mbps).c_str(), format_gbps(cfg_.min_link_speed_mbps).c_str());
}

std::string Agent::silent_summary() const {
    std::vector<std::string> parts, failed;
    for (const auto& n : nics_) {
        if (!n.lldp_silent.empty()) parts.push_back(n.ifname + " (" + n.lldp_silent + ")");
        if (n.addr && !n.configured && !n.config_error.empty()) failed.push_back(n.ifname + ": " + n.config_error);
    }
    std::string out = parts.empty() ? "" : strfmt("LLDP silent on %zu NIC(s): ", parts.size()) + join(parts, "; ");
    if (!failed.empty()) out += (out.empty() ? "" : " ") + strfmt("Not configured: %s", join(failed, "; ").c_str());
    return out;
}

std::string Agent::check_pcie(NicState& n) {
    ensure_pcie();
    if (!cfg_.require_full_pcie) return "";
    if (pcie_late_ && !n.pcie.known())
        return "its PCIe link state did not answer in " + format_go_duration(cfg_.sysfs_read_timeout_ns) +
               " (a function in error recovery?)";
    if (n.pcie.degraded())
        return strfmt("its PCIe link trained at %s: RDMA moves at a fraction of the rail's rate (reseat the card, check the "
                      "riser and the slot's BIOS link setting)", n.pcie.str().c_str());
    if (n.gpu_pcie.narrower())
        return strfmt("the PCIe link of its GPU %s trained at x%d of x%d: GPUDirect RDMA to and from it is throttled "
                      "(reseat the GPU, check the riser)", n.gpu_bdf.c_str(), n.gpu_pcie.width, n.gpu_pcie.max_width);
    return "";
}

bool Agent::l2_link_ok(NicState& n) {
    n.config_error = check_link_speed(n);
    if (n.config_error.empty()) n.config_error = check_pcie(n);
    if (!n.config_error.empty()) NLOG_W("Interface '%s' not ready: %s", n.ifname.c_str(), n.config_error.c_str());
    return n.link.up() && !n.no_carrier && n.config_error.empty();
}

bool Agent::wait_carrier(int stop_fd) {
    // Admin-up is not a link: a NIC without carrier (unplugged cable, switch port down, optic
    // dead) carries nothing, so L2 readiness needs IFF_LOWER_UP on every NIC.  The reference
    // publishes its label right after link-up (cmd/discover/main.go:198-206,239-246).
    std::unique_ptr<nl::LinkWatcher> watcher;
    try {
        watcher = ops_.subscribe_links();
    } catch (const std::exception& e) {
        NLOG_W("link events unavailable, carrier read once: %s", e.what());
    }
    for (auto& n : nics_) {  // the state after subscribing: no transition can be missed
        try {
            auto l = ops_.link_by_name(n.ifname);
            n.link.flags = l.flags;
            n.link.operstate = l.operstate;
        } catch (const std::exception&) {
        }
    }
    auto dark = [](const NicState& n) { return n.link.up() && !n.link.lower_up(); };
    auto missing = [&] { return std::any_of(nics_.begin(), nics_.end(), dark); };
    // While the links train, the readiness probe says so ("waiting for carrier", a start-up
    // reason for the operator), not "no carrier": that only once carrier_wait_ns has passed.
    int waiting = 0;
    for (auto& n : nics_) waiting += (n.awaiting_carrier = dark(n));
    if (waiting) {
        NLOG_I("Waiting up to %s for carrier on %d interface(s)", format_go_duration(cfg_.carrier_wait_ns).c_str(), waiting);
        write_status();
    }
    const int64_t deadline = mono_ns() + cfg_.carrier_wait_ns;
    while (watcher && missing() && mono_ns() < deadline) {
        if (fd_readable(stop_fd)) return false;
        const int64_t slice = std::min<int64_t>(deadline, mono_ns() + 100000000LL);  // stop_fd checked every 100 ms
        bool changed = false;
        for (auto& ev : watcher->wait(slice))
            for (auto& n : nics_)
                if (!ev.deleted && n.link.index == ev.link.index) {
                    n.link.flags = ev.link.flags;
                    n.link.operstate = ev.link.operstate;
                    if (n.awaiting_carrier && !dark(n)) {
                        n.awaiting_carrier = false;
                        changed = true;
                        NLOG_I("Interface '%s' has carrier after %s", n.ifname.c_str(),
                               format_go_duration(mono_ns() - t0_).c_str());
                    }
                }
        if (changed && missing()) write_status();  // the probe's reason names only the NICs still training
    }
    for (auto& n : nics_) {
        n.awaiting_carrier = false;
        n.no_carrier = dark(n);
        n.configured = n.link.up() && !n.no_carrier;
        if (n.no_carrier)
            NLOG_W("Interface '%s' has no carrier after %s (%s)", n.ifname.c_str(),
                   format_go_duration(cfg_.carrier_wait_ns).c_str(), n.link.operstate_str().c_str());
    }
    return true;
}

}  // namespace netop::agent

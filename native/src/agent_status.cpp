// Agent: how it reports -- status.json and the readiness probe's one-line reason, the
// /metrics text, and the per-NIC result log.
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

std::map<std::string, std::string> Agent::status_node() const {
    std::map<std::string, std::string> m;
    if (!cfg_.node_name.empty()) m["node"] = cfg_.node_name;
    if (!gdr_.kernel.empty()) {
        m["gpudirect_rdma"] = gdr_.mode();
        m["kernel"] = gdr_.kernel;
    }
    if (cfg_.xgmi_expect_links >= 0) {
        m["xgmi_pairs"] = std::to_string(xgmi_.pairs_connected) + "/" + std::to_string(xgmi_.pairs_expected);
        int gpus = 0, up = 0, down = 0, width = 0, speed = 0;
        for (const auto& h : xgmi_health_) {
            if (!h.known) continue;
            ++gpus;
            up += h.links_up();
            down += h.links_down();
            width = width ? std::min(width, h.width) : h.width;
            speed = speed ? std::min(speed, h.speed_gbps) : h.speed_gbps;
        }
        if (gpus)
            m["xgmi_links"] = strfmt("%d up, %d down on %d GPUs, x%d at %d Gb/s (gpu_metrics)", up, down, gpus, width, speed);
        else if (!xgmi_unread_.empty())
            m["xgmi_links"] = "not checked: " + xgmi_unread_;
        if (!xgmi_error_.empty()) m["xgmi_error"] = xgmi_error_;
    }
    if (!no_rdma_.empty()) m["nics_without_rdma"] = join(no_rdma_, ",");
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

void Agent::log_results() {
    // The reference's summary (cmd/discover/main.go logResults) at -v=3 only: below that it would
    // still cost an address dump per NIC on the way to the label.
    if (log::verbosity() < 3) return;
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

uint64_t Agent::late_reads_total() const {
    uint64_t n = 0;
    for (const auto& [what, count] : late_reads_) n += count;
    return n;
}

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
    metric("netop_agent_nic_pcie_degraded", "gauge",
           "1 when the NIC's PCIe link, or its GPU's, trained below the speed or width it supports");
    for (const auto& n : nics_)
        if (n.pcie.known() || n.gpu_pcie.known())
            o += strfmt("netop_agent_nic_pcie_degraded{nic=\"%s\"} %d\n", httpd::escape_label(n.ifname).c_str(),
                        n.pcie.degraded() || n.gpu_pcie.narrower() ? 1 : 0);
    metric("netop_agent_link_flaps_total", "counter", "link losses observed after readiness");
    o += strfmt("netop_agent_link_flaps_total %d\n", flaps_);
    metric("netop_agent_label_withdrawals_total", "counter", "times the monitor withdrew the readiness label");
    o += strfmt("netop_agent_label_withdrawals_total %d\n", label_withdrawals_);
    metric("netop_agent_label_suppressed_total", "counter",
           "recoveries not republished because the node flapped again within --label-holddown");
    o += strfmt("netop_agent_label_suppressed_total %d\n", label_suppressed_);
    metric("netop_agent_sysfs_reads_late_total", "counter",
           "sysfs reads that did not answer within --sysfs-read-timeout (a wedged SMU, a function in PCIe error recovery)");
    for (const char* what : {"gpu_metrics", "pcie", "kfd", "topology"}) {
        auto it = late_reads_.find(what);
        o += strfmt("netop_agent_sysfs_reads_late_total{read=\"%s\"} %llu\n", what,
                    (unsigned long long)(it == late_reads_.end() ? 0 : it->second));
    }
    if (cfg_.require_rdma) {
        metric("netop_agent_nic_rdma", "gauge", "1 when the NIC has an RDMA device (--require-rdma: the label waits for every NIC's)");
        for (const auto& n : nics_)
            o += strfmt("netop_agent_nic_rdma{nic=\"%s\"} %d\n", httpd::escape_label(n.ifname).c_str(), n.rdma_dev.empty() ? 0 : 1);
    }
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
        bool any = false;
        for (const auto& h : xgmi_health_) any |= h.known;
        if (any) {
            metric("netop_agent_xgmi_links", "gauge", "xGMI links of a GPU by trained state (gpu_metrics)");
            for (const auto& h : xgmi_health_)
                if (h.known)
                    for (const char* st : {"up", "down"})
                        o += strfmt("netop_agent_xgmi_links{gpu=\"%s\",state=\"%s\"} %d\n", httpd::escape_label(h.bdf).c_str(),
                                    st, st[0] == 'u' ? h.links_up() : h.links_down());
            metric("netop_agent_xgmi_link_width", "gauge", "Trained xGMI link width of a GPU (lanes, gpu_metrics)");
            for (const auto& h : xgmi_health_)
                if (h.known)
                    o += strfmt("netop_agent_xgmi_link_width{gpu=\"%s\"} %d\n", httpd::escape_label(h.bdf).c_str(), h.width);
        }
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
        // Beside it, one line for the readiness probe to print while the node is not ready: the
        // kubelet records probe output in the Pod's events ("Readiness probe failed: ...").  The
        // reason goes first: a probe that finds the status file must find the reason as well, or
        // it reports a bare "label not published" -- not a start-up reason, so the operator would
        // count a node still starting as degraded.
        const std::string why = ready_ ? "" : not_ready_reason();
        if (!why.empty()) write_file_atomic(reason_path(cfg_.status_file), why + "\n");
        write_file_atomic(cfg_.status_file, artifacts::generate_status(nics_, phases_, t0_, cfg_.mode, ready_, status_node()) + "\n");
        if (why.empty()) ::unlink(reason_path(cfg_.status_file).c_str());
    } catch (const std::exception& e) {
        NLOG_W("Could not write status file: %s", e.what());
    }
}

std::string reason_path(const std::string& status_file) { return status_file + ".not-ready"; }

std::string Agent::not_ready_reason() const {
    if (!config_error_.empty()) return config_error_;
    std::vector<std::string> parts;
    if (!xgmi_error_.empty()) parts.push_back("xGMI: " + xgmi_error_);
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
        else if (!n.pcie_error.empty())
            why = n.pcie_error;
        else if (!n.addr_error.empty() && !n.configured)
            why = n.addr_error;
        else if (n.cache_stale)
            why = "the switch has not confirmed the cached Port Description";
        else if (!n.peer_error.empty())
            why = n.peer_error;
        else if (cfg_.require_rdma && n.rdma_dev.empty() && (cfg_.mode != "L3" || n.configured))
            why = rdma_reason();
        else if (cfg_.mode == "L3" && !n.configured)
            why = n.lldp_seen                           ? "not configured yet"
                  : n.link.up() && !n.link.lower_up() ? "waiting for carrier"  // no frame can come yet
                                                        : "waiting for LLDP";
        if (!why.empty()) parts.push_back(n.ifname + ": " + why);
    }
    if (parts.empty() && holddown_until_ > 0)
        parts.push_back(strfmt("label hold-down: healthy again after %d withdrawal(s), republished in %.1fs without a flap",
                               label_withdrawals_, double(std::max<int64_t>(0, holddown_until_ - mono_ns())) / 1e9));
    return join(parts, "; ");
}

}  // namespace netop::agent

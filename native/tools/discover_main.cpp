// `discover` — the MI355X network operator's node agent (DaemonSet container entrypoint).
//
// Reference: cmd/discover/main.go (cobra command `discover`).  Same flag names and
// defaults (:281-298) plus klog's -v/--v; MI355X additions are documented in --help.
#include <signal.h>
#include <sys/signalfd.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <iostream>

#include "netop/agent.hpp"
#include "netop/cli.hpp"
#include "netop/log.hpp"

using namespace netop;

int main(int argc, char** argv) {
    agent::Config cfg;
    int verbosity = 0;
    bool show_help = false, show_version = false, logtostderr = true, skip_headers = false;
    std::string log_file, logging_format = "text", discovery_mode = "affine", nic_drivers, token_policy = "compat-then-last",
                                         max_path = "PXB", vmodule, stderrthreshold;

    cli::FlagSet fs("discover");
    // klog flags first (the reference adds the Go flag set before its own, SortFlags=false).
    fs.add_int("v", &verbosity, "number for the log level verbosity");
    fs.shorthand('v', "v");
    fs.add_bool("logtostderr", &logtostderr, "log to standard error instead of files");
    fs.add_bool("alsologtostderr", &logtostderr, "log to standard error as well as files", true);
    fs.add_string("log_file", &log_file, "If non-empty, use this log file");
    fs.add_bool("skip_headers", &skip_headers, "If true, avoid header prefixes in the log messages");
    fs.add_string("vmodule", &vmodule, "comma-separated list of pattern=N settings (accepted, ignored)", true);
    fs.add_string("stderrthreshold", &stderrthreshold, "accepted for klog compatibility", true);
    fs.add_string("logging-format", &logging_format, "log format: text (klog) or json");

    fs.add_string("mode", &cfg.mode, "'L2' for network layer 2 or 'L3' for network layer 3 (L3) using LLDP");
    fs.add_bool("configure", &cfg.configure, "Configure L3 network with LLDP or set interfaces up with L2 networks");
    fs.add_bool("disable-networkmanager", &cfg.disable_nm, "Disable Host's NetworkManager for interfaces");
    fs.add_string("interfaces", &cfg.interfaces, "Comma separated list of additional network interfaces");
    fs.add_duration("wait", &cfg.wait_ns, "Time to wait for LLDP packets");
    fs.add_string("rccl-net", &cfg.rccl_net, "RCCL scale-out NIC file path (NIC_NET_CONFIG JSON)");
    fs.alias("gaudinet", "rccl-net");
    fs.add_bool("keep-running", &cfg.keep_running, "Keep running after any configurations are done");
    fs.add_string("systemd-networkd", &cfg.networkd, "Write systemd networkd configuration files to given directory");
    fs.add_int("mtu", &cfg.mtu, "MTU value to set for interfaces");

    fs.add_string("nic-discovery", &discovery_mode, "scale-out NIC discovery: affine (NICs sharing a PCIe switch with an amdgpu GPU), accel (netdevs under the accelerator PCI function), rdma (RDMA-capable NICs of --nic-drivers that are neither a GPU's rail nor the node's own NIC -- default route, a non-/30 address or a route the agent does not install: host NICs), none");
    fs.add_string("accel-driver", &cfg.discovery.accel_driver, "accelerator PCI driver to enumerate");
    fs.add_string("nic-drivers", &nic_drivers, "comma separated NIC driver allow-list for affine discovery (default: common RoCE drivers)");
    fs.add_string("max-path", &max_path, "farthest GPU<->NIC PCIe path type accepted: PIX, PXB, PHB, NODE, SYS");
    fs.add_string("token-policy", &token_policy, "Port Description address token: compat (token 1), compat-then-last, any");
    fs.add_bool("lldp-promisc", &cfg.lldp_promisc, "put interfaces in promiscuous mode while listening for LLDP");
    fs.add_bool("pipeline", &cfg.pipeline, "configure each interface as soon as its LLDP frame arrives");
    fs.add_bool("label-without-peers", &cfg.label_without_peers, "publish the readiness label even when no LLDP peer was found (reference behaviour)");
    fs.add_bool("fsync-artifacts", &cfg.fsync_artifacts, "fsync artifact, label and status files before renaming them into place (off: they are rewritten on every start)");
    fs.add_string("nfd-features-dir", &cfg.labels.dir, "NFD local feature source directory");
    fs.add_string("nfd-label-file", &cfg.labels.file, "readiness label file name inside the features directory");
    fs.add_string("nfd-label", &cfg.labels.key, "readiness label key (published as KEY=true; KEY.mode, KEY.nics, ... alongside)");
    fs.add_string("rccl-env", &cfg.rccl_env, "write an RCCL environment file (NCCL_IB_HCA, NCCL_IB_GID_INDEX, ...)");
    fs.add_string("rccl-topo", &cfg.rccl_topo, "write an RCCL topology file (NCCL_TOPO_FILE XML: the PCIe tree of the GPUs and scale-out NICs)");
    fs.add_string("rccl-topo-env-path", &cfg.rccl_topo_env_path, "NCCL_TOPO_FILE value written into the RCCL environment file (the path jobs mount; default --rccl-topo)");
    fs.add_string("rccl-socket-ifname", &cfg.socket_ifname, "NCCL_SOCKET_IFNAME in the RCCL environment file: auto (L3: the configured scale-out NICs, GPU order), none, or a list");
    fs.add_int("rail-table-base", &cfg.rail_table_base,
               "L3: per-rail source routing; NIC k (its GPU index) gets routing table and rule priority base+k (0 = off)");
    fs.add_string("rccl-env-extra", &cfg.rccl_env_extra, "site settings appended to the RCCL environment file: KEY=VALUE[,...] (NCCL_*, RCCL_*, HSA_*)");
    fs.add_string("status-file", &cfg.status_file, "write a JSON status document (per-NIC results, phase timings)");
    fs.add_string("nm-keyfile-dir", &cfg.nm_keyfile_dir, "with --disable-networkmanager, also persist an unmanaged-devices keyfile here (removed on exit)");
    fs.add_bool("nm-restore", &cfg.nm_restore, "with --disable-networkmanager: on exit, remove the keyfile and set the interfaces managed by NetworkManager again (default: they stay unmanaged across restarts)");
    fs.add_int("xgmi-expect", &cfg.xgmi_expect_links, "verify the xGMI mesh before labelling: -1 off, 0 full mesh, N GPU pairs; the links' trained state (amdgpu gpu_metrics) too: a link down fails the check");
    fs.add_bool("require-full-pcie", &cfg.require_full_pcie, "configure (and label) a NIC only if its PCIe link trained at the speed and width it supports, and its GPU's at full width; degraded links are reported either way (status.json, metrics)");
    fs.add_int("xgmi-min-link-width", &cfg.xgmi_min_link_width, "with --xgmi-expect: the narrowest trained xGMI link width (lanes) a GPU may run at, from gpu_metrics; 0 = any");
    fs.add_duration("xgmi-health-interval", &cfg.xgmi_health_interval_ns, "with the monitor: how often the xGMI links' state (with --xgmi-expect) and the rails' PCIe links (with --require-full-pcie) are read again; a link down or retrained narrower withdraws the readiness label until it is back (0 = at start only)");
    fs.add_duration("sysfs-read-timeout", &cfg.sysfs_read_timeout_ns, "bound on each sysfs read firmware or hardware answers (gpu_metrics: an SMU query per GPU; PCIe link state; the KFD topology): a read still blocked then is reported and the label follows the policy, the start and the monitor never wait behind it");
    fs.add_duration("label-holddown", &cfg.label_holddown_ns, "with the monitor: after the readiness label was withdrawn, republish it only once the node has been healthy this long without a flap (0 = at once; the first publication is never delayed)");
    fs.add_int("xgmi-down-samples", &cfg.xgmi_down_samples, "with the monitor: consecutive gpu_metrics samples that must see an xGMI link down before it counts (a status read during a GPU reset is not a flap)");
    fs.add_bool("allow-policy-routed", &cfg.allow_policy_routed, "configure a NIC that has a default route in a per-NIC policy-routing table even when it holds the node's own address (not a /30, or the source its rule selects); by default such a NIC is refused like the node's uplink");
    fs.add_bool("require-rdma", &cfg.require_rdma, "every scale-out NIC must have an RDMA device (its RDMA driver loaded) before the readiness label and rccl.env: the NICs are configured, the probe says 'waiting for RDMA device', and the monitor labels the node once the devices appear");
    fs.add_duration("rdma-wait", &cfg.rdma_wait_ns, "with --require-rdma: how long after the start a missing RDMA device is 'waiting' (start-up) before it is reported as the fault 'no RDMA device (load its RDMA driver)'");
    fs.add_duration("rdma-poll-interval", &cfg.rdma_poll_ns, "with --require-rdma: how often the waiting agent looks for the RDMA devices", true);
    fs.add_duration("link-wait", &cfg.link_wait_ns, "time to wait for link state echoes from the kernel");
    fs.add_duration("carrier-wait", &cfg.carrier_wait_ns, "L2: time every admin-up NIC may take to get a carrier (optic and switch port link training) before it is reported as 'no carrier'; meanwhile the readiness probe says 'waiting for carrier' (with the monitor a NIC still dark afterwards is labelled when its carrier comes)");
    fs.add_duration("verify-peers", &cfg.verify_peers_ns,
                    "L3: before publishing readiness, require every NIC's switch-side /30 address to answer ARP within this time (0 = off)");
    fs.add_duration("gid-wait", &cfg.gid_wait_ns, "time to wait for the RoCE v2 GID of a newly configured address");
    fs.add_bool("lldp-announce", &cfg.lldp_announce, "transmit our own LLDPDU on each NIC (makes 802.1AB-2009 switches answer within ~1s)");
    fs.add_bool("lldp-restart-fast", &cfg.announce_shutdown_first, "send a shutdown LLDPDU before the first announcement so a switch holding a stale entry (agent restart) fast-starts again");
    fs.add_bool("keep-config", &cfg.keep_config, "on exit withdraw only the readiness label: addresses, routes, rail rules and links stay for the next agent, which adopts the /30 its LLDP cache confirms (hitless agent restarts; needs --lldp-cache in L3)");
    fs.add_bool("cleanup", &cfg.cleanup, "one-shot: remove what --keep-config agents left on the node (IPv4 addresses of the discovered NICs, tagged rail rules and routes, label, artifacts, LLDP cache, networkd files) and exit");
    std::string node_lock = "auto";
    fs.add_string("node-lock", &node_lock, "node-wide lock (abstract unix socket) held while the agent runs, so agents configuring the same NICs never overlap (exiting vs starting agent, agent vs --cleanup, two policies on one node): auto (named after --nfd-label-file), none, or a name");
    fs.add_duration("rediscover-interval", &cfg.rediscover_ns, "host-nic discovery that left every NIC to the node or to amd-so: how often the idle agent looks again; when a NIC of its own appears it exits so that its restart configures it (0 = never)");
    fs.add_duration("node-lock-wait", &cfg.node_lock_wait_ns, "how long to wait for the node lock (and each NIC lock) before failing");
    cfg.nic_locks = true;
    fs.add_bool("nic-lock", &cfg.nic_locks, "hold a node-wide lock per configured NIC (abstract unix socket netop-nic:<ifname>) so two agents, whatever their policies and label files, never configure one NIC");
    bool include_gpu_rails = false;
    fs.add_bool("rdma-include-gpu-rails", &include_gpu_rails, "with --nic-discovery=rdma, also take RDMA NICs that sit next to a GPU (its scale-out rail, which an amd-so agent owns); default: left alone");
    fs.add_bool("check-peer-mtu", &cfg.check_peer_mtu, "refuse a NIC whose switch port advertises (LLDP 802.3 Maximum Frame Size) frames smaller than its MTU needs");
    int min_speed_gbps = 0;
    fs.add_int("min-link-speed-gbps", &min_speed_gbps, "minimum negotiated link speed of every scale-out NIC (sysfs speed); a slower NIC is left unconfigured (L3) or fails the start (L2); 0 = off");
    fs.add_string("rail-switch-pattern", &cfg.rail_switch_pattern, "L3 rail cabling check: the NIC of GPU k must reach a switch whose LLDP System Name matches this ECMAScript regex with {rail} = k (e.g. 'leaf-r{rail}-.*'); a mismatch leaves the NIC unconfigured");
    fs.add_bool("dry-run", &cfg.dry_run, "discover, check xGMI / GPUDirect RDMA and write the topology file and status only: no link, address, NetworkManager or label change, no LLDP (needs no privileges)");
    fs.add_string("lldp-cache", &cfg.lldp_cache, "with --keep-running: remember each NIC's confirmed Port Description in this file and configure from it at start (the switch must confirm it within --lldp-cache-confirm)");
    fs.add_duration("lldp-cache-max-age", &cfg.lldp_cache_max_age_ns, "ignore LLDP cache entries older than this");
    fs.add_duration("lldp-cache-confirm", &cfg.lldp_cache_confirm_ns, "withdraw readiness if no LLDP frame confirms a cached Port Description within this time");
    fs.add_string("node-name", &cfg.node_name, "LLDP System Name (default $NODE_NAME, else the hostname)");
    fs.add_bool("monitor", &cfg.monitor, "with --keep-running: keep announcing LLDP, withdraw the label on link loss, re-configure on Port Description changes");
    fs.add_duration("lldp-tx-interval", &cfg.lldp_tx_interval_ns, "LLDP keep-alive transmit interval while monitoring");
    fs.add_string("metrics-bind-address", &cfg.metrics_addr, "serve /metrics, /healthz, /readyz on this address (e.g. :9102; empty = off)");
    fs.add_string("require-gdr", &cfg.require_gdr, "refuse readiness without GPUDirect RDMA: any, peermem, dmabuf (empty = report only)");
    fs.add_bool("disable-fw-lldp", &cfg.disable_fw_lldp, "L3: turn off NIC-firmware LLDP agents while running (i40e disable-fw-lldp, ice fw-lldp-agent, --fw-lldp-priv-flag rules); other DCB NICs (e.g. mlx5_core) only with --fw-lldp-dcbx-host");
    fs.add_bool("fw-lldp-dcbx-host", &cfg.fw_lldp_dcbx_host, "with --disable-fw-lldp: on a NIC without a firmware-LLDP private flag whose DCBX an embedded agent runs (mlx5_core firmware mode), hand DCBX to the host (the firmware stops negotiating PFC/ETS with the switch); restored on exit");
    fs.add_bool("restore-mtu", &cfg.restore_mtu, "on a clean exit (not --keep-config), put each NIC's MTU back to what it was when the agent started (host-nic policies: the node's own NICs)");
    fs.add_string("link-state", &cfg.link_state, "file keeping each NIC's link state (up/down) from before the first agent brought it up, across crashes and --keep-config restarts (put back on the last clean exit or by --cleanup)");
    fs.add_string("mtu-state", &cfg.mtu_state, "with --restore-mtu: file keeping each NIC's MTU from before the first agent changed it, across --keep-config restarts (restored on the last clean exit or by --cleanup)");
    fs.add_string("fw-lldp-priv-flag", &cfg.fw_lldp_flags, "extra ethtool private-flag rules NAME=0|1[,...] for --disable-fw-lldp");
    fs.add_string("fw-lldp-state", &cfg.fw_lldp_state, "with --keep-config: keep the originals of what --disable-fw-lldp changed in this file across restarts instead of restoring them on exit; --cleanup restores them");
    bool ready_check = false;
    fs.add_bool("ready-check", &ready_check, "exit 0 if the readiness label is published, 1 otherwise (readinessProbe)");
    fs.add_bool("help", &show_help, "help for discover");
    fs.shorthand('h', "help");
    fs.add_bool("version", &show_version, "print version");

    try {
        fs.parse(argc, argv);
    } catch (const std::invalid_argument& e) {
        std::fprintf(stderr, "Error: %s\n%s", e.what(), fs.usage().c_str());
        return 2;
    }
    if (show_help) {
        std::cout << "Discover and optionally configure network devices\n\n" << fs.usage();
        return 0;
    }
    if (ready_check) {
        if (path_exists(cfg.labels.path())) return 0;
        // The kubelet keeps a failing probe's output in the Pod's events: say why.
        std::optional<std::string> why;
        if (!cfg.status_file.empty()) why = read_file(agent::reason_path(cfg.status_file));
        // No status file yet: the agent has not got as far as writing one (a start-up state for
        // the operator, like "waiting for LLDP"), not a failure.
        if (!why && !cfg.status_file.empty() && !path_exists(cfg.status_file)) why = std::string(agent::kStartingReason);
        std::string line = why ? trim(*why) : "readiness label " + cfg.labels.path() + " not published";
        if (line.size() > 900) line = line.substr(0, 900) + " ...";
        std::printf("not ready: %s\n", line.c_str());
        return 1;
    }
    if (show_version) {
        std::cout << "discover (amd network operator) " << NETOP_VERSION << "\n";
        return 0;
    }
    log::set_verbosity(verbosity);
    log::set_skip_headers(skip_headers);
    if (!log_file.empty()) log::set_log_file(log_file);
    if (logging_format == "json") log::set_format(log::Format::Json);

    auto dm = topo::parse_discovery_mode(discovery_mode);
    auto tp = l3::parse_token_policy(token_policy);
    if (!dm || !tp) {
        std::fprintf(stderr, "Error: invalid --nic-discovery or --token-policy\n");
        return 2;
    }
    if (cfg.rail_table_base < 0 || cfg.rail_table_base > 200) {
        std::fprintf(stderr, "Error: --rail-table-base must be 0 (off) or 1..200\n");
        return 2;
    }
    if (node_lock == "auto")
        cfg.node_lock = cfg.labels.file;
    else if (node_lock != "none")
        cfg.node_lock = node_lock;
    if (min_speed_gbps < 0 || min_speed_gbps > 3200) {
        std::fprintf(stderr, "Error: --min-link-speed-gbps must be 0 (off) or 1..3200\n");
        return 2;
    }
    cfg.min_link_speed_mbps = int64_t(min_speed_gbps) * 1000;
    cfg.discovery.mode = *dm;
    cfg.discovery.exclude_gpu_rails = !include_gpu_rails;
    cfg.token_policy = *tp;
    if (!nic_drivers.empty()) cfg.discovery.nic_drivers = split(nic_drivers, ',');
    static const std::map<std::string, topo::PathType> paths{{"PIX", topo::PathType::PIX}, {"PXB", topo::PathType::PXB},
                                                             {"PHB", topo::PathType::PHB}, {"NODE", topo::PathType::NODE},
                                                             {"SYS", topo::PathType::SYS}};
    auto pit = paths.find(to_upper(max_path));
    if (pit == paths.end()) {
        std::fprintf(stderr, "Error: invalid --max-path '%s'\n", max_path.c_str());
        return 2;
    }
    cfg.discovery.max_path = pit->second;
    if (cfg.node_name.empty()) {
        const char* nn = std::getenv("NODE_NAME");  // set by the DaemonSet (downward API)
        char host[256] = {};
        if (nn && *nn)
            cfg.node_name = nn;
        else if (::gethostname(host, sizeof host - 1) == 0)
            cfg.node_name = host;
    }

    // SIGTERM/SIGINT are consumed through a signalfd so every wait in the state machine
    // (LLDP epoll, idle) can observe them without async-signal-safety concerns.
    sigset_t mask;
    sigemptyset(&mask);
    sigaddset(&mask, SIGTERM);
    sigaddset(&mask, SIGINT);
    sigprocmask(SIG_BLOCK, &mask, nullptr);
    int sfd = signalfd(-1, &mask, SFD_CLOEXEC | SFD_NONBLOCK);

    try {
        nl::Rtnl rtnl;
        agent::Agent a(cfg, rtnl, agent::make_packet_source(cfg.lldp_promisc), [] { return nm::connect_system_bus(); });
        a.run(sfd);
    } catch (const std::exception& e) {
        NLOG_E("%s", e.what());
        std::fprintf(stderr, "Error: %s\n", e.what());
        return 1;
    }
    return 0;
}

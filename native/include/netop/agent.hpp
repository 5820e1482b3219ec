// The node agent ("discover") state machine.
//
// Reference: cmd/discover/main.go:cmdRun (:161-259) — sanitize, pre-cleanup, discover,
// [unmanage from NM], links up, MTU, flush IPv4, [L3: LLDP -> /30 + routes -> artifacts],
// readiness label, idle until SIGTERM, post-cleanup.
//
// MI355X-first differences (each documented at its call site):
//   * LLDP frames are consumed from one epoll loop and each NIC is configured the moment
//     its frame arrives (Config::pipeline), instead of a barrier over all NICs
//     (main.go:84-122);
//   * scale-out NICs are found by PCIe affinity to amdgpu functions (topology.hpp);
//   * RCCL artifacts replace gaudinet.json; RoCE v2 GID indices are resolved per NIC;
//   * optional xGMI-mesh verification gates the readiness label;
//   * in L3 mode zero LLDP peers is an error instead of a silently-published label
//     (main.go:212,239-246) unless Config::label_without_peers (compat) is set.
#pragma once

#include <sys/types.h>

#include <cstdint>
#include <functional>
#include <future>
#include <map>
#include <memory>
#include <mutex>
#include <optional>
#include <set>
#include <string>
#include <vector>

#include "netop/arp.hpp"
#include "netop/artifacts.hpp"
#include "netop/bounded.hpp"
#include "netop/ethtool.hpp"
#include "netop/httpd.hpp"
#include "netop/l3.hpp"
#include "netop/lldp.hpp"
#include "netop/netlink.hpp"
#include "netop/nm.hpp"
#include "netop/packet.hpp"
#include "netop/state.hpp"
#include "netop/topology.hpp"

namespace netop::agent {

struct Config {
    // Reference flags (cmd/discover/main.go:281-298) with the same defaults.
    std::string mode = "L3";
    bool configure = false;
    bool disable_nm = false;
    std::string interfaces;              // comma separated extra interfaces
    int64_t wait_ns = 30LL * 1000000000; // --wait
    std::string rccl_net;                // --rccl-net (alias --gaudinet)
    bool keep_running = false;
    std::string networkd;                // --systemd-networkd
    int mtu = 1500;

    // MI355X additions.
    topo::DiscoveryOptions discovery;
    std::string sysfs_root;              // "" = $SYSFS_ROOT or /sys/
    l3::TokenPolicy token_policy = l3::TokenPolicy::CompatThenLast;
    bool lldp_promisc = false;
    bool pipeline = true;
    bool label_without_peers = false;
    bool fsync_artifacts = false;  // fsync every artifact / label / status write (see set_durable_writes)
    artifacts::Labels labels;
    std::string rccl_env;                // --rccl-env
    std::string rccl_topo;               // --rccl-topo: NCCL_TOPO_FILE XML written here
    std::string rccl_topo_env_path;      // --rccl-topo-env-path: path jobs see (default rccl_topo)
    // --rccl-socket-ifname: NCCL_SOCKET_IFNAME in rccl.env.  "auto": L3 -> the configured scale-out
    // NICs in GPU order (every node lists rail 0 first, so bootstrap meets on one /16); L2 -> not
    // written (no IPv4).  "none" / "" -> not written.  Anything else: a literal interface list.
    std::string socket_ifname = "auto";
    std::string status_file;             // --status-file (JSON)
    std::string nm_keyfile_dir;          // --nm-keyfile-dir
    // --nm-restore: on exit, remove the keyfile and set Managed=true again.  Off by default: an
    // agent exits on every rolling update, drain and reboot, and NetworkManager must not reclaim
    // the scale-out NICs (and start DHCP on them) before the next agent runs; the reference
    // leaves Managed=false in place too.  For handing the NICs back when the policy goes.
    bool nm_restore = false;
    int xgmi_expect_links = -1;          // -1 off; 0 = full mesh among discovered GPUs; N = exact pairs
    // With the xGMI check, the links' trained state from gpu_metrics (topo::XgmiLinkHealth): a link
    // down fails the check; a width below this (lanes, 0 = any) too.  The monitor reads the state
    // again every xgmi_health_interval_ns and withdraws the label while a link is down.
    int xgmi_min_link_width = 0;
    // Configure (and label) a NIC only if its PCIe link trained at the speed and width it and its
    // slot support, and its GPU's at full width (a GPU may lower its link speed when idle).
    bool require_full_pcie = false;
    int64_t xgmi_health_interval_ns = 5LL * 1000000000;
    // Bound on each sysfs read that firmware or hardware answers (gpu_metrics: an SMU query per
    // GPU; PCIe link state; the KFD topology): a read that has not returned by then is reported
    // ("gpu_metrics of <bdf> did not answer in 5s") and the label follows the policy, instead of the
    // start or the monitor hanging behind it (netop/bounded.hpp).
    int64_t sysfs_read_timeout_ns = 5LL * 1000000000;
    // Flap dampening: after the monitor withdrew the label, it is republished only once the node
    // has been healthy for this long without a break (a flapping optic or a GPU reset would
    // otherwise toggle the node's scheduling eligibility as fast as the link flaps).  The first
    // publication is not delayed.  0 = republish at once.
    int64_t label_holddown_ns = 10LL * 1000000000;
    // The monitor counts an xGMI link as down only after this many consecutive gpu_metrics samples
    // saw it down (a transient status during a GPU reset is not a flap); the start needs one.
    int xgmi_down_samples = 2;
    int64_t link_wait_ns = 3LL * 1000000000;  // netlink echo wait (network.go:251)
    // L2: how long a NIC that is admin-up may train its link before it counts as "no carrier".
    // Separate from the 3 s echo wait: 200/400G optics with FEC and link training commonly take
    // 5-15 s (longer through auto-negotiation retries), so 3 s made every start look degraded.
    int64_t carrier_wait_ns = 30LL * 1000000000;
    // The RDMA core adds the RoCE v2 GID of a new IPv4 address asynchronously (netdev notifier
    // -> GID cache work item); wait this long for it before writing rccl.env without a GID.
    int64_t gid_wait_ns = 3LL * 1000000000;
    // L3: before the label, every configured NIC's switch-side /30 address must answer ARP
    // within this time (0 = no check, the reference's behaviour); requests every retry.
    int64_t verify_peers_ns = 0;
    int64_t verify_peers_retry_ns = 100LL * 1000000;
    bool lldp_announce = true;           // transmit our own LLDPDU (triggers switch fast start)
    int64_t announce_interval_ns = 1000000000LL;  // re-announce to still-silent NICs
    int announce_count = 6;  // rounds at 0, +25 ms, +125 ms, +425 ms, +1.4 s, +2.4 s (interval 1 s)
    bool announce_shutdown_first = true;  // clear a stale neighbour entry left by a crashed run
    std::string node_name;               // LLDP System Name ($NODE_NAME, else hostname)
    // Keep-running monitor: LLDP keep-alive transmission, link-failure detection (the label is
    // withdrawn while a NIC is down and republished when it recovers), re-configuration when a
    // switch port's Port Description changes.  The reference only waits for SIGTERM.
    bool monitor = true;
    int64_t lldp_tx_interval_ns = 30LL * 1000000000;  // msgTxInterval
    int64_t monitor_tick_ns = 200LL * 1000000;        // link-event polling granularity
    std::string metrics_addr;                         // "" = off; e.g. ":9102" (/metrics, /healthz, /readyz)
    // Turn off NIC-firmware LLDP agents (ethtool private flags) while the agent runs, so the
    // switch's LLDPDUs reach the host (ethtool.hpp).  L3 only.
    // GPUDirect RDMA: "" = report only; "any" = require peer-memory or dma-buf; "peermem" /
    // "dmabuf" = require that mechanism.  Checked before LLDP, like the xGMI mesh.
    std::string require_gdr;
    // Every scale-out NIC must have an RDMA device before the readiness label: a RoCE NIC whose
    // RDMA driver is not loaded leaves RCCL only TCP sockets on that rail.  (The reference labels
    // after configuring the RDMA NICs HCCL uses, cmd/discover/main.go:212-246; Gaudi's integrated
    // NICs are RDMA by construction.)  The NICs are configured either way; the label and rccl.env
    // wait, the probe says "waiting for RDMA device", and the monitor publishes the label once the
    // devices appear (a driver container loading the module).  Past rdma_wait_ns from the start the
    // reason turns into the fault "no RDMA device (load its RDMA driver)".  Off: a warning only.
    bool require_rdma = false;
    int64_t rdma_wait_ns = 300LL * 1000000000;
    int64_t rdma_poll_ns = 250LL * 1000000;  // how often the waiting agent looks for the devices
    bool disable_fw_lldp = false;
    // With disable_fw_lldp, on a NIC without a firmware-LLDP private flag whose DCBX an embedded
    // agent runs (mlx5_core in firmware mode): hand DCBX to the host.  Opt-in: the firmware then
    // stops negotiating PFC/ETS with the switch (ethtool.hpp).
    bool fw_lldp_dcbx_host = false;
    // On a clean exit (not --keep-config), put every NIC's MTU back to what it was at the start
    // (host-nic policies: the node's own NICs).
    bool restore_mtu = false;
    // With restore_mtu: "ifname mtu" lines keeping each NIC's MTU from before the first agent that
    // changed it, across --keep-config restarts, for the last clean exit or the --cleanup Job.
    std::string mtu_state;
    // "ifname up|down" lines keeping each NIC's administrative state from before the first agent
    // brought it up, across crashes and --keep-config restarts (a restarted agent finds the link up
    // and would take that for the original).  The last clean exit, or --cleanup, puts the recorded
    // state back and removes the file.  Empty: the state this process found (the reference).
    std::string link_state;
    std::string fw_lldp_flags;                        // extra rules "NAME=0|1,..."
    // With keep_config: the originals of what --disable-fw-lldp changed are kept in this file
    // across agent restarts (a restart does not flip the NICs back and forth: some drivers reset
    // the port when the flag flips) and put back by --cleanup.  Without keep_config the record
    // still outlives an agent that fails (the next one must not take the changed flags for the
    // originals) and is restored and removed on a clean exit.
    std::string fw_lldp_state;
    std::string rccl_env_extra;                       // "KEY=VALUE,..." appended to rccl.env
    // Per-rail source routing (L3): NIC k gets routing table base+k (k = its GPU index; NICs
    // without a GPU get the indices after the last GPU's) holding its /30 and its /16 via the
    // switch, and a rule "from <local>/32 lookup base+k" at priority base+k.  Traffic sourced
    // from a rail's address then leaves through that rail even though every rail's /16 route is
    // also in the main table.  Tables and priorities base..base+N-1 are reserved for the agent;
    // its rules and routes carry protocol kRailProtocol and it never deletes any other.  0 = off
    // (the reference's main-table-only routing).
    int rail_table_base = 0;
    // Discovery, the xGMI / GPUDirect checks and the topology file only; no link, address, NM
    // or label change and no LLDP (no privileges needed): what the agent would configure here.
    bool dry_run = false;
    // Keep the data plane across agent restarts (rolling updates, drains, agent crashes): on exit
    // only the readiness label is withdrawn; addresses, routes, rail rules and link state stay,
    // and the next agent adopts them (the /30 its LLDP cache holds for a NIC is not flushed, so
    // RoCE QPs bound to it survive).  The reference tears everything down on every SIGTERM
    // (main.go:143-159), which breaks running RCCL jobs whenever the DaemonSet rolls.
    bool keep_config = false;
    // One-shot teardown of what --keep-config agents left on the node (the operator runs it when
    // the policy is deleted): IPv4 addresses of the discovered NICs, rules and routes tagged
    // kRailProtocol, the label, the agent's artifacts, LLDP cache and networkd files.
    bool cleanup = false;
    // LLDP cache (artifacts.hpp): configure from the last confirmed Port Description at start,
    // then require a real frame to confirm it within lldp_cache_confirm_ns (else the NIC counts
    // as degraded and the label is withdrawn until one arrives).  "" = off.  Used only with
    // --keep-running and the monitor (which does the confirming).
    std::string lldp_cache;
    int64_t lldp_cache_max_age_ns = 7LL * 24 * 3600 * 1000000000;  // older entries are ignored
    int64_t lldp_cache_confirm_ns = 95LL * 1000000000;              // 3 x msgTxInterval + 5 s
    // Node-wide mutual exclusion between agents that configure the same NICs (an exiting and a
    // starting agent, an agent and the --cleanup Job, two policies selecting one node): an
    // abstract unix socket of this name, held for the agent's lifetime.  hostNetwork Pods share
    // the node's network namespace, so the name is node-wide, and the kernel releases it when the
    // process dies, SIGKILL included.  "" = off (discover's --node-lock defaults it from the
    // label file, so an amd-so and a host-nic agent never wait for each other).
    std::string node_lock;
    // One owner per NIC: an abstract unix socket per interface ("netop-nic:<ifname>"), taken in
    // name order after discovery and held for the agent's lifetime, whatever the label file.  An
    // amd-so and a host-nic agent (or two host-nic policies) that select the same NIC can then
    // never configure it concurrently: the second waits node_lock_wait_ns and fails naming the
    // NIC.  Off here (unit tests run several agents in one process); discover turns it on.
    bool nic_locks = false;
    // Rail cabling check (L3): the NIC of GPU k must be cabled to a switch whose LLDP System Name
    // matches this ECMAScript regex with "{rail}" replaced by k (e.g. "leaf-r{rail}-.*" for a
    // rail-optimized fabric).  A NIC on the wrong leaf still works but crosses the spine, so a
    // mismatch leaves it unconfigured and is named in the error.  "" = off.
    std::string rail_switch_pattern;
    // Minimum negotiated link speed (Mb/s, sysfs class/net/<if>/speed): a 400G rail that came up
    // at 200G (a marginal cable or optic, a port renegotiated down) halves that GPU's scale-out
    // bandwidth while everything else looks healthy.  A slower NIC is left unconfigured (L3) or
    // fails the start (L2), named in the error; a speed the driver does not report is allowed
    // with a warning.  0 = off.
    int64_t min_link_speed_mbps = 0;
    // Refuse a NIC whose switch port advertises (LLDP 802.3 Maximum Frame Size TLV) a maximum
    // frame smaller than the NIC's frames (max_frame_for_mtu: MTU + header + FCS [+ 802.1Q tag]):
    // jumbo RoCE frames would be dropped by the switch, which shows as hung or crawling RCCL jobs
    // rather than as an error.
    bool check_peer_mtu = true;
    int64_t node_lock_wait_ns = 60LL * 1000000000;
    // host-nic with nothing of its own to configure: how often the idle agent looks again (a NIC
    // freed by the node, a driver loaded late); it then exits so its restart configures the NIC.
    // 0 = never.
    int64_t rediscover_ns = 30LL * 1000000000;
    // A NIC with a default route in a per-NIC policy-routing table that also holds the node's own
    // address (not a /30, or the source its rule selects) is refused like an uplink; this takes
    // it anyway (a rail whose site routing the operator knows to be its own).
    bool allow_policy_routed = false;
};

// Where the agent leaves the one-line reason the node is not ready (beside --status-file), and
// what `discover --ready-check --status-file=...` prints when it fails.
std::string reason_path(const std::string& status_file);
// --ready-check's reason while the agent has not written its status file yet.
inline constexpr const char* kStartingReason = "agent starting";

// FRA_PROTOCOL / rtm_protocol tag on the agent's rail rules and rail-table routes ("installed by
// the AMD network operator"): cleanup only ever removes rules and routes carrying it.
constexpr uint8_t kRailProtocol = 0xa3;

// Sanitises in place (MTU clamp to [1500, 9000], mode upper-cased); throws on a bad mode.
void sanitize(Config& c);

// The rail cabling check's regular expressions are ECMAScript (std::regex): "" when `pattern`
// compiles, else the library's reason.  The webhook's grammar check is tested against these.
std::string ecmascript_regex_error(const std::string& pattern);
std::optional<bool> ecmascript_full_match(const std::string& pattern, const std::string& text);  // nullopt: no compile
constexpr int kMaxRails = 16;  // GPU indices a rail pattern is checked for
// "" when --rail-switch-pattern compiles for every rail index 0..kMaxRails-1.
std::string rail_pattern_error(const std::string& pattern);

// Source of LLDP frames (AF_PACKET in production, scripted in tests).
class LldpSource {
   public:
    virtual ~LldpSource() = default;
    virtual void add(const std::string& ifname, int ifindex, const MacAddr& own_mac) = 0;
    virtual pkt::ListenResult run(int64_t deadline,
                                  const std::function<bool(const std::string&, const lldp::Frame&)>& on_frame,
                                  int stop_fd) = 0;
    // Transmits our own LLDPDU on an interface (no-op for sources that cannot transmit).
    virtual void announce(const std::string& ifname, const std::vector<uint8_t>& frame) {}
    virtual pkt::ListenerStats stats() const { return {}; }
    // Per-interface counters; nullopt for sources that keep none.
    virtual std::optional<pkt::ListenerStats> stats_for(const std::string& ifname) const {
        (void)ifname;
        return std::nullopt;
    }
};

// The LLDPDU the agent advertises for one of its NICs.  Announcing ourselves makes an
// IEEE 802.1AB-2009 switch see a *new neighbour* and enter fast transmission (txFast), so
// its Port Description arrives within ~1 s instead of up to msgTxInterval (30 s).
// ttl = 0 builds the shutdown LLDPDU sent on cleanup.  mtu > 0 adds the IEEE 802.3 Maximum
// Frame Size TLV (MTU + 18: header and FCS), so the switch's neighbour table shows what frames
// the host sends and a mismatch is visible from the switch side too.
// IEEE 802.3 Maximum Frame Size for an MTU: Ethernet header (14) + payload + FCS (4), and an
// 802.1Q tag (4) when the NIC sends tagged frames.  Both what the agent advertises and the least
// a switch port must accept (Config::check_peer_mtu).
int max_frame_for_mtu(int mtu, bool vlan_tagged);
lldp::Frame make_node_frame(const std::string& node_name, const std::string& ifname, const MacAddr& mac,
                            const std::string& gpu_bdf, uint16_t ttl = 120, int mtu = 0);
std::unique_ptr<LldpSource> make_packet_source(bool promisc);

using NmFactory = std::function<std::unique_ptr<nm::NetworkManagerIf>()>;

class AgentError : public std::runtime_error {
   public:
    using std::runtime_error::runtime_error;
};

class Agent {
   public:
    struct TopoResult {  // what the topology worker hands back
        std::string xml, fp;            // the file and its inputs (the ".key" sidecar)
        std::vector<std::string> names;  // the interfaces it was generated for
        bool reused = false;             // the file on disk is current: nothing to write
    };
    Agent(Config cfg, nl::NetOps& ops, std::unique_ptr<LldpSource> lldp, NmFactory nm_factory);
    ~Agent();

    // Runs the whole state machine.  `stop_fd` becomes readable on SIGTERM/SIGINT (a
    // signalfd in production, a pipe/eventfd in tests).  Throws AgentError on fatal errors.
    void run(int stop_fd);

    const std::vector<NicState>& nics() const { return nics_; }
    const std::map<std::string, int64_t>& phases() const { return phases_; }
    bool ready() const { return ready_; }
    const topo::XgmiReport& xgmi() const { return xgmi_; }
    const topo::GdrReport& gdr() const { return gdr_; }
    const std::vector<std::pair<std::string, std::string>>& excluded() const { return excluded_; }

    // Replaces the ethtool ioctl table (tests inject fakes).
    void set_ethtool_ops(std::unique_ptr<ethtool::Ops> ops) { ethtool_ = std::move(ops); }
    const std::vector<ethtool::FwLldpResult>& fw_lldp() const { return fw_lldp_; }

    // Test hook: called once per monitor iteration (lets tests inject link events / stop).
    std::function<void(int)> on_monitor_tick;
    // The ARP prober behind --verify-peers (arp::probe_all; tests inject a fake switch).
    std::function<bool(std::vector<arp::Probe>&, int64_t timeout_ns, int64_t retry_ns, int stop_fd)> arp_probe;
    int link_flaps() const { return flaps_; }
    int reconfigurations() const { return reconfigs_; }

    // Exposed for unit tests (reference-named helpers).
    void interfaces_up();
    void interfaces_restore_down();
    void interfaces_set_mtu();
    void remove_existing_ips(const std::map<std::string, Ipv4Prefix>& keep = {});
    bool configure_interface(NicState& n);
    int configure_all();  // returns number configured
    void assign_rail_indices();

   private:
    void pre_cleanups();
    void post_cleanups();
    void cleanup_node();                    // --cleanup
    std::map<std::string, Ipv4Prefix> cached_addresses() const;  // --keep-config: addresses to adopt
    std::vector<std::string> collect_interfaces(bool quiet = false);
    // host-nic, nothing of its own: waits for SIGTERM, looking again every rediscover_ns.  True
    // when a NIC of its own has appeared (the caller exits; the restart configures it).
    bool idle_until_own_nic(int stop_fd);
    void get_network_configs(const std::vector<std::string>& names);
    void detect_lldp(int stop_fd);
    void diagnose_silent();            // after --wait expired: why each silent NIC heard nothing
    std::string check_link_speed(NicState& n);  // "" or why n is below --min-link-speed-gbps
    // L2: up, carrier, and fast enough (sets n.config_error to the speed shortfall, else clears it).
    bool l2_link_ok(NicState& n);
    std::string silent_summary() const;
    std::string not_ready_reason() const;  // per NIC, for the readiness probe ("" when none known)  // "" or "LLDP silent on k NIC(s): ... Not configured: ..." for the exit error
    void on_lldp(NicState& n, const lldp::Frame& f);
    void add_route(NicState& n, int mask);
    uint32_t rail_table(const NicState& n) const;
    void add_rail_routing(NicState& n);
    void remove_rail_routing(NicState& n);  // what was installed for n
    void remove_rail_routing();             // every NIC's
    // gid_wait_ns < 0: --gid-wait.  The monitor passes 0 (one look, never blocking its loop) and
    // looks again for the GIDs still missing (gid_retry_until_).
    void write_artifacts(int64_t gid_wait_ns = -1);
    void write_l2_artifacts(int64_t gid_wait_ns = -1);
    bool look_up_gids();        // one look for every configured RDMA NIC's missing GID; true if one was found
    bool gids_missing() const;  // a configured RDMA NIC without its GID index
    int64_t gid_retry_until_ = 0;
    // L2: waits up to carrier_wait_ns for carrier on every up NIC (reported as "waiting for
    // carrier" meanwhile); marks the others no_carrier.
    // False when stop_fd fired meanwhile.
    bool wait_carrier(int stop_fd);
    void write_rccl_env_file();
    std::string write_topo();  // returns the NCCL_TOPO_FILE value for rccl.env ("" = none)
    // The topology XML depends only on sysfs and the NIC set, both fixed once discovery is done:
    // it is generated on a worker thread from then on (overlapping link-up and the LLDP wait)
    // and written at artifact time, so its sysfs walk is off the node-ready critical path.
    void start_topo();
    void write_host_config();  // systemd-networkd files and the LLDP cache
    void dry_run_report();
    const std::string& topo_xml();  // joins the worker; "" when generation failed
    std::vector<std::string> socket_ifnames() const;
    void check_xgmi();     // dry run: join the prefetched KFD topology and gpu_metrics now
    void join_xgmi();      // the prefetched KFD topology, evaluated (right after link-up)
    void evaluate_xgmi();  // the mesh check
    // start_prefetch(): each read on its own detached thread (netop/bounded.hpp), all joined by
    // prefetch_deadline_ at the latest (a late KFD read fails the start, a late PCIe read leaves the
    // links unknown, a late gpu_metrics read names the GPU).
    bounded::Call<topo::XgmiReport> xgmi_call_;
    int64_t prefetch_deadline_ = 0;
    void start_prefetch();
    void log_results();
    void mark(const std::string& phase);
    void write_status();
    void monitor(int stop_fd);
    bool publish_label();
    void announce_all(uint16_t ttl);
    bool nic_healthy(const NicState& n) const;
    // --verify-peers: ARP-probes the switch side of every NIC in `which` for up to `timeout_ns`;
    // returns how many did not answer (-1 when interrupted by stop_fd).
    int verify_peers(const std::vector<NicState*>& which, int64_t timeout_ns, int stop_fd);

    std::map<std::string, std::string> labels_extra_;
    int flaps_ = 0;
    int reconfigs_ = 0;
    std::unique_ptr<httpd::Server> httpd_;
    std::unique_ptr<ethtool::Ops> ethtool_;
    std::vector<ethtool::FwLldpResult> fw_lldp_;
    // Records of an earlier agent for NICs this one does not select (the policy's interface list
    // changed, a NIC was renamed) that could not be restored at start: kept in --fw-lldp-state
    // so --cleanup can try again.
    std::vector<ethtool::FwLldpResult> fw_lldp_carried_;
    // The record: this agent's changes (with_current) and the carried ones; removed when empty.
    void save_fw_lldp_state(bool with_current = true);
    void load_mtu_state();       // orig_mtu of every NIC from --mtu-state (recording new ones)
    void restore_mtus();         // each NIC's orig_mtu back; the state file's entries with it
    void restore_mtu_state();    // --cleanup: every entry of --mtu-state back, then the file goes
    void load_link_state();      // orig_flags' IFF_UP of every NIC from --link-state (recording new ones)
    void forget_link_state();    // after interfaces_restore_down: drop the NICs back in their original state
    void restore_link_state();   // --cleanup: every NIC recorded down goes down, then the file goes
    std::vector<std::pair<std::string, std::string>> rccl_env_extra_;
    void disable_fw_lldp();
    void restore_fw_lldp_from_state();
    bool persist_fw_lldp() const { return cfg_.keep_config && !cfg_.fw_lldp_state.empty(); }
    void restore_network_manager();
    int apply_lldp_cache(const std::set<int>& listening);  // NICs addressed from the cache (by ifindex)
    // A frame for a NIC that already has an address: confirms a cached Port Description or moves
    // the NIC to the new one.  True when the NIC's status changed.
    bool refresh_from_frame(NicState& n, const lldp::Frame& f);
    void save_lldp_cache();
    bool nm_keyfile_written_ = false;
    std::vector<std::string> nm_unmanaged_;
    int node_lock_fd_ = -1;
    std::vector<int> nic_lock_fds_;
    std::string config_error_;  // a setting the agent cannot work with: it configures nothing
    void idle(int stop_fd);
    void acquire_node_lock(int stop_fd);
    void acquire_nic_locks(int stop_fd);
    // Binds the abstract socket `name` (waiting up to `deadline` while another process holds it);
    // the fd, or throws AgentError(busy) at the deadline.
    int take_lock(const std::string& name, int64_t deadline, int stop_fd, const std::string& waiting,
                  const std::string& busy);
    // The node's own interfaces.  Every mode refuses to touch a NIC that carries a default route,
    // itself or through a device stacked on it (refuse_uplinks); rdma discovery also leaves out NICs
    // enslaved to a bond / bridge / team and NICs holding addresses or routes the agent never
    // installs, or carrying a stacked device that does (node_owned_reason), unless --interfaces
    // names them.
    std::vector<int> uplinks_;
    bool uplinks_read_ = false;
    const std::vector<int>& uplinks();
    std::string node_owned_reason(const nl::LinkInfo& l, int depth = 0);
    // nullopt when no default route leaves through `l`; else "" (directly) or the path through
    // the devices stacked on it (" via bond0", " via ens1.100 via br0").
    std::optional<std::string> uplink_path(const nl::LinkInfo& l, int depth = 0);
    std::vector<nl::LinkInfo> stacked_on(const nl::LinkInfo& l);  // its master and sysfs upper devices
    void refuse_uplinks();
    std::vector<std::pair<std::string, std::string>> excluded_;  // discovered but left alone, and why

   public:
    // Prometheus text exposition of the agent state (served on Config::metrics_addr).
    std::string render_metrics() const;
    int metrics_port() const;

    Config cfg_;
    nl::NetOps& ops_;
    std::unique_ptr<LldpSource> lldp_;
    NmFactory nm_factory_;
    std::unique_ptr<arp::Prober> arp_;  // --verify-peers sockets, opened on first use
    std::vector<NicState> nics_;
    topo::DiscoveryResult disc_;
    double cpu_ms_at_ready_ = -1;  // user + system CPU of the process when the label went up
    std::vector<std::string> dry_run_missing_;  // discovered, but not in this network namespace
    bounded::Call<TopoResult> topo_call_;  // the topology worker (start_topo), joined with a deadline
    bool topo_late_ = false;                // it missed that deadline once: later joins only look
    bool monitoring_ = false;               // in monitor(): joins wait briefly, a late file follows
    std::optional<TopoResult> topo_;
    topo::XgmiReport xgmi_;
    std::vector<topo::XgmiLinkHealth> xgmi_health_;
    std::string xgmi_error_;  // what the last gpu_metrics read found wrong (empty: fine or not read)
    std::string xgmi_unread_;  // why no GPU's link state could be decoded (an unknown gpu_metrics layout)
    // `min_down`: consecutive samples a link must have been seen down (xgmi_down_streak_).
    std::string xgmi_health_problem(int min_down = 1) const;
    void note_xgmi_sample();  // updates xgmi_down_streak_ from xgmi_health_
    std::map<std::string, std::vector<int>> xgmi_down_streak_;  // per GPU BDF, per link slot
    // The start's gpu_metrics read (start_prefetch; an SMU query per GPU): joined by
    // finish_xgmi_health() before the label decision.
    bounded::Call<std::vector<topo::XgmiLinkHealth>> xgmi_health_call_;
    void finish_xgmi_health();
    std::vector<std::string> xgmi_health_bdfs() const;
    std::string check_pcie(NicState& n);  // "" when fine or not required
    // The NICs' and their GPUs' PCIe links (start_prefetch), joined by ensure_pcie() at first use.
    bounded::Call<std::vector<std::pair<topo::PcieLink, topo::PcieLink>>> pcie_call_;
    bool pcie_joined_ = false;
    bool pcie_late_ = false;  // the start's PCIe link read did not answer in time
    void ensure_pcie();
    // Monitor: the periodic gpu_metrics / PCIe reads, on a worker (results through an eventfd).
    struct HealthSample {
        std::vector<topo::XgmiLinkHealth> xgmi;
        std::vector<std::pair<topo::PcieLink, topo::PcieLink>> pcie;  // per NIC (nics_ order)
        std::vector<bool> pcie_late;  // per NIC: its read had not returned by the deadline
        bool xgmi_read = false, pcie_read = false;
    };
    // Applies a sample; true when the node's health changed.
    bool apply_health(const HealthSample& s);
    // Label hold-down (Config::label_holddown_ns): when the node last turned healthy after a
    // withdrawal (0 = not holding), how often a recovery was cut short by another flap, and the
    // withdrawals.
    int64_t holddown_until_ = 0;
    int label_suppressed_ = 0;
    int label_withdrawals_ = 0;
    // Bounded sysfs reads that missed --sysfs-read-timeout, by what was read ("gpu_metrics",
    // "pcie", "kfd", "topology"): a wedged SMU or a function in error recovery, as a counter.
    std::map<std::string, uint64_t> late_reads_;
    uint64_t late_reads_total() const;
    // GPU rails whose NIC has no RDMA device (its RDMA driver is not loaded): RCCL could only use
    // them over TCP sockets.  Reported always; fatal with --require-gdr.
    std::vector<std::string> no_rdma_;
    void check_rdma();
    // --require-rdma: the configured NICs still without an RDMA device (empty when not required).
    std::vector<std::string> rdma_missing() const;
    // Looks again for the RDMA device of every NIC without one; true when one appeared (the
    // topology file, which names the HCAs, is then generated again).
    bool refresh_rdma();
    std::string rdma_reason() const;  // the probe's per-NIC reason while a device is missing
    topo::GdrReport gdr_;
    void check_gdr();
    std::map<std::string, std::string> status_node() const;
    std::map<std::string, int64_t> phases_;
    int64_t t0_ = 0, t_last_ = 0;
    bool ready_ = false;
    bool aborted_ = false;
};

}  // namespace netop::agent

// Per-interface state carried through the agent's pipeline.
//
// Mirrors the reference's networkConfiguration (cmd/discover/network.go:65-74) and adds
// the MI355X-specific fields: the paired GPU, the RDMA device / RoCE v2 GID index and
// per-NIC timestamps used by the node-ready latency measurement.
#pragma once

#include <cstdint>
#include <optional>
#include <string>
#include <vector>

#include "netop/common.hpp"
#include "netop/l3.hpp"
#include "netop/netlink.hpp"
#include "netop/topology.hpp"

namespace netop {

struct NicState {
    std::string ifname;
    nl::LinkInfo link;
    unsigned orig_flags = 0;
    int orig_mtu = 0;  // at discovery: put back on a clean exit with --restore-mtu
    bool expect_response = false;

    // LLDP
    bool lldp_seen = false;
    std::string port_description;
    std::optional<MacAddr> peer_mac;
    std::string peer_system_name;
    std::string peer_port_id;
    bool lldp_from_cache = false;  // addressed from --lldp-cache, not yet confirmed by a frame
    bool cache_stale = false;      // the switch did not confirm the cached Port Description in time
    int64_t t_cache_applied = 0;

    // L3
    std::optional<l3::P2pAddressing> addr;
    std::string addr_error;
    bool configured = false;
    std::string config_error;
    // --verify-peers: the switch-side /30 address answered ARP (0 = not checked / no answer)
    bool peer_verified = false;
    int64_t peer_rtt_ns = 0;      // last ARP request -> answer
    int64_t peer_verify_ns = 0;   // first ARP request -> answer (retries included)
    // The ARP answer came from another MAC than the LLDP peer's (ChassisID/PortID MAC): a
    // proxy-ARP or misaddressed port, or a switch answering from its router MAC.  Reported, not
    // fatal (switches may legitimately answer ARP from a different MAC than their LLDP one).
    bool peer_mac_mismatch = false;
    std::optional<MacAddr> peer_arp_mac;
    std::string peer_error;

    // Topology
    int gpu_index = -1;
    int64_t speed_mbps = -1;
    int peer_max_frame = -1;  // the switch port's LLDP 802.3 Maximum Frame Size, -1 when not sent  // negotiated link speed when checked (--min-link-speed-gbps), -1 unknown
    std::string gpu_bdf;
    std::string rdma_dev;
    int rdma_port = 1;
    std::optional<int> gid_index;
    int numa_node = -1;     // NUMA node of the GPU (pin the rank's CPU threads there)
    std::string pcie_path;  // GPU <-> NIC PCIe path type (PIX / PXB / ...)
    // PCIe links of the NIC and of its GPU as trained (read at discovery; --require-full-pcie)
    topo::PcieLink pcie, gpu_pcie;
    // The monitor found the link (or its GPU's) retrained below its maximum after readiness
    // (--require-full-pcie): the label waits for it.  "" = fine.
    std::string pcie_error;
    // Per-rail source routing: this NIC's rail k (its GPU index; NICs without a GPU get indices
    // above every GPU's) and what the agent installed for it, so exactly that is removed later.
    int rail_index = -1;
    std::optional<nl::RuleSpec> rail_rule;
    std::vector<nl::RouteSpec> rail_routes;

    // NIC firmware LLDP agent (--disable-fw-lldp): summary of what was done
    std::string fw_lldp;
    // DCBX mode of the NIC (DCB netlink), in words: read by --disable-fw-lldp, or when the NIC
    // stays silent; "" = not read / no DCB interface.
    std::string dcbx;
    bool dcbx_embedded = false;  // an embedded agent holds DCBX (not handed to the host by us)
    // L3, --wait expired without a frame: the NIC's driver and what it did hear meanwhile
    // (Agent::diagnose_silent), e.g. "mlx5_core: no LLDPDU in 90s while 412 frames arrived ...".
    std::string driver;
    std::optional<uint64_t> rx_at_listen;  // link rx_packets when the LLDP wait began
    std::string lldp_silent;

    // L2: admin-up, no carrier (IFF_LOWER_UP) yet, and still within --carrier-wait: the optic
    // and the switch port are training (seconds on 200/400G PAM4 links).  Start-up, not a fault.
    bool awaiting_carrier = false;
    // L2: admin-up but no carrier within --carrier-wait: an unplugged cable, a dead switch port.
    // Not configured, not counted for readiness until the carrier comes.
    bool no_carrier = false;

    // Monitor
    bool degraded = false;  // link went down / lost carrier after readiness
    int flaps = 0;

    // Timing (CLOCK_MONOTONIC ns; 0 = never)
    int64_t t_lldp = 0;
    int64_t t_configured = 0;
};

}  // namespace netop

// Node topology discovery from sysfs: amdgpu GPUs, scale-out NICs, GPU<->NIC PCIe
// affinity, RDMA devices / RoCE GID indices, and the xGMI mesh from the KFD topology.
//
// Reference: the Gaudi agent globs netdevs *under* the accelerator's PCI function
// ($SYSFS_ROOT/bus/pci/drivers/habanalabs/????:??:??.?/net/*, cmd/discover/network.go:84-119)
// because Gaudi NICs are integrated.  MI355X has no integrated NICs: each OAM GPU sits
// behind a PCIe switch together with a discrete RoCE NIC, so the scale-out NICs are the
// netdevs that share a PCIe switch with an amdgpu function.  The reference-compatible
// "netdevs under the accelerator function" mode is kept (DiscoveryMode::Accel) and the
// SYSFS_ROOT override is preserved for fake-sysfs tests.
#pragma once

#include <cstdint>
#include <map>
#include <optional>
#include <string>
#include <vector>

#include "netop/common.hpp"

namespace netop::topo {

std::string sysfs_root();  // $SYSFS_ROOT or "/sys/"

struct PciDev {
    std::string bdf;                 // "0000:0a:00.0"
    std::string path;                // resolved path, e.g. <root>/devices/pci0000:00/.../0000:0a:00.0
    std::vector<std::string> chain;  // path components from the host bridge ("pci0000:00") down to bdf
    std::string driver;
    uint32_t vendor = 0, device = 0, pci_class = 0;
    uint32_t subsystem_vendor = 0, subsystem_device = 0;
    int numa = -1;
    // PCIe link capability of the function and of the port above it (sysfs max_link_speed /
    // max_link_width of the device and of its parent directory); "" / 0 when unreadable.
    std::string max_link_speed, port_max_link_speed;  // e.g. "32.0 GT/s PCIe"
    int max_link_width = 0, port_max_link_width = 0;
    bool topo_attrs = false;  // subsystem ids and link attributes were read (read_pci_dev(..., true))
    // The link as RCCL records it (NCCL xml.cc): the slower of device and port speed (the
    // device's string when neither parses), the narrower width.
    std::string rccl_link_speed() const;
    int rccl_link_width() const;
};

struct Gpu {
    int index = 0;  // ordinal (sorted by BDF), matches HIP/RCCL enumeration on a standard node
    PciDev pci;
};

struct Nic {
    std::string ifname;
    PciDev pci;
    MacAddr mac;
    std::string rdma_dev;  // e.g. "mlx5_3" (empty when not an RDMA NIC)
    int rdma_port = 1;
};

// NCCL/RCCL path types, ordered best-first.
enum class PathType { PIX = 0, PXB = 1, PHB = 2, NODE = 3, SYS = 4 };
const char* to_string(PathType p);

struct GpuNicPair {
    int gpu = -1;  // index into gpus
    int nic = -1;  // index into nics
    PathType path = PathType::SYS;
    int common_depth = 0;
};

// Affine: GPU-paired scale-out NICs.  Accel: reference layout (netdevs under the accelerator
// function).  Rdma: every RDMA-capable NIC of the driver allow-list that is not a GPU's scale-out
// rail (the host-nic configuration type).  None: --interfaces only.
enum class DiscoveryMode { Affine, Accel, Rdma, None };
std::optional<DiscoveryMode> parse_discovery_mode(std::string_view s);

struct DiscoveryOptions {
    DiscoveryMode mode = DiscoveryMode::Affine;
    std::string accel_driver = "amdgpu";
    // Empty = any PCI network driver.
    std::vector<std::string> nic_drivers{"mlx5_core", "bnxt_en", "ionic", "ice", "irdma", "i40e", "qede", "cxgb4"};
    PathType max_path = PathType::PXB;  // NICs farther than this from every GPU are not scale-out NICs
    // Rdma mode: leave out every NIC within `gpu_rail_path` of an accelerator function.  Those are
    // the GPUs' scale-out rails, which the amd-so agent owns (whatever driver list it runs with);
    // the reference can never reach them from another agent either, since it only ever enumerates
    // netdevs under the accelerator's own PCI functions (cmd/discover/network.go:34,88-119).
    bool exclude_gpu_rails = true;
    PathType gpu_rail_path = PathType::PXB;
};

// `topo_attrs`: also read the subsystem ids and the link attributes, which only the topology
// file needs (discovery skips them: six fewer sysfs reads per device on the critical path).
std::optional<PciDev> read_pci_dev(const std::string& root, const std::string& device_path, bool topo_attrs = true);
// The same for a path that is already canonical (no symlink to resolve), e.g. PciDev::path.
std::optional<PciDev> read_pci_dir(const std::string& canonical_path, bool topo_attrs = true, bool with_driver = true);
// Adds the topology attributes to a device discovery read without them; false if unreadable.
bool read_topo_attrs(PciDev& d);
// The PCI device behind a netdev (<root>/class/net/<ifname>/device); nullopt for virtual links.
std::optional<PciDev> netdev_pci(const std::string& root, const std::string& ifname);
// The negotiated link speed in Mb/s (<root>/class/net/<if>/speed), or -1 when the driver does not
// report one (link down, virtual NIC, no such file).
int64_t netdev_speed_mbps(const std::string& root, const std::string& ifname);
// The RDMA device of a netdev's PCI function (<root>/class/net/<ifname>/device/infiniband/*):
// present once the NIC's RDMA driver (mlx5_ib, ionic_rdma, bnxt_re) has registered it.  "" when
// there is none (yet).
std::string netdev_rdma_device(const std::string& root, const std::string& ifname);
// Devices stacked on a netdev (its sysfs upper_<name> links): the bond, bridge or team it is
// enslaved to, VLANs and macvlans on it.  Sorted; empty when there are none or no sysfs entry.
std::vector<std::string> netdev_uppers(const std::string& root, const std::string& ifname);
// The ancestors RCCL puts above `d` in its topology tree, outermost first.  RCCL (NCCL's
// ncclTopoGetXmlFromSys) climbs the sysfs path two components at a time — a switch's downstream
// port and the switch above it count as one bridge — and stops at the root complex, whose
// "pciDDDD:BB" component is not a BDF; the CPU node there is the outermost ancestor's NUMA node.
// Mirroring that walk keeps a topology file the agent writes identical to RCCL's own view.
// `cache` (optional) holds bridges already read, by sysfs path: GPUs and NICs share switches.
std::vector<PciDev> rccl_pci_parents(const PciDev& d, std::map<std::string, PciDev>* cache = nullptr);

// The CPU identity RCCL records on each <cpu> node of its topology (NCCL's ncclTopoGetXmlFromCpu):
// uname machine, and on x86_64 the CPUID vendor string and family / model ids computed the way
// NCCL does (family + extended family << 4, model + extended model << 4 — e.g. 191 / 2 on the
// MI355X boxes' Zen 5 CPUs, not /proc/cpuinfo's 26).  RCCL refuses a topology file whose <cpu>
// lacks them ("Attribute arch of node cpu not found"): it fills CPU attributes only for CPU
// nodes it creates itself.
struct CpuIdentity {
    std::string arch;    // "x86_64"
    std::string vendor;  // "AuthenticAMD"
    int family = -1, model = -1;
};
CpuIdentity cpu_identity();  // of the machine running this code
// <root>/devices/system/node/node<N>/cpumap ("ffffffff,..."); "" if unknown.
std::string numa_cpumap(const std::string& root, int numa);
std::vector<Gpu> discover_gpus(const std::string& root, const std::string& driver = "amdgpu");
std::vector<Nic> discover_pci_nics(const std::string& root, const std::vector<std::string>& drivers);
PathType path_between(const PciDev& a, const PciDev& b, int* common_depth = nullptr);
// Greedy best-first unique pairing: each GPU gets the closest free NIC within max_path.
std::vector<GpuNicPair> pair_gpus_nics(const std::vector<Gpu>& gpus, const std::vector<Nic>& nics, PathType max_path);

// Reference-compatible: netdev names found under the accelerator driver's PCI functions.
std::vector<std::string> accel_netdevs(const std::string& root, const std::string& driver);

struct DiscoveryResult {
    std::vector<Gpu> gpus;
    std::vector<Nic> nics;            // every candidate PCI NIC seen
    std::vector<GpuNicPair> pairs;    // GPU -> NIC assignment (Affine mode)
    std::vector<std::string> ifnames; // selected scale-out interfaces, in GPU order
    // Candidates discovery left out, with the reason (Rdma mode: the GPUs' scale-out rails).
    std::vector<std::pair<std::string, std::string>> excluded;
};
DiscoveryResult discover(const DiscoveryOptions& opt, const std::string& root = sysfs_root());

// RoCE v2 GID index on (rdma_dev, port) whose GID is the IPv4-mapped address `ip`.
std::optional<int> find_rocev2_gid_index(const std::string& root, const std::string& rdma_dev, int port, Ipv4 ip);

// ---------------------------------------------------------------------------
// xGMI mesh from the KFD topology (/sys/class/kfd/kfd/topology/nodes/*)
// ---------------------------------------------------------------------------
constexpr int kIoLinkTypeXgmi = 11;  // HSA_IOLINK_TYPE_XGMI (hsakmttypes.h)
constexpr int kIoLinkTypePcie = 2;

struct KfdNode {
    int node = -1;
    uint32_t gpu_id = 0;
    uint32_t simd_count = 0;
    uint32_t vendor_id = 0, device_id = 0;
    uint32_t location_id = 0, domain = 0;
    uint64_t hive_id = 0;
    uint32_t num_xcc = 0;
    std::string bdf() const;  // from domain + location_id
    bool is_gpu() const { return simd_count > 0; }
};

struct KfdLink {
    int from = -1, to = -1, type = 0, weight = 0;
    uint32_t min_bw_mbs = 0, max_bw_mbs = 0;
};

struct XgmiReport {
    std::vector<KfdNode> gpus;              // GPU nodes, sorted by BDF
    std::vector<KfdLink> links;             // every xGMI link seen (either direction)
    int pairs_expected = 0;                 // n*(n-1)/2 among GPUs of the same hive
    int pairs_connected = 0;                // unordered GPU pairs with an xGMI link
    std::vector<std::pair<std::string, std::string>> missing;  // BDF pairs without a link
    uint64_t min_link_bw_mbs = 0;           // slowest advertised xGMI link
    bool full_mesh() const { return pairs_connected == pairs_expected; }
    // Per-GPU aggregate advertised xGMI bandwidth (MB/s, one direction) — the busbw ceiling
    // input for the all-reduce validation.
    uint64_t per_gpu_bw_mbs() const;
};

XgmiReport read_xgmi(const std::string& root = sysfs_root());

// The trained state of one GPU's xGMI links, from amdgpu's gpu_metrics blob (sysfs, readable
// without privileges): what amd-smi reports as link status, width and bit rate, read without the
// library.  KFD's topology (read_xgmi) says which links exist; this says whether they are up and
// at what width.  The blob's layout is versioned (format.content); only revisions this reader
// knows are decoded -- 1.8, which MI355X firmware reports (layout checked against amd-smi on a
// live node: tests/fixtures/gpu_metrics_v1_8.bin) -- anything else is reported as not read.
// Negotiated vs maximum PCIe link of a PCI function (current_link_speed / _width against
// max_link_*).  A card that trained below what it and its slot support (a loose card or riser,
// a bad lane, a BIOS slot setting) moves RDMA or GPUDirect traffic at a fraction of its rate.
struct PcieLink {
    double speed_gts = 0, max_speed_gts = 0;  // GT/s; 0 when the attribute is missing
    int width = 0, max_width = 0;
    bool known() const { return speed_gts > 0 && width > 0 && max_speed_gts > 0 && max_width > 0; }
    bool slower() const { return known() && speed_gts + 1e-6 < max_speed_gts; }
    bool narrower() const { return known() && width < max_width; }
    bool degraded() const { return slower() || narrower(); }
    std::string str() const;  // "32.0 GT/s x16", or "16.0 GT/s x8 of 32.0 GT/s x16" when degraded
};
PcieLink read_pcie_link(const std::string& root, const std::string& bdf);

constexpr int kMaxXgmiLinks = 8;
struct XgmiLinkHealth {
    std::string bdf;
    std::string revision;          // "1.8"
    bool known = false;            // decoded (a known revision, not truncated)
    std::string error;             // why not
    bool late = false;             // the read did not return in time (see the bounded overload)
    int width = 0;                 // lanes per link
    int speed_gbps = 0;            // per-lane rate (amd-smi's bit_rate)
    std::vector<int> status;       // per link slot: 1 up, 0 down, -1 no link in this slot
    std::vector<uint64_t> read_kb, write_kb;  // accumulated traffic per slot
    int links_up() const;
    int links_down() const;
};
XgmiLinkHealth parse_gpu_metrics(const std::string& blob);
// One entry per BDF, from <root>/bus/pci/devices/<bdf>/gpu_metrics.
std::vector<XgmiLinkHealth> read_xgmi_health(const std::string& root, const std::vector<std::string>& bdfs);
// The same with the GPUs read concurrently (netop/bounded.hpp), for at most `timeout_ns`: a GPU
// whose gpu_metrics has not answered by then (a wedged or resetting SMU) is reported `late`, and
// its read is not started again until the one still blocked returns.
std::vector<XgmiLinkHealth> read_xgmi_health(const std::string& root, const std::vector<std::string>& bdfs,
                                             int64_t timeout_ns);

// GPUDirect RDMA readiness: can the RoCE NICs DMA straight into MI355X HBM?  Without it RCCL
// stages every inter-node transfer through host memory, costing bandwidth and latency.
// Two mechanisms exist on ROCm:
//   * peer-memory: the amdgpu driver registers "amdkfd" with ib_core's peer-memory client API
//     (/sys/kernel/mm/memory_peers/amdkfd/version, MLNX_OFED / amdgpu-dkms);
//   * dma-buf:     upstream RDMA dma-buf memory regions, kernel >= 5.12 with ib_uverbs loaded.
struct GdrReport {
    bool peer_mem = false;
    std::string peer_mem_version;
    bool ib_uverbs = false;
    std::string kernel;          // release string the dma-buf decision used
    bool dmabuf = false;
    std::string mode() const { return peer_mem ? "peermem" : dmabuf ? "dmabuf" : "none"; }
};
// `kernel_release` = "" reads uname(2).
// L2 mode (no IPv4 on the NICs): the RoCE v2 GID of the port's IPv6 link-local address
// (fe80::/64) is the one RCCL must use.
std::optional<int> find_rocev2_linklocal_gid_index(const std::string& root, const std::string& rdma_dev, int port);
GdrReport detect_gdr(const std::string& root = sysfs_root(), const std::string& kernel_release = "");
bool kernel_at_least(const std::string& release, int major, int minor);

}  // namespace netop::topo

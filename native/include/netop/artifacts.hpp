// Node-local artifacts written by the agent.
//
//   rccl-net.json   This operator's own per-node NIC contract (RCCL does not read it): the
//                   reference's gaudinet.json entry schema (cmd/discover/gaudinet.go:28-37) —
//                   NIC_MAC, NIC_IP, SUBNET_MASK, GATEWAY_MAC first, in that order — extended
//                   with NIC_NAME, GATEWAY_IP, GPU_BDF, RDMA_DEV and GID_INDEX.  Consumers:
//                   the validation tooling (parallel/rail.py, validate.py) and users' launchers.
//   rccl.env        KEY=VALUE environment for RCCL jobs on this node — what RCCL itself
//                   consumes: NCCL_IB_HCA in GPU order, NCCL_IB_GID_INDEX for RoCE v2,
//                   NCCL_SOCKET_IFNAME, NCCL_TOPO_FILE.
//   rccl-topo.xml   NCCL_TOPO_FILE (generate_rccl_topo below).
//   *.network       systemd-networkd units (cmd/discover/systemd-networkd.go:49-74), same text.
//   NFD label file  features.d readiness label (cmd/discover/main.go:43-45,239-246).
#pragma once

#include <map>
#include <string>
#include <vector>

#include "netop/state.hpp"
#include "netop/topology.hpp"

namespace netop::artifacts {

// Minimal streaming JSON writer (compact output, like Go's encoding/json.Marshal).
class Json {
   public:
    Json& begin_object();
    Json& end_object();
    Json& begin_array();
    Json& end_array();
    Json& key(const std::string& k);
    Json& value(const std::string& s);
    Json& value(const char* s) { return value(std::string(s)); }
    Json& value(int64_t v);
    Json& value(int v) { return value(int64_t(v)); }
    Json& value(uint64_t v);
    Json& value(double v);
    Json& value(bool b);
    Json& null();
    const std::string& str() const { return out_; }
    static std::string escape(const std::string& s);

   private:
    void sep();
    std::string out_;
    std::vector<bool> first_{true};
    bool after_key_ = false;
};

// Entries are sorted by (gpu_index, ifname) so the file is deterministic.
std::string generate_rccl_net(const std::vector<NicState>& nics, bool extended = true);
void write_rccl_net(const std::string& path, const std::vector<NicState>& nics, bool extended = true);

// `extra`: site settings appended verbatim (e.g. NCCL_IB_TC for the fabric's RoCE traffic class);
// keys must look like NCCL_* / RCCL_* / HSA_*, values must be single-line (parse_env_extra).
// `socket_ifnames`: NCCL_SOCKET_IFNAME (exact-match list, "=a,b"): the interfaces RCCL bootstraps
// over and, without RDMA, moves data over.  Empty = not written.
// GID: one index shared by every scale-out NIC is pinned with NCCL_IB_GID_INDEX.  When the
// indices differ (or one is not known yet) RCCL's own per-NIC selection is steered instead:
// NCCL_IB_ROCE_VERSION_NUM=2 and NCCL_IB_ADDR_FAMILY = AF_INET (L3 /30s) or AF_INET6
// (`link_local`, L2: the fe80:: GID), both read by RCCL 2.26 / 2.27.
std::string generate_rccl_env(const std::vector<NicState>& nics, const std::string& topo_file,
                              const std::vector<std::pair<std::string, std::string>>& extra = {},
                              const std::vector<std::string>& socket_ifnames = {}, bool link_local = false);
void write_rccl_env(const std::string& path, const std::vector<NicState>& nics, const std::string& topo_file,
                    const std::vector<std::pair<std::string, std::string>>& extra = {},
                    const std::vector<std::string>& socket_ifnames = {}, bool link_local = false);

// NCCL_TOPO_FILE: the node's PCIe tree as RCCL models it (RCCL's topology-XML dialect, the
// format NCCL_TOPO_DUMP_FILE writes): one <cpu numaid> per root-complex NUMA node, the switches
// above each GPU and scale-out NIC folded the way RCCL folds them (topo::rccl_pci_parents), the
// GPUs' PCI functions, and under each NIC's function a <nic><net name=...> whose name is what
// RCCL's network plugin calls the device (the RDMA device for the IB plugin, else the netdev).
// RCCL loads the file, then fills every attribute the file leaves out (GPU dev/rank/arch, link
// speeds, NIC speed/GDR) from the running system and drops devices its job does not use, so the
// file pins the PCIe affinity — which NIC is next to which GPU — without ever naming a device
// index that differs per job.  The <cpu> nodes carry arch / vendor / familyid / modelid / affinity
// because RCCL does not fill those for CPU nodes it reads from a file and fails init without
// them (measured on the box: "Attribute arch of node cpu not found").  xGMI links are left out:
// RCCL detects them itself for the GPUs of each communicator, and whether it would also keep
// file-provided links (doubling the link count it plans rings with) cannot be checked without
// a multi-GPU run.  Verified on an MI355X box with torch's RCCL 2.26.6 and ROCm's 2.27.7: the
// file loads and RCCL's dump places the GPU exactly as the file does (profiles/r2_rccl_topo_box.md).
constexpr int kRcclTopoXmlVersion = 2;  // <system version="2">: RCCL 2.26 / 2.27 (ROCm 7)
struct TopoNic {
    topo::PciDev pci;
    std::string net_name;  // RCCL network device name
    int port = 0;          // RDMA port (0 = not written)
};
// `cpu` goes on every <cpu> node (RCCL requires arch / vendor / familyid / modelid there), with
// the NUMA node's cpumap from `sysfs_root` as its affinity.
std::string generate_rccl_topo(const std::vector<topo::Gpu>& gpus, const std::vector<TopoNic>& nics,
                               const topo::CpuIdentity& cpu, const std::string& sysfs_root,
                               int version = kRcclTopoXmlVersion);
void write_rccl_topo(const std::string& path, const std::vector<topo::Gpu>& gpus, const std::vector<TopoNic>& nics,
                     const topo::CpuIdentity& cpu, const std::string& sysfs_root, int version = kRcclTopoXmlVersion);
// The NICs of `names` as RCCL sees them: PCI function from the discovery result (or sysfs for an
// extra --interfaces NIC), net name = RDMA device when the NIC has one, else the netdev name.
std::vector<TopoNic> topo_nics(const topo::DiscoveryResult& d, const std::vector<std::string>& names,
                               const std::string& sysfs_root);
// "K=V,K2=V2" -> pairs; throws std::invalid_argument on a bad key or value.
std::vector<std::pair<std::string, std::string>> parse_env_extra(const std::string& spec);

std::string networkd_filename(const std::string& dir, const std::string& ifname);
std::string generate_networkd(const NicState& nic);
// Validates every interface first, writes one unit per interface and rolls back on error
// (systemd-networkd.go:76-94).  Returns the interfaces written.
std::vector<std::string> write_networkd(const std::string& dir, const std::vector<NicState>& nics);
void delete_networkd(const std::string& dir, const std::vector<std::string>& ifnames);

// NFD local feature source.
struct Labels {
    std::string dir = "/etc/kubernetes/node-feature-discovery/features.d/";
    std::string file = "scale-out-readiness.txt";
    std::string key = "amd.feature.node.kubernetes.io/gpu-scale-out";  // published as "<key>=true"
    std::string path() const;
};
extern const char* const kScaleOutReadyLabel;  // "amd.feature.node.kubernetes.io/gpu-scale-out=true"
std::string generate_labels(const std::map<std::string, std::string>& extra,
                            const std::string& key = "amd.feature.node.kubernetes.io/gpu-scale-out");
// Writes the label file only when the features.d directory exists (main.go:240).  Returns
// true when written.
bool write_labels(const Labels& l, const std::map<std::string, std::string>& extra);
bool remove_labels(const Labels& l);

// LLDP cache (--lldp-cache): the last Port Description each NIC confirmed from a real frame,
// so a restarted agent (DaemonSet upgrade, crash, node reboot) configures at once instead of
// waiting up to msgTxInterval for a switch that does not fast-start; the monitor then expects
// the switch to confirm it.  One line per NIC, tab-separated:
//   <nic mac> <ifname> <unix seconds> <peer mac|-> <system name> <port id> <port description>
struct LldpCacheEntry {
    std::string nic_mac, ifname;
    int64_t unix_s = 0;
    std::string peer_mac, system_name, port_id, port_description;
};
std::vector<LldpCacheEntry> read_lldp_cache(const std::string& path);  // [] when absent / unreadable
void write_lldp_cache(const std::string& path, const std::vector<LldpCacheEntry>& entries);
// The file's text (the switch controls System Name, Port ID and Port Description: a tab or line
// break in them can never make another field or another NIC's line).
std::string encode_lldp_cache(const std::vector<LldpCacheEntry>& entries);
std::vector<LldpCacheEntry> decode_lldp_cache(const std::string& text);

// Agent status document (phase timings, per-NIC results) for observability and the bench.
std::string generate_status(const std::vector<NicState>& nics, const std::map<std::string, int64_t>& phases_ns,
                            int64_t t0_mono, const std::string& mode, bool ready,
                            const std::map<std::string, std::string>& node = {});

}  // namespace netop::artifacts

// Node-local artifacts written by the agent.
//
//   rccl-net.json   RCCL scale-out NIC contract.  Same NIC_NET_CONFIG entry schema as the
//                   reference's gaudinet.json (cmd/discover/gaudinet.go:28-37) — NIC_MAC,
//                   NIC_IP, SUBNET_MASK, GATEWAY_MAC first, in that order — extended with
//                   NIC_NAME, GATEWAY_IP, GPU_BDF, RDMA_DEV and GID_INDEX.
//   rccl.env        KEY=VALUE environment for RCCL jobs on this node (NCCL_IB_HCA in GPU
//                   order, NCCL_IB_GID_INDEX for RoCE v2, ...).
//   *.network       systemd-networkd units (cmd/discover/systemd-networkd.go:49-74), same text.
//   NFD label file  features.d readiness label (cmd/discover/main.go:43-45,239-246).
#pragma once

#include <map>
#include <string>
#include <vector>

#include "netop/state.hpp"

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
std::string generate_rccl_env(const std::vector<NicState>& nics, const std::string& topo_file,
                              const std::vector<std::pair<std::string, std::string>>& extra = {});
void write_rccl_env(const std::string& path, const std::vector<NicState>& nics, const std::string& topo_file,
                    const std::vector<std::pair<std::string, std::string>>& extra = {});
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

// Agent status document (phase timings, per-NIC results) for observability and the bench.
std::string generate_status(const std::vector<NicState>& nics, const std::map<std::string, int64_t>& phases_ns,
                            int64_t t0_mono, const std::string& mode, bool ready,
                            const std::map<std::string, std::string>& node = {});

}  // namespace netop::artifacts

// libnetop_smi.so / netop-xgmi-counters — xGMI link state and traffic counters via amd-smi.
//
// BASELINE.json asks for validation "with rccl-tests and rocm-smi link counters": after the
// operator has configured a node, an all-reduce must move bytes over *every* xGMI link.
// netop_smi_snapshot() returns, per visible GPU, the link status (up / down / disabled), the
// link width / speed and the accumulated per-link read / write counters (KB); bench.py takes
// a snapshot before and after the timed all-reduce loop and reports the per-link traffic.
// Kept out of the node agent (which has no ROCm dependency) — this links libamd_smi.
#include <amd_smi/amdsmi.h>

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

namespace {

std::string bdf_str(amdsmi_bdf_t b) {
    char buf[32];
    std::snprintf(buf, sizeof buf, "%04llx:%02x:%02x.%x", (unsigned long long)b.domain_number, (unsigned)b.bus_number,
                  (unsigned)b.device_number, (unsigned)b.function_number);
    return buf;
}

const char* status_char(amdsmi_xgmi_link_status_type_t s) {
    switch (s) {
        case AMDSMI_XGMI_LINK_UP: return "U";
        case AMDSMI_XGMI_LINK_DOWN: return "D";
        default: return "X";
    }
}

}  // namespace

extern "C" {

// Writes a JSON document into `out` (NUL-terminated, truncated to `cap`).  Returns the
// amdsmi_status_t of the first failing call (0 = success).
int netop_smi_snapshot(char* out, size_t cap) {
    std::string j = "{\"gpus\":[";
    amdsmi_status_t st = amdsmi_init(AMDSMI_INIT_AMD_GPUS);
    if (st != AMDSMI_STATUS_SUCCESS) {
        std::snprintf(out, cap, "{\"error\":\"amdsmi_init failed: %d\"}", int(st));
        return int(st);
    }
    uint32_t nsock = 0;
    amdsmi_get_socket_handles(&nsock, nullptr);
    std::vector<amdsmi_socket_handle> socks(nsock);
    amdsmi_get_socket_handles(&nsock, socks.data());
    bool first = true;
    for (auto s : socks) {
        uint32_t np = 0;
        amdsmi_get_processor_handles(s, &np, nullptr);
        std::vector<amdsmi_processor_handle> ps(np);
        amdsmi_get_processor_handles(s, &np, ps.data());
        for (auto p : ps) {
            amdsmi_bdf_t bdf{};
            amdsmi_get_gpu_device_bdf(p, &bdf);
            j += first ? "" : ",";
            first = false;
            j += "{\"bdf\":\"" + bdf_str(bdf) + "\"";
            amdsmi_xgmi_link_status_t ls{};
            if (amdsmi_get_gpu_xgmi_link_status(p, &ls) == AMDSMI_STATUS_SUCCESS) {
                j += ",\"link_status\":\"";
                for (uint32_t i = 0; i < ls.total_links && i < AMDSMI_MAX_NUM_XGMI_LINKS; ++i) j += status_char(ls.status[i]);
                j += "\"";
            }
            amdsmi_gpu_metrics_t m{};
            if (amdsmi_get_gpu_metrics_info(p, &m) == AMDSMI_STATUS_SUCCESS) {
                char buf[128];
                std::snprintf(buf, sizeof buf, ",\"xgmi_link_width\":%u,\"xgmi_link_speed\":%u", unsigned(m.xgmi_link_width),
                              unsigned(m.xgmi_link_speed));
                j += buf;
                j += ",\"xgmi_read_kb\":[";
                for (int i = 0; i < AMDSMI_MAX_NUM_XGMI_LINKS; ++i) {
                    std::snprintf(buf, sizeof buf, "%s%llu", i ? "," : "", (unsigned long long)m.xgmi_read_data_acc[i]);
                    j += buf;
                }
                j += "],\"xgmi_write_kb\":[";
                for (int i = 0; i < AMDSMI_MAX_NUM_XGMI_LINKS; ++i) {
                    std::snprintf(buf, sizeof buf, "%s%llu", i ? "," : "", (unsigned long long)m.xgmi_write_data_acc[i]);
                    j += buf;
                }
                j += "]";
            }
            amdsmi_link_metrics_t lm{};
            if (amdsmi_get_link_metrics(p, &lm) == AMDSMI_STATUS_SUCCESS) {
                j += ",\"links\":[";
                for (uint32_t i = 0; i < lm.num_links && i < AMDSMI_MAX_NUM_XGMI_PHYSICAL_LINK; ++i) {
                    char buf[256];
                    std::snprintf(buf, sizeof buf,
                                  "%s{\"peer\":\"%s\",\"type\":%d,\"bit_rate_gbps\":%u,\"max_bw_gbps\":%u,\"read_kb\":%llu,"
                                  "\"write_kb\":%llu}",
                                  i ? "," : "", bdf_str(lm.links[i].bdf).c_str(), int(lm.links[i].link_type),
                                  lm.links[i].bit_rate, lm.links[i].max_bandwidth,
                                  (unsigned long long)lm.links[i].read, (unsigned long long)lm.links[i].write);
                    j += buf;
                }
                j += "]";
            }
            j += "}";
        }
    }
    j += "]}";
    amdsmi_shut_down();
    std::snprintf(out, cap, "%s", j.c_str());
    return 0;
}

}  // extern "C"

#ifdef NETOP_SMI_MAIN
int main() {
    std::vector<char> buf(1 << 20);
    int rc = netop_smi_snapshot(buf.data(), buf.size());
    std::printf("%s\n", buf.data());
    return rc ? 1 : 0;
}
#endif

// `netop-xgmi-probe` — GPU-side xGMI link validation for a node (single process, every
// visible GPU).  Prints JSON: per-link pull bandwidth, per-GPU aggregate bandwidth with all
// peers pulled concurrently, and byte-exact integrity of every transfer.  The agent can gate
// its readiness label on this (`discover --xgmi-expect`), the operator docs use it as the
// post-configuration check.  On a 1-GPU box it degenerates to a loopback HBM copy.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

extern "C" int netop_xgmi_probe(uint64_t bytes, int iters, int max_gpus, double* bw_single, double* bw_all, int* n_out,
                                unsigned long long* total_errors);
extern "C" int netop_xgmi_probe_push(uint64_t bytes, int iters, int max_gpus, double* bw_push, int* n_out,
                                     unsigned long long* total_errors);

int main(int argc, char** argv) {
    uint64_t bytes = 256ull << 20;
    int iters = 10, max_gpus = 8;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        if (a.rfind("--bytes=", 0) == 0) bytes = std::strtoull(a.c_str() + 8, nullptr, 0);
        else if (a.rfind("--iters=", 0) == 0) iters = std::atoi(a.c_str() + 8);
        else if (a.rfind("--max-gpus=", 0) == 0) max_gpus = std::atoi(a.c_str() + 11);
        else {
            std::fprintf(stderr, "usage: netop-xgmi-probe [--bytes=N] [--iters=N] [--max-gpus=N]\n");
            return 2;
        }
    }
    std::vector<double> single(64 * 64, 0.0), all(64, 0.0);
    int n = 0;
    unsigned long long errors = 0;
    int rc = netop_xgmi_probe(bytes, iters, max_gpus, single.data(), all.data(), &n, &errors);
    if (rc != 0) {
        std::fprintf(stderr, "netop_xgmi_probe failed: hip error %d\n", rc);
        return 1;
    }
    std::printf("{\"gpus\":%d,\"bytes\":%llu,\"iters\":%d,\"errors\":%llu,\"link_GBps\":[", n, (unsigned long long)bytes,
                iters, errors);
    for (int d = 0; d < n; ++d) {
        std::printf("%s[", d ? "," : "");
        for (int p = 0; p < n; ++p) std::printf("%s%.1f", p ? "," : "", single[size_t(d * n + p)]);
        std::printf("]");
    }
    std::printf("],\"aggregate_GBps\":[");
    for (int d = 0; d < n; ++d) std::printf("%s%.1f", d ? "," : "", all[size_t(d)]);
    // Push: every GPU writes to all of its peers at once.
    std::vector<double> push(64, 0.0);
    int n2 = 0;
    unsigned long long perr = 0;
    rc = netop_xgmi_probe_push(bytes, iters, max_gpus, push.data(), &n2, &perr);
    if (rc != 0) {
        std::fprintf(stderr, "netop_xgmi_probe_push failed: hip error %d\n", rc);
        return 1;
    }
    std::printf("],\"push_aggregate_GBps\":[");
    for (int d = 0; d < n2; ++d) std::printf("%s%.1f", d ? "," : "", push[size_t(d)]);
    std::printf("],\"push_errors\":%llu}\n", perr);
    return errors || perr ? 3 : 0;
}

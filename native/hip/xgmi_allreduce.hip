// `netop-xgmi-allreduce` — a direct xGMI all-reduce for one 8x MI355X node, used to check the
// links the operator verified and to compare against RCCL on the same node.
//
// Why: an MI355X node is a full mesh.  Each GPU has 7 point-to-point xGMI links, one per peer.
// A ring all-reduce moves data over 2 links per ring at a time and needs many concurrent rings to
// load all 7 links.  A two-shot all-reduce in which every GPU talks to every peer at once loads
// all 7 links by construction:
//   reduce-scatter: GPU d owns chunk d of the message and reduces it from all n inputs;
//   all-gather:     GPU d fetches every other reduced chunk from the GPU that owns it.
// Each phase moves (n-1)/n of the message over n-1 links at once, so the algorithm's bus
// bandwidth limit is the per-GPU aggregate link bandwidth: 7 x 76 GB/s = 532 GB/s.
//
// Two data-movement schemes, both measured because xGMI read and write bandwidth differ:
//   pull  RS: GPU d loads chunk d of every peer's input (remote loads), sums in fp32,
//             and stores bf16 locally.
//         AG: GPU d copies chunk p from GPU p, for every peer p (remote loads).
//   push  RS: GPU p writes chunk q of its input into slot p of GPU q's scratch (remote stores),
//             then GPU q reduces its n slots locally.
//         AG: GPU q writes its reduced chunk into every peer's output (remote stores).
// Phases are ordered with events across streams and devices, never with in-kernel spinning
// on remote flags, so a lost peer can stall a stream but cannot hang a wavefront.
//
// Correctness: every size runs three rounds with different seeds on the same buffers, and
// each GPU's output is checked exactly against the bf16 pattern sum (netop_verify_pattern_at).
// Reusing the buffers this way catches stale remote lines in L2.
//
// --ranks N with fewer GPUs maps rank r to GPU (r % gpus).  This runs the full n-rank
// algorithm, including all chunking and cross-stream ordering, on a single GPU.  That is how
// the algorithm is tested on a 1-GPU box.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

extern "C" {
int netop_fill_pattern_at(void* buf, uint64_t n_elems, uint32_t seed, int rank_lo, int n_ranks, uint64_t elem_offset,
                          hipStream_t stream);
int netop_verify_pattern_at(const void* buf, uint64_t n_elems, uint32_t seed, int rank_lo, int n_ranks,
                            uint64_t elem_offset, unsigned long long* errors, hipStream_t stream);
int netop_sum_bf16(const void* const* srcs, int nsrc, void* dst, uint64_t n_elems, int wg_per_cu, hipStream_t stream);
}

namespace {

#define HIPCHECK(x)                                                                                \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                          \
        }                                                                                          \
    } while (0)

constexpr int kThreads = 256;
constexpr int kMaxRanks = 8;

struct Ptrs {
    const uint4* p[kMaxRanks];
};
struct DstPtrs {
    uint4* p[kMaxRanks];
};

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Several independent copies in one launch: blockIdx.y selects the (src, dst) pair.  Every byte
// is moved once: nontemporal loads and stores (copy_tune.hip, profiles/r6_copy_tune.jsonl).
__global__ __launch_bounds__(kThreads) void multi_copy_kernel(Ptrs src, DstPtrs dst, uint64_t n_vec) {
    const u32x4* __restrict__ s = reinterpret_cast<const u32x4*>(src.p[blockIdx.y]);
    u32x4* __restrict__ d = reinterpret_cast<u32x4*>(dst.p[blockIdx.y]);
    const uint64_t stride = uint64_t(gridDim.x) * kThreads;
    for (uint64_t i = uint64_t(blockIdx.x) * kThreads + threadIdx.x; i < n_vec; i += stride)
        __builtin_nontemporal_store(__builtin_nontemporal_load(&s[i]), &d[i]);
}

struct Rank {
    int dev = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev = nullptr;  // marks the end of this rank's current phase
    char* in = nullptr;       // message input (bytes)
    char* out = nullptr;      // result
    char* scratch = nullptr;  // push mode: n slots of one chunk
    unsigned long long* err = nullptr;
};

struct Args {
    uint64_t min_bytes = 1 << 20, max_bytes = 1ull << 30;
    double factor = 4;
    int iters = 20, warmup = 5, ranks = 0, per_cu = 4;
    std::string mode = "both";
};

int cu_count(int dev) {
    int c = 0;
    if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0) c = 256;
    return c;
}

class Node {
   public:
    Node(int n_ranks, int n_gpus, uint64_t max_bytes, int per_cu) : n_(n_ranks), per_cu_(per_cu) {
        ranks_.resize(n_);
        for (int r = 0; r < n_; ++r) ranks_[r].dev = r % n_gpus;
        for (int g = 0; g < n_gpus; ++g) cus_.push_back(cu_count(g));
        // Peer access between every pair of distinct GPUs in use.
        for (int a = 0; a < n_gpus && a < n_; ++a) {
            HIPCHECK(hipSetDevice(a));
            for (int b = 0; b < n_gpus && b < n_; ++b) {
                if (a == b) continue;
                int can = 0;
                HIPCHECK(hipDeviceCanAccessPeer(&can, a, b));
                if (!can) {
                    std::fprintf(stderr, "GPU %d cannot access GPU %d: no xGMI/P2P path\n", a, b);
                    std::exit(1);
                }
                hipError_t e = hipDeviceEnablePeerAccess(b, 0);
                if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) HIPCHECK(e);
                (void)hipGetLastError();
            }
        }
        bytes_cap_ = max_bytes;
        for (auto& r : ranks_) {
            HIPCHECK(hipSetDevice(r.dev));
            HIPCHECK(hipStreamCreateWithFlags(&r.stream, hipStreamNonBlocking));
            HIPCHECK(hipEventCreateWithFlags(&r.ev, hipEventDisableTiming));
            HIPCHECK(hipMalloc(&r.in, max_bytes));
            HIPCHECK(hipMalloc(&r.out, max_bytes));
            HIPCHECK(hipMalloc(&r.scratch, max_bytes));
            HIPCHECK(hipMalloc(&r.err, sizeof(unsigned long long)));
        }
    }
    ~Node() {
        for (auto& r : ranks_) {
            (void)hipSetDevice(r.dev);
            (void)hipStreamSynchronize(r.stream);
            (void)hipFree(r.in);
            (void)hipFree(r.out);
            (void)hipFree(r.scratch);
            (void)hipFree(r.err);
            (void)hipEventDestroy(r.ev);
            (void)hipStreamDestroy(r.stream);
        }
    }

    int n() const { return n_; }

    // Message size rounded so that every chunk is a whole number of 16-B vectors.
    uint64_t round_bytes(uint64_t bytes) const {
        uint64_t q = 16ull * n_;
        uint64_t b = (std::max<uint64_t>(bytes, q) + q - 1) / q * q;
        return std::min(b, bytes_cap_ / q * q);
    }

    // Every rank's stream waits until every rank has finished its current phase.
    void barrier() {
        for (auto& r : ranks_) {
            HIPCHECK(hipSetDevice(r.dev));
            HIPCHECK(hipEventRecord(r.ev, r.stream));
        }
        for (auto& r : ranks_) {
            HIPCHECK(hipSetDevice(r.dev));
            for (auto& p : ranks_)
                if (&p != &r) HIPCHECK(hipStreamWaitEvent(r.stream, p.ev, 0));
        }
    }

    void allreduce(uint64_t bytes, bool push) {
        const uint64_t chunk = bytes / n_;     // bytes per chunk
        const uint64_t cvec = chunk / 16;      // 16-B vectors per chunk
        // Entry condition: every rank's input is complete (the previous round ended with a
        // barrier, and fill() ends with one).
        if (!push) {
            for (int d = 0; d < n_; ++d) {
                Rank& r = ranks_[d];
                HIPCHECK(hipSetDevice(r.dev));
                Ptrs src{};
                for (int p = 0; p < n_; ++p)
                    src.p[p] = reinterpret_cast<const uint4*>(ranks_[p].in + uint64_t(d) * chunk);
                launch_reduce(r, src, reinterpret_cast<uint4*>(r.out + uint64_t(d) * chunk), cvec);
            }
            barrier();
            for (int d = 0; d < n_; ++d) gather_pull(d, chunk, cvec);
        } else {
            for (int p = 0; p < n_; ++p) scatter_push(p, chunk, cvec);
            barrier();
            for (int q = 0; q < n_; ++q) {
                Rank& r = ranks_[q];
                HIPCHECK(hipSetDevice(r.dev));
                Ptrs src{};
                for (int p = 0; p < n_; ++p)
                    src.p[p] = p == q ? reinterpret_cast<const uint4*>(r.in + uint64_t(q) * chunk)
                                      : reinterpret_cast<const uint4*>(r.scratch + uint64_t(p) * chunk);
                launch_reduce(r, src, reinterpret_cast<uint4*>(r.out + uint64_t(q) * chunk), cvec);
            }
            // The all-gather pushes read only the owner's own reduced chunk, and they write peer
            // chunks that no other phase touches.  So no barrier is needed before them.
            for (int q = 0; q < n_; ++q) gather_push(q, chunk, cvec);
        }
        // Nobody may overwrite inputs/scratch/outputs of this round before every peer is done.
        barrier();
    }

    void fill(uint32_t seed, uint64_t bytes) {
        for (int d = 0; d < n_; ++d) {
            Rank& r = ranks_[d];
            HIPCHECK(hipSetDevice(r.dev));
            HIPCHECK(hipError_t(netop_fill_pattern_at(r.in, bytes / 2, seed, d, 1, 0, r.stream)));
            HIPCHECK(hipMemsetAsync(r.out, 0xff, bytes, r.stream));  // poison: a missed chunk cannot pass
        }
        barrier();
    }

    unsigned long long verify(uint32_t seed, uint64_t bytes) {
        unsigned long long total = 0;
        for (auto& r : ranks_) {
            HIPCHECK(hipSetDevice(r.dev));
            HIPCHECK(hipMemsetAsync(r.err, 0, sizeof(unsigned long long), r.stream));
            HIPCHECK(hipError_t(netop_verify_pattern_at(r.out, bytes / 2, seed, 0, n_, 0, r.err, r.stream)));
            unsigned long long h = 0;
            HIPCHECK(hipMemcpyAsync(&h, r.err, sizeof h, hipMemcpyDeviceToHost, r.stream));
            HIPCHECK(hipStreamSynchronize(r.stream));
            total += h;
        }
        return total;
    }

    void sync() {
        for (auto& r : ranks_) {
            HIPCHECK(hipSetDevice(r.dev));
            HIPCHECK(hipStreamSynchronize(r.stream));
        }
    }

   private:
    int grid(const Rank& r, uint64_t work_vec, int split = 1) const {
        uint64_t need = (work_vec + kThreads - 1) / kThreads;
        uint64_t cap = std::max<uint64_t>(1, uint64_t(cus_[r.dev]) * per_cu_ / split);
        return int(std::max<uint64_t>(1, std::min(need, cap)));
    }
    void launch_reduce(Rank& r, const Ptrs& src, uint4* dst, uint64_t cvec) {
        // The n-way sum is the library kernel (libnetop_hip.so: netop_sum_bf16), numerics-tested
        // against PyTorch; here its sources are peer pointers.
        const void* srcs[kMaxRanks];
        for (int s = 0; s < n_; ++s) srcs[s] = src.p[s];
        HIPCHECK(hipError_t(netop_sum_bf16(srcs, n_, dst, cvec * 8, per_cu_, r.stream)));
    }
    void gather_pull(int d, uint64_t chunk, uint64_t cvec) {
        if (n_ == 1) return;
        Rank& r = ranks_[d];
        HIPCHECK(hipSetDevice(r.dev));
        Ptrs src{};
        DstPtrs dst{};
        int k = 0;
        for (int p = 0; p < n_; ++p) {
            if (p == d) continue;
            src.p[k] = reinterpret_cast<const uint4*>(ranks_[p].out + uint64_t(p) * chunk);
            dst.p[k] = reinterpret_cast<uint4*>(r.out + uint64_t(p) * chunk);
            ++k;
        }
        hipLaunchKernelGGL(multi_copy_kernel, dim3(grid(r, cvec, k), k), dim3(kThreads), 0, r.stream, src, dst, cvec);
        HIPCHECK(hipGetLastError());
    }
    void scatter_push(int p, uint64_t chunk, uint64_t cvec) {
        if (n_ == 1) return;
        Rank& r = ranks_[p];
        HIPCHECK(hipSetDevice(r.dev));
        Ptrs src{};
        DstPtrs dst{};
        int k = 0;
        for (int q = 0; q < n_; ++q) {
            if (q == p) continue;
            src.p[k] = reinterpret_cast<const uint4*>(r.in + uint64_t(q) * chunk);
            dst.p[k] = reinterpret_cast<uint4*>(ranks_[q].scratch + uint64_t(p) * chunk);
            ++k;
        }
        hipLaunchKernelGGL(multi_copy_kernel, dim3(grid(r, cvec, k), k), dim3(kThreads), 0, r.stream, src, dst, cvec);
        HIPCHECK(hipGetLastError());
    }
    void gather_push(int q, uint64_t chunk, uint64_t cvec) {
        if (n_ == 1) return;
        Rank& r = ranks_[q];
        HIPCHECK(hipSetDevice(r.dev));
        Ptrs src{};
        DstPtrs dst{};
        int k = 0;
        for (int p = 0; p < n_; ++p) {
            if (p == q) continue;
            src.p[k] = reinterpret_cast<const uint4*>(r.out + uint64_t(q) * chunk);
            dst.p[k] = reinterpret_cast<uint4*>(ranks_[p].out + uint64_t(q) * chunk);
            ++k;
        }
        hipLaunchKernelGGL(multi_copy_kernel, dim3(grid(r, cvec, k), k), dim3(kThreads), 0, r.stream, src, dst, cvec);
        HIPCHECK(hipGetLastError());
    }

    int n_, per_cu_;
    uint64_t bytes_cap_ = 0;
    std::vector<Rank> ranks_;
    std::vector<int> cus_;
};

uint64_t parse_size(const char* s) {
    char* end = nullptr;
    double v = std::strtod(s, &end);
    if (end && (*end == 'K' || *end == 'k')) v *= 1024;
    if (end && (*end == 'M' || *end == 'm')) v *= 1024.0 * 1024;
    if (end && (*end == 'G' || *end == 'g')) v *= 1024.0 * 1024 * 1024;
    return uint64_t(v);
}

}  // namespace

int main(int argc, char** argv) {
    Args a;
    int soak = 0;
    for (int i = 1; i < argc; ++i) {
        std::string k = argv[i];
        auto val = [&]() -> const char* {
            if (i + 1 >= argc) {
                std::fprintf(stderr, "missing value for %s\n", k.c_str());
                std::exit(2);
            }
            return argv[++i];
        };
        if (k == "-b") a.min_bytes = parse_size(val());
        else if (k == "-e") a.max_bytes = parse_size(val());
        else if (k == "-f") a.factor = std::atof(val());
        else if (k == "-n") a.iters = std::atoi(val());
        else if (k == "-w") a.warmup = std::atoi(val());
        else if (k == "--ranks") a.ranks = std::atoi(val());
        else if (k == "--mode") a.mode = val();
        else if (k == "--wg-per-cu") a.per_cu = std::atoi(val());
        else if (k == "--soak") soak = std::atoi(val());
        else {
            std::fprintf(stderr,
                         "usage: netop-xgmi-allreduce [-b min] [-e max] [-f factor] [-n iters] [-w warmup]\n"
                         "         [--ranks N (default: all GPUs, <= 8)] [--mode pull|push|both] [--wg-per-cu K]\n"
                         "         [--soak N (N calls of random sizes up to -e, pull and push in turn, each checked)]\n");
            return k == "-h" || k == "--help" ? 0 : 2;
        }
    }
    if (a.mode != "pull" && a.mode != "push" && a.mode != "both") return 2;
    if (a.factor <= 1 || a.iters < 1 || a.min_bytes > a.max_bytes || a.per_cu < 1 || soak < 0) return 2;
    int ngpu = 0;
    HIPCHECK(hipGetDeviceCount(&ngpu));
    if (ngpu < 1) return 1;
    int n = a.ranks > 0 ? a.ranks : std::min(ngpu, kMaxRanks);
    if (n > kMaxRanks) {
        std::fprintf(stderr, "--ranks %d > %d\n", n, kMaxRanks);
        return 2;
    }
    const int gpus_used = std::min(ngpu, n);
    Node node(n, gpus_used, a.max_bytes + 16ull * n, a.per_cu);
    std::fprintf(stderr, "# netop-xgmi-allreduce: %d rank(s) on %d GPU(s), bf16 sum, two-shot, %d WG/CU\n", n, gpus_used,
                 a.per_cu);
    std::fprintf(stderr, "#%5s %12s %10s %10s %10s %8s\n", "mode", "size(B)", "time(us)", "algbw", "busbw", "#wrong");
    unsigned long long total_wrong = 0;
    if (soak > 0) {
        // Every call on fresh data and checked exactly: random sizes (the same sequence on every
        // run), pull and push in turn, every third call issued again straight after the previous
        // one on the same buffers.  What a timed loop cannot show: a cross-stream event or
        // buffer-reuse race that corrupts one call in thousands.
        uint64_t rng = 0x5eed5eed5eedull;
        auto t0 = std::chrono::steady_clock::now();
        unsigned long long calls[2] = {0, 0}, wrong[2] = {0, 0};
        for (int i = 0; i < soak; ++i) {
            rng ^= rng << 13;
            rng ^= rng >> 7;
            rng ^= rng << 17;
            const bool push = a.mode == "push" || (a.mode == "both" && (i & 1));
            const uint64_t bytes = node.round_bytes(16ull * n + rng % a.max_bytes);
            uint32_t seed = 0x50a10000u + uint32_t(i);
            node.fill(seed, bytes);
            node.allreduce(bytes, push);
            if (i % 3 == 2) {
                seed ^= 0x00ff00ffu;
                node.fill(seed, bytes);
                node.allreduce(bytes, push);
            }
            wrong[push] += node.verify(seed, bytes);
            ++calls[push];
        }
        const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        total_wrong = wrong[0] + wrong[1];
        std::printf("{\"op\":\"xgmi_all_reduce_soak\",\"ranks\":%d,\"gpus\":%d,\"max_bytes\":%llu,\"calls\":{\"pull\":%llu,"
                    "\"push\":%llu},\"wrong\":{\"pull\":%llu,\"push\":%llu},\"seconds\":%.2f}\n",
                    n, gpus_used, (unsigned long long)a.max_bytes, calls[0], calls[1], wrong[0], wrong[1], secs);
        return total_wrong ? 3 : 0;
    }
    std::vector<std::string> modes;
    if (a.mode != "push") modes.push_back("pull");
    if (a.mode != "pull") modes.push_back("push");
    for (const auto& m : modes) {
        const bool push = m == "push";
        for (uint64_t req = a.min_bytes; req <= a.max_bytes;) {
            uint64_t bytes = node.round_bytes(req);
            unsigned long long wrong = 0;
            for (uint32_t round = 0; round < 3; ++round) {  // same buffers, new data each round
                uint32_t seed = 0xa11e0000u + round * 7919u + uint32_t(bytes);
                node.fill(seed, bytes);
                node.allreduce(bytes, push);
                wrong += node.verify(seed, bytes);
            }
            for (int i = 0; i < a.warmup; ++i) node.allreduce(bytes, push);
            node.sync();
            auto t0 = std::chrono::steady_clock::now();
            for (int i = 0; i < a.iters; ++i) node.allreduce(bytes, push);
            node.sync();
            double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / a.iters;
            double algbw = double(bytes) / (us * 1e-6) / 1e9;
            double busbw = algbw * 2.0 * (n - 1) / n;
            total_wrong += wrong;
            std::fprintf(stderr, " %5s %12llu %10.2f %10.2f %10.2f %8llu\n", m.c_str(), (unsigned long long)bytes, us,
                         algbw, busbw, wrong);
            std::printf("{\"op\":\"xgmi_all_reduce\",\"mode\":\"%s\",\"bytes\":%llu,\"ranks\":%d,\"gpus\":%d,"
                        "\"time_us\":%.3f,\"algbw_GBps\":%.4f,\"busbw_GBps\":%.4f,\"wrong\":%llu}\n",
                        m.c_str(), (unsigned long long)bytes, n, gpus_used, us, algbw, busbw, wrong);
            std::fflush(stdout);
            uint64_t next = uint64_t(double(req) * a.factor);
            req = next > req ? next : req + 1;
        }
    }
    return total_wrong ? 3 : 0;
}

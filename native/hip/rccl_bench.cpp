// `netop-rccl-bench` — native RCCL collective bandwidth harness for MI355X nodes.
//
// The reference enables the collective library only through a file contract (gaudinet.json,
// reference cmd/discover/gaudinet.go:28-89) and never measures it.  This
// is the MI355X side's proof that the configured fabric carries collectives: rccl-tests
// semantics (sizes swept by a factor, out-of-place or in-place, algbw = bytes / time,
// busbw = algbw x the per-collective bus factor) with a byte-exact bf16 check of every
// result using the pattern kernels of libnetop_hip.so.
//
// Two launch shapes:
//   * single process, every local GPU:  netop-rccl-bench -g 8           (ncclCommInitAll)
//   * one process per GPU (torchrun, a Job per node, ...):
//       netop-rccl-bench --nranks N --rank R --device D --id-file /shared/path
//     rank 0 writes the ncclUniqueId to --id-file (atomic rename), the others poll it.
//     RANK / WORLD_SIZE / LOCAL_RANK from the environment are used when the flags are absent.
//
// --graph captures the timed iterations of each size into one HIP graph per GPU and replays
// it, removing host launch cost from small-message latency.
//
// Output: an rccl-tests-style table on stderr, one JSON object per size on stdout (rank 0).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

extern "C" {
int netop_fill_pattern_at(void* buf, uint64_t n_elems, uint32_t seed, int rank_lo, int n_ranks, uint64_t elem_offset,
                          hipStream_t stream);
int netop_verify_pattern_at(const void* buf, uint64_t n_elems, uint32_t seed, int rank_lo, int n_ranks,
                            uint64_t elem_offset, unsigned long long* errors, hipStream_t stream);
}

namespace {

#define HIPCHECK(x)                                                                                    \
    do {                                                                                               \
        hipError_t e_ = (x);                                                                           \
        if (e_ != hipSuccess) {                                                                        \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));     \
            std::exit(1);                                                                              \
        }                                                                                              \
    } while (0)
#define NCCLCHECK(x)                                                                                   \
    do {                                                                                               \
        ncclResult_t r_ = (x);                                                                         \
        if (r_ != ncclSuccess) {                                                                       \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, ncclGetErrorString(r_));    \
            std::exit(1);                                                                              \
        }                                                                                              \
    } while (0)

enum class Op { AllReduce, AllGather, ReduceScatter, Broadcast, AllToAll };

struct OpInfo {
    const char* name;
    Op op;
};
constexpr OpInfo kOps[] = {{"all_reduce", Op::AllReduce},
                           {"all_gather", Op::AllGather},
                           {"reduce_scatter", Op::ReduceScatter},
                           {"broadcast", Op::Broadcast},
                           {"alltoall", Op::AllToAll}};

// rccl-tests (src/*.cu, PERFORMANCE.md) bus-bandwidth factors: the fraction of the data every
// rank must move over its slowest link.
double bus_factor(Op op, int n) {
    switch (op) {
        case Op::AllReduce: return 2.0 * (n - 1) / n;
        case Op::AllGather:
        case Op::ReduceScatter:
        case Op::AllToAll: return double(n - 1) / n;
        case Op::Broadcast: return 1.0;
    }
    return 1.0;
}

uint64_t parse_size(const char* s) {
    char* end = nullptr;
    double v = std::strtod(s, &end);
    switch (end && *end ? *end : 0) {
        case 'K': case 'k': v *= 1024; break;
        case 'M': case 'm': v *= 1024.0 * 1024; break;
        case 'G': case 'g': v *= 1024.0 * 1024 * 1024; break;
        default: break;
    }
    return uint64_t(v);
}

struct Args {
    uint64_t min_bytes = 8, max_bytes = 128ull << 20;
    double factor = 2;
    int iters = 20, warmup = 5, ngpus = 1, check = 1, inplace = 0, graph = 0, root = 0;
    int nranks = -1, rank = -1, device = -1;
    Op op = Op::AllReduce;
    const char* op_name = "all_reduce";
    std::string id_file, dtype = "bf16";
};

void usage() {
    std::fprintf(stderr,
                 "usage: netop-rccl-bench [-b minbytes] [-e maxbytes] [-f factor] [-n iters] [-w warmup]\n"
                 "         [-g gpus] [-o all_reduce|all_gather|reduce_scatter|broadcast|alltoall]\n"
                 "         [-d bf16|float] [-c 0|1] [--inplace] [--graph] [--root R]\n"
                 "         [--nranks N --rank R --device D --id-file PATH]\n");
}

bool parse(int argc, char** argv, Args& a) {
    for (int i = 1; i < argc; ++i) {
        std::string k = argv[i];
        auto val = [&](const char* name) -> const char* {
            if (i + 1 >= argc) {
                std::fprintf(stderr, "missing value for %s\n", name);
                std::exit(2);
            }
            return argv[++i];
        };
        if (k == "-b" || k == "--minbytes") a.min_bytes = parse_size(val("-b"));
        else if (k == "-e" || k == "--maxbytes") a.max_bytes = parse_size(val("-e"));
        else if (k == "-f" || k == "--stepfactor") a.factor = std::atof(val("-f"));
        else if (k == "-n" || k == "--iters") a.iters = std::atoi(val("-n"));
        else if (k == "-w" || k == "--warmup_iters") a.warmup = std::atoi(val("-w"));
        else if (k == "-g" || k == "--ngpus") a.ngpus = std::atoi(val("-g"));
        else if (k == "-c" || k == "--check") a.check = std::atoi(val("-c"));
        else if (k == "-d" || k == "--datatype") a.dtype = val("-d");
        else if (k == "--inplace") a.inplace = 1;
        else if (k == "--graph") a.graph = 1;
        else if (k == "--root") a.root = std::atoi(val("--root"));
        else if (k == "--nranks") a.nranks = std::atoi(val("--nranks"));
        else if (k == "--rank") a.rank = std::atoi(val("--rank"));
        else if (k == "--device") a.device = std::atoi(val("--device"));
        else if (k == "--id-file") a.id_file = val("--id-file");
        else if (k == "-o" || k == "--op") {
            std::string o = val("-o");
            bool ok = false;
            for (const auto& oi : kOps)
                if (o == oi.name) a.op = oi.op, a.op_name = oi.name, ok = true;
            if (!ok) return false;
        } else if (k == "-h" || k == "--help") {
            usage();
            std::exit(0);
        } else {
            std::fprintf(stderr, "unknown argument %s\n", k.c_str());
            return false;
        }
    }
    if (a.dtype != "bf16" && a.dtype != "float") return false;
    if (a.factor <= 1.0 || a.iters < 1 || a.warmup < 0 || a.min_bytes > a.max_bytes || a.ngpus < 1) return false;
    return true;
}

// One rank of the communicator living in this process.
struct Rank {
    int dev = 0, rank = 0;
    ncclComm_t comm = nullptr;
    hipStream_t stream = nullptr;
    void* send = nullptr;
    void* recv = nullptr;
    unsigned long long* err = nullptr;
    hipGraphExec_t graph = nullptr;
};

void write_id_file(const std::string& path, const ncclUniqueId& id) {
    std::string tmp = path + ".tmp." + std::to_string(getpid());
    {
        std::ofstream f(tmp, std::ios::binary | std::ios::trunc);
        f.write(id.internal, sizeof id.internal);
        if (!f) {
            std::fprintf(stderr, "cannot write %s\n", tmp.c_str());
            std::exit(1);
        }
    }
    if (std::rename(tmp.c_str(), path.c_str()) != 0) {
        std::perror("rename id file");
        std::exit(1);
    }
}

ncclUniqueId read_id_file(const std::string& path, int timeout_s) {
    ncclUniqueId id;
    auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(timeout_s);
    while (std::chrono::steady_clock::now() < deadline) {
        std::ifstream f(path, std::ios::binary);
        if (f && f.read(id.internal, sizeof id.internal) && f.gcount() == sizeof id.internal) return id;
        std::this_thread::sleep_for(std::chrono::milliseconds(20));
    }
    std::fprintf(stderr, "timed out waiting for %s\n", path.c_str());
    std::exit(1);
}

int env_int(const char* k, int dflt) {
    const char* v = std::getenv(k);
    return v && *v ? std::atoi(v) : dflt;
}

// Element counts per rank: `count` is the per-rank send count for all_gather and the
// per-rank receive count for reduce_scatter (rccl-tests convention: the reported size is
// the larger, full buffer).
struct Shape {
    uint64_t send_elems, recv_elems, report_bytes, count;
};

Shape shape_for(Op op, uint64_t bytes, int n, size_t esize) {
    // Every per-rank chunk must be a multiple of 8 elements (16-B vectors of bf16).
    uint64_t elems = std::max<uint64_t>(bytes / esize, 1);
    uint64_t chunk_align = 8ull * ((op == Op::AllReduce || op == Op::Broadcast) ? 1 : n);
    elems = (elems + chunk_align - 1) / chunk_align * chunk_align;
    Shape s{};
    switch (op) {
        case Op::AllReduce:
        case Op::Broadcast: s = {elems, elems, elems * esize, elems}; break;
        case Op::AllGather: s = {elems / n, elems, elems * esize, elems / n}; break;
        case Op::ReduceScatter: s = {elems, elems / n, elems * esize, elems / n}; break;
        case Op::AllToAll: s = {elems, elems, elems * esize, elems / n}; break;
    }
    return s;
}

void launch(const Args& a, Op op, Rank& r, const Shape& s, ncclDataType_t dt) {
    const void* sb = a.inplace ? r.recv : r.send;
    // In-place layouts follow the NCCL rules: all_gather sends from its own chunk of the output,
    // reduce_scatter receives into its own chunk of the input.
    size_t es = dt == ncclBfloat16 ? 2 : 4;
    switch (op) {
        case Op::AllReduce: NCCLCHECK(ncclAllReduce(sb, r.recv, s.count, dt, ncclSum, r.comm, r.stream)); break;
        case Op::Broadcast: NCCLCHECK(ncclBroadcast(sb, r.recv, s.count, dt, a.root, r.comm, r.stream)); break;
        case Op::AllGather:
            if (a.inplace) sb = static_cast<char*>(r.recv) + size_t(r.rank) * s.count * es;
            NCCLCHECK(ncclAllGather(sb, r.recv, s.count, dt, r.comm, r.stream));
            break;
        case Op::ReduceScatter: {
            void* rb = a.inplace ? static_cast<char*>(r.send) + size_t(r.rank) * s.count * es : r.recv;
            NCCLCHECK(ncclReduceScatter(r.send, rb, s.count, dt, ncclSum, r.comm, r.stream));
            break;
        }
        case Op::AllToAll: NCCLCHECK(ncclAllToAll(a.inplace ? r.recv : r.send, r.recv, s.count, dt, r.comm, r.stream)); break;
    }
}

// Fill inputs with the rank's pattern.  For in-place ops the input lives in the buffer the
// op reads from (recv for all_reduce/broadcast/all_gather/alltoall, send for reduce_scatter).
void fill_inputs(const Args& a, Op op, Rank& r, const Shape& s, int n) {
    uint32_t seed = 0x5eed0000u + uint32_t(s.count);
    HIPCHECK(hipSetDevice(r.dev));
    auto fill = [&](void* p, uint64_t elems, uint64_t off) {
        HIPCHECK(hipError_t(netop_fill_pattern_at(p, elems, seed, r.rank, 1, off, r.stream)));
    };
    switch (op) {
        case Op::AllReduce:
        case Op::Broadcast:
        case Op::AllToAll: fill(a.inplace ? r.recv : r.send, s.send_elems, 0); break;
        case Op::AllGather:
            fill(a.inplace ? static_cast<char*>(r.recv) + size_t(r.rank) * s.count * 2 : r.send, s.send_elems, 0);
            break;
        case Op::ReduceScatter: fill(r.send, s.send_elems, 0); break;
    }
}

// Count mismatching elements of this rank's output.
void verify_outputs(const Args& a, Op op, Rank& r, const Shape& s, int n) {
    uint32_t seed = 0x5eed0000u + uint32_t(s.count);
    auto check = [&](const void* p, uint64_t elems, int lo, int cnt, uint64_t off) {
        HIPCHECK(hipError_t(netop_verify_pattern_at(p, elems, seed, lo, cnt, off, r.err, r.stream)));
    };
    const char* out = static_cast<const char*>(r.recv);
    switch (op) {
        case Op::AllReduce: check(out, s.recv_elems, 0, n, 0); break;
        case Op::Broadcast: check(out, s.recv_elems, a.root, 1, 0); break;
        case Op::AllGather:
            for (int k = 0; k < n; ++k) check(out + size_t(k) * s.count * 2, s.count, k, 1, 0);
            break;
        case Op::ReduceScatter:
            check(a.inplace ? static_cast<const char*>(r.send) + size_t(r.rank) * s.count * 2 : out, s.count, 0, n,
                  uint64_t(r.rank) * s.count);
            break;
        case Op::AllToAll:
            // Chunk k of my output is chunk `rank` of rank k's input.
            for (int k = 0; k < n; ++k) check(out + size_t(k) * s.count * 2, s.count, k, 1, uint64_t(r.rank) * s.count);
            break;
    }
}

void group_launch(const Args& a, std::vector<Rank>& ranks, const Shape& s, ncclDataType_t dt) {
    if (ranks.size() > 1) NCCLCHECK(ncclGroupStart());
    for (auto& r : ranks) {
        HIPCHECK(hipSetDevice(r.dev));
        launch(a, a.op, r, s, dt);
    }
    if (ranks.size() > 1) NCCLCHECK(ncclGroupEnd());
}

void sync_all(std::vector<Rank>& ranks) {
    for (auto& r : ranks) {
        HIPCHECK(hipSetDevice(r.dev));
        HIPCHECK(hipStreamSynchronize(r.stream));
    }
}

}  // namespace

int main(int argc, char** argv) {
    Args a;
    if (!parse(argc, argv, a)) {
        usage();
        return 2;
    }
    if (a.nranks < 0) a.nranks = env_int("WORLD_SIZE", -1);
    if (a.rank < 0) a.rank = env_int("RANK", -1);
    if (a.device < 0) a.device = env_int("LOCAL_RANK", 0);
    const bool multi_proc = a.nranks > 0 && a.rank >= 0 && !a.id_file.empty();
    const ncclDataType_t dt = a.dtype == "bf16" ? ncclBfloat16 : ncclFloat32;
    const size_t esize = a.dtype == "bf16" ? 2 : 4;
    if (a.check && dt != ncclBfloat16) a.check = 0;  // exact-pattern check is defined for bf16

    int ndev = 0;
    HIPCHECK(hipGetDeviceCount(&ndev));
    std::vector<Rank> ranks;
    int world = 0, my_first_rank = 0;
    if (multi_proc) {
        if (a.device >= ndev) {
            std::fprintf(stderr, "device %d not present (%d visible)\n", a.device, ndev);
            return 1;
        }
        world = a.nranks;
        my_first_rank = a.rank;
        ncclUniqueId id;
        if (a.rank == 0) {
            NCCLCHECK(ncclGetUniqueId(&id));
            write_id_file(a.id_file, id);
        } else {
            id = read_id_file(a.id_file, 120);
        }
        Rank r;
        r.dev = a.device;
        r.rank = a.rank;
        HIPCHECK(hipSetDevice(r.dev));
        NCCLCHECK(ncclCommInitRank(&r.comm, world, id, a.rank));
        ranks.push_back(r);
    } else {
        if (a.ngpus > ndev) {
            std::fprintf(stderr, "-g %d: only %d GPUs visible\n", a.ngpus, ndev);
            return 1;
        }
        world = a.ngpus;
        std::vector<ncclComm_t> comms(world);
        std::vector<int> devs(world);
        for (int i = 0; i < world; ++i) devs[i] = i;
        NCCLCHECK(ncclCommInitAll(comms.data(), world, devs.data()));
        for (int i = 0; i < world; ++i) {
            Rank r;
            r.dev = i;
            r.rank = i;
            r.comm = comms[i];
            ranks.push_back(r);
        }
    }
    if (a.root < 0 || a.root >= world) {
        std::fprintf(stderr, "--root %d outside [0,%d)\n", a.root, world);
        return 2;
    }

    // Buffers sized for the largest message (+ chunk rounding), allocated once.
    Shape big = shape_for(a.op, a.max_bytes, world, esize);
    const size_t buf_bytes = std::max(big.send_elems, big.recv_elems) * esize + 256;
    for (auto& r : ranks) {
        HIPCHECK(hipSetDevice(r.dev));
        HIPCHECK(hipStreamCreateWithFlags(&r.stream, hipStreamNonBlocking));
        HIPCHECK(hipMalloc(&r.send, buf_bytes));
        HIPCHECK(hipMalloc(&r.recv, buf_bytes));
        HIPCHECK(hipMalloc(&r.err, sizeof(unsigned long long)));
        HIPCHECK(hipMemset(r.send, 0, buf_bytes));
        HIPCHECK(hipMemset(r.recv, 0, buf_bytes));
    }
    const bool print = my_first_rank == 0;
    int nccl_version = 0;
    ncclGetVersion(&nccl_version);
    if (print) {
        std::fprintf(stderr, "# netop-rccl-bench: op %s, dtype %s, %d rank(s)%s, RCCL %d, %s%s\n", a.op_name,
                     a.dtype.c_str(), world, multi_proc ? " (one process per GPU)" : " (single process)", nccl_version,
                     a.inplace ? "in-place" : "out-of-place", a.graph ? ", hipGraph" : "");
        std::fprintf(stderr, "#%12s %12s %10s %10s %10s %8s\n", "size(B)", "count", "time(us)", "algbw", "busbw", "#wrong");
    }

    double peak_busbw = 0;
    uint64_t total_wrong = 0;
    for (uint64_t bytes = a.min_bytes; bytes <= a.max_bytes;) {
        Shape s = shape_for(a.op, bytes, world, esize);
        // Correctness pass first (fresh inputs, one op, verify), then the timed loop.
        unsigned long long wrong = 0;
        if (a.check) {
            for (auto& r : ranks) {
                HIPCHECK(hipSetDevice(r.dev));
                HIPCHECK(hipMemsetAsync(r.err, 0, sizeof(unsigned long long), r.stream));
                fill_inputs(a, a.op, r, s, world);
            }
            group_launch(a, ranks, s, dt);
            for (auto& r : ranks) {
                HIPCHECK(hipSetDevice(r.dev));
                verify_outputs(a, a.op, r, s, world);
                unsigned long long h = 0;
                HIPCHECK(hipMemcpyAsync(&h, r.err, sizeof h, hipMemcpyDeviceToHost, r.stream));
                HIPCHECK(hipStreamSynchronize(r.stream));
                wrong += h;
            }
        }
        for (int i = 0; i < a.warmup; ++i) group_launch(a, ranks, s, dt);
        sync_all(ranks);

        double us;
        if (a.graph) {
            // One graph per GPU holding all timed iterations, captured from the same group calls.
            for (auto& r : ranks) {
                HIPCHECK(hipSetDevice(r.dev));
                HIPCHECK(hipStreamBeginCapture(r.stream, hipStreamCaptureModeGlobal));
            }
            for (int i = 0; i < a.iters; ++i) group_launch(a, ranks, s, dt);
            for (auto& r : ranks) {
                HIPCHECK(hipSetDevice(r.dev));
                hipGraph_t g;
                HIPCHECK(hipStreamEndCapture(r.stream, &g));
                HIPCHECK(hipGraphInstantiate(&r.graph, g, nullptr, nullptr, 0));
                HIPCHECK(hipGraphDestroy(g));
                HIPCHECK(hipGraphLaunch(r.graph, r.stream));  // graph warm-up
            }
            sync_all(ranks);
            auto t0 = std::chrono::steady_clock::now();
            for (auto& r : ranks) {
                HIPCHECK(hipSetDevice(r.dev));
                HIPCHECK(hipGraphLaunch(r.graph, r.stream));
            }
            sync_all(ranks);
            us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / a.iters;
            for (auto& r : ranks) {
                HIPCHECK(hipSetDevice(r.dev));
                HIPCHECK(hipGraphExecDestroy(r.graph));
                r.graph = nullptr;
            }
        } else {
            auto t0 = std::chrono::steady_clock::now();
            for (int i = 0; i < a.iters; ++i) group_launch(a, ranks, s, dt);
            sync_all(ranks);
            us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / a.iters;
        }
        double algbw = us > 0 ? double(s.report_bytes) / (us * 1e-6) / 1e9 : 0;
        double busbw = algbw * bus_factor(a.op, world);
        peak_busbw = std::max(peak_busbw, busbw);
        total_wrong += wrong;
        if (print) {
            std::fprintf(stderr, " %12llu %12llu %10.2f %10.2f %10.2f %8llu\n", (unsigned long long)s.report_bytes,
                         (unsigned long long)s.count, us, algbw, busbw, wrong);
            std::printf(
                "{\"op\":\"%s\",\"bytes\":%llu,\"count\":%llu,\"dtype\":\"%s\",\"ranks\":%d,\"time_us\":%.3f,"
                "\"algbw_GBps\":%.4f,\"busbw_GBps\":%.4f,\"wrong\":%llu,\"checked\":%s,\"inplace\":%s,\"graph\":%s}\n",
                a.op_name, (unsigned long long)s.report_bytes, (unsigned long long)s.count, a.dtype.c_str(), world, us,
                algbw, busbw, wrong, a.check ? "true" : "false", a.inplace ? "true" : "false",
                a.graph ? "true" : "false");
            std::fflush(stdout);
        }
        uint64_t next = uint64_t(double(bytes) * a.factor);
        bytes = next > bytes ? next : bytes + 1;
    }
    if (print) std::fprintf(stderr, "# peak busbw %.2f GB/s, out of bounds values: %llu\n", peak_busbw, (unsigned long long)total_wrong);
    for (auto& r : ranks) {
        HIPCHECK(hipSetDevice(r.dev));
        NCCLCHECK(ncclCommDestroy(r.comm));
        HIPCHECK(hipFree(r.send));
        HIPCHECK(hipFree(r.recv));
        HIPCHECK(hipFree(r.err));
        HIPCHECK(hipStreamDestroy(r.stream));
    }
    return total_wrong ? 3 : 0;
}

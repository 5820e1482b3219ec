// MI355X validation kernels for the network operator (gfx950, wave64).
//
// The operator's job ends at "RCCL sees every link".  These kernels are what the node
// tooling and the bench use to *prove* it on the GPU side:
//
//   * netop_fill_pattern / netop_verify_sum — bf16 all-reduce correctness check.  Each rank
//     fills a deterministic small-integer pattern (exact in bf16 for any reduction order);
//     the verifier recomputes Σ_ranks pattern and counts mismatches.  16-byte vector
//     accesses (8 x bf16 per lane), one contiguous chunk per workgroup, one atomic per
//     workgroup.
//   * netop_copy — 16-B/lane streaming copy used by the xGMI link probe: with peer access
//     enabled the loads of a peer pointer travel over the xGMI link to that peer, so one
//     copy per peer on its own stream drives all 7 links of an MI355X concurrently.
//   * netop_sum_bf16 — n-way bf16 sum with fp32 accumulation (the reduce-scatter step of the
//     direct xGMI all-reduce, sources are peer pointers there).
//
// No CUDA/hipify heritage: plain HIP for gfx950, 256-thread workgroups (4 waves), grids
// sized as a multiple of the 256 CUs.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

namespace {

constexpr int kThreads = 256;

// Pattern of (element, rank): integers in [-4, 3] -> exact in bf16, sums of up to 64 ranks
// stay exact (|sum| <= 256 = 2^8).  Per 16-byte vector (group g of 8 elements; every buffer and
// offset is a multiple of 8 elements) one rank-independent hash h(g); rank r's word is h(g) * m_r
// with m_r = m_0 + r d (m_0 odd, d twice an odd number: every m_r odd; both from the seed), and
// element e of the group is its 3-bit field at bit 5 + 3 e, minus 4.  Summing over ranks works on
// the fields in place (SWAR): the even and the odd fields of every rank are added as 6-bit slots
// of two words (bits 5-28 and 8-31; 9 ranks fit a slot), and rank r + 1's word is rank r's plus
// h d, so a rank costs one add and two and-adds -- no multiply, no shift, no per-element work.
// pattern_tune.hip measured the steps on MI355X: a hash and eight extractions per rank ("v1") ->
// one multiply per rank ("v2", profiles/r4_pattern_tune_v1_v2.jsonl: 8-rank fill 2.5 -> 4.3 TB/s,
// verify 2.4 -> 5.2) -> one add per rank (this, "v4", profiles/r4_pattern_tune_v4.jsonl: 8-rank
// verify 4.95 -> 5.86 TB/s, 16 ranks fill 3.1 -> 4.6 and verify 3.1 -> 4.0).
// PyTorch reference: network_operator_amd/parallel/collectives.py:pattern_reference.
__device__ __forceinline__ uint32_t group_hash(uint64_t g) {
    uint32_t x = uint32_t(g) * 0x9E3779B1u ^ uint32_t(g >> 32) * 0x85EBCA77u;
    x ^= x >> 15;
    x *= 0x2C1B3C6Du;
    x ^= x >> 12;
    return x;
}

__device__ __forceinline__ uint32_t base_mult(uint32_t seed) {  // m_0
    const uint32_t k = (seed + 0x632BE5ABu) * 0xC2B2AE3Du;
    return (k ^ (k >> 16)) | 1u;
}

__device__ __forceinline__ uint32_t step_mult(uint32_t seed) {  // d
    const uint32_t k = (seed ^ 0x27D4EB2Fu) * 0x165667B1u;
    return ((k ^ (k >> 15)) << 1) | 2u;
}

constexpr uint32_t kEvenSlots = (7u << 5) | (7u << 11) | (7u << 17) | (7u << 23);  // fields 0, 2, 4, 6
constexpr uint32_t kOddSlots = kEvenSlots << 3;                                     // fields 1, 3, 5, 7

__device__ __forceinline__ uint16_t int_to_bf16(int v) {
    // Small integers are exact; convert through f32 bits (truncation is exact here).
    float f = float(v);
    return uint16_t(__float_as_uint(f) >> 16);
}

__device__ __forceinline__ float bf16_to_float(uint16_t h) { return __uint_as_float(uint32_t(h) << 16); }

// s[k] = Σ_{r in [rank_lo, rank_lo + n_ranks)} pattern(8 g + k, r): one rank's data (n_ranks =
// 1) or the reduction over a contiguous rank range (all-reduce / reduce-scatter expectation).
__device__ __forceinline__ void group_sum(uint64_t g, uint32_t seed, int rank_lo, int n_ranks, int s[8]) {
    const uint32_t h = group_hash(g);
    const uint32_t d = step_mult(seed);
    const uint32_t dx = h * d;
    uint32_t x = h * (base_mult(seed) + uint32_t(rank_lo) * d);  // rank rank_lo's word
#pragma unroll
    for (int k = 0; k < 8; ++k) s[k] = -4 * n_ranks;
    for (int r0 = 0; r0 < n_ranks; r0 += 9) {  // 9 x 7 = 63 fits a 6-bit slot
        uint32_t even = 0, odd = 0;
        const int r1 = r0 + 9 < n_ranks ? r0 + 9 : n_ranks;
        for (int r = r0; r < r1; ++r) {
            even += x & kEvenSlots;
            odd += x & kOddSlots;
            x += dx;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            s[2 * k] += int((even >> (5 + 6 * k)) & 63u);
            s[2 * k + 1] += int((odd >> (8 + 6 * k)) & 63u);
        }
    }
}

// The vectors of one workgroup: one contiguous chunk of the buffer (a multiple of the workgroup
// size), the workgroup's lanes striding through it together.  pattern_tune.hip ("chunk" mode,
// profiles/r4_pattern_tune_chunk.jsonl): against a grid-stride walk over the whole buffer the
// HBM writes of the fill run 4.6 -> 5.6 TB/s (1 GiB, 16 workgroups per CU), the one-rank verify
// 6.1 -> 6.5 TB/s; the copy kernel below stays grid-strided (there the chunked walk was slower).
// In the library (profiles/r4_pattern_kernels_chunk.json, rocprofv3): 1 GiB fill 4.44 -> 5.34
// TB/s at one rank and 4.54 -> 4.89 at eight, one-rank verify 5.78 -> 6.23; the eight-rank
// verify is ALU-bound and reads the same with either walk (4.6-4.85 TB/s from box to box).
struct ChunkWalk {
    uint64_t first, end;
    __device__ explicit ChunkWalk(uint64_t n_vec) {
        const uint64_t per = ((n_vec + gridDim.x - 1) / gridDim.x + kThreads - 1) / kThreads * kThreads;
        const uint64_t b = uint64_t(blockIdx.x) * per;
        first = b + threadIdx.x;
        end = b + per < n_vec ? b + per : n_vec;
    }
};

// Element e of the buffer holds the pattern sum of element e + elem_offset: the offset lets a
// chunk of a collective's output be checked against the slice of the global pattern it came
// from.  elem_offset is a multiple of 8, so vector v is group (elem_offset / 8 + v).
__global__ __launch_bounds__(kThreads) void fill_kernel(uint4* __restrict__ out, uint64_t n_vec, uint32_t seed, int rank_lo,
                                                        int n_ranks, uint64_t elem_offset) {
    const ChunkWalk walk(n_vec);
    const uint64_t g0 = elem_offset >> 3;
    u32x4* __restrict__ vout = reinterpret_cast<u32x4*>(out);
    for (uint64_t v = walk.first; v < walk.end; v += kThreads) {
        int s[8];
        group_sum(g0 + v, seed, rank_lo, n_ranks, s);
        u32x4 w;
        w.x = uint32_t(int_to_bf16(s[0])) | (uint32_t(int_to_bf16(s[1])) << 16);
        w.y = uint32_t(int_to_bf16(s[2])) | (uint32_t(int_to_bf16(s[3])) << 16);
        w.z = uint32_t(int_to_bf16(s[4])) | (uint32_t(int_to_bf16(s[5])) << 16);
        w.w = uint32_t(int_to_bf16(s[6])) | (uint32_t(int_to_bf16(s[7])) << 16);
        __builtin_nontemporal_store(w, &vout[v]);  // streamed once; read back by another kernel
    }
}

__global__ __launch_bounds__(kThreads) void verify_kernel(const uint4* __restrict__ in, uint64_t n_vec, uint32_t seed,
                                                          int rank_lo, int n_ranks, uint64_t elem_offset,
                                                          unsigned long long* __restrict__ errors) {
    __shared__ unsigned int wave_err[kThreads / 64];
    const ChunkWalk walk(n_vec);
    const uint64_t g0 = elem_offset >> 3;
    unsigned int err = 0;
    const u32x4* __restrict__ vin = reinterpret_cast<const u32x4*>(in);
    for (uint64_t v = walk.first; v < walk.end; v += kThreads) {
        // Read once: nontemporal (pattern_tune.hip: 5.6 -> 6.1 TB/s at one rank).
        const u32x4 q = __builtin_nontemporal_load(&vin[v]);
        uint32_t w[4] = {q.x, q.y, q.z, q.w};
        int s[8];
        group_sum(g0 + v, seed, rank_lo, n_ranks, s);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            err += bf16_to_float(uint16_t(w[k] & 0xffff)) != float(s[2 * k]);
            err += bf16_to_float(uint16_t(w[k] >> 16)) != float(s[2 * k + 1]);
        }
    }
    // wave64 reduction, then one atomic per workgroup.
    for (int off = 32; off > 0; off >>= 1) err += __shfl_down(err, off, 64);
    if ((threadIdx.x & 63) == 0) wave_err[threadIdx.x >> 6] = err;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned int s = 0;
        for (int i = 0; i < kThreads / 64; ++i) s += wave_err[i];
        if (s) atomicAdd(errors, (unsigned long long)s);
    }
}

__global__ __launch_bounds__(kThreads) void copy_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                        uint64_t n_vec) {
    // One 16-B load per lane per iteration with 4 workgroups per CU: the best of the
    // unroll {1,2,4,8} x workgroups/CU {4,8,16,32} x {regular, nontemporal store} sweep on
    // MI355X HBM (2.86 TB/s copy = 5.7 TB/s of traffic, profiles/r1_copy_tune.jsonl).  Round 6
    // added nontemporal loads to the sweep: with nontemporal loads and stores 3.08 TB/s
    // (profiles/r6_copy_tune.jsonl).  Every byte is moved once.
    const u32x4* __restrict__ s = reinterpret_cast<const u32x4*>(src);
    u32x4* __restrict__ d = reinterpret_cast<u32x4*>(dst);
    const uint64_t stride = uint64_t(gridDim.x) * kThreads;
    for (uint64_t v = uint64_t(blockIdx.x) * kThreads + threadIdx.x; v < n_vec; v += stride)
        __builtin_nontemporal_store(__builtin_nontemporal_load(&s[v]), &d[v]);
}

// ---- n-way bf16 sum (reduce-scatter step of the direct xGMI all-reduce) ----------------------
constexpr int kMaxSrc = 8;
struct SrcPtrs {
    const uint4* p[kMaxSrc];
};

__device__ __forceinline__ void add_bf16x8(float (&acc)[8], const uint4& v) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        acc[2 * k] += __uint_as_float(w[k] << 16);
        acc[2 * k + 1] += __uint_as_float(w[k] & 0xffff0000u);
    }
}

__device__ __forceinline__ uint32_t pack_bf16x2_rne(float a, float b) {
    uint32_t ua = __float_as_uint(a), ub = __float_as_uint(b);
    // NaN stays NaN (quiet), everything else rounds to nearest even.
    ua = (ua & 0x7fffffffu) > 0x7f800000u ? (ua | 0x00400000u) : ua + 0x7fffu + ((ua >> 16) & 1u);
    ub = (ub & 0x7fffffffu) > 0x7f800000u ? (ub | 0x00400000u) : ub + 0x7fffu + ((ub >> 16) & 1u);
    return (ua >> 16) | (ub & 0xffff0000u);
}

// dst[i] = Σ_s src[s][i] in fp32 (s = 0..NSRC-1, in order), bf16 RNE out.  All NSRC x UNROLL
// 16-B loads of a lane are issued before the adds: with peer pointers those are remote xGMI
// reads, and having many in flight per lane is what hides the link round trip.  The sources are
// read once: nontemporal loads.  Shape from sum_tune.hip on the box (local HBM, 256 MiB per
// buffer, profiles/r6_sum_tune.jsonl): nontemporal loads, UNROLL 2 up to 4 sources and 1 above
// (8 loads in flight per lane already), 2 workgroups per CU: (n + 1) x buffer bytes at 6.45 / 6.12
// / 5.88 TB/s for 2 / 4 / 8 sources, against 5.24 / 4.86 / 4.83 with regular loads, UNROLL 2 and
// 4 workgroups per CU; every variant bit-identical.
template <int NSRC, int UNROLL>
__global__ __launch_bounds__(kThreads) void sum_bf16_kernel(SrcPtrs src, uint4* __restrict__ dst, uint64_t n_vec) {
    const uint64_t stride = uint64_t(gridDim.x) * kThreads * UNROLL;
    for (uint64_t base = uint64_t(blockIdx.x) * kThreads * UNROLL + threadIdx.x; base < n_vec; base += stride) {
        uint4 v[UNROLL][NSRC];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const uint64_t i = base + uint64_t(u) * kThreads;
            if (i < n_vec) {
#pragma unroll
                for (int s = 0; s < NSRC; ++s) {
                    const u32x4 q = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src.p[s]) + i);
                    v[u][s] = make_uint4(q.x, q.y, q.z, q.w);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const uint64_t i = base + uint64_t(u) * kThreads;
            if (i >= n_vec) continue;
            float acc[8] = {};
#pragma unroll
            for (int s = 0; s < NSRC; ++s) add_bf16x8(acc, v[u][s]);
            dst[i] = make_uint4(pack_bf16x2_rne(acc[0], acc[1]), pack_bf16x2_rne(acc[2], acc[3]),
                                pack_bf16x2_rne(acc[4], acc[5]), pack_bf16x2_rne(acc[6], acc[7]));
        }
    }
}

using SumFn = void (*)(SrcPtrs, uint4*, uint64_t);
constexpr int sum_unroll(int n) { return n <= 4 ? 2 : 1; }
template <int N>
SumFn sum_for() {
    return sum_bf16_kernel<N, sum_unroll(N)>;
}
SumFn sum_fn(int n) {
    switch (n) {
        case 1: return sum_for<1>();
        case 2: return sum_for<2>();
        case 3: return sum_for<3>();
        case 4: return sum_for<4>();
        case 5: return sum_for<5>();
        case 6: return sum_for<6>();
        case 7: return sum_for<7>();
        default: return sum_for<8>();
    }
}

int grid_for(uint64_t n_vec, int per_cu = 8) {
    // CU count per device, cached: hipGetDeviceProperties is far too slow for a launch path.
    static int cached[64] = {};
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < 64) {
        if (!cached[dev]) {
            int c = 0;
            if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && c > 0) cached[dev] = c;
        }
        if (cached[dev]) cus = cached[dev];
    }
    uint64_t need = (n_vec + kThreads - 1) / kThreads;
    uint64_t cap = uint64_t(cus) * per_cu;
    return int(need < cap ? (need ? need : 1) : cap);
}

// The probes walk every GPU with hipSetDevice; the caller (a torch.distributed rank) must get
// its own current device back on every return path, or its next collective runs elsewhere.
struct DeviceRestore {
    int prev = -1;
    DeviceRestore() {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    }
    ~DeviceRestore() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

}  // namespace

extern "C" {

// All functions return a hipError_t value (0 = success).  Sizes are in bf16 elements and
// must be multiples of 8 (16-byte vectors); pointers must be 16-byte aligned.

int netop_hip_version() { return 1; }

// General forms: element i holds Σ_{r in [rank_lo, rank_lo+n_ranks)} pattern(i + elem_offset, r).
// elem_offset must be a multiple of 8 as well.
int netop_fill_pattern_at(void* buf, uint64_t n_elems, uint32_t seed, int rank_lo, int n_ranks, uint64_t elem_offset,
                          hipStream_t stream) {
    if ((n_elems & 7) || (elem_offset & 7) || (reinterpret_cast<uintptr_t>(buf) & 15) || n_ranks < 1 || rank_lo < 0)
        return int(hipErrorInvalidValue);
    uint64_t nv = n_elems / 8;
    if (nv == 0) return int(hipSuccess);
    hipLaunchKernelGGL(fill_kernel, dim3(grid_for(nv, 16)), dim3(kThreads), 0, stream, static_cast<uint4*>(buf), nv, seed,
                       rank_lo, n_ranks, elem_offset);
    return int(hipGetLastError());
}

// Adds the number of mismatching elements to *errors (a device pointer the caller zeroes).
int netop_verify_pattern_at(const void* buf, uint64_t n_elems, uint32_t seed, int rank_lo, int n_ranks,
                            uint64_t elem_offset, unsigned long long* errors, hipStream_t stream) {
    if ((n_elems & 7) || (elem_offset & 7) || (reinterpret_cast<uintptr_t>(buf) & 15) || n_ranks < 1 || rank_lo < 0)
        return int(hipErrorInvalidValue);
    uint64_t nv = n_elems / 8;
    if (nv == 0) return int(hipSuccess);
    hipLaunchKernelGGL(verify_kernel, dim3(grid_for(nv, 16)), dim3(kThreads), 0, stream,
                       static_cast<const uint4*>(buf), nv, seed, rank_lo, n_ranks, elem_offset, errors);
    return int(hipGetLastError());
}

int netop_fill_pattern(void* buf, uint64_t n_elems, uint32_t seed, int rank, hipStream_t stream) {
    return netop_fill_pattern_at(buf, n_elems, seed, rank, 1, 0, stream);
}

int netop_fill_expected_sum(void* buf, uint64_t n_elems, uint32_t seed, int world, hipStream_t stream) {
    return netop_fill_pattern_at(buf, n_elems, seed, 0, world, 0, stream);
}

// Counts elements that differ from Σ_{r<world} pattern(i, r).
int netop_verify_sum(const void* buf, uint64_t n_elems, uint32_t seed, int world, unsigned long long* errors,
                     hipStream_t stream) {
    return netop_verify_pattern_at(buf, n_elems, seed, 0, world, 0, errors, stream);
}

// dst = Σ srcs (bf16, fp32 accumulation in source order, RNE).  1 <= nsrc <= 8; sizes in bf16
// elements, multiple of 8; all pointers 16-byte aligned (sources may be peer pointers).
// wg_per_cu <= 0 selects the default (4 workgroups per CU).
int netop_sum_bf16(const void* const* srcs, int nsrc, void* dst, uint64_t n_elems, int wg_per_cu, hipStream_t stream) {
    if (nsrc < 1 || nsrc > kMaxSrc || (n_elems & 7) || (reinterpret_cast<uintptr_t>(dst) & 15))
        return int(hipErrorInvalidValue);
    SrcPtrs p{};
    for (int s = 0; s < nsrc; ++s) {
        if (!srcs[s] || (reinterpret_cast<uintptr_t>(srcs[s]) & 15)) return int(hipErrorInvalidValue);
        p.p[s] = static_cast<const uint4*>(srcs[s]);
    }
    const uint64_t nv = n_elems / 8;
    if (nv == 0) return int(hipSuccess);
    const uint64_t unroll = uint64_t(sum_unroll(nsrc));
    hipLaunchKernelGGL(sum_fn(nsrc), dim3(grid_for((nv + unroll - 1) / unroll, wg_per_cu > 0 ? wg_per_cu : 2)),
                       dim3(kThreads), 0, stream, p, static_cast<uint4*>(dst), nv);
    return int(hipGetLastError());
}

int netop_copy(const void* src, void* dst, uint64_t bytes, hipStream_t stream) {
    if ((bytes & 15) || (reinterpret_cast<uintptr_t>(src) & 15) || (reinterpret_cast<uintptr_t>(dst) & 15))
        return int(hipErrorInvalidValue);
    uint64_t nv = bytes / 16;
    hipLaunchKernelGGL(copy_kernel, dim3(grid_for(nv, 4)), dim3(kThreads), 0, stream, static_cast<const uint4*>(src),
                       static_cast<uint4*>(dst), nv);
    return int(hipGetLastError());
}

// xGMI link probe, single process, all visible GPUs.  For every ordered pair (dst, src) with
// src != dst (or the loopback dst == src when only one GPU is visible) GPU `dst` pulls
// `bytes` from GPU `src` with netop_copy, `iters` times.  Two phases:
//   phase 1: one pair at a time           -> per-link GB/s in bw_single[dst * n + src]
//   phase 2: every dst pulls from all of its peers concurrently (one stream per peer)
//            -> aggregate GB/s per dst in bw_all[dst]
// Data integrity is checked on every pull (pattern fill + verify on the destination).
// Returns hipSuccess, or the first error.  `n_out` receives the number of GPUs probed.
int netop_xgmi_probe(uint64_t bytes, int iters, int max_gpus, double* bw_single, double* bw_all, int* n_out,
                     unsigned long long* total_errors) {
    DeviceRestore restore;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) return int(e);
    if (max_gpus > 0 && n > max_gpus) n = max_gpus;
    if (n > 64) n = 64;  // the per-GPU tables below
    *n_out = n;
    *total_errors = 0;
    bytes &= ~uint64_t(15);
    if (n == 0 || bytes == 0 || iters < 1) return int(hipErrorInvalidValue);

    // Every pair must be peer-accessible before any kernel reads a peer's memory: a pull over a
    // pair without peer access would fault the GPU (and may reset the node), so refuse instead.
    for (int d = 0; d < n; ++d)
        for (int p = 0; p < n; ++p) {
            if (p == d) continue;
            int can = 0;
            if ((e = hipDeviceCanAccessPeer(&can, d, p)) != hipSuccess) return int(e);
            if (!can) return int(hipErrorPeerAccessUnsupported);
        }
    void* src[64] = {};
    void* dst[64] = {};
    unsigned long long* err[64] = {};
    for (int d = 0; d < n; ++d) {
        if ((e = hipSetDevice(d)) != hipSuccess) return int(e);
        for (int p = 0; p < n; ++p) {
            if (p == d) continue;
            hipError_t pe = hipDeviceEnablePeerAccess(p, 0);
            if (pe != hipSuccess && pe != hipErrorPeerAccessAlreadyEnabled) return int(pe);
            (void)hipGetLastError();
        }
        // Each dst needs one receive buffer per peer for the concurrent phase.
        if ((e = hipMalloc(&src[d], bytes)) != hipSuccess) return int(e);
        if ((e = hipMalloc(&dst[d], bytes * size_t(n > 1 ? n - 1 : 1))) != hipSuccess) return int(e);
        if ((e = hipMalloc(&err[d], sizeof(unsigned long long))) != hipSuccess) return int(e);
        if ((e = (hipError_t)netop_fill_pattern(src[d], bytes / 2, 1234u, d, nullptr)) != hipSuccess) return int(e);
        if ((e = hipDeviceSynchronize()) != hipSuccess) return int(e);
    }

    // Phase 1: single links.
    for (int d = 0; d < n; ++d) {
        hipSetDevice(d);
        hipStream_t s;
        hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
        hipEvent_t t0, t1;
        hipEventCreate(&t0);
        hipEventCreate(&t1);
        for (int p = 0; p < n; ++p) {
            if (p == d && n > 1) {
                bw_single[d * n + p] = 0;
                continue;
            }
            netop_copy(src[p], dst[d], bytes, s);  // warm-up
            hipEventRecord(t0, s);
            for (int it = 0; it < iters; ++it) netop_copy(src[p], dst[d], bytes, s);
            hipEventRecord(t1, s);
            if ((e = hipEventSynchronize(t1)) != hipSuccess) return int(e);
            float ms = 0;
            hipEventElapsedTime(&ms, t0, t1);
            bw_single[d * n + p] = ms > 0 ? double(bytes) * iters / (double(ms) * 1e-3) / 1e9 : 0;
        }
        hipEventDestroy(t0);
        hipEventDestroy(t1);
        hipStreamDestroy(s);
    }

    // Phase 2: all peers concurrently into distinct buffers, then verify each buffer.
    for (int d = 0; d < n; ++d) {
        hipSetDevice(d);
        int peers = n > 1 ? n - 1 : 1;
        hipStream_t ss[64];
        for (int k = 0; k < peers; ++k) hipStreamCreateWithFlags(&ss[k], hipStreamNonBlocking);
        hipEvent_t t0, t1;
        hipEventCreate(&t0);
        hipEventCreate(&t1);
        hipEventRecord(t0, nullptr);
        for (int k = 0; k < peers; ++k) hipStreamWaitEvent(ss[k], t0, 0);
        for (int it = 0; it < iters; ++it) {
            int k = 0;
            for (int p = 0; p < n; ++p) {
                if (p == d && n > 1) continue;
                netop_copy(src[p], static_cast<char*>(dst[d]) + size_t(k) * bytes, bytes, ss[k]);
                ++k;
            }
        }
        for (int k = 0; k < peers; ++k) {
            hipEvent_t done;
            hipEventCreate(&done);
            hipEventRecord(done, ss[k]);
            hipStreamWaitEvent(nullptr, done, 0);
            hipEventDestroy(done);
        }
        hipEventRecord(t1, nullptr);
        if ((e = hipEventSynchronize(t1)) != hipSuccess) return int(e);
        float ms = 0;
        hipEventElapsedTime(&ms, t0, t1);
        bw_all[d] = ms > 0 ? double(bytes) * iters * peers / (double(ms) * 1e-3) / 1e9 : 0;
        // Integrity: buffer k must equal peer p's source bytes (host compare: this is a
        // validation path, not a hot path).
        std::vector<uint8_t> got(bytes), want(bytes);
        int k = 0;
        for (int p = 0; p < n; ++p) {
            if (p == d && n > 1) continue;
            hipMemcpy(got.data(), static_cast<char*>(dst[d]) + size_t(k) * bytes, bytes, hipMemcpyDeviceToHost);
            hipSetDevice(p);
            hipMemcpy(want.data(), src[p], bytes, hipMemcpyDeviceToHost);
            hipSetDevice(d);
            unsigned long long h = 0;
            for (size_t i = 0; i < bytes; ++i) h += got[i] != want[i];
            *total_errors += h;
            ++k;
        }
        hipEventDestroy(t0);
        hipEventDestroy(t1);
        for (int k2 = 0; k2 < peers; ++k2) hipStreamDestroy(ss[k2]);
    }
    for (int d = 0; d < n; ++d) {
        hipSetDevice(d);
        hipFree(src[d]);
        hipFree(dst[d]);
        hipFree(err[d]);
    }
    return int(hipSuccess);
}

// Push counterpart of phase 2: GPU `src` runs one copy per peer, each on its own stream,
// writing into the peer's memory (remote stores over the link to that peer), all peers at
// once.  bw_push[src] = aggregate GB/s leaving GPU src.  xGMI writes are posted and may reach a
// different bandwidth than reads; the direct all-reduce has a pull and a push mode for that
// reason.  Integrity is checked byte-exact on every destination.
int netop_xgmi_probe_push(uint64_t bytes, int iters, int max_gpus, double* bw_push, int* n_out,
                          unsigned long long* total_errors) {
    DeviceRestore restore;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) return int(e);
    if (max_gpus > 0 && n > max_gpus) n = max_gpus;
    *n_out = n;
    *total_errors = 0;
    bytes &= ~uint64_t(15);
    if (n == 0 || bytes == 0 || iters < 1 || n > 64) return int(hipErrorInvalidValue);
    std::vector<void*> src(n, nullptr), dst(n, nullptr);
    const int peers = n > 1 ? n - 1 : 1;
    for (int d = 0; d < n; ++d) {
        if ((e = hipSetDevice(d)) != hipSuccess) return int(e);
        for (int p = 0; p < n; ++p) {
            if (p == d) continue;
            hipError_t pe = hipDeviceEnablePeerAccess(p, 0);
            if (pe != hipSuccess && pe != hipErrorPeerAccessAlreadyEnabled) return int(pe);
            (void)hipGetLastError();
        }
        if ((e = hipMalloc(&src[d], bytes)) != hipSuccess) return int(e);
        // Receive area: one slot per possible writer.
        if ((e = hipMalloc(&dst[d], bytes * size_t(n))) != hipSuccess) return int(e);
        if ((e = (hipError_t)netop_fill_pattern(src[d], bytes / 2, 4321u, d, nullptr)) != hipSuccess) return int(e);
        if ((e = hipDeviceSynchronize()) != hipSuccess) return int(e);
    }
    for (int s = 0; s < n; ++s) {
        hipSetDevice(s);
        std::vector<hipStream_t> ss(peers);
        for (auto& st : ss) hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
        hipEvent_t t0, t1;
        hipEventCreate(&t0);
        hipEventCreate(&t1);
        hipEventRecord(t0, nullptr);
        for (auto& st : ss) hipStreamWaitEvent(st, t0, 0);
        for (int it = 0; it < iters; ++it) {
            int k = 0;
            for (int p = 0; p < n; ++p) {
                if (p == s && n > 1) continue;
                netop_copy(src[s], static_cast<char*>(dst[p]) + size_t(s) * bytes, bytes, ss[k++]);
            }
        }
        for (auto& st : ss) {
            hipEvent_t done;
            hipEventCreate(&done);
            hipEventRecord(done, st);
            hipStreamWaitEvent(nullptr, done, 0);
            hipEventDestroy(done);
        }
        hipEventRecord(t1, nullptr);
        if ((e = hipEventSynchronize(t1)) != hipSuccess) return int(e);
        float ms = 0;
        hipEventElapsedTime(&ms, t0, t1);
        bw_push[s] = ms > 0 ? double(bytes) * iters * peers / (double(ms) * 1e-3) / 1e9 : 0;
        hipEventDestroy(t0);
        hipEventDestroy(t1);
        for (auto& st : ss) hipStreamDestroy(st);
    }
    // Integrity: slot s of every destination p must equal src[s].
    std::vector<uint8_t> got(bytes), want(bytes);
    for (int s = 0; s < n; ++s) {
        hipSetDevice(s);
        hipMemcpy(want.data(), src[s], bytes, hipMemcpyDeviceToHost);
        for (int p = 0; p < n; ++p) {
            if (p == s && n > 1) continue;
            hipSetDevice(p);
            hipMemcpy(got.data(), static_cast<char*>(dst[p]) + size_t(s) * bytes, bytes, hipMemcpyDeviceToHost);
            unsigned long long h = 0;
            for (size_t i = 0; i < bytes; ++i) h += got[i] != want[i];
            *total_errors += h;
        }
    }
    for (int d = 0; d < n; ++d) {
        hipSetDevice(d);
        hipFree(src[d]);
        hipFree(dst[d]);
    }
    return int(hipSuccess);
}

}  // extern "C"

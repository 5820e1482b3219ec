// Tuning sweep for the xGMI probe's streaming copy (gfx950): loads in flight per lane (UNROLL)
// x workgroups per CU, nontemporal vs regular stores, and (round 6) nontemporal vs regular
// loads.  HBM loopback on one GPU (the link version cannot be measured on a 1-GPU box).  Prints
// one JSON line per variant.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                                 \
        }                                                                             \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int UNROLL, bool NT, bool NTL = false>
__global__ __launch_bounds__(256) void copy_u(const u32x4* __restrict__ src, u32x4* __restrict__ dst, uint64_t n) {
    const uint64_t stride = uint64_t(gridDim.x) * 256;
    uint64_t v = uint64_t(blockIdx.x) * 256 + threadIdx.x;
    for (; v + (UNROLL - 1) * stride < n; v += UNROLL * stride) {
        u32x4 r[UNROLL];
#pragma unroll
        for (int k = 0; k < UNROLL; ++k) r[k] = NTL ? __builtin_nontemporal_load(&src[v + k * stride]) : src[v + k * stride];
#pragma unroll
        for (int k = 0; k < UNROLL; ++k) {
            if (NT)
                __builtin_nontemporal_store(r[k], &dst[v + k * stride]);
            else
                dst[v + k * stride] = r[k];
        }
    }
    for (; v < n; v += stride) dst[v] = src[v];
}

template <int U, bool NT, bool NTL = false>
int run(const u32x4* s, u32x4* d, uint64_t n, int blocks, int iters, hipEvent_t a, hipEvent_t b) {
    hipLaunchKernelGGL((copy_u<U, NT, NTL>), dim3(blocks), dim3(256), 0, 0, s, d, n);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    for (int i = 0; i < iters; ++i) hipLaunchKernelGGL((copy_u<U, NT, NTL>), dim3(blocks), dim3(256), 0, 0, s, d, n);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    double gbs = double(n) * 16 * iters / (ms * 1e-3) / 1e9;
    std::printf("{\"unroll\":%d,\"nt\":%d,\"ntload\":%d,\"blocks\":%d,\"copy_GBps\":%.1f,\"traffic_GBps\":%.1f}\n", U,
                int(NT), int(NTL), blocks, gbs, 2 * gbs);
    return 0;
}

int main() {
    const uint64_t bytes = 1ull << 30;
    const uint64_t n = bytes / 16;
    u32x4 *s, *d;
    CHECK(hipMalloc(&s, bytes));
    CHECK(hipMalloc(&d, bytes));
    CHECK(hipMemset(s, 1, bytes));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    for (int bpc : {2, 4, 8, 16, 32}) {
        int blocks = 256 * bpc;
        if (run<1, false, true>(s, d, n, blocks, 10, a, b)) return 1;
        if (run<2, false, true>(s, d, n, blocks, 10, a, b)) return 1;
        if (run<4, false, true>(s, d, n, blocks, 10, a, b)) return 1;
        if (run<1, true, true>(s, d, n, blocks, 10, a, b)) return 1;
        if (run<2, true, true>(s, d, n, blocks, 10, a, b)) return 1;
        if (run<1, false>(s, d, n, blocks, 10, a, b)) return 1;
        if (run<2, false>(s, d, n, blocks, 10, a, b)) return 1;
        if (run<4, false>(s, d, n, blocks, 10, a, b)) return 1;
        if (run<8, false>(s, d, n, blocks, 10, a, b)) return 1;
        if (run<2, true>(s, d, n, blocks, 10, a, b)) return 1;
        if (run<4, true>(s, d, n, blocks, 10, a, b)) return 1;
    }
    return 0;
}

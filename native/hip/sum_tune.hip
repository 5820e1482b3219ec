// Tuning sweep for the n-way bf16 sum (netop_sum_bf16: the reduce step of the direct xGMI
// all-reduce) on gfx950: loads in flight per lane (UNROLL) x walk (grid-stride vs one contiguous
// chunk per workgroup) x nontemporal loads x nontemporal stores x workgroups per CU, for 2, 4 and
// 8 sources.  Local HBM on one GPU (over xGMI the peer reads are link-bound instead).  Every
// variant's output is compared bit for bit with the first one's.  One JSON line per variant.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHECK(x)                                                                           \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int kThreads = 256;
constexpr int kMaxSrc = 8;
struct Srcs {
    const u32x4* p[kMaxSrc];
};

__device__ __forceinline__ uint32_t rne2(float a, float b) {
    uint32_t ua = __float_as_uint(a), ub = __float_as_uint(b);
    ua = (ua & 0x7fffffffu) > 0x7f800000u ? (ua | 0x00400000u) : ua + 0x7fffu + ((ua >> 16) & 1u);
    ub = (ub & 0x7fffffffu) > 0x7f800000u ? (ub | 0x00400000u) : ub + 0x7fffu + ((ub >> 16) & 1u);
    return (ua >> 16) | (ub & 0xffff0000u);
}

template <int NSRC, int UNROLL, bool CHUNK, bool NTL, bool NTS>
__global__ __launch_bounds__(kThreads) void sum_k(Srcs src, u32x4* __restrict__ dst, uint64_t n) {
    constexpr uint64_t kStep = uint64_t(kThreads) * UNROLL;
    uint64_t b, end, stride;
    if (CHUNK) {
        const uint64_t per = ((n + gridDim.x - 1) / gridDim.x + kStep - 1) / kStep * kStep;
        b = uint64_t(blockIdx.x) * per + threadIdx.x;
        end = uint64_t(blockIdx.x) * per + per < n ? uint64_t(blockIdx.x) * per + per : n;
        stride = kStep;
    } else {
        b = uint64_t(blockIdx.x) * kStep + threadIdx.x;
        end = n;
        stride = uint64_t(gridDim.x) * kStep;
    }
    for (; b < end; b += stride) {
        u32x4 v[UNROLL][NSRC];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const uint64_t i = b + uint64_t(u) * kThreads;
            if (i < end) {
#pragma unroll
                for (int s = 0; s < NSRC; ++s) v[u][s] = NTL ? __builtin_nontemporal_load(&src.p[s][i]) : src.p[s][i];
            }
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const uint64_t i = b + uint64_t(u) * kThreads;
            if (i >= end) continue;
            float acc[8] = {};
#pragma unroll
            for (int s = 0; s < NSRC; ++s) {
                const uint32_t w[4] = {v[u][s].x, v[u][s].y, v[u][s].z, v[u][s].w};
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    acc[2 * k] += __uint_as_float(w[k] << 16);
                    acc[2 * k + 1] += __uint_as_float(w[k] & 0xffff0000u);
                }
            }
            u32x4 o;
            o.x = rne2(acc[0], acc[1]);
            o.y = rne2(acc[2], acc[3]);
            o.z = rne2(acc[4], acc[5]);
            o.w = rne2(acc[6], acc[7]);
            if (NTS)
                __builtin_nontemporal_store(o, &dst[i]);
            else
                dst[i] = o;
        }
    }
}

__global__ void fill_k(u32x4* p, uint64_t n, uint32_t seed) {
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
        uint32_t x = uint32_t(i) * 2654435761u ^ seed;
        u32x4 w;
        // bf16 pairs with a small exponent range: sums stay finite, roundings happen
        w.x = ((x & 0x7fffu) | 0x3c00u) | (((x >> 3) & 0x7fffu) | 0x3c00u) << 16;
        w.y = w.x ^ 0x00050005u;
        w.z = w.x ^ 0x80008000u;
        w.w = w.x + 0x00010001u;
        p[i] = w;
    }
}

using Fn = void (*)(Srcs, u32x4*, uint64_t);

template <int NSRC>
void variants(std::vector<std::pair<const char*, Fn>>& out) {
#define V(U, C, L, S) out.push_back({#U "," #C "," #L "," #S, sum_k<NSRC, U, C, L, S>})
#define V4(U) V(U, false, false, false); V(U, false, true, false); V(U, false, false, true); V(U, false, true, true); \
              V(U, true, false, false); V(U, true, true, false); V(U, true, false, true); V(U, true, true, true)
    V4(1);
    V4(2);
    V4(4);
#undef V4
#undef V
}

int main(int argc, char** argv) {
    const uint64_t bytes = argc > 1 ? std::strtoull(argv[1], nullptr, 10) << 20 : 256ull << 20;
    const int iters = argc > 2 ? std::atoi(argv[2]) : 10;
    const uint64_t n = bytes / 16;
    int cus = 256;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    std::vector<u32x4*> bufs(kMaxSrc);
    for (int s = 0; s < kMaxSrc; ++s) {
        CHECK(hipMalloc(&bufs[s], bytes));
        hipLaunchKernelGGL(fill_k, dim3(1024), dim3(256), 0, 0, bufs[s], n, 0x9e3779b9u * uint32_t(s + 1));
    }
    u32x4 *out, *ref;
    CHECK(hipMalloc(&out, bytes));
    CHECK(hipMalloc(&ref, bytes));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    std::vector<unsigned char> h_out(bytes), h_ref(bytes);
    for (int nsrc : {2, 4, 8}) {
        std::vector<std::pair<const char*, Fn>> vs;
        if (nsrc == 2) variants<2>(vs);
        if (nsrc == 4) variants<4>(vs);
        if (nsrc == 8) variants<8>(vs);
        Srcs p{};
        for (int s = 0; s < nsrc; ++s) p.p[s] = bufs[s];
        bool have_ref = false;
        for (auto& [name, fn] : vs) {
            for (int wg : {2, 4, 8, 16}) {
                int unroll = name[0] - '0';
                uint64_t need = (n + uint64_t(kThreads) * unroll - 1) / (uint64_t(kThreads) * unroll);
                int blocks = int(std::min<uint64_t>(need, uint64_t(cus) * wg));
                CHECK(hipMemset(out, 0xff, bytes));
                hipLaunchKernelGGL(fn, dim3(blocks), dim3(kThreads), 0, 0, p, have_ref ? out : ref, n);
                CHECK(hipDeviceSynchronize());
                bool same = true;
                if (have_ref) {
                    CHECK(hipMemcpy(h_out.data(), out, bytes, hipMemcpyDeviceToHost));
                    same = std::memcmp(h_out.data(), h_ref.data(), bytes) == 0;
                } else {
                    CHECK(hipMemcpy(h_ref.data(), ref, bytes, hipMemcpyDeviceToHost));
                    have_ref = true;
                }
                std::vector<float> ms(iters);
                for (int i = 0; i < iters; ++i) {
                    CHECK(hipEventRecord(a));
                    hipLaunchKernelGGL(fn, dim3(blocks), dim3(kThreads), 0, 0, p, out, n);
                    CHECK(hipEventRecord(b));
                    CHECK(hipEventSynchronize(b));
                    CHECK(hipEventElapsedTime(&ms[i], a, b));
                }
                std::sort(ms.begin(), ms.end());
                const double t = ms[ms.size() / 2] * 1e-3;
                std::printf("{\"sources\":%d,\"unroll_chunk_ntload_ntstore\":\"%s\",\"wg_per_cu\":%d,\"median_us\":%.2f,"
                            "\"TBps\":%.3f,\"same\":%s}\n",
                            nsrc, name, wg, t * 1e6, double(nsrc + 1) * double(bytes) / t / 1e12, same ? "true" : "false");
                std::fflush(stdout);
            }
        }
    }
    return 0;
}

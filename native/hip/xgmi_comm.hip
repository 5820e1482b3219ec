// Building blocks of the multi-process direct xGMI all-reduce (network_operator_amd/parallel/
// xgmi_comm.py): one process per GPU, as torch.distributed jobs run, instead of the
// single-process driver in xgmi_allreduce.hip.
//
//   * IPC export / import of device buffers, so every rank can address every peer's input and
//     output buffers directly over its xGMI link (peer pointers, no staging copies);
//   * a multi-pair copy kernel (all-gather phase: one launch pulls the n-1 reduced chunks);
//   * a shared-memory barrier between the ranks of one node.  The phases are ordered on the
//     host: stream synchronize -> barrier -> next launch.  No kernel ever spins on a flag
//     written by another process, so a rank that dies leaves its peers with a barrier timeout
//     (an error), never with a wavefront that cannot finish.
//
// The reduce phase uses netop_sum_bf16 from netop_hip.hip (same shared object).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

namespace {

constexpr int kThreads = 256;
constexpr int kMaxPairs = 8;

struct CopyPairs {
    const uint4* src[kMaxPairs];
    uint4* dst[kMaxPairs];
};

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// blockIdx.y selects the (src, dst) pair; within a pair, a grid-stride loop of 16-B vectors.
// Two loads in flight per lane: with peer sources each is an xGMI round trip.  Every byte is
// moved once: nontemporal loads and stores (copy_tune.hip on the box, profiles/r6_copy_tune.jsonl:
// 3.08 against 2.86 TB/s of copy with regular ones, HBM loopback).
__global__ __launch_bounds__(kThreads) void multi_copy_kernel(CopyPairs pairs, uint64_t n_vec) {
    const u32x4* __restrict__ s = reinterpret_cast<const u32x4*>(pairs.src[blockIdx.y]);
    u32x4* __restrict__ d = reinterpret_cast<u32x4*>(pairs.dst[blockIdx.y]);
    // Each workgroup covers 2 x kThreads consecutive vectors per step.
    const uint64_t stride = uint64_t(gridDim.x) * kThreads * 2;
    for (uint64_t i = uint64_t(blockIdx.x) * kThreads * 2 + threadIdx.x; i < n_vec; i += stride) {
        const uint64_t j = i + uint64_t(kThreads);
        const u32x4 a = __builtin_nontemporal_load(&s[i]);
        u32x4 b;
        const bool two = j < n_vec;
        if (two) b = __builtin_nontemporal_load(&s[j]);
        __builtin_nontemporal_store(a, &d[i]);
        if (two) __builtin_nontemporal_store(b, &d[j]);
    }
}

int cus_of_current_device() {
    static int cached[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (!cached[dev]) {
        int c = 0;
        if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && c > 0)
            cached[dev] = c;
        else
            return 256;
    }
    return cached[dev];
}

// Sense-reversing barrier in a shared mapping; `count` and `sense` on separate cache lines.
struct alignas(64) ShmBarrier {
    std::atomic<int> count;
    char pad0[60];
    std::atomic<int> sense;
    char pad1[60];
    int world;
};
static_assert(sizeof(std::atomic<int>) == 4, "lock-free int expected");

struct BarrierHandle {
    ShmBarrier* b;
    int local_sense;
};

}  // namespace

extern "C" {

// Exports the allocation that contains `ptr`: *handle (sizeof(hipIpcMemHandle_t) = 64 bytes)
// and the byte offset of `ptr` inside it (torch's caching allocator hands out sub-blocks).
int netop_ipc_export(const void* ptr, void* handle, uint64_t* offset) {
    if (!ptr || !handle || !offset) return int(hipErrorInvalidValue);
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    hipError_t e = hipMemGetAddressRange(&base, &size, const_cast<void*>(ptr));
    if (e != hipSuccess) return int(e);
    hipIpcMemHandle_t h;
    e = hipIpcGetMemHandle(&h, reinterpret_cast<void*>(base));
    if (e != hipSuccess) return int(e);
    std::memcpy(handle, &h, sizeof h);
    *offset = uint64_t(static_cast<const char*>(ptr) - static_cast<const char*>(reinterpret_cast<void*>(base)));
    return int(hipSuccess);
}

int netop_ipc_handle_size() { return int(sizeof(hipIpcMemHandle_t)); }

// The PCI bus id ("0000:0d:00.0") of the GPU whose memory `ptr` is: what an exporter publishes
// beside its handle, so the importer can check peer access to that GPU before mapping.
int netop_ipc_device_bus_id(const void* ptr, char* out, int len) {
    if (!ptr || !out || len < 13) return int(hipErrorInvalidValue);
    hipPointerAttribute_t a{};
    hipError_t e = hipPointerGetAttributes(&a, ptr);
    if (e != hipSuccess) return int(e);
    return int(hipDeviceGetPCIBusId(out, len, a.device));
}

// Maps a peer's exported allocation into this process (peer access enabled lazily) and
// returns the address of the exported pointer (*base is what netop_ipc_close needs).
// `peer_bus_id` names the exporter's GPU: like the single-process probe (netop_hip.hip), nothing
// is mapped unless this process's GPU can access it -- the exporter's GPU not visible here, or a
// pair without peer access, is refused with hipErrorPeerAccessUnsupported before any kernel could
// read across it (a pull over a pair without peer access faults the GPU and may reset the node).
int netop_ipc_open(const void* handle, uint64_t offset, const char* peer_bus_id, void** ptr, void** base) {
    if (!handle || !ptr || !base || !peer_bus_id) return int(hipErrorInvalidValue);
    int cur = 0, peer = -1;
    hipError_t e = hipGetDevice(&cur);
    if (e != hipSuccess) return int(e);
    if (hipDeviceGetByPCIBusId(&peer, peer_bus_id) != hipSuccess || peer < 0) {
        (void)hipGetLastError();  // the lookup's error is the refusal below, not a sticky one
        return int(hipErrorPeerAccessUnsupported);
    }
    if (peer != cur) {
        int can = 0;
        if ((e = hipDeviceCanAccessPeer(&can, cur, peer)) != hipSuccess) return int(e);
        if (!can) return int(hipErrorPeerAccessUnsupported);
    }
    hipIpcMemHandle_t h;
    std::memcpy(&h, handle, sizeof h);
    void* b = nullptr;
    e = hipIpcOpenMemHandle(&b, h, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) return int(e);
    *base = b;
    *ptr = static_cast<char*>(b) + offset;
    return int(hipSuccess);
}

int netop_ipc_close(void* base) { return int(hipIpcCloseMemHandle(base)); }

// dst[k] = src[k] for k < n pairs, `bytes` each (multiple of 16, 16-B aligned; sources may be
// peer pointers).  One launch; wg_per_cu <= 0 selects 4 workgroups per CU over all pairs.
int netop_multi_copy(const void* const* srcs, void* const* dsts, int n, uint64_t bytes, int wg_per_cu,
                     hipStream_t stream) {
    if (n < 0 || n > kMaxPairs || (bytes & 15)) return int(hipErrorInvalidValue);
    if (n == 0 || bytes == 0) return int(hipSuccess);
    CopyPairs p{};
    for (int k = 0; k < n; ++k) {
        if (!srcs[k] || !dsts[k] || (reinterpret_cast<uintptr_t>(srcs[k]) & 15) ||
            (reinterpret_cast<uintptr_t>(dsts[k]) & 15))
            return int(hipErrorInvalidValue);
        p.src[k] = static_cast<const uint4*>(srcs[k]);
        p.dst[k] = static_cast<uint4*>(dsts[k]);
    }
    const uint64_t nv = bytes / 16;
    const uint64_t per_pair_cap = std::max<uint64_t>(1, uint64_t(cus_of_current_device()) * (wg_per_cu > 0 ? wg_per_cu : 4) / n);
    const uint64_t need = (nv + 2 * kThreads - 1) / (2 * kThreads);
    const unsigned gx = unsigned(std::max<uint64_t>(1, std::min(need, per_pair_cap)));
    hipLaunchKernelGGL(multi_copy_kernel, dim3(gx, unsigned(n)), dim3(kThreads), 0, stream, p, nv);
    return int(hipGetLastError());
}

// ---- node-local barrier ------------------------------------------------------------------------
// Rank 0 creates `name` (POSIX shm), every rank opens it; after all have opened, rank 0 may
// unlink the name (the mapping stays).  Returns an opaque handle or nullptr (errno set).
void* netop_shm_barrier_open(const char* name, int world, int create) {
    if (!name || world < 1) return nullptr;
    int fd = create ? ::shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600) : ::shm_open(name, O_RDWR, 0600);
    if (fd < 0) return nullptr;
    if (create && ::ftruncate(fd, sizeof(ShmBarrier)) != 0) {
        ::close(fd);
        ::shm_unlink(name);
        return nullptr;
    }
    void* m = ::mmap(nullptr, sizeof(ShmBarrier), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    ::close(fd);
    if (m == MAP_FAILED) return nullptr;
    auto* b = static_cast<ShmBarrier*>(m);
    if (create) {
        b->count.store(0, std::memory_order_relaxed);
        b->world = world;
        b->sense.store(0, std::memory_order_release);
    }
    auto* h = new BarrierHandle{b, 0};
    return h;
}

int netop_shm_unlink(const char* name) { return ::shm_unlink(name) == 0 ? 0 : errno; }

// 0 on success, ETIMEDOUT after timeout_ms (the barrier is then unusable for this rank).
int netop_shm_barrier_wait(void* handle, int timeout_ms) {
    auto* h = static_cast<BarrierHandle*>(handle);
    if (!h) return EINVAL;
    ShmBarrier* b = h->b;
    const int s = h->local_sense ^ 1;
    h->local_sense = s;
    if (b->count.fetch_add(1, std::memory_order_acq_rel) == b->world - 1) {
        b->count.store(0, std::memory_order_relaxed);
        b->sense.store(s, std::memory_order_release);
        return 0;
    }
    const auto end = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
    for (unsigned spin = 0;; ++spin) {
        if (b->sense.load(std::memory_order_acquire) == s) return 0;
        if ((spin & 1023) == 1023) {
            if (std::chrono::steady_clock::now() > end) return ETIMEDOUT;
            ::sched_yield();
        }
    }
}

void netop_shm_barrier_close(void* handle) {
    auto* h = static_cast<BarrierHandle*>(handle);
    if (!h) return;
    ::munmap(h->b, sizeof(ShmBarrier));
    delete h;
}

}  // extern "C"

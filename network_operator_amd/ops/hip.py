"""ctypes binding of ``libnetop_hip.so`` (native/hip/netop_hip.hip, gfx950).

The kernels validate what the operator configures: all-reduce results over RCCL (bf16
pattern fill / verify, exact for any reduction order) and xGMI link integrity and bandwidth
(peer-pull copy).  Every entry point raises if the library is missing — on a GPU box these
ops never fall back to eager PyTorch.
"""

from __future__ import annotations

import ctypes
import threading

from ..utils.paths import hip_library, native_bin

_lib = None
_lock = threading.Lock()


class HipError(RuntimeError):
    pass


def lib() -> ctypes.CDLL:
    global _lib
    with _lock:
        if _lib is None:
            L = ctypes.CDLL(str(hip_library()))
            u64, i32, u32, vp = ctypes.c_uint64, ctypes.c_int, ctypes.c_uint32, ctypes.c_void_p
            L.netop_hip_version.restype = i32
            L.netop_fill_pattern.argtypes = [vp, u64, u32, i32, vp]
            L.netop_fill_pattern.restype = i32
            L.netop_fill_expected_sum.argtypes = [vp, u64, u32, i32, vp]
            L.netop_fill_expected_sum.restype = i32
            L.netop_verify_sum.argtypes = [vp, u64, u32, i32, vp, vp]
            L.netop_verify_sum.restype = i32
            L.netop_fill_pattern_at.argtypes = [vp, u64, u32, i32, i32, u64, vp]
            L.netop_fill_pattern_at.restype = i32
            L.netop_verify_pattern_at.argtypes = [vp, u64, u32, i32, i32, u64, vp, vp]
            L.netop_verify_pattern_at.restype = i32
            L.netop_sum_bf16.argtypes = [ctypes.POINTER(vp), i32, vp, u64, i32, vp]
            L.netop_sum_bf16.restype = i32
            L.netop_copy.argtypes = [vp, vp, u64, vp]
            L.netop_copy.restype = i32
            L.netop_xgmi_probe.argtypes = [u64, i32, i32, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                           ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_ulonglong)]
            L.netop_xgmi_probe.restype = i32
            L.netop_xgmi_probe_push.argtypes = [u64, i32, i32, ctypes.POINTER(ctypes.c_double),
                                                ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_ulonglong)]
            L.netop_xgmi_probe_push.restype = i32
            # xgmi_comm.hip: IPC buffers, multi-pair copy, node-local barrier
            L.netop_ipc_handle_size.restype = i32
            L.netop_ipc_export.argtypes = [vp, vp, ctypes.POINTER(u64)]
            L.netop_ipc_export.restype = i32
            L.netop_ipc_device_bus_id.argtypes = [vp, ctypes.c_char_p, i32]
            L.netop_ipc_device_bus_id.restype = i32
            L.netop_ipc_open.argtypes = [vp, u64, ctypes.c_char_p, ctypes.POINTER(vp), ctypes.POINTER(vp)]
            L.netop_ipc_open.restype = i32
            L.netop_ipc_close.argtypes = [vp]
            L.netop_ipc_close.restype = i32
            L.netop_multi_copy.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(vp), i32, u64, i32, vp]
            L.netop_multi_copy.restype = i32
            L.netop_shm_barrier_open.argtypes = [ctypes.c_char_p, i32, i32]
            L.netop_shm_barrier_open.restype = vp
            L.netop_shm_barrier_wait.argtypes = [vp, i32]
            L.netop_shm_barrier_wait.restype = i32
            L.netop_shm_barrier_close.argtypes = [vp]
            L.netop_shm_barrier_close.restype = None
            L.netop_shm_unlink.argtypes = [ctypes.c_char_p]
            L.netop_shm_unlink.restype = i32
            _lib = L
    return _lib


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise HipError(f"{what} failed with hipError {rc}")


def _stream(tensor):
    import torch

    return ctypes.c_void_p(torch.cuda.current_stream(tensor.device).cuda_stream)


def _check_buf(t):
    import torch

    if t.dtype != torch.bfloat16 or not t.is_cuda or not t.is_contiguous():
        raise ValueError("expected a contiguous bfloat16 CUDA tensor")
    if t.numel() % 8 or t.data_ptr() % 16:
        raise ValueError("numel must be a multiple of 8 and the buffer 16-byte aligned")


def fill_pattern(t, seed: int, rank: int) -> None:
    """Fill ``t`` (bf16) with rank ``rank``'s deterministic integer pattern in [-4, 3]."""
    _check_buf(t)
    _check(lib().netop_fill_pattern(ctypes.c_void_p(t.data_ptr()), t.numel(), seed & 0xFFFFFFFF, rank, _stream(t)),
           "netop_fill_pattern")


def fill_expected_sum(t, seed: int, world: int) -> None:
    """Fill ``t`` with Σ_{r<world} pattern(r) — what an all-reduce(sum) must produce."""
    _check_buf(t)
    _check(lib().netop_fill_expected_sum(ctypes.c_void_p(t.data_ptr()), t.numel(), seed & 0xFFFFFFFF, world, _stream(t)),
           "netop_fill_expected_sum")


def verify_sum(t, seed: int, world: int) -> int:
    """Number of elements of ``t`` that differ from the expected all-reduce sum (synchronises)."""
    import torch

    _check_buf(t)
    err = torch.zeros(1, dtype=torch.int64, device=t.device)
    _check(lib().netop_verify_sum(ctypes.c_void_p(t.data_ptr()), t.numel(), seed & 0xFFFFFFFF, world,
                                  ctypes.c_void_p(err.data_ptr()), _stream(t)), "netop_verify_sum")
    return int(err.item())


def fill_pattern_at(t, seed: int, rank_lo: int, n_ranks: int = 1, elem_offset: int = 0) -> None:
    """``t[i] = Σ_{r in [rank_lo, rank_lo+n_ranks)} pattern(i + elem_offset, r)`` — the slice of the
    global pattern a collective's output chunk must equal (all-gather / reduce-scatter / all-to-all)."""
    _check_buf(t)
    if elem_offset % 8:
        raise ValueError("elem_offset must be a multiple of 8")
    _check(lib().netop_fill_pattern_at(ctypes.c_void_p(t.data_ptr()), t.numel(), seed & 0xFFFFFFFF, rank_lo, n_ranks,
                                       elem_offset, _stream(t)), "netop_fill_pattern_at")


def verify_pattern_at(t, seed: int, rank_lo: int, n_ranks: int = 1, elem_offset: int = 0) -> int:
    """Mismatch count of ``t`` against :func:`fill_pattern_at`'s definition (synchronises)."""
    import torch

    _check_buf(t)
    if elem_offset % 8:
        raise ValueError("elem_offset must be a multiple of 8")
    err = torch.zeros(1, dtype=torch.int64, device=t.device)
    _check(lib().netop_verify_pattern_at(ctypes.c_void_p(t.data_ptr()), t.numel(), seed & 0xFFFFFFFF, rank_lo, n_ranks,
                                         elem_offset, ctypes.c_void_p(err.data_ptr()), _stream(t)),
           "netop_verify_pattern_at")
    return int(err.item())


def sum_bf16(srcs, out, wg_per_cu: int = 0) -> None:
    """``out = Σ srcs`` for 1..8 bf16 tensors of equal size: fp32 accumulation in list order,
    round-to-nearest-even to bf16 (the reduce step of the direct xGMI all-reduce)."""
    if not 1 <= len(srcs) <= 8:
        raise ValueError("1..8 sources")
    for t in (*srcs, out):
        _check_buf(t)
        if t.numel() != out.numel():
            raise ValueError("all tensors must have the same number of elements")
    arr = (ctypes.c_void_p * len(srcs))(*[t.data_ptr() for t in srcs])
    _check(lib().netop_sum_bf16(arr, len(srcs), ctypes.c_void_p(out.data_ptr()), out.numel(), wg_per_cu, _stream(out)),
           "netop_sum_bf16")


def copy(src, dst) -> None:
    """16-byte-vector device copy (src may live on a peer GPU with peer access enabled)."""
    nbytes = src.numel() * src.element_size()
    if dst.numel() * dst.element_size() < nbytes:
        raise ValueError("destination too small")
    _check(lib().netop_copy(ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(dst.data_ptr()), nbytes, _stream(dst)),
           "netop_copy")


def multi_copy(srcs, dsts, wg_per_cu: int = 0) -> None:
    """``dsts[k] <- srcs[k]`` for up to 8 equal-size pairs in one launch (the all-gather step of
    the multi-process xGMI all-reduce; sources may be peer memory)."""
    if len(srcs) != len(dsts) or len(srcs) > 8:
        raise ValueError("up to 8 (src, dst) pairs")
    if not srcs:
        return
    nbytes = srcs[0].numel() * srcs[0].element_size()
    for s, d in zip(srcs, dsts):
        if not (s.is_cuda and d.is_cuda and s.is_contiguous() and d.is_contiguous()):
            raise ValueError("contiguous CUDA tensors expected")
        if s.numel() * s.element_size() != nbytes or d.numel() * d.element_size() != nbytes:
            raise ValueError("all pairs must have the same byte size")
        if s.data_ptr() % 16 or d.data_ptr() % 16 or nbytes % 16:
            raise ValueError("16-byte aligned buffers and sizes expected")
    vp = ctypes.c_void_p
    a = (vp * len(srcs))(*[vp(s.data_ptr()) for s in srcs])
    b = (vp * len(dsts))(*[vp(d.data_ptr()) for d in dsts])
    _check(lib().netop_multi_copy(a, b, len(srcs), nbytes, wg_per_cu, _stream(dsts[0])), "netop_multi_copy")


def xgmi_probe(nbytes: int = 256 << 20, iters: int = 10, max_gpus: int = 8) -> dict:
    """Pull-bandwidth and integrity probe over every visible GPU pair (see netop_hip.hip)."""
    n = 64
    single = (ctypes.c_double * (n * n))()
    agg = (ctypes.c_double * n)()
    n_out = ctypes.c_int(0)
    errors = ctypes.c_ulonglong(0)
    _check(lib().netop_xgmi_probe(nbytes, iters, max_gpus, single, agg, ctypes.byref(n_out), ctypes.byref(errors)),
           "netop_xgmi_probe")
    g = n_out.value
    return {
        "gpus": g,
        "bytes": nbytes,
        "iters": iters,
        "errors": errors.value,
        "link_GBps": [[single[d * g + p] for p in range(g)] for d in range(g)],
        "aggregate_GBps": [agg[d] for d in range(g)],
    }


def xgmi_probe_isolated(nbytes: int = 256 << 20, iters: int = 10, max_gpus: int = 8, timeout: float = 120) -> dict:
    """``xgmi_probe`` + ``xgmi_probe_push`` in a child process (``netop-xgmi-probe``): the caller
    keeps no context on the peer GPUs, and a fault or hang in the probe ends the child, not the
    caller (bench.py's rank 0 still has to print its result).  Byte errors come back as data
    (exit status 3), any other failure raises."""
    import json
    import subprocess

    r = subprocess.run([str(native_bin("netop-xgmi-probe")), f"--bytes={nbytes}", f"--iters={iters}",
                        f"--max-gpus={max_gpus}"], capture_output=True, text=True, timeout=timeout)
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    if r.returncode not in (0, 3) or not lines:
        raise RuntimeError(f"netop-xgmi-probe rc={r.returncode}: {r.stderr[-400:]}")
    return json.loads(lines[-1])


def xgmi_probe_push(nbytes: int = 256 << 20, iters: int = 10, max_gpus: int = 8) -> dict:
    """Every GPU writes to all of its peers at once (remote stores): aggregate GB/s per GPU."""
    push = (ctypes.c_double * 64)()
    n_out = ctypes.c_int(0)
    errors = ctypes.c_ulonglong(0)
    _check(lib().netop_xgmi_probe_push(nbytes, iters, max_gpus, push, ctypes.byref(n_out), ctypes.byref(errors)),
           "netop_xgmi_probe_push")
    return {"gpus": n_out.value, "bytes": nbytes, "iters": iters, "errors": errors.value,
            "push_aggregate_GBps": [push[d] for d in range(n_out.value)]}

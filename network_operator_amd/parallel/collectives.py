"""RCCL-over-xGMI validation: rccl-tests bandwidth math and timed collectives.

The operator's contract ends where RCCL starts: after the node agent has configured the
scale-out NICs and verified the xGMI mesh, collectives must see every link.  This module
measures that with the same definitions as rccl-tests (``src/common.cu``-style formulas):

    algbw = bytes / time
    busbw = algbw * factor(op, n)       all_reduce: 2(n-1)/n, all_gather / reduce_scatter /
                                        all_to_all: (n-1)/n, broadcast / reduce: 1

One process per GPU, ``torch.distributed`` with the ``nccl`` backend (= RCCL on ROCm).
Timings are bracketed by barrier + device synchronize and the MAX over ranks is reported.
"""

from __future__ import annotations

import math
import time
from dataclasses import asdict, dataclass
from typing import Callable, Iterable, List, Optional

BUS_FACTORS: dict[str, Callable[[int], float]] = {
    "all_reduce": lambda n: 2.0 * (n - 1) / n,
    "all_gather": lambda n: (n - 1) / n,
    "reduce_scatter": lambda n: (n - 1) / n,
    "all_to_all": lambda n: (n - 1) / n,
    "broadcast": lambda n: 1.0,
    "reduce": lambda n: 1.0,
}


def bus_factor(op: str, n: int) -> float:
    if n < 1:
        raise ValueError("n must be >= 1")
    return BUS_FACTORS[op](n)


@dataclass
class CollectiveResult:
    op: str
    bytes: int          # per-rank message size (rccl-tests "size")
    n_ranks: int
    iters: int
    time_s: float       # per-iteration time, max over ranks
    algbw_GBps: float
    busbw_GBps: float
    verified: Optional[bool] = None
    errors: Optional[int] = None

    def as_dict(self) -> dict:
        return asdict(self)


def bandwidths(op: str, nbytes: int, n: int, seconds: float) -> tuple[float, float]:
    if seconds <= 0:
        return float("inf"), float("inf")
    algbw = nbytes / seconds / 1e9
    return algbw, algbw * bus_factor(op, n)


def xgmi_busbw_ceiling_GBps(n: int, link_GBps: float = 76.0) -> float:
    """Upper bound on all-reduce busbw inside one MI355X node.

    Each GPU has one xGMI link to each of its n-1 peers (KFD advertises 76 GB/s per
    direction per link on MI355X).  A bandwidth-optimal all-reduce moves 2(n-1)/n * S bytes
    out of every GPU, and at most (n-1) * link_GBps can leave a GPU at once, so
    busbw <= (n-1) * link_GBps.  n = 1 has no links (busbw is 0 by definition).
    """
    return 0.0 if n <= 1 else (n - 1) * link_GBps


def _max_over_ranks(value: float, device) -> float:
    import torch
    import torch.distributed as dist

    if not dist.is_initialized() or dist.get_world_size() == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def time_collective(op: str, tensor, iters: int, warmup: int, group=None, out=None) -> float:
    """Runs ``warmup`` untimed + ``iters`` timed collectives; returns max-over-ranks s/iter."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group) if dist.is_initialized() else 1

    def once():
        if op == "all_reduce":
            dist.all_reduce(tensor, group=group)
        elif op == "all_gather":
            dist.all_gather_into_tensor(out, tensor, group=group)
        elif op == "reduce_scatter":
            dist.reduce_scatter_tensor(out, tensor, group=group)
        elif op == "all_to_all":
            dist.all_to_all_single(out, tensor, group=group)
        elif op == "broadcast":
            dist.broadcast(tensor, src=0, group=group)
        else:
            raise ValueError(op)

    for _ in range(warmup):
        once()
    if dist.is_initialized():
        dist.barrier(group=group)
    sync(tensor.device)
    t0 = time.perf_counter()
    for _ in range(iters):
        once()
    sync(tensor.device)
    dt = (time.perf_counter() - t0) / max(iters, 1)
    if dist.is_initialized():
        dist.barrier(group=group)
    return _max_over_ranks(dt, tensor.device) if world > 1 else dt


def sync(device) -> None:
    import torch

    if getattr(device, "type", str(device)) == "cuda":
        torch.cuda.synchronize(device)


def pattern_reference(n: int, seed: int, rank: int):
    """PyTorch (CPU) reference of the HIP pattern in native/hip/netop_hip.hip (group_hash /
    base_mult / step_mult / group_sum): element i is the 3-bit field at bit 5 + 3 (i & 7) of
    group_hash(i >> 3) * (base_mult(seed) + rank * step_mult(seed)), minus 4."""
    import torch

    M32 = 0xFFFFFFFF
    i = torch.arange(n, dtype=torch.int64)
    g = i >> 3  # one hash per 8-element group
    h = ((g & M32) * 0x9E3779B1) & M32
    h = h ^ ((((g >> 32) & M32) * 0x85EBCA77) & M32)
    h = h ^ (h >> 15)
    h = (h * 0x2C1B3C6D) & M32
    h = h ^ (h >> 12)
    k = (((seed + 0x632BE5AB) & M32) * 0xC2B2AE3D) & M32
    m0 = (k ^ (k >> 16)) | 1
    k = (((seed ^ 0x27D4EB2F) & M32) * 0x165667B1) & M32
    d = (((k ^ (k >> 15)) << 1) | 2) & M32
    m = (m0 + rank * d) & M32
    x = (h * m) & M32  # int64 wraps on overflow; the low 32 bits are exact
    return (((x >> (5 + 3 * (i & 7))) & 7) - 4).to(torch.float32)


def verify_all_reduce(numel: int, device, seed: int = 2024, group=None) -> tuple[bool, int]:
    """Fills rank-specific patterns, all-reduces, verifies Σ over ranks exactly.

    On a GPU the fill and the check are the HIP kernels of ``libnetop_hip.so`` (bf16; no
    fallback — a missing library raises).  On the CPU (gloo rehearsals of the multi-rank
    path) the same pattern comes from ``pattern_reference`` in fp32."""
    import torch
    import torch.distributed as dist

    numel -= numel % 8
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if getattr(device, "type", str(device)) == "cuda":
        from ..ops import hip

        buf = torch.empty(numel, dtype=torch.bfloat16, device=device)
        hip.fill_pattern(buf, seed, rank)
        if dist.is_initialized():
            dist.all_reduce(buf, group=group)
        errors = hip.verify_sum(buf, seed, world)
    else:
        buf = pattern_reference(numel, seed, rank)
        if dist.is_initialized():
            dist.all_reduce(buf, group=group)
        want = sum(pattern_reference(numel, seed, r) for r in range(world))
        errors = int((buf != want).sum().item())
    total = int(_max_over_ranks(float(errors), device)) if world > 1 else errors
    return total == 0, total


def sweep_sizes(min_bytes: int, max_bytes: int, factor: int = 2) -> List[int]:
    out, s = [], max(min_bytes, 16)
    while s <= max_bytes:
        out.append(s)
        s *= factor
    return out


def run_sweep(op: str, sizes: Iterable[int], iters: int, warmup: int, device, group=None,
              dtype=None) -> List[CollectiveResult]:
    import torch
    import torch.distributed as dist

    dtype = dtype or torch.bfloat16
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    esize = torch.tensor([], dtype=dtype).element_size()
    results = []
    for nbytes in sizes:
        # rccl-tests "size": the full buffer — all_gather's output, reduce_scatter's input,
        # all_to_all's per-rank send (= receive) buffer, the all_reduce buffer.
        numel = max(1, nbytes // esize)
        numel = int(math.ceil(numel / world) * world)
        out = None
        if op == "all_gather":
            t = torch.zeros(numel // world, dtype=dtype, device=device)
            out = torch.empty(numel, dtype=dtype, device=device)
        elif op == "reduce_scatter":
            t = torch.zeros(numel, dtype=dtype, device=device)
            out = torch.empty(numel // world, dtype=dtype, device=device)
        else:
            t = torch.zeros(numel, dtype=dtype, device=device)
            if op == "all_to_all":
                out = torch.empty_like(t)
        dt = time_collective(op, t, iters, warmup, group=group, out=out)
        algbw, busbw = bandwidths(op, numel * esize, world, dt)
        results.append(CollectiveResult(op, numel * esize, world, iters, dt, algbw, busbw))
        del t, out
    return results

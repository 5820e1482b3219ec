"""Driver for the native RCCL harness ``netop-rccl-bench`` (native/hip/rccl_bench.cpp).

The harness links RCCL directly (``ncclCommInitAll`` for every local GPU in one process, or
``ncclCommInitRank`` with a file-based unique-id exchange for one process per GPU), sweeps
message sizes like rccl-tests and checks every result exactly with the bf16 pattern kernels.
This module runs it and parses its JSON lines; ``bench.py --native-rccl`` reports it next to
the torch.distributed numbers.
"""

from __future__ import annotations

import json
import os
import subprocess
from dataclasses import dataclass
from typing import List, Optional

from ..utils.paths import native_bin

OPS = ("all_reduce", "all_gather", "reduce_scatter", "broadcast", "alltoall")


@dataclass
class Row:
    op: str
    bytes: int
    count: int
    ranks: int
    time_us: float
    algbw_GBps: float
    busbw_GBps: float
    wrong: int
    checked: bool
    inplace: bool
    graph: bool


def command(op: str = "all_reduce", gpus: int = 1, min_bytes: int = 8, max_bytes: int = 128 << 20, factor: float = 2,
            iters: int = 20, warmup: int = 5, check: bool = True, inplace: bool = False, graph: bool = False,
            dtype: str = "bf16", nranks: Optional[int] = None, rank: Optional[int] = None,
            device: Optional[int] = None, id_file: Optional[str] = None) -> List[str]:
    if op not in OPS:
        raise ValueError(f"unknown op {op!r}")
    cmd = [str(native_bin("netop-rccl-bench")), "-o", op, "-g", str(gpus), "-b", str(min_bytes), "-e", str(max_bytes),
           "-f", str(factor), "-n", str(iters), "-w", str(warmup), "-c", "1" if check else "0", "-d", dtype]
    if inplace:
        cmd.append("--inplace")
    if graph:
        cmd.append("--graph")
    if nranks is not None:
        cmd += ["--nranks", str(nranks), "--rank", str(rank), "--device", str(device or 0), "--id-file", str(id_file)]
    return cmd


# RCCL knobs whose effect on large intra-node all-reduce is worth knowing per node type.
ENV_PROBES = (
    {},
    {"NCCL_MIN_NCHANNELS": "64"},
    {"NCCL_MIN_NCHANNELS": "112"},
    {"NCCL_BUFFSIZE": str(8 << 20)},
    {"NCCL_ALGO": "Ring"},
    {"HSA_NO_SCRATCH_RECLAIM": "1"},
)


def env_probe(gpus: int, nbytes: int, iters: int = 10, probes=ENV_PROBES, timeout: float = 120,
              budget_s: Optional[float] = None, base_env: Optional[dict] = None) -> List[dict]:
    """busbw of one all-reduce size under each RCCL environment variant (fresh process each:
    RCCL caches its parameters at first use), on top of ``base_env`` (the agent's artifacts).
    Variants not started within ``budget_s`` seconds are reported as skipped."""
    import time

    out = []
    t0 = time.monotonic()
    for extra in probes:
        if budget_s is not None and time.monotonic() - t0 > budget_s:
            out.append({"env": extra, "skipped": "time budget spent"})
            continue
        try:
            rows = run(op="all_reduce", gpus=gpus, min_bytes=nbytes, max_bytes=nbytes, iters=iters, warmup=3,
                       check=False, env=dict(base_env or {}, **extra), timeout=timeout)
            out.append({"env": extra, "busbw_GBps": rows[-1].busbw_GBps if rows else None,
                        "time_us": rows[-1].time_us if rows else None})
        except Exception as e:
            out.append({"env": extra, "error": str(e)[-300:]})
    return out


def choose_env(probes: List[dict], min_gain: float = 1.03) -> dict:
    """The variant to use: the fastest measured one if it beats the defaults ({}) by at least
    ``min_gain``, else the defaults.  Returns {"chosen": env, "baseline_busbw_GBps": x,
    "best_busbw_GBps": y}."""
    base = next((p.get("busbw_GBps") for p in probes if p["env"] == {}), None) or 0.0
    best = max((p for p in probes if p.get("busbw_GBps")), key=lambda p: p["busbw_GBps"], default=None)
    chosen = best["env"] if best and base and best["busbw_GBps"] >= min_gain * base else {}
    return {"chosen": dict(chosen), "baseline_busbw_GBps": base,
            "best_busbw_GBps": best["busbw_GBps"] if best else None}


def parse(stdout: str) -> List[Row]:
    rows = []
    for line in stdout.splitlines():
        line = line.strip()
        if line.startswith("{"):
            d = json.loads(line)
            rows.append(Row(d["op"], d["bytes"], d["count"], d["ranks"], d["time_us"], d["algbw_GBps"], d["busbw_GBps"],
                            d["wrong"], d["checked"], d["inplace"], d["graph"]))
    return rows


def run(timeout: float = 300, env: Optional[dict] = None, **kw) -> List[Row]:
    """Runs the harness; ``env`` adds variables (RCCL knobs) on top of this process's environment."""
    full_env = dict(os.environ, **(env or {}))
    r = subprocess.run(command(**kw), capture_output=True, text=True, timeout=timeout, env=full_env)
    if r.returncode not in (0, 3):
        raise RuntimeError(f"netop-rccl-bench failed ({r.returncode}): {r.stderr[-2000:]}")
    return parse(r.stdout)

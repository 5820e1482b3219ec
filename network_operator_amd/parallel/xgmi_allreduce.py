"""Driver for ``netop-xgmi-allreduce`` (native/hip/xgmi_allreduce.hip): a two-shot all-reduce
that drives every xGMI link of an MI355X node at once (pull or push data movement), checked
exactly, reported next to RCCL by ``bench.py``."""

from __future__ import annotations

import json
import subprocess
from typing import List, Optional

from ..utils.paths import native_bin


def command(ranks: Optional[int] = None, min_bytes: int = 1 << 20, max_bytes: int = 1 << 30, factor: float = 4,
            iters: int = 20, warmup: int = 5, mode: str = "both", wg_per_cu: int = 4) -> List[str]:
    if mode not in ("pull", "push", "both"):
        raise ValueError(mode)
    cmd = [str(native_bin("netop-xgmi-allreduce")), "-b", str(min_bytes), "-e", str(max_bytes), "-f", str(factor),
           "-n", str(iters), "-w", str(warmup), "--mode", mode, "--wg-per-cu", str(wg_per_cu)]
    if ranks:
        cmd += ["--ranks", str(ranks)]
    return cmd


def parse(stdout: str) -> List[dict]:
    return [json.loads(line) for line in stdout.splitlines() if line.strip().startswith("{")]


def run(timeout: float = 300, **kw) -> List[dict]:
    r = subprocess.run(command(**kw), capture_output=True, text=True, timeout=timeout)
    if r.returncode not in (0, 3):
        raise RuntimeError(f"netop-xgmi-allreduce failed ({r.returncode}): {r.stderr[-2000:]}")
    return parse(r.stdout)


def soak(ranks: Optional[int] = None, max_bytes: int = 64 << 20, calls: int = 1000, timeout: float = 60) -> dict:
    """``--soak``: `calls` all-reduces of random sizes up to `max_bytes`, pull and push in turn,
    every one on fresh data and checked exactly.  Returns the binary's document (``wrong`` per
    mode; the binary exits 3 when any element was wrong, which is reported, not raised)."""
    cmd = [str(native_bin("netop-xgmi-allreduce")), "-e", str(max_bytes), "--mode", "both", "--soak", str(calls)]
    if ranks:
        cmd += ["--ranks", str(ranks)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout)
    docs = parse(r.stdout)
    if r.returncode not in (0, 3) or not docs:
        raise RuntimeError(f"netop-xgmi-allreduce --soak failed ({r.returncode}): {r.stderr[-2000:]}")
    return docs[-1]

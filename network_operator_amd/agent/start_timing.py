"""The node agent's start on a node's real sysfs, repeated: every phase that needs no privileges,
as the agent itself times them (status.json ``phases_ms``), and the wall time of the process.

``discover --dry-run`` with the operator's MI355X flags (``--require-rdma``, ``--xgmi-expect=0``,
``--rccl-topo``, ``--rccl-env``): discovery, the KFD xGMI mesh, GPUDirect RDMA detection, the GPUs'
``gpu_metrics`` link state (bounded, concurrent), the PCIe link reads and the RCCL topology file.
Link-up, LLDP and the netlink writes need NET_ADMIN / NET_RAW; the netns harness measures them.
Used by ``bench.py`` (``node_ready_gpu_side.agent_binary``) and ``tools/agent_start_box.py``."""

from __future__ import annotations

import json
import os
import subprocess
import tempfile
import time
from pathlib import Path
from typing import Optional

from ..utils.paths import native_bin


def _pct(xs, q):
    xs = sorted(xs)
    return round(xs[min(len(xs) - 1, int(q * (len(xs) - 1) + 0.5))], 4) if xs else None


def measure(runs: int = 30, sysfs: str = "", timeout: float = 60) -> dict:
    """Per-phase p50 / p95 / max (ms) over `runs` dry runs, and the process wall time."""
    env = dict(os.environ)
    if sysfs:
        env["SYSFS_ROOT"] = sysfs
    phases: dict = {}
    wall = []
    last: dict = {}
    with tempfile.TemporaryDirectory() as tmp:
        for i in range(runs):
            st = Path(tmp) / "status.json"
            cmd = [str(native_bin("discover")), "--dry-run", "--mode=L3", "--require-rdma", "--xgmi-expect=0",
                   f"--rccl-topo={tmp}/rccl-topo.xml", f"--rccl-env={tmp}/rccl.env", f"--status-file={st}"]
            t = time.perf_counter()
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env)
            wall.append((time.perf_counter() - t) * 1e3)
            if r.returncode != 0:
                return {"error": f"run {i}: rc {r.returncode}", "stderr": r.stderr[-2000:]}
            last = json.loads(st.read_text())
            for k, v in (last.get("phases_ms") or {}).items():
                phases.setdefault(k, []).append(float(v))
            # The topology file is reused within a boot when nothing changed (its key file): the
            # first run generates it, later ones check the key.  Measure generation every time.
            for f in ("rccl-topo.xml", "rccl-topo.xml.key"):
                (Path(tmp) / f).unlink(missing_ok=True)
    return {
        "what": "discover --dry-run on this node's real sysfs (unprivileged phases of the agent's start)",
        "runs": runs,
        "phases_ms": {k: {"p50": _pct(v, 0.5), "p95": _pct(v, 0.95), "max": round(max(v), 4)} for k, v in phases.items()},
        "process_wall_ms": {"p50": _pct(wall, 0.5), "p95": _pct(wall, 0.95), "max": round(max(wall), 4)},
        "xgmi_pairs": last.get("xgmi_pairs"),
        "xgmi_links": last.get("xgmi_links"),
        "gpudirect_rdma": last.get("gpudirect_rdma"),
        "nics_in_this_netns": len(last.get("interfaces") or []),
        "nics_not_in_this_netns": [x for x in (last.get("not_in_netns") or "").split(",") if x],
        "nics_without_rdma": last.get("nics_without_rdma"),
    }


def main(argv: Optional[list] = None) -> int:
    import argparse

    ap = argparse.ArgumentParser(prog="python -m network_operator_amd.agent.start_timing")
    ap.add_argument("--runs", type=int, default=30)
    ap.add_argument("--sysfs", default="")
    a = ap.parse_args(argv)
    out = measure(a.runs, a.sysfs)
    print(json.dumps(out))
    return 1 if "error" in out else 0


if __name__ == "__main__":
    raise SystemExit(main())

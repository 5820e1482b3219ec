#!/usr/bin/env python3
"""A/B of two node-agent builds on the netns harness: node-ready latency and the agent's phase
timings, the two builds' bring-ups interleaved (A, B, B, A, ...) so that machine load drifts
affect both alike.

Each bring-up is ``testing.netns.run_isolated`` (a private network namespace, N veth NICs in a
fake sysfs copy of an 8xMI355X node, a fast-starting synthetic LLDP switch), with
``NETOP_BIN_DIR`` pointing at one build's ``discover``.  Build the other side from its commit,
e.g. ``git worktree add /tmp/old <sha> && cmake -S /tmp/old/native -B /tmp/oldb -G Ninja
-DNETOP_PYTHON=OFF -DNETOP_OUT=/tmp/oldb/out && cmake --build /tmp/oldb``.

    python bench/agent_ab.py --a /tmp/oldb/out/bin --b network_operator_amd/_lib/bin --runs 16
"""

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from network_operator_amd.testing import netns  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--a", required=True, help="directory holding build A's discover")
    ap.add_argument("--b", required=True, help="directory holding build B's discover")
    ap.add_argument("--runs", type=int, default=16, help="bring-ups per build")
    ap.add_argument("--nics", type=int, default=8)
    ap.add_argument("--mode", choices=["L2", "L3"], default="L3")
    ap.add_argument("--seed", type=int, default=7)
    a = ap.parse_args()
    ok, why = netns.available()
    if not ok:
        print(json.dumps({"error": f"netns harness unavailable: {why}"}))
        return 2
    sides = {"a": {"dir": os.path.abspath(a.a), "latency_ms": [], "phases_ms": {}},
             "b": {"dir": os.path.abspath(a.b), "latency_ms": [], "phases_ms": {}}}
    for k in range(a.runs):
        for name in (("a", "b") if k % 2 == 0 else ("b", "a")):
            s = sides[name]
            os.environ["NETOP_BIN_DIR"] = s["dir"]
            r = netns.run_isolated(n_nics=a.nics, seed=a.seed * 1000 + k, interval="30s", fast_start=True, verbose=0,
                                   mode=a.mode, link_state=False,  # (flags builds before rounds 5 and 6 lack)
                                   require_rdma=False)
            if not r["ready"]:
                raise RuntimeError(f"{name} run {k} did not become ready: {r['agent_log'][-2000:]}")
            s["latency_ms"].append(r["latency_s"] * 1e3)
            for ph, v in ((r.get("status") or {}).get("phases_ms") or {}).items():
                s["phases_ms"].setdefault(ph, []).append(v)
    os.environ.pop("NETOP_BIN_DIR", None)
    out = {"nics": a.nics, "mode": a.mode, "runs_per_build": a.runs, "switch": "fast start"}
    for name, s in sides.items():
        out[name] = {"dir": s["dir"], "latency_p50_ms": round(statistics.median(s["latency_ms"]), 3),
                     "latency_max_ms": round(max(s["latency_ms"]), 3),
                     "phases_p50_ms": {ph: round(statistics.median(v), 3) for ph, v in sorted(s["phases_ms"].items())}}
    out["b_minus_a_p50_ms"] = round(out["b"]["latency_p50_ms"] - out["a"]["latency_p50_ms"], 3)
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())

"""Local-HBM rate of the n-way bf16 sum (netop_sum_bf16, the reduce step of the direct xGMI
all-reduce) on one GPU: n source buffers, one output, each `--mib` MiB.  Traffic per call is
(n + 1) x the buffer; the rate is that over the median of `--iters` calls (HIP events).  Sweeps
the workgroups per CU.  Prints one JSON object.

    python tools/sum_rate_box.py [--mib 256] [--iters 20]"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from network_operator_amd.ops import hip  # noqa: E402


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--sources", default="2,4,8")
    ap.add_argument("--wg-per-cu", default="0,2,4,8,16")
    a = ap.parse_args(argv)
    n_elems = a.mib * (1 << 20) // 2
    rows = []
    for n in [int(x) for x in a.sources.split(",")]:
        srcs = [torch.randn(n_elems, device="cuda", dtype=torch.float32).to(torch.bfloat16) for _ in range(n)]
        out = torch.empty(n_elems, device="cuda", dtype=torch.bfloat16)
        acc = srcs[0].float()
        for s in srcs[1:]:  # the kernel's order: fp32 adds source by source, one RNE rounding
            acc += s.float()
        ref = acc.to(torch.bfloat16)
        del acc
        for wg in [int(x) for x in a.wg_per_cu.split(",")]:
            hip.sum_bf16(srcs, out, wg)
            torch.cuda.synchronize()
            exact = bool(torch.equal(out, ref))
            times = []
            for _ in range(a.iters):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                hip.sum_bf16(srcs, out, wg)
                e1.record()
                e1.synchronize()
                times.append(e0.elapsed_time(e1) * 1e-3)
            t = sorted(times)[len(times) // 2]
            rows.append({"sources": n, "wg_per_cu": wg or "library default (2)", "mib": a.mib, "median_us": round(t * 1e6, 2),
                         "TBps": round((n + 1) * a.mib * (1 << 20) / t / 1e12, 3), "exact_vs_fp32_sum": exact})
        del srcs, out, ref
        torch.cuda.empty_cache()
    print(json.dumps({"what": "netop_sum_bf16 on local HBM: (n+1) x buffer bytes per call", "rows": rows}))
    return 0


if __name__ == "__main__":
    sys.exit(main())

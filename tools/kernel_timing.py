"""Times the HIP validation kernels (fill / verify, one rank and an 8-rank expected sum) at the
bench's sizes and prints achieved HBM bandwidth from HIP events; run under rocprofv3 for the
per-kernel table."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from network_operator_amd.ops import hip  # noqa: E402


def timed(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e-3


out = []
for nbytes in (64 << 20, 1 << 30):
    t = torch.empty(nbytes // 2, dtype=torch.bfloat16, device="cuda")
    for world in (1, 8):
        f = timed(lambda: hip.fill_expected_sum(t, 7, world))
        v = timed(lambda: hip.verify_sum(t, 7, world))
        assert hip.verify_sum(t, 7, world) == 0
        out.append({"bytes": nbytes, "ranks": world, "fill_us": round(f * 1e6, 2), "fill_TBps": round(nbytes / f / 1e12, 2),
                    "verify_call_us_incl_sync": round(v * 1e6, 2)})
    del t
print(json.dumps(out))

#!/usr/bin/env python3
"""Node scale-out-ready latency (the first half of BASELINE.json's metric).

Fresh node bring-ups in private network namespaces (veth "NICs", synthetic 802.1AB switch,
fake sysfs of a real 8x MI355X node, the real C++ agent).  Measures t(agent start) ->
t(NFD readiness label written), against two switch behaviours:

* fast_start_switch: IEEE 802.1AB-2009 switch (fast transmission on a new neighbour);
* legacy_switch:     periodic LLDP only (msgTxInterval, 30 s by default).

For every run the harness also reports ``reference_model_s``: when the switch's first
*periodic* LLDPDU reached the last NIC — the earliest an agent that never transmits
(the reference's pcap listener) could have configured the node, before adding libpcap's
delivery delay.  Prints one JSON document.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from network_operator_amd.testing import netns  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--nics", type=int, default=8)
    ap.add_argument("--runs", type=int, default=5)
    ap.add_argument("--interval", default="30s")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--mode", choices=["L2", "L3"], default="L3")
    ap.add_argument("--matrix", action="store_true",
                    help="L2 and L3 x {1,2,4,8} NICs, fast-start switch only (BASELINE.md measurement plan)")
    a = ap.parse_args()
    ok, why = netns.available()
    if not ok:
        print(json.dumps({"error": f"netns harness unavailable: {why}"}))
        return 2
    if a.matrix:
        rows = []
        for mode in ("L2", "L3"):
            for n in (1, 2, 4, 8):
                r = netns.node_ready_bench(n_nics=n, runs=a.runs, interval=a.interval, seed=a.seed, legacy=False,
                                           mode=mode)
                f = r["fast_start_switch"]
                rows.append({"mode": mode, "nics": n, "runs": a.runs, "p50_s": f["p50_s"], "p95_s": f["p95_s"],
                             "max_s": f["max_s"],
                             # L2 has no LLDP phase: the reference's LLDP-bound model does not apply.
                             "reference_model_p50_s": f["reference_model_p50_s"] if mode == "L3" else None})
        print(json.dumps({"interval": a.interval, "matrix": rows}))
        return 0
    res = netns.node_ready_bench(n_nics=a.nics, runs=a.runs, interval=a.interval, seed=a.seed, mode=a.mode)
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    sys.exit(main())

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
    a = ap.parse_args()
    ok, why = netns.available()
    if not ok:
        print(json.dumps({"error": f"netns harness unavailable: {why}"}))
        return 2
    res = netns.node_ready_bench(n_nics=a.nics, runs=a.runs, interval=a.interval, seed=a.seed)
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    sys.exit(main())

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

``--e2e`` measures the same from the control plane's side: the time from creating the
NetworkClusterPolicy to the scale-out label on the Node object and to the policy's
``All good`` (operator, DaemonSet, simulated kubelet + NFD, real agent; ``testing/e2e.py``).
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
    ap.add_argument("--e2e", action="store_true",
                    help="whole chain from `kubectl apply` of the policy: operator, DaemonSet, simulated kubelet and "
                         "NFD, real agent (testing/e2e.py); reports policy -> Node label and -> status 'All good'")
    ap.add_argument("--fabric-nodes", type=int, default=0,
                    help="with --e2e: N simulated nodes on one routing leaf, one policy (testing/e2e.py run_fabric)")
    a = ap.parse_args()
    ok, why = netns.available()
    if not ok:
        print(json.dumps({"error": f"netns harness unavailable: {why}"}))
        return 2
    if a.e2e:
        import statistics

        from network_operator_amd.testing import e2e

        if a.fabric_nodes:
            runs = [e2e.run_isolated(fabric=True, n_nodes=a.fabric_nodes, n_nics=a.nics, seed=a.seed * 1000 + k,
                                     collective=False) for k in range(a.runs)]
            out = {"nodes": a.fabric_nodes, "nics_per_node": a.nics, "runs": a.runs}
            for k in ("policy_to_all_nodes_labelled_s", "policy_to_all_good_s", "delete_to_all_nodes_clean_s"):
                xs = [r[k] for r in runs]
                ok_xs = sorted(x for x in xs if x is not None)
                out[k] = {"p50": statistics.median(ok_xs) if ok_xs else None, "max": ok_xs[-1] if ok_xs else None,
                          "failed": sum(1 for x in xs if x is None), "all": xs}
            print(json.dumps(out))
            return 0
        keys = ("policy_to_daemonset_s", "policy_to_agent_start_s", "policy_to_node_label_s", "policy_to_all_good_s",
                "delete_to_agent_stopped_s", "delete_to_label_removed_s")
        runs = [e2e.run_isolated(n_nics=a.nics, mode=a.mode, seed=a.seed * 1000 + k, interval=a.interval)
                for k in range(a.runs)]
        out = {"mode": a.mode, "nics": a.nics, "runs": a.runs, "interval": a.interval}
        for k in keys:
            xs = [r[k] for r in runs]
            ok_xs = sorted(x for x in xs if x is not None)
            out[k] = {"p50": statistics.median(ok_xs) if ok_xs else None, "max": ok_xs[-1] if ok_xs else None,
                      "failed": sum(1 for x in xs if x is None), "all": xs}
        print(json.dumps(out))
        return 0
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

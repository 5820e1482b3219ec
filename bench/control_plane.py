#!/usr/bin/env python3
"""Control-plane scale: how fast the operator converges on a large cluster, and its footprint.

A fake API server (``testing/fakeapi.py``: watch, status subresource, DaemonSet and pod
simulation) runs in this process with N GPU nodes; the real manager runs as a separate process
(``python -m network_operator_amd.operator.manager``) against it, so its RSS is its own.
Measured:

* ``daemonsets_s``:  P policies created -> P agent DaemonSets exist;
* ``targets_s``:     -> every policy's status.targets == the nodes of its pool;
* ``all_good_s``:    every agent on every node reports ready -> every policy "All good";
* ``manager_rss_mib``: the manager's peak RSS (VmHWM), against the Deployment's 128Mi limit
  (reference config/operator/manager/manager.yaml:95-101);
* ``requests``: API requests the manager made (informers, not polling);
* ``manager_cpu_s``: the manager's own CPU time over the run.  The wall-clock phases include the
  fake API server, a single Python process that also plays the DaemonSet controller and streams
  every Pod (realistic ones, kilobytes each) to the watchers.

With ``--keep-config`` the policies use ``keepConfigOnRestart``, and the run goes on to delete
them: ``delete_to_cleanup_jobs_s`` (every node's cleanup Job exists), then the simulated kubelets
complete them, and ``cleanup_done_to_gone_s`` (every policy finalized and gone).

The policies alternate between ``amd-so`` and ``host-nic`` and the nodes are split into
ceil(P/2) pools: each node runs one agent of each type (two policies of one type never share a
node -- the newer is held off, holdoff.hold_off_terms), so a run has 2N agent Pods for P >= 2.
(Until round 4 every policy was an amd-so on every node: P*N Pods, now a conflict by design.)

The reference has no equivalent measurement (controller-runtime + envtest, no scale test).

    python bench/control_plane.py --nodes 1000 --policies 4
"""

import argparse
import asyncio
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from network_operator_amd.api.v1alpha1 import types as T  # noqa: E402
from network_operator_amd.operator import kube  # noqa: E402
from network_operator_amd.testing.fakeapi import FakeApiServer  # noqa: E402

LABEL = "amd.feature.node.kubernetes.io/gpu-ready"


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cpu_s(pid: int) -> float:
    """utime + stime of the process (the manager's own CPU, apart from the fake API server's)."""
    with open(f"/proc/{pid}/stat") as f:
        fields = f.read().rsplit(")", 1)[1].split()
    return (int(fields[11]) + int(fields[12])) / os.sysconf("SC_CLK_TCK")


def _hwm_mib(pid: int) -> float:
    with open(f"/proc/{pid}/status") as f:
        line = next(x for x in f if x.startswith("VmHWM:"))
    return int(line.split()[1]) / 1024


async def _until(pred, timeout: float, poll: float = 0.005) -> float:
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < timeout:
        if pred():
            return time.perf_counter() - t0
        await asyncio.sleep(poll)
    raise TimeoutError(f"did not converge: {getattr(pred, '__name__', pred)} at line {pred.__code__.co_firstlineno}")


async def run(nodes: int, policies: int, timeout: float, keep: bool = False, validation: bool = False,
              overlap: bool = False) -> dict:
    """``overlap``: every policy an amd-so on every node (the pre-round-5 layout): the oldest holds
    the nodes, the others are held off all of them (targets 0), so the run measures what the
    hold-off costs at scale -- its node LISTs and the conflict reports -- instead of 2N agents."""
    fake = FakeApiServer(bookmark_interval=5.0)
    url = await fake.start()
    pools = max(1, (policies + 1) // 2)
    for i in range(nodes):
        fake.add_node(f"gpu-node-{i:04d}", {LABEL: "true", "pool": str(i % pools)})
    pool_size = {k: sum(1 for i in range(nodes) if i % pools == k) for k in range(pools)}
    env = dict(os.environ, PYTHONPATH=ROOT, OPERATOR_NAMESPACE="amd-network-operator", ENABLE_WEBHOOKS="false")
    # The manager's log goes to a file: a pipe nobody reads fills up and blocks it (one log line
    # per cleanup Job at scale).
    import tempfile

    log = tempfile.NamedTemporaryFile(prefix="netop-cp-manager-", suffix=".log", delete=False)
    proc = subprocess.Popen([sys.executable, "-m", "network_operator_amd.operator.manager", "--master", url,
                             f"--health-probe-bind-address=127.0.0.1:{_port()}", "--metrics-bind-address=0"],
                            env=env, stdout=subprocess.DEVNULL, stderr=log)
    try:
        await asyncio.sleep(1.0)  # manager start: informers list + watch
        n_req0 = len(fake.requests)
        cpu0 = _cpu_s(proc.pid)
        P = kube.NETWORKCLUSTERPOLICIES
        names = [f"policy-{k}" for k in range(policies)]
        want = {n: pool_size[k // 2] for k, n in enumerate(names)}
        amd = [n for k, n in enumerate(names) if k % 2 == 0]
        if overlap:
            want = {n: nodes if k == 0 else 0 for k, n in enumerate(names)}
            amd = list(names)
        t0 = time.perf_counter()
        for k, n in enumerate(names):
            sel = {LABEL: "true", "pool": str(k // 2)}
            if overlap:
                pol = T.new_policy(n, keepConfigOnRestart=keep, node_selector={LABEL: "true"},
                                   validation={"enabled": True} if validation else None)
                fake._create(P, pol.to_dict(), None)
                continue
            if k % 2 == 0:
                pol = T.new_policy(n, keepConfigOnRestart=keep, node_selector=sel,
                                   validation={"enabled": True} if validation else None)
            else:
                pol = T.new_host_nic_policy(n, keepConfigOnRestart=keep, node_selector=sel)
            fake._create(P, pol.to_dict(), None)

        def ds_all():
            return all(fake.get_object(kube.DAEMONSETS, n, "amd-network-operator") for n in names)

        def targets_all():
            return all((fake.get_object(P, n).get("status") or {}).get("targets") == want[n] for n in names)

        await _until(ds_all, timeout)
        t_ds = time.perf_counter() - t0
        await _until(targets_all, timeout)
        t_targets = time.perf_counter() - t0
        t1 = time.perf_counter()
        for i in range(nodes):
            for k, n in enumerate(names):
                if (k == 0) if overlap else (i % pools == k // 2):
                    fake.node_ready[(f"amd-network-operator/{n}", f"gpu-node-{i:04d}")] = True
        fake._sync_daemonsets()

        def good_all():  # a policy held off every node has no targets (and says why in its errors)
            return all((fake.get_object(P, n).get("status") or {}).get("state") ==
                       ("All good" if want[n] else "No targets") for n in names)

        await _until(good_all, timeout)
        t_good = time.perf_counter() - t1
        if validation:  # every ready node gets its validation Job; the simulated kubelets pass them
            t_v = time.perf_counter()
            await _until(lambda: len(fake._table(kube.JOBS)) == sum(want[n] for n in amd), timeout, poll=0.05)
            jobs_s = time.perf_counter() - t_v
            for j in fake.list_objects(kube.JOBS):
                fake.set_job_result(j["metadata"]["name"], "amd-network-operator", True)

            def validated_all():
                for n in amd:
                    c = {x["type"]: x for x in (fake.get_object(P, n).get("status") or {}).get("conditions") or []}
                    if (c.get("FabricValidated") or {}).get("reason") != "AllNodesValidated":
                        return False
                return True
            await _until(validated_all, timeout, poll=0.05)
        await asyncio.sleep(0.5)
        if overlap:
            out_conflicts = {n: len([e for e in (fake.get_object(P, n).get("status") or {}).get("errors") or []
                                     if "also selected by policy" in e]) for n in names}
        out = {"nodes": nodes, "policies": policies, "pods": sum(want.values()), "daemonsets_s": round(t_ds, 4),
               "targets_s": round(t_targets, 4), "all_good_s": round(t_good, 4)}
        if overlap:
            out["layout"] = "overlap: every policy amd-so on every node"
            out["conflict_entries"] = out_conflicts
        if validation:
            out.update(ready_to_validation_jobs_s=round(jobs_s, 4),
                       jobs_done_to_validated_s=round(time.perf_counter() - t_v - jobs_s, 4))
        if keep:
            await _until(lambda: all(len((fake.get_object(P, n).get("status") or {}).get("keptNodes") or []) == want[n]
                                     for n in names), timeout)
            t2 = time.perf_counter()
            for n in names:
                fake._delete_or_mark(P, n, "")
            await _until(lambda: len(fake._table(kube.JOBS)) == sum(want.values()), timeout, poll=0.05)
            out["delete_to_cleanup_jobs_s"] = round(time.perf_counter() - t2, 4)
            t3 = time.perf_counter()
            for j in fake.list_objects(kube.JOBS):
                fake.set_job_result(j["metadata"]["name"], "amd-network-operator", True)
            await _until(lambda: not any(fake.get_object(P, n) for n in names), timeout, poll=0.05)
            out["cleanup_done_to_gone_s"] = round(time.perf_counter() - t3, 4)
        await asyncio.sleep(0.5)
        rss = _hwm_mib(proc.pid)
        out.update(manager_rss_mib=round(rss, 1), manager_limit_mib=128, requests=len(fake.requests) - n_req0,
                   manager_cpu_s=round(_cpu_s(proc.pid) - cpu0, 2))
        return out
    except Exception:
        log.flush()
        print(open(log.name, errors="replace").read()[-4000:], file=sys.stderr)
        raise
    finally:
        proc.terminate()
        try:
            proc.wait(10)
        except subprocess.TimeoutExpired:
            proc.kill()
        await fake.stop()


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--nodes", type=int, default=1000)
    ap.add_argument("--policies", type=int, default=4)
    ap.add_argument("--timeout", type=float, default=300)
    ap.add_argument("--keep-config", action="store_true", help="keepConfigOnRestart policies, then delete them")
    ap.add_argument("--validation", action="store_true", help="fabric validation Jobs on every ready node")
    ap.add_argument("--overlap", action="store_true",
                    help="every policy an amd-so on every node: one holds them, the others are held off")
    a = ap.parse_args()
    print(json.dumps(asyncio.run(run(a.nodes, a.policies, a.timeout, a.keep_config, a.validation, a.overlap))))
    return 0


if __name__ == "__main__":
    sys.exit(main())

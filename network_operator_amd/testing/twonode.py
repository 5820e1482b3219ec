"""Two-node L3 fabric harness: two agents, one routing switch, a collective across the nodes.

BASELINE.json config "L3 mode, 2 nodes: /16 route install + cross-node RoCE, rccl-tests
all-reduce across nodes", reproduced without hardware::

    node A netns (this process)         switch netns (child)            node B netns (child)
    enp5s0np0 .. (veth)          <->    swp0 .. swpN-1
                                        swpN .. swp2N-1          <->    enp5s0np0 .. (veth)
    discover (agent A)                  netop-lldp-tx --assign-ip       discover (agent B)
                                        ip_forward = 1 (the leaf
                                        routes between the /30s)

Both agents learn their /30s from LLDP and install the ``/16 via <switch port>`` routes.  A
``torch.distributed`` gloo all-reduce then runs between one process per node.  The process
on node A (rank 0) and the process on node B (rank 1) bind to their first scale-out NIC
(``GLOO_SOCKET_IFNAME``).  They rendezvous on node A's scale-out address, so every byte of the
collective crosses the configured fabric: node A NIC, /16 route, switch forwarding, node B NIC.
RoCE itself cannot be emulated on veths.  The IP layer that RCCL's RoCE v2 traffic is routed
over is exactly what this exercises.

Run through ``run_isolated_two_nodes()`` (a fresh namespace per run).
"""

from __future__ import annotations

import argparse
import json
import os
import random
import shutil
import signal
import subprocess
import sys
import tempfile
import time
from pathlib import Path

from .netns import CLONE_NEWNET, _native, _wait_for, random_plan, unshare_cmd

_WORKER = r"""
import json, os, sys, time
import torch, torch.distributed as dist
from datetime import timedelta
rank = int(os.environ["RANK"])
t0 = time.monotonic()
dist.init_process_group("gloo", init_method=os.environ["INIT"], rank=rank, world_size=2,
                        timeout=timedelta(seconds=60))
t_init = time.monotonic() - t0
x = torch.full((1 << 20,), float(rank + 1))
dist.all_reduce(x)
ok = bool(torch.all(x == 3.0))
big = torch.ones(16 << 20)            # 64 MiB of fp32
dist.all_reduce(big); dist.barrier()
t1 = time.monotonic()
for _ in range(3):
    dist.all_reduce(big)
dt = (time.monotonic() - t1) / 3
nbytes = big.numel() * 4
out = {"rank": rank, "ok": ok and bool(torch.all(big == 2.0 ** 4)), "init_s": t_init, "allreduce_64MiB_s": dt,
       "busbw_GBps": nbytes / dt / 1e9 * 2 * (2 - 1) / 2}
print(json.dumps(out), flush=True)
dist.destroy_process_group()
"""


def _worker_env(rank: int, ifname: str, master: str, port: int) -> dict:
    root = Path(__file__).resolve().parents[2]
    return dict(os.environ, RANK=str(rank), GLOO_SOCKET_IFNAME=ifname, INIT=f"tcp://{master}:{port}",
                PYTHONPATH=str(root), OMP_NUM_THREADS="1")


def _agent_args(tmp: Path, tag: str, wait: str) -> list:
    from ..utils.paths import native_bin

    feat = tmp / f"features-{tag}"
    feat.mkdir(exist_ok=True)
    return [str(native_bin("discover")), "--configure=true", "--keep-running", "--mode=L3", "--mtu=9000",
            f"--wait={wait}", f"--rccl-net={tmp / f'rccl-net-{tag}.json'}", f"--rccl-env={tmp / f'rccl-{tag}.env'}",
            f"--status-file={tmp / f'status-{tag}.json'}", f"--nfd-features-dir={feat}", "--xgmi-expect=0", "-v=1"]


def run_two_nodes(n_nics: int = 2, seed: int | None = None, wait: str = "30s", collective: bool = True) -> dict:
    """Must already run inside a private network namespace (node A)."""
    import ctypes
    import ctypes.util

    from . import fakesysfs
    from ..utils.paths import native_bin

    nat = _native()
    rng = random.Random(seed)
    rt = nat.Rtnl()
    rt.link_set_up(rt.link_by_name("lo")["index"])
    libc = ctypes.CDLL(ctypes.util.find_library("c"), use_errno=True)
    tmp = Path(tempfile.mkdtemp(prefix="netop-2node-"))
    res: dict = {"n_nics": n_nics}
    children = []
    agents = []
    try:
        for tag in ("A", "B"):
            fakesysfs.build_mi355x_node(tmp / f"sys{tag}", n_gpus=n_nics)
        nics = [p["nic"] for p in nat.discover(str(tmp / "sysA"))["pairs"]][:n_nics]
        plan = random_plan(2 * n_nics, rng)
        res["plan"] = plan
        res["nics"] = nics

        def fork_ns(body):
            r, w = os.pipe()
            r2, w2 = os.pipe()
            pid = os.fork()
            if pid == 0:
                code = 1
                try:
                    os.close(r)
                    os.close(w2)
                    if libc.unshare(CLONE_NEWNET) != 0:
                        os._exit(3)
                    os.write(w, b"1")
                    os.read(r2, 1)  # "go": our veth ends have arrived
                    code = body() or 0
                except BaseException as e:  # noqa: BLE001 - report and exit the child
                    sys.stderr.write(f"child failed: {e!r}\n")
                finally:
                    os._exit(code)
            os.close(w)
            os.close(r2)
            os.read(r, 1)
            children.append(pid)
            return pid, w2

        # Switch: forwards between the /30s it owns (the leaf's routing), LLDP on every port.
        ports = [f"swp{i}" for i in range(2 * n_nics)]
        tx = [str(native_bin("netop-lldp-tx")), "--interval=30s", "--fast-start", "--assign-ip",
              f"--seed={rng.randrange(1, 1 << 30)}"] + [f"--port={p}={pl['desc']}" for p, pl in zip(ports, plan)]

        def switch():
            with open("/proc/sys/net/ipv4/ip_forward", "w") as f:
                f.write("1")
            devnull = os.open(os.devnull, os.O_WRONLY)
            os.dup2(devnull, 1)
            os.execv(tx[0], tx)

        sw_pid, sw_go = fork_ns(switch)

        # Node B: rename its veths to the real NIC names, run agent B, then the rank-1 worker.
        b_result = tmp / "B.json"
        port = 29500 + rng.randrange(0, 400)
        master = plan[0]["local"]  # node A's first scale-out address

        def node_b():
            rtb = _native().Rtnl()
            rtb.link_set_up(rtb.link_by_name("lo")["index"])
            for i, name in enumerate(nics):
                rtb.link_set_name(rtb.link_by_name(f"tb{i}")["index"], name)
            env = dict(os.environ, SYSFS_ROOT=str(tmp / "sysB"), NODE_NAME="mi355x-node-b")
            t0 = time.monotonic()
            ag = subprocess.Popen(_agent_args(tmp, "B", wait), env=env, stdout=subprocess.PIPE,
                                  stderr=subprocess.STDOUT, text=True)
            label = tmp / "features-B" / "scale-out-readiness.txt"
            t_ready = _wait_for(label, 5 + float(wait.rstrip("s")), ag)
            out = {"ready_s": (t_ready - t0) if t_ready else None}
            if t_ready and collective:
                w = subprocess.run([sys.executable, "-c", _WORKER], env=_worker_env(1, nics[0], master, port),
                                   capture_output=True, text=True, timeout=180)
                out["worker_rc"] = w.returncode
                out["worker"] = json.loads(w.stdout.strip().splitlines()[-1]) if w.returncode == 0 else w.stderr[-2000:]
            st = rtb.route_list()
            out["routes"] = [r for r in st if r.get("gateway")]
            ag.send_signal(signal.SIGTERM)
            log, _ = ag.communicate(timeout=30)
            out["agent_rc"] = ag.returncode
            out["agent_log"] = log[-3000:]
            b_result.write_text(json.dumps(out))
            return 0

        b_pid, b_go = fork_ns(node_b)

        # Wire the fabric.
        for i, name in enumerate(nics):
            rt.veth_add(name, ports[i])
            rt.link_set_netns_pid(rt.link_by_name(ports[i])["index"], sw_pid)
            rt.veth_add(f"tb{i}", ports[n_nics + i])
            rt.link_set_netns_pid(rt.link_by_name(ports[n_nics + i])["index"], sw_pid)
            rt.link_set_netns_pid(rt.link_by_name(f"tb{i}")["index"], b_pid)
        os.write(sw_go, b"1")
        os.write(b_go, b"1")

        env = dict(os.environ, SYSFS_ROOT=str(tmp / "sysA"), NODE_NAME="mi355x-node-a")
        t0 = time.monotonic()
        ag = subprocess.Popen(_agent_args(tmp, "A", wait), env=env, stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, text=True)
        agents.append(ag)
        t_ready = _wait_for(tmp / "features-A" / "scale-out-readiness.txt", 5 + float(wait.rstrip("s")), ag)
        res["A_ready_s"] = (t_ready - t0) if t_ready else None
        res["A_routes"] = [r for r in rt.route_list() if r.get("gateway")]
        if t_ready and collective:
            w = subprocess.run([sys.executable, "-c", _WORKER], env=_worker_env(0, nics[0], master, port),
                               capture_output=True, text=True, timeout=180)
            res["A_worker_rc"] = w.returncode
            res["A_worker"] = json.loads(w.stdout.strip().splitlines()[-1]) if w.returncode == 0 else w.stderr[-2000:]
        _, status = os.waitpid(b_pid, 0)
        children.remove(b_pid)
        res["B_exit"] = os.waitstatus_to_exitcode(status)
        res["B"] = json.loads(b_result.read_text()) if b_result.exists() else None
        ag.send_signal(signal.SIGTERM)
        log, _ = ag.communicate(timeout=30)
        res["A_agent_rc"] = ag.returncode
        res["A_agent_log"] = log[-3000:]
        for f in ("rccl-net-A.json", "rccl-net-B.json"):
            p = tmp / f
            res[f.split(".")[0].replace("-", "_")] = json.loads(p.read_text()) if p.exists() else None
        return res
    finally:
        for a in agents:
            if a.poll() is None:
                a.kill()
        for pid in children:
            try:
                os.kill(pid, signal.SIGKILL)
                os.waitpid(pid, 0)
            except OSError:
                pass
        shutil.rmtree(tmp, ignore_errors=True)


def run_isolated_two_nodes(timeout: float = 400, **kw) -> dict:
    cmd = [*unshare_cmd(), sys.executable, "-m", "network_operator_amd.testing.twonode", "--json", json.dumps(kw)]
    root = Path(__file__).resolve().parents[2]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=root,
                       env=dict(os.environ, PYTHONPATH=str(root)))
    if r.returncode != 0:
        raise RuntimeError(f"two-node scenario failed rc={r.returncode}: {r.stderr[-3000:]}")
    return json.loads(r.stdout.strip().splitlines()[-1])


def _main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default="{}")
    a = ap.parse_args(argv)
    print(json.dumps(run_two_nodes(**json.loads(a.json))))
    return 0


if __name__ == "__main__":
    sys.exit(_main())

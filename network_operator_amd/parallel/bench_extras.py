"""bench.py's diagnostics, each one a child process with a hard deadline.

The headline (the timed all-reduce with the agent's artifacts applied) is measured first, in the
rank processes.  Everything else rank 0 reports — RCCL with its defaults (the A/B), the HIP xGMI
link probe, the native RCCL harness, the direct xGMI all-reduce, the multi-process IPC
all-reduce, the netns node-ready harness — runs afterwards through :class:`Runner`:

* every extra is a separate process in its own session (``start_new_session``), and the whole
  tree below it is killed (psutil walk + ``killpg``) when its time is up;
* its time is ``min(own cap, deadline - now)``: an extra can never push the single JSON line
  past ``bench.py --deadline-s``;
* an extra that was killed is reported as ``{"error": "deadline"}`` (the global deadline) or
  ``{"error": "timed out"}`` (its own cap), never silently dropped.

``python -m network_operator_amd.parallel.bench_extras NAME JSON_KWARGS`` runs one extra and
prints its result as one JSON line.  Test hooks: ``NETOP_BENCH_HANG_EXTRA=NAME`` makes that extra
(or a bench.py started as that extra) sleep forever, to rehearse a hung first contact;
``NETOP_BENCH_FAKE_EXTRA_S=NAME=SECONDS[,...]`` makes the named extras stand-ins that take that
long and report ``{"fake": true}`` (the CPU rehearsal of the GPU extras' order and deadline).
"""

from __future__ import annotations

import json
import os
import signal
import subprocess
import sys
import threading
import time
from typing import Dict, List, Optional

HANG_ENV = "NETOP_BENCH_HANG_EXTRA"
FAKE_EXTRA_ENV = "NETOP_BENCH_FAKE_EXTRA_S"
NAME_ENV = "NETOP_BENCH_EXTRA_NAME"
LAUNCH_ENV = ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK", "ROLE_WORLD_SIZE",
              "MASTER_ADDR", "MASTER_PORT", "GROUP_WORLD_SIZE", "ROLE_NAME", "NETOP_BENCH_STORE")


def maybe_hang() -> None:
    """The test hook: a process started as extra NAME sleeps forever when NAME is the one to hang."""
    want = os.environ.get(HANG_ENV)
    if want and os.environ.get(NAME_ENV) == want:
        while True:
            time.sleep(3600)


def fake_seconds(name: str) -> Optional[float]:
    """The test hook: how long extra NAME's stand-in takes, when it has one."""
    for item in (os.environ.get(FAKE_EXTRA_ENV) or "").split(","):
        k, _, v = item.partition("=")
        if k.strip() == name and v.strip():
            return float(v)
    return None


def clean_env(env: Optional[dict] = None) -> dict:
    """The launcher's rank variables removed: a child bench.py must not think it is a rank."""
    env = dict(os.environ if env is None else env)
    return {k: v for k, v in env.items() if k not in LAUNCH_ENV and not k.startswith("TORCHELASTIC_")}


def kill_tree(p: subprocess.Popen) -> None:
    """SIGKILL the process, its session's group and every descendant (some extras start their own
    sessions for their ranks)."""
    procs = []
    try:
        import psutil

        root = psutil.Process(p.pid)
        procs = root.children(recursive=True)
    except Exception:
        pass
    try:
        os.killpg(p.pid, signal.SIGKILL)
    except (ProcessLookupError, PermissionError):
        pass
    for c in procs:
        try:
            c.kill()
        except Exception:
            pass
    try:
        p.kill()
    except ProcessLookupError:
        pass
    try:
        p.wait(10)
    except subprocess.TimeoutExpired:
        pass


def last_json(text: str) -> Optional[dict]:
    for line in reversed(text.splitlines()):
        line = line.strip()
        if line.startswith("{"):
            try:
                return json.loads(line)
            except ValueError:
                continue
    return None


class Runner:
    """Runs extras one after another against one absolute deadline (``time.monotonic()``)."""

    def __init__(self, deadline: float, base_env: Optional[dict] = None, margin_s: float = 3.0):
        self.deadline = deadline
        self.base_env = clean_env(base_env)
        repo = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        pp = self.base_env.get("PYTHONPATH")
        self.base_env["PYTHONPATH"] = repo + (os.pathsep + pp if pp else "")
        self.margin_s = margin_s
        self.live: Dict[int, subprocess.Popen] = {}
        self.lock = threading.Lock()
        self.log: List[dict] = []

    def left(self) -> float:
        return self.deadline - self.margin_s - time.monotonic()

    def run(self, name: str, cmd: List[str], cap_s: float, env: Optional[dict] = None) -> dict:
        """Runs ``cmd`` as extra ``name``; returns its last stdout JSON line, or an error record."""
        left = self.left()
        if left < 2:
            return {"error": "deadline", "detail": "not started: the bench deadline was reached"}
        budget = min(cap_s, left)
        full_env = dict(self.base_env, **(env or {}))
        full_env[NAME_ENV] = name
        t0 = time.monotonic()
        p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=full_env,
                             start_new_session=True)
        with self.lock:
            self.live[p.pid] = p
        try:
            so, se = p.communicate(timeout=budget)
        except subprocess.TimeoutExpired:
            kill_tree(p)
            try:
                p.communicate(timeout=5)
            except Exception:
                pass
            hit_deadline = budget < cap_s
            rec = {"error": "deadline" if hit_deadline else "timed out", "timed_out": True,
                   "seconds": round(time.monotonic() - t0, 1), "limit_s": round(budget, 1)}
            self.log.append({"extra": name, **rec})
            return rec
        finally:
            with self.lock:
                self.live.pop(p.pid, None)
        secs = round(time.monotonic() - t0, 1)
        self.log.append({"extra": name, "rc": p.returncode, "seconds": secs})
        doc = last_json(so)
        if doc is None:
            return {"error": f"rc={p.returncode}, no JSON result: {(se or so)[-400:]}", "seconds": secs}
        if p.returncode != 0 and "error" not in doc:
            doc = dict(doc, rc=p.returncode)
        return doc

    def extra(self, name: str, cap_s: float, env: Optional[dict] = None, **kwargs) -> dict:
        """Runs one of this module's extras (``EXTRAS[name]``) in a child process."""
        cmd = [sys.executable, "-m", "network_operator_amd.parallel.bench_extras", name, json.dumps(kwargs)]
        return self.run(name, cmd, cap_s, env)

    def kill_all(self) -> None:
        with self.lock:
            live = list(self.live.values())
        for p in live:
            kill_tree(p)


# ------------------------------------------------------------------------------------------
# The extras (run inside the child process)
# ------------------------------------------------------------------------------------------
def xgmi_probe(world: int) -> dict:
    """HIP xGMI link probe over the first ``world`` GPUs: per-link pull bandwidth and the
    all-peers pull / push aggregates, byte-exact."""
    from ..ops import hip as H

    r = H.xgmi_probe_isolated(64 << 20, iters=5, max_gpus=world, timeout=110)
    links = sorted(x for d, row in enumerate(r["link_GBps"]) for p, x in enumerate(row) if p != d)
    return {"gpus": r["gpus"], "errors": r["errors"] + r["push_errors"],
            "link_GBps": {"min": links[0], "median": links[len(links) // 2], "max": links[-1]} if links else None,
            "aggregate_GBps": {"min": min(r["aggregate_GBps"]), "max": max(r["aggregate_GBps"])},
            "push_aggregate_GBps": {"min": min(r["push_aggregate_GBps"]), "max": max(r["push_aggregate_GBps"])}}


def native_rccl(world: int, env_probe: bool = False) -> dict:
    """ROCm's RCCL linked directly (netop-rccl-bench, one process over ``world`` GPUs), every size
    checked exactly; runs with whatever RCCL environment the runner gave it (the artifacts)."""
    from . import rccl_bench

    rows = rccl_bench.run(op="all_reduce", gpus=world, min_bytes=1 << 20, max_bytes=1 << 30, factor=32, iters=20,
                          warmup=5, timeout=110)
    out = {"rows": [{"bytes": r.bytes, "time_us": r.time_us, "algbw_GBps": r.algbw_GBps, "busbw_GBps": r.busbw_GBps,
                     "wrong": r.wrong} for r in rows],
           "peak_busbw_GBps": max((r.busbw_GBps for r in rows), default=0.0),
           "rccl_env": {k: v for k, v in os.environ.items() if k.startswith(("NCCL_", "RCCL_"))}}
    if world > 1 and env_probe:
        out["env_probe"] = rccl_bench.env_probe(world, 1 << 30)
    return out


def _soak(fn) -> dict:
    try:
        return fn()
    except Exception as e:  # the timed rows stand without it
        return {"error": str(e)[-300:]}


def xgmi_allreduce(world: int, nbytes: int) -> dict:
    from . import xgmi_allreduce as XA

    out = {"rows": XA.run(ranks=world, min_bytes=nbytes, max_bytes=nbytes, iters=10, warmup=3, timeout=80)}
    # Then 1000 calls over the real links, every one checked (random sizes up to 64 MiB).
    out["soak"] = _soak(lambda: XA.soak(ranks=world, max_bytes=min(nbytes, 64 << 20), calls=1000, timeout=30))
    return out


def xgmi_comm(world: int, nbytes: int) -> dict:
    from . import xgmi_comm as XC

    out = XC.run(world, nbytes=nbytes, min_bytes=1 << 20, iters=10, warmup=3, timeout=80)
    out["soak"] = _soak(lambda: XC.run(world, nbytes=min(nbytes, 64 << 20), timeout=30, soak=1000))
    return out


def node_ready(n_nics: int, runs: int, required: bool = False) -> dict:
    from ..testing import netns

    why = netns.unavailable()  # structured: {"code", "why"}, never scraped from a child's last line
    if why is not None:
        if required:
            raise RuntimeError(why["why"])
        return {"unavailable": why}
    return {"result": netns.node_ready_bench(n_nics=max(n_nics, 1), runs=runs, legacy=False)}


def sleep(seconds: float) -> dict:
    """A do-nothing extra (tests)."""
    time.sleep(seconds)
    return {"slept": seconds}


EXTRAS = {"xgmi_probe": xgmi_probe, "native_rccl": native_rccl, "xgmi_allreduce": xgmi_allreduce,
          "xgmi_comm": xgmi_comm, "node_ready": node_ready, "sleep": sleep}


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    name = argv[0]
    kwargs = json.loads(argv[1]) if len(argv) > 1 else {}
    maybe_hang()
    fake = fake_seconds(name)
    if fake is not None:
        time.sleep(fake)
        print(json.dumps({"fake": True, "extra": name, "kwargs": kwargs}), flush=True)
        return 0
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    if root not in sys.path:
        sys.path.insert(0, root)
    try:
        doc = EXTRAS[name](**kwargs)
    except Exception as e:  # reported, never fatal to the bench
        print(json.dumps({"error": f"{type(e).__name__}: {str(e)[-500:]}"}), flush=True)
        return 1
    print(json.dumps(doc), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())

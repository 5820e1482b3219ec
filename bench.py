#!/usr/bin/env python3
"""Headline benchmark: RCCL all-reduce bus bandwidth on MI355X *with the operator's artifacts
applied* (+ node-ready latency).

BASELINE.json metric: "node scale-out-ready latency (s) + rccl all-reduce busbw GB/s at
1/2/4/8 GPU", config "L3 mode, 8xMI355X single node: all xGMI + host RoCE links configured,
rccl-tests 8-GPU all-reduce".

* **What is measured is the configured fabric, not stock RCCL.**  Before any rank creates an
  RCCL communicator, rank 0 runs the node agent itself, unprivileged, on this node
  (``discover --dry-run --rccl-topo=… --rccl-env=…``: its ``NCCL_TOPO_FILE`` and the
  intra-node part of ``rccl.env``), and hands the files to every rank through the rendezvous
  store; every rank exports them, and rank 0 also sets ``NCCL_TOPO_DUMP_FILE``.  The reference's
  node artifact exists for the collective library in the same way (HCCL reads gaudinet.json,
  reference cmd/discover/gaudinet.go:28-89).  ``--artifacts DIR`` applies an existing artifact
  directory instead (``rccl.env`` + ``rccl-tuned.env``, e.g. /etc/amd/scale-out on a configured
  node); ``--artifacts off`` runs RCCL's defaults.
* One process per GPU, ``torch.distributed`` backend ``nccl`` (= RCCL over xGMI on ROCm).
  Under ``torchrun --nproc-per-node N`` the launcher's ranks are used (WORLD_SIZE must equal
  ``--gpus``); a bare ``python bench.py --gpus N`` starts the N rank processes itself.
  ``config.model`` names the BASELINE.json config of the world size that actually ran.  A
  *step* is one in-place bf16 all-reduce of ``--bytes`` per rank (default 1 GiB, rccl-tests'
  large-message regime); ``--warmup`` untimed steps, then exactly ``--steps`` timed steps
  bracketed by barrier + ``torch.cuda.synchronize()``, max over ranks.
* ``value`` is the job aggregate the driver's contract asks for: rccl-tests busbw (algbw *
  2(n-1)/n, a per-GPU figure) times n, with the artifacts applied.  The per-GPU figures, the
  ones rccl-tests prints and BASELINE's metric names, are ``busbw_GBps`` (artifacts) and
  ``busbw_rccl_defaults_GBps`` (the same loop in fresh rank processes without them); the A/B on
  the aggregate basis is ``value`` vs ``aggregate_busbw_rccl_defaults_GBps``.  The ceiling
  ``busbw_ceiling_GBps`` is per GPU too: (n-1) xGMI links x their rate.
  ``agent_artifacts`` says what was applied (file bytes, per-rank record) and what RCCL made of
  it (its dump: xGMI links seen per GPU — n-1 expected — and GPU / NIC ancestry vs the file's).
  At n > 1 the run exits non-zero (after printing its line) only when the file is to blame:
  RCCL sees fewer xGMI links under it than without it (``xgmi_links_check.file_blamed``), or
  the artifacts were not applied.  A dump that cannot settle it is reported, not failed.
* Order and deadline: verification and the timed loop come first; every diagnostic after it
  (RCCL defaults, xGMI probe, native harness, direct / IPC all-reduce, netns node-ready) is a
  child process killed at ``--deadline-s`` (``parallel/bench_extras.py``), and a watchdog in
  rank 0 prints the line with whatever was measured when the deadline passes.  Exactly one JSON
  line, always.
* At n = 1 there are no links and busbw is 0 by definition; the single-rank all-reduce is a
  no-op, so algbw is reported as null with the reason, and ``node_ready_gpu_side`` times the
  agent phases that run unprivileged on the box (``agent_binary``: ten dry runs of the real
  ``discover`` with the operator's flags, its own phase timings and the process wall time).  The netns node-ready harness needs a private
  network namespace and is reported null with the reason where that is unavailable.
* Data are synthetic (RCCL moves the same bytes whatever their values).
"""

from __future__ import annotations

import argparse
import json
import os
import shutil
import socket
import sys
import tempfile
import threading
import time
from typing import Optional

METRIC = "node scale-out-ready latency (s) + rccl all-reduce busbw GB/s at 1/2/4/8 GPU"
STORE_KEY = "netop/bench/artifacts"
STORE_FILE_ENV = "NETOP_BENCH_STORE"  # FileStore path of a rendezvous without a launcher
# Test hooks (CPU rehearsal of the xGMI link check): XML files read as RCCL's topology dump of the
# run with the artifacts / of the RCCL-defaults run.
FAKE_DUMP_ENV = "NETOP_BENCH_FAKE_RCCL_DUMP"
FAKE_DUMP_DEFAULTS_ENV = "NETOP_BENCH_FAKE_RCCL_DUMP_DEFAULTS"
# CPU rehearsal of the N-GPU line (tests): plan the GPU extras as on a node with this many GPUs
# (their stand-ins come from bench_extras.FAKE_EXTRA_ENV), give rank r the GPU BDF FAKE_BDFS[r],
# and read amd-smi's counters around the timed loop from a JSON file {"before": .., "after": ..}.
FAKE_GPUS_ENV = "NETOP_BENCH_FAKE_GPUS"
FAKE_SMI_ENV = "NETOP_BENCH_FAKE_SMI"
FAKE_BDFS = [f"0000:{0x0a + 0x19 * k:02x}:00.0" for k in range(8)]


def plan_extras(args, world: int, gpu: bool, device_count: int) -> list:
    """Rank 0's diagnostics after the headline, in the order they run (each bounded by the
    deadline, so the later ones are the first to go when time runs short).  The direct xGMI
    all-reduces (single process and IPC) run only where the job holds every GPU of the node --
    the last of the driver's N = 1, 2, 4, 8 runs -- unless forced with --xgmi-allreduce 1."""
    plan = []
    if args.rccl_defaults and args.artifacts != "off":
        plan.append("rccl_defaults")
    if gpu and args.native_rccl:
        plan.append("native_rccl")
    if gpu and world > 1 and args.xgmi_probe:
        plan.append("xgmi_probe")
    direct = args.xgmi_allreduce == "1" or (args.xgmi_allreduce == "auto" and world == device_count)
    if gpu and world > 1 and direct:
        plan += ["xgmi_allreduce", "xgmi_comm"]
    if args.node_ready != "off":
        plan.append("node_ready")
    return plan


def _fake_smi() -> Optional[dict]:
    path = os.environ.get(FAKE_SMI_ENV)
    if not path:
        return None
    with open(path) as f:
        return json.load(f)

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


CONFIG_1 = "L3 mode, 1xMI355X: mock-switch LLDP /30 Port-Description -> one NIC up + NFD scale-out label"


def config_name(n: int) -> str:
    """The BASELINE.json config this run measures, from the world size actually running."""
    if n == 1:  # BASELINE.json configs[1]
        return CONFIG_1
    if n == 8:  # BASELINE.json configs[2]
        return ("L3 mode, 8xMI355X single node: all xGMI + host RoCE links configured, "
                "rccl-tests 8-GPU all-reduce")
    return (f"L3 mode, {n}xMI355X single node (first {n} GPUs of the 8-GPU node): xGMI links among {n} GPUs, "
            f"rccl-tests {n}-GPU all-reduce")


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawn_ranks(n: int, argv: list[str], device: str, deadline: float) -> int:
    """``python bench.py --gpus N`` without a launcher: start N rank processes (one per GPU,
    torchrun-style env) and wait for them.  This process never touches the GPU (counting devices
    does not initialise HIP on this image), so the ranks are ordinary children, not an exec.
    Only rank 0 prints the JSON line; if any rank fails the others are stopped, and ranks still
    alive 30 s after the deadline (rank 0's watchdog has printed by then) are killed."""
    import signal
    import subprocess

    if device == "cuda":
        import torch

        have = torch.cuda.device_count()
        if have < n:
            print(f"bench.py --gpus {n}: only {have} GPU(s) visible", file=sys.stderr)
            return 2
    port = _free_port()
    store_dir = tempfile.mkdtemp(prefix="netop-bench-store-")
    procs = {}
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   **{STORE_FILE_ENV: os.path.join(store_dir, "store")})
        procs[r] = subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env)
    rc, killed = 0, set()
    try:
        while procs:
            for r, p in list(procs.items()):
                code = p.poll()
                if code is None:
                    continue
                del procs[r]
                if code != 0 and rc == 0 and r not in killed:
                    rc = code if code > 0 else 128 - code
                    for q in procs.values():  # one rank died: the rest would hang in the next collective
                        q.send_signal(signal.SIGTERM)
            if procs and time.monotonic() > deadline + 30:
                for r, q in procs.items():
                    killed.add(r)
                    q.kill()
            time.sleep(0.05)
    except KeyboardInterrupt:
        for q in procs.values():
            q.send_signal(signal.SIGTERM)
        raise
    finally:
        for q in procs.values():
            try:
                q.wait(30)
            except subprocess.TimeoutExpired:
                q.kill()
        shutil.rmtree(store_dir, ignore_errors=True)
    return rc


def node_ready_gpu_side(sysfs: str = "/sys/") -> dict:
    """Times the node agent's phases that need no privileges, against the real sysfs of the
    box: GPU<->NIC PCIe-affinity discovery, KFD xGMI mesh check, GPUDirect RDMA detection,
    and the RCCL artifacts (rccl.env + NCCL_TOPO_FILE XML) and NFD label written to a scratch
    directory.  A component of node-ready latency, not the metric: link-up, LLDP and the netlink
    writes need NET_ADMIN/NET_RAW and run in the netns harness (``--node-ready``)."""
    from network_operator_amd.agent import native

    m = native()
    out: dict = {"what": "agent phases that need no privileges, real /sys of this box (component, not the metric)",
                 "phases_ms": {}}

    def timed(name, fn):
        t = time.perf_counter()
        r = fn()
        out["phases_ms"][name] = round((time.perf_counter() - t) * 1e3, 4)
        return r

    d = timed("discover", lambda: m.discover(sysfs, "affine"))
    x = timed("xgmi", lambda: m.read_xgmi(sysfs))
    g = timed("gdr", lambda: m.detect_gdr(sysfs))
    with tempfile.TemporaryDirectory() as tmp:
        def topo_file():
            xml = m.rccl_topo_xml(sysfs)
            with open(os.path.join(tmp, "rccl-topo.xml"), "w") as f:
                f.write(xml)
            return xml

        out["rccl_topo_xml_bytes"] = len(timed("rccl_topo", topo_file))
        lab = os.path.join(tmp, "scale-out-readiness.txt")

        def label():
            with open(lab + ".tmp", "w") as f:
                f.write("amd.feature.node.kubernetes.io/gpu-scale-out=true\n")
            os.replace(lab + ".tmp", lab)

        timed("label", label)
    out["total_ms"] = round(sum(out["phases_ms"].values()), 4)
    # The agent binary itself, 10 dry runs with the operator's flags (its own phase timings and
    # the process wall time, exec to exit): network_operator_amd/agent/start_timing.py.
    try:
        from network_operator_amd.agent import start_timing

        out["agent_binary"] = start_timing.measure(runs=10, sysfs=sysfs if sysfs != "/sys/" else "")
    except Exception as e:  # reported, never fatal to the line
        out["agent_binary"] = {"error": str(e)[-300:]}
    out["gpus"] = len(d["gpus"])
    out["nics_paired"] = len(d["pairs"])
    out["xgmi_pairs"] = f"{x['pairs_connected']}/{x['pairs_expected']}"
    out["gpudirect_rdma"] = g["mode"]
    return out


_LAUNCH_ENV = ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK", "ROLE_WORLD_SIZE",
               "MASTER_ADDR", "MASTER_PORT", STORE_FILE_ENV)


def _probe_cmd(world: int, nbytes: int, steps: int, device: str, warmup: int = 2) -> list:
    """bench.py as a bare measurement of the timed loop: every extra and diagnostic off."""
    return [sys.executable, os.path.abspath(__file__), "--gpus", str(world), "--steps", str(steps), "--warmup",
            str(warmup), "--bytes", str(nbytes), "--sweep", "", "--collectives", "", "--node-ready", "off",
            "--xgmi-probe", "0", "--native-rccl", "0", "--xgmi-allreduce", "0", "--rccl-autotune", "0",
            "--gpu-side", "0", "--rccl-defaults", "0", "--strict", "0", "--device", device]


def torch_env_probe(world: int, nbytes: int, budget_s: float, device: str = "cuda", variants=None,
                    steps: int = 5, artifacts: str = "off", base_env: Optional[dict] = None) -> list:
    """busbw of the timed loop itself (torch.distributed, this torch's RCCL, bf16, `nbytes`) under
    each RCCL knob variant of ``rccl_bench.ENV_PROBES``: bench.py runs again in a fresh set of
    `world` rank processes per variant, with the variant in its environment on top of
    `artifacts` (an artifact directory, or "off") and every extra measurement off.  Variants not
    started within `budget_s` are reported as skipped.  A hung variant is killed with its whole
    process tree (its ranks hold GPUs)."""
    from network_operator_amd.parallel import bench_extras, rccl_bench

    runner = bench_extras.Runner(time.monotonic() + budget_s + 30, base_env=base_env, margin_s=0)
    out = []
    t0 = time.monotonic()
    for extra in (variants if variants is not None else rccl_bench.ENV_PROBES):
        if budget_s - (time.monotonic() - t0) <= 0:
            out.append({"env": extra, "skipped": "time budget spent"})
            continue
        j = runner.run("autotune", _probe_cmd(world, nbytes, steps, device) + ["--artifacts", artifacts],
                       cap_s=budget_s + 30, env=extra)
        if "error" in j:
            out.append({"env": extra, "error": j["error"] if j["error"] != "deadline" else "timed out"})
            continue
        out.append({"env": extra, "busbw_GBps": j["busbw_GBps"], "time_us": j["ms_per_step"] * 1e3,
                    "artifacts_applied": bool((j.get("agent_artifacts") or {}).get("applied"))})
    return out


AUTOTUNE_KEY = "netop/bench/autotune"


def _rccl_autotune(store, rank: int, world: int, nbytes: int, budget_s: float = 150.0, device: str = "cuda",
                   variants=None, artifacts: str = "off", base_env: Optional[dict] = None) -> dict:
    """RCCL reads its parameters once per process, at communicator creation, so they must be
    chosen before init_process_group.

    Rank 0 measures the knob variants of ``rccl_bench.ENV_PROBES`` with bench.py itself
    (``torch_env_probe``: the same torch, RCCL build, dtype, message *and the same agent
    artifacts* as the timed loop) over the node's first `world` GPUs.  Each variant runs in fresh
    processes, and all of them must fit in ``budget_s``.  A variant must beat the artifacts alone
    by >= 3 % (``rccl_bench.choose_env``).  Rank 0 publishes the choice through the rendezvous
    store (one per launcher run, so the driver's back-to-back N = 2, 4, 8 runs cannot see each
    other's), and every rank exports it.  This is what the validation Job writes to a node's
    ``rccl-tuned.env`` (``validate.py --tune-rccl``): what jobs on a configured node source."""
    if rank == 0:
        try:
            from network_operator_amd.parallel import rccl_bench

            probes = torch_env_probe(world, nbytes, budget_s, device=device, variants=variants, artifacts=artifacts,
                                     base_env=base_env)
            doc = dict(rccl_bench.choose_env(probes), probes=probes)
        except Exception as e:  # never leave the other ranks waiting: no knobs, and say why
            doc = {"chosen": {}, "error": str(e)[-300:]}
        store.set(AUTOTUNE_KEY, json.dumps(doc))
    else:
        doc = json.loads(store.get(AUTOTUNE_KEY))
    for k, v in doc["chosen"].items():
        os.environ[k] = v
    return doc


# ------------------------------------------------------------------------------------------
# The operator's artifacts, before RCCL starts
# ------------------------------------------------------------------------------------------
def _store(world: int, timeout_s: float):
    """The rendezvous store (torchrun's agent store under torchrun; without a launcher a
    FileStore, so no TCP port picked here can be taken by another process before rank 0 binds
    it: that failed a box run with EADDRINUSE), shared with init_process_group: it carries the
    artifacts from rank 0 to every rank before any RCCL communicator exists."""
    from datetime import timedelta

    import torch.distributed as dist

    f = os.environ.get(STORE_FILE_ENV)
    if f:
        rank = int(os.environ.get("RANK", "0"))
        store, _, _ = next(dist.rendezvous(f"file://{f}", rank=rank, world_size=world,
                                           timeout=timedelta(seconds=timeout_s)))
    else:
        store, _, _ = next(dist.rendezvous("env://", timeout=timedelta(seconds=timeout_s)))
    return store


def _artifacts(store, rank: int, args) -> dict:
    """Rank 0 produces (``--artifacts agent``) or loads (``--artifacts DIR``) the RCCL artifacts
    and publishes them; every rank applies them to its environment before RCCL initialises.
    Returns rank 0's description (with ``applied``) and this rank's record."""
    from network_operator_amd.parallel import fabric_artifacts as FA

    if rank == 0:
        try:
            if args.artifacts == "agent":
                work = tempfile.mkdtemp(prefix="netop-bench-")
                doc = FA.generate(work, sysfs_root=args.sysfs_root or None)
                doc.update(dir=work, scratch=True)
            else:
                env = FA.load_env_dir(args.artifacts)
                doc = {"source": f"artifact directory {args.artifacts}", "dir": args.artifacts, "env": env,
                       "topo_file": env.get("NCCL_TOPO_FILE")}
                if not env:
                    doc["error"] = f"no {FA.ENV_FILE} in {args.artifacts}"
                tf = env.get("NCCL_TOPO_FILE")
                doc["topo_file_bytes"] = os.path.getsize(tf) if tf and os.path.isfile(tf) else 0
                doc["topo_sha256"] = FA._sha256(tf) if tf else None
        except Exception as e:
            doc = {"error": f"{type(e).__name__}: {str(e)[-500:]}"}
        store.set(STORE_KEY, json.dumps(doc))
    else:
        doc = json.loads(store.get(STORE_KEY))
    if "error" in doc:
        return {"doc": doc, "record": {"rank": rank, "applied": False}}
    rec = FA.apply(doc["env"])
    rec.update(rank=rank, applied=True)
    return {"doc": doc, "record": rec}


class _Once:
    """Rank 0's single JSON line: printed once, by the main thread or the deadline watchdog."""

    def __init__(self, out=None):
        self.lock = threading.Lock()
        self.done = False
        self.out = out

    def emit(self, line: dict) -> bool:
        with self.lock:
            if self.done:
                return False
            print(json.dumps(line), file=self.out or sys.stdout, flush=True)
            self.done = True
            return True


def run_config(args, world: int, st: dict) -> tuple:
    """(config.model, what ran, what did not) for the line.  At n = 1 the BASELINE.json configs[1]
    name is claimed only when its node-ready half (LLDP on the mock switch, NIC up, the NFD
    label) was measured in this run; otherwise the line names what did run.
    At n = 2 / 4 the name follows the world size; at n = 8 the configs[2] name, which says the
    host RoCE links are configured, carries what this run did instead when node-ready did not run."""
    a = st.get("artifacts") or {}
    ran = ["rccl_all_reduce"] + (["agent_artifacts"] if a.get("applied") else [])
    skipped = []
    if st.get("node_ready"):
        ran += ["lldp", "nic_up", "label"]
    else:
        skipped += ["lldp", "nic_up", "label"]
    if st.get("gpu_side") and "error" not in st["gpu_side"]:
        ran.append("agent_gpu_side_phases")
    why = st.get("node_ready_note") or ("--node-ready off" if args.node_ready == "off" else "not reached")
    backend = "RCCL" if args.device == "cuda" else "gloo (CPU rehearsal)"
    if st.get("node_ready") or world in (2, 4):
        return config_name(world), ran, skipped
    if world > 1:
        # configs[2] names the node's host RoCE links as configured: keep the name (the all-reduce
        # over xGMI is what it measures) and say that this run did not configure them.
        via = "with the agent's artifacts" if a.get("applied") else "without the agent's artifacts"
        return (f"{config_name(world)} [this run: {backend} all-reduce over xGMI {via}; host RoCE links not "
                f"configured by it (node-ready not run: {why})]"), ran, skipped
    model = (f"{backend} all-reduce with the agent's artifacts, 1xMI355X (node-ready not run: {why})"
             if a.get("applied") else f"{backend} all-reduce, 1xMI355X (node-ready not run: {why})")
    return model, ran, skipped


def _line(args, world: int, st: dict) -> dict:
    """The JSON line from whatever has been measured so far (``st``)."""
    h = st.get("headline")
    cuda = args.device == "cuda"
    from network_operator_amd.parallel import collectives as C

    ceiling = C.xgmi_busbw_ceiling_GBps(world)
    busbw = h["busbw"] if h else None
    model, ran, skipped = run_config(args, world, st)
    line = {
        "metric": METRIC,
        # The driver's contract: the whole job's aggregate over its N GPUs.  rccl-tests' busbw is
        # a per-GPU figure (what each GPU's links carry), so the job's is N times it.
        "value": round(busbw * world, 3) if h else None,
        "value_definition": "aggregate busbw of the job: rccl-tests busbw (per GPU) x n_gpus",
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": h["per_step"] * 1e3 if h else None,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16" if cuda else "fp32",
        "data": "synthetic (zeros for the timed loop; exact pattern check before timing)",
        "config": {"model": model, "ran": ran, "skipped": skipped, "global_batch": None, "seq_len": None,
                   "parallelism": f"dp{world}", "gpus": world, "message_bytes_per_rank": h["nbytes"] if h else None,
                   "op": "all_reduce(sum)",
                   "backend": "torch.distributed nccl (RCCL)" if cuda else "torch.distributed gloo (CPU rehearsal)",
                   "rccl_env": ("agent artifacts (discover --dry-run)" if args.artifacts == "agent"
                                else "RCCL defaults" if args.artifacts == "off" else f"artifacts from {args.artifacts}")
                   + (f" + autotuned {(st.get('tuned') or {}).get('chosen')}" if (st.get("tuned") or {}).get("chosen")
                      else "")},
        "agent_artifacts": st.get("artifacts"),
        "busbw_GBps": busbw,
        "busbw_basis": "per GPU (rccl-tests); value and aggregate_* are x n_gpus",
        "busbw_rccl_defaults_GBps": (st.get("rccl_defaults") or {}).get("busbw_GBps"),
        "aggregate_busbw_rccl_defaults_GBps": (
            round(st["rccl_defaults"]["busbw_GBps"] * world, 3)
            if (st.get("rccl_defaults") or {}).get("busbw_GBps") is not None else None),
        "rccl_defaults": st.get("rccl_defaults"),
        "algbw_GBps": h["algbw"] if h else None,
        "algbw_note": h.get("algbw_note") if h else None,
        # rccl-tests busbw is per rank; the whole job moves n times that over the links.
        "aggregate_busbw_GBps": busbw * world if h else None,
        "busbw_ceiling_GBps": ceiling,
        "busbw_vs_ceiling": (busbw / ceiling) if h and ceiling else None,
        "verified": st.get("verified"),
        "verify_errors": st.get("verify_errors"),
        "sweep": st.get("sweep", []),
        "collectives": st.get("collectives", []),
        "xgmi_probe": st.get("xgmi_probe"),
        "native_rccl": st.get("native_rccl"),
        "rccl_autotune": st.get("tuned"),
        "xgmi_allreduce": st.get("xgmi_allreduce"),
        "xgmi_allreduce_multiprocess": st.get("xgmi_comm"),
        "node_ready": st.get("node_ready"),
        "node_ready_unavailable": st.get("node_ready_unavailable"),
        "node_ready_gpu_side": st.get("gpu_side"),
        "xgmi_traffic": st.get("xgmi_traffic"),
        "deadline_s": args.deadline_s,
        "elapsed_s": round(time.monotonic() - st["t_start"], 2),
        "extras_log": st.get("extras_log", []),
        "notes": "; ".join(x for x in [
            "n=1: busbw is 0 by definition (rccl-tests factor 2(n-1)/n)" if world == 1 else "",
            "reference publishes no numbers (BASELINE.md) so vs_baseline is null",
            st.get("node_ready_note") or "", st.get("smi_note") or ""] if x),
        "rccl_version": st.get("rccl_version"),
    }
    if st.get("error"):
        line["error"] = st["error"]
    return line


def _watchdog(rank: int, deadline: float, st: dict, once: _Once, runner_box: list, args, world: int) -> None:
    """At the deadline: rank 0 kills every running extra and prints the line with what has been
    measured; every rank then exits (0 if the timed loop finished, 1 if it never did)."""
    def fire():
        delay = deadline - time.monotonic() + (0 if rank == 0 else 20)
        if delay > 0:
            time.sleep(delay)
        if st.get("finished"):  # printed; only a hung teardown is left
            sys.stdout.flush()
            os._exit(st.get("rc", 0))
        if rank == 0:
            if runner_box:
                runner_box[0].kill_all()
            for name in st.get("pending", ()):
                st.setdefault(name, {"error": "deadline", "detail": "killed at --deadline-s"})
            if not st.get("headline"):
                st["error"] = f"deadline ({args.deadline_s} s) passed before the timed loop finished"
            if once.emit(_line(args, world, st)):
                print(f"bench.py: --deadline-s {args.deadline_s} reached; printed what was measured", file=sys.stderr)
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0 if st.get("headline") else 1)

    threading.Thread(target=fire, name="bench-deadline", daemon=True).start()


def main(argv=None) -> int:
    t_start = time.monotonic()
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--bytes", type=int, default=1 << 30, help="all-reduce message size per rank")
    ap.add_argument("--artifacts", default="agent",
                    help="RCCL environment of the timed loop: 'agent' (run discover --dry-run on this node and apply "
                         "its NCCL_TOPO_FILE / rccl.env), an artifact directory (rccl.env + rccl-tuned.env), or 'off' "
                         "(RCCL defaults)")
    ap.add_argument("--sysfs-root", default=os.environ.get("SYSFS_ROOT", ""),
                    help="sysfs the agent reads for --artifacts agent (default the real /sys)")
    ap.add_argument("--topo-dump", default="", help="with --artifacts off: RCCL topology dump path (rank 0)")
    ap.add_argument("--rccl-defaults", type=int, default=1,
                    help="also run the timed loop in fresh rank processes with RCCL's defaults (the A/B)")
    ap.add_argument("--strict", type=int, default=1,
                    help="GPU, n > 1: exit 1 (after printing the line) when the artifacts could not be applied or RCCL "
                         "sees fewer xGMI links per GPU under them than without them")
    ap.add_argument("--deadline-s", type=float, default=450.0,
                    help="hard wall-clock limit: extras are killed and the line printed by then")
    ap.add_argument("--sweep", default="4096,1048576,67108864", help="extra sizes (bytes) reported alongside")
    ap.add_argument("--node-ready", choices=["auto", "on", "off"], default="auto")
    ap.add_argument("--node-ready-runs", type=int, default=5)
    ap.add_argument("--collectives", default="all_gather,reduce_scatter,all_to_all",
                    help="other collectives reported at --bytes (n > 1 only)")
    ap.add_argument("--xgmi-probe", type=int, default=1, help="run the HIP xGMI link probe on rank 0 (n > 1)")
    ap.add_argument("--native-rccl", type=int, default=1,
                    help="also run the native netop-rccl-bench harness (ROCm's RCCL, artifacts applied) on rank 0")
    ap.add_argument("--rccl-env-probe", type=int, default=0,
                    help="n > 1: also measure the 1 GiB busbw under RCCL knob variants (a fresh process each)")
    ap.add_argument("--extras-budget", type=float, default=0.0, help=argparse.SUPPRESS)  # superseded by --deadline-s
    ap.add_argument("--rccl-autotune", type=int, default=1,
                    help="GPU, n > 1: before RCCL starts, rank 0 measures RCCL knob variants on top of the agent's "
                         "artifacts by running this bench again per variant (within --rccl-autotune-budget s) and "
                         "every rank uses the fastest (>= 3%% better than the artifacts alone): what the validation "
                         "Job writes to rccl-tuned.env; 0 = the artifacts' environment only")
    ap.add_argument("--rccl-autotune-budget", type=float, default=120.0)
    ap.add_argument("--gpu-side", type=int, default=1, help="rank 0: time the agent's unprivileged phases on this box")
    # CPU rehearsal of the autotune plumbing (tests): run it with gloo too, on the first K variants.
    ap.add_argument("--autotune-cpu-variants", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--xgmi-allreduce", choices=["0", "1", "auto"], default="auto",
                    help="also run the hand-written direct xGMI all-reduces (single process and one process per "
                         "GPU over HIP IPC) after the headline; auto = only when the job spans every visible GPU "
                         "(the last of the driver's N = 1, 2, 4, 8 runs): their first contact with real peers must "
                         "not be able to leave a GPU in a state that costs a later run its number")
    # CPU rehearsal of the multi-rank path (tests): gloo backend, fp32 on the host.
    ap.add_argument("--device", choices=["cuda", "cpu"], default="cuda", help=argparse.SUPPRESS)
    raw_argv = list(sys.argv[1:] if argv is None else argv)
    args = ap.parse_args(raw_argv)
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    deadline = t_start + args.deadline_s

    from network_operator_amd.parallel import bench_extras

    bench_extras.maybe_hang()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return _spawn_ranks(args.gpus, raw_argv, args.device, deadline)

    # A rank's stdout carries exactly the one JSON line: what libraries print there (RCCL's
    # version banner, gloo's connection notes) and child processes that inherit it go to stderr.
    json_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus={args.gpus} but the launcher started WORLD_SIZE={world} ranks", file=sys.stderr)
        return 2
    base_env = dict(os.environ)  # before any artifact or knob is exported: what the extras start from
    own_store = None
    if "WORLD_SIZE" not in os.environ:  # one rank, no launcher: a rendezvous of its own (a FileStore)
        own_store = tempfile.mkdtemp(prefix="netop-bench-store-")
        os.environ.update(RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
                          **{STORE_FILE_ENV: os.path.join(own_store, "store")})

    import torch
    import torch.distributed as dist

    from network_operator_amd.parallel import collectives as C
    from network_operator_amd.parallel import fabric_artifacts as FA

    st: dict = {"t_start": t_start, "pending": []}
    once = _Once(json_out)
    runner_box: list = []
    _watchdog(rank, deadline, st, once, runner_box, args, world)

    cuda = args.device == "cuda"
    fake_gpus = 0 if cuda else int(os.environ.get(FAKE_GPUS_ENV) or 0)
    if cuda and not torch.cuda.is_available():
        print("bench.py needs an MI355X GPU (torch.cuda.is_available() is False)", file=sys.stderr)
        return 2

    # 0. RCCL's environment, fixed before any communicator exists: the operator's artifacts, then
    #    (n > 1) the knob autotune on top of them, both handed to every rank through the rendezvous
    #    store.
    store = _store(world, timeout_s=max(60.0, deadline - time.monotonic()))
    art, dump_path = None, None
    if args.artifacts != "off":
        art = _artifacts(store, rank, args)
        doc = art["doc"]
        if rank == 0 and "error" not in doc:
            dump_path = os.path.join(doc["dir"] if doc.get("scratch") else tempfile.mkdtemp(prefix="netop-bench-"),
                                     FA.DUMP_FILE)
    elif rank == 0 and args.topo_dump:
        dump_path = args.topo_dump
    if world > 1 and (args.rccl_autotune if cuda else args.autotune_cpu_variants):
        from network_operator_amd.parallel import rccl_bench

        variants = None if cuda else rccl_bench.ENV_PROBES[:args.autotune_cpu_variants]
        art_dir = art["doc"].get("dir") if art and "error" not in art["doc"] else None
        st["tuned"] = _rccl_autotune(store, rank, world, args.bytes, args.rccl_autotune_budget, device=args.device,
                                     variants=variants, artifacts=art_dir or "off", base_env=base_env)
    if dump_path:
        os.environ["NCCL_TOPO_DUMP_FILE"] = dump_path

    if cuda:
        torch.cuda.set_device(local_rank)
        device, dtype = torch.device("cuda", local_rank), torch.bfloat16
        dist.init_process_group("nccl", store=store, rank=rank, world_size=world, device_id=device)
        # Host-side group for waiting while rank 0 runs its extras: an RCCL barrier would leave a
        # spinning kernel on every other GPU and disturb what those tools measure.
        host_pg = dist.new_group(backend="gloo")
        st["rccl_version"] = ".".join(str(x) for x in torch.cuda.nccl.version()) if hasattr(torch.cuda, "nccl") else None
    else:
        device, dtype = torch.device("cpu"), torch.float32
        dist.init_process_group("gloo", store=store, rank=rank, world_size=world)
        host_pg = None
    esize = torch.tensor([], dtype=dtype).element_size()
    records = [None] * world
    mine = dict(art["record"] if art else {"rank": rank, "applied": False})
    if cuda:
        from network_operator_amd.parallel.rail import device_bdf

        mine["bdf"] = device_bdf(local_rank)
    elif fake_gpus:
        mine["bdf"] = FAKE_BDFS[local_rank % len(FAKE_BDFS)]
    dist.all_gather_object(records, mine, group=host_pg)
    job_bdfs = [r.get("bdf") for r in records if r and r.get("bdf")]

    # 1. Correctness of the collective path (exact, HIP pattern kernels on the GPU).
    verified, errors = C.verify_all_reduce(min(args.bytes // 2, 64 << 20), device)
    st["verified"], st["verify_errors"] = verified, errors

    # 2. Headline: K timed all-reduce steps of --bytes per rank.
    numel = (args.bytes // esize) // 8 * 8
    buf = torch.zeros(numel, dtype=dtype, device=device)
    for _ in range(args.warmup):
        dist.all_reduce(buf)
    smi_before = None
    fake_smi = _fake_smi() if rank == 0 and not cuda else None
    if rank == 0 and cuda:  # xGMI counters (amd-smi), outside the timed region
        try:
            from network_operator_amd.ops import smi

            smi_before = smi.snapshot()
        except Exception as e:
            st["smi_note"] = f"amd-smi counters unavailable: {e}"
    elif fake_smi is not None:
        from network_operator_amd.ops import smi

        smi_before = fake_smi["before"]
    dist.barrier()
    C.sync(device)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        dist.all_reduce(buf)
    C.sync(device)
    dt = time.perf_counter() - t0
    dist.barrier()
    if rank == 0 and smi_before is not None:
        try:
            t = smi.traffic(smi_before, fake_smi["after"] if fake_smi is not None else smi.snapshot())
            st["xgmi_traffic"] = {"links_up": t["links_up"], "links_with_traffic": t["links_with_traffic"],
                                  "GB_per_gpu": [round(sum(g["bytes_per_link"]) / 1e9, 3) for g in t["gpus"]],
                                  "job": FA.traffic_view(job_bdfs, t)}
        except Exception as e:
            st["smi_note"] = f"amd-smi counters unavailable: {e}"
    t = torch.tensor([dt], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    per_step = float(t.item()) / max(args.steps, 1)
    nbytes = numel * esize
    algbw, busbw = C.bandwidths("all_reduce", nbytes, world, per_step)
    del buf
    headline = {"busbw": busbw, "algbw": algbw, "per_step": per_step, "nbytes": nbytes}
    if world == 1:
        # A single-rank in-place all-reduce moves no bytes (RCCL returns at once): bytes/time would
        # be a number with no meaning (round 1 printed 93 TB/s, 12x HBM peak).  Null, and why.
        headline["algbw"] = None
        headline["algbw_note"] = ("n=1: the timed in-place all-reduce is a no-op in RCCL (no peer, no copy), so algbw "
                                  "is not a bandwidth; ms_per_step is its launch latency. busbw is 0 by definition")
    st["headline"] = headline
    if rank == 0 and os.environ.get(bench_extras.HANG_ENV) == "rank0-after-headline":  # test hook: a hung step
        while True:
            time.sleep(3600)

    # 3. Size sweep (latency / medium messages), same definitions.
    sizes = [int(s) for s in args.sweep.split(",") if s.strip()]
    if sizes:
        st["sweep"] = [{"bytes": r.bytes, "time_us": r.time_s * 1e6, "algbw_GBps": None if world == 1 else r.algbw_GBps,
                        "busbw_GBps": r.busbw_GBps}
                       for r in C.run_sweep("all_reduce", sizes, iters=max(args.steps, 10), warmup=max(args.warmup, 3),
                                            device=device, dtype=dtype)]

    # 4. The other collectives RCCL runs over the same links (rccl-tests definitions), n > 1.
    if world > 1:
        others = []
        for op in [o.strip() for o in args.collectives.split(",") if o.strip()]:
            before = None
            if rank == 0 and smi_before is not None and fake_smi is None:  # no collective starts before rank 0 joins it
                try:
                    before = smi.snapshot()
                except Exception:
                    before = None
            r = C.run_sweep(op, [nbytes], iters=max(args.steps // 2, 5), warmup=2, device=device, dtype=dtype)[0]
            row = {"op": op, "bytes": r.bytes, "time_us": r.time_s * 1e6, "algbw_GBps": r.algbw_GBps,
                   "busbw_GBps": r.busbw_GBps}
            if before is not None:  # does this collective use every xGMI link of the job too?
                try:
                    row["xgmi_links"] = FA.traffic_view(job_bdfs, smi.traffic(before, smi.snapshot()))
                except Exception as e:
                    row["xgmi_links"] = {"error": str(e)[-200:]}
            others.append(row)
        st["collectives"] = others

    # 5. What was applied, and what RCCL made of it (rank 0).
    if rank == 0:
        if art is not None:
            doc = dict(art["doc"])
            doc.pop("scratch", None)
            recs = [r for r in records if r]
            shas = {r.get("topo_sha256") for r in recs if r.get("applied")}
            doc.update(applied=bool(recs) and all(r.get("applied") for r in recs) and "error" not in doc,
                       ranks_applied=sum(1 for r in recs if r.get("applied")), ranks_same_file=len(shas) <= 1,
                       per_rank=[{"rank": r["rank"], "applied": r.get("applied"),
                                  "NCCL_TOPO_FILE": (r.get("env") or {}).get("NCCL_TOPO_FILE"),
                                  "topo_sha256": r.get("topo_sha256")} for r in recs])
            st["artifacts"] = doc
        else:
            st["artifacts"] = {"applied": False, "source": "RCCL defaults (--artifacts off)"}
        if dump_path:
            # CPU rehearsal of the link check (tests): a prepared file stands in for RCCL's dump.
            fake = os.environ.get(FAKE_DUMP_ENV if art is not None else FAKE_DUMP_DEFAULTS_ENV)
            st["artifacts"]["rccl_dump"] = (FA.read_view(fake or dump_path, st["artifacts"].get("topo_file"))
                                            or {"error": f"RCCL wrote no topology dump to {dump_path}"}) \
                if cuda or fake else {"note": "gloo: no RCCL topology on the CPU rehearsal"}

    # 6. Diagnostics, rank 0, each a child process bounded by the deadline (bench_extras.Runner).
    if rank == 0:
        runner = bench_extras.Runner(deadline, base_env=base_env)
        runner_box.append(runner)
        art_env = art["doc"]["env"] if art and "error" not in art["doc"] else {}
        plan = plan_extras(args, world, gpu=cuda or fake_gpus > 0,
                           device_count=torch.cuda.device_count() if cuda else fake_gpus)
        st["pending"] = list(plan)
        for name in plan:
            if name == "rccl_defaults":
                ddump = os.path.join(tempfile.mkdtemp(prefix="netop-bench-defaults-"), "rccl-topo-dump-defaults.xml")
                cmd = _probe_cmd(world, args.bytes, args.steps, args.device, warmup=args.warmup) + [
                    "--artifacts", "off", "--topo-dump", ddump, "--deadline-s", str(max(runner.left() - 2, 10))]
                j = runner.run(name, cmd, cap_s=180)
                res = j if "error" in j else {
                    "busbw_GBps": j.get("busbw_GBps"), "ms_per_step": j.get("ms_per_step"),
                    "verified": j.get("verified"), "rccl_dump": (j.get("agent_artifacts") or {}).get("rccl_dump")}
                shutil.rmtree(os.path.dirname(ddump), ignore_errors=True)
            elif name == "native_rccl":
                res = runner.extra(name, 150, env=art_env, world=world, env_probe=bool(args.rccl_env_probe))
                res["with_artifacts"] = bool(art_env)
            elif name == "xgmi_probe":
                res = runner.extra(name, 120, world=world)
            elif name in ("xgmi_allreduce", "xgmi_comm"):
                res = runner.extra(name, 120, world=world, nbytes=nbytes)
            else:  # node_ready
                res = runner.extra(name, 150, n_nics=world, runs=args.node_ready_runs, required=args.node_ready == "on")
                if "unavailable" in res:
                    u = res["unavailable"]
                    st["node_ready_note"] = f"node-ready harness unavailable: {u['why']}" if isinstance(u, dict) \
                        else f"node-ready harness unavailable: {u}"
                    st["node_ready_unavailable"] = u
                    res = None
                elif "result" in res:
                    res = res["result"]
                elif "error" in res:
                    st["node_ready_note"] = f"node-ready harness failed: {res['error']}"
                    res = None
            st[name] = res
            st["pending"].remove(name)
        st["extras_log"] = runner.log
        if args.gpu_side:
            try:
                st["gpu_side"] = node_ready_gpu_side()
            except Exception as e:
                st["gpu_side"] = {"error": str(e)[-300:]}

    # 7. The link check: RCCL must see >= n-1 xGMI links per GPU under the agent's file.  The run
    # fails (after its line) only when the file itself is to blame -- it costs links RCCL sees
    # without it -- or was not applied; a dump that cannot settle it is reported in the line.
    rc = 0 if verified else 1
    if rank == 0 and (cuda or os.environ.get(FAKE_DUMP_ENV)) and art is not None:
        a = st["artifacts"]
        v = FA.links_verdict(world, a.get("rccl_dump"), (st.get("rccl_defaults") or {}).get("rccl_dump"),
                             (st.get("xgmi_traffic") or {}).get("job"))
        a["xgmi_links_check"] = v
        if world > 1 and args.strict and (not a.get("applied") or v.get("file_blamed")):
            why = v.get("why") if a.get("applied") else f"artifacts not applied: {a.get('error')}"
            st["error"] = f"agent artifacts check failed: {why}"
            rc = 1

    try:  # everyone waits for rank 0's extras on the host (no spinning RCCL kernel)
        dist.barrier(group=host_pg)
    except Exception as e:  # rank 0 already gone (watchdog): the measurement stands
        if rank != 0:
            print(f"bench.py rank {rank}: final barrier: {e}", file=sys.stderr)
    if rank == 0:
        once.emit(_line(args, world, st))
        if st.get("error"):
            print(f"bench.py: {st['error']}", file=sys.stderr)
    st["rc"] = rc
    st["finished"] = True
    dist.destroy_process_group()
    if rank == 0 and art is not None and art["doc"].get("scratch"):
        shutil.rmtree(art["doc"]["dir"], ignore_errors=True)
    if own_store:
        shutil.rmtree(own_store, ignore_errors=True)
    return rc


if __name__ == "__main__":
    sys.exit(main())

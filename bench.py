#!/usr/bin/env python3
"""Headline benchmark: RCCL all-reduce bus bandwidth on MI355X (+ node-ready latency).

BASELINE.json metric: "node scale-out-ready latency (s) + rccl all-reduce busbw GB/s at
1/2/4/8 GPU", config "L3 mode, 8xMI355X single node: all xGMI + host RoCE links configured,
rccl-tests 8-GPU all-reduce".

* One process per GPU, ``torch.distributed`` backend ``nccl`` (= RCCL over xGMI on ROCm).
  Under ``torchrun --nproc-per-node N`` the launcher's ranks are used (WORLD_SIZE must equal
  ``--gpus``); a bare ``python bench.py --gpus N`` starts the N rank processes itself.
  ``config.model`` names the BASELINE.json config of the world size that actually ran.  A *step* is one in-place bf16 all-reduce of
  ``--bytes`` per rank (default 1 GiB, rccl-tests' large-message regime); ``--warmup``
  untimed steps, then exactly ``--steps`` timed steps bracketed by barrier +
  ``torch.cuda.synchronize()``, max over ranks.
* ``value`` is busbw = algbw * 2(n-1)/n (rccl-tests definition, per rank;
  ``aggregate_busbw_GBps`` is n times that).  At n = 1 there are no links and busbw is 0 by
  definition; the single-rank all-reduce is a no-op, so algbw is reported as null with the
  reason and ``node_ready_gpu_side`` times the agent phases that run unprivileged on the box.
* Before timing, the result of one all-reduce of rank-specific patterns is verified exactly
  with the HIP kernels in ``libnetop_hip.so`` (fails loudly if the library is missing).
* The node-ready latency half of the metric needs a private network namespace (root /
  user namespaces + AF_PACKET); it runs with ``--node-ready`` where that is available and is
  reported as null with the reason otherwise (the GPU pool's boxes run unprivileged).
* Data are synthetic (RCCL moves the same bytes whatever their values).
"""

from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import time

METRIC = "node scale-out-ready latency (s) + rccl all-reduce busbw GB/s at 1/2/4/8 GPU"


def config_name(n: int) -> str:
    """The BASELINE.json config this run measures, from the world size actually running."""
    if n == 1:  # BASELINE.json configs[1]
        return "L3 mode, 1xMI355X: mock-switch LLDP /30 Port-Description -> one NIC up + NFD scale-out label"
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


def _spawn_ranks(n: int, argv: list[str], device: str) -> int:
    """``python bench.py --gpus N`` without a launcher: start N rank processes (one per GPU,
    torchrun-style env) and wait for them.  This process never touches the GPU (counting devices
    does not initialise HIP on this image), so the ranks are ordinary children, not an exec.
    Only rank 0 prints the JSON line; if any rank fails the others are stopped."""
    import signal
    import subprocess

    if device == "cuda":
        import torch

        have = torch.cuda.device_count()
        if have < n:
            print(f"bench.py --gpus {n}: only {have} GPU(s) visible", file=sys.stderr)
            return 2
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env))
    rc = 0
    try:
        while procs:
            for p in list(procs):
                code = p.poll()
                if code is None:
                    continue
                procs.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code
                    for q in procs:  # one rank died: the rest would hang in the next collective
                        q.send_signal(signal.SIGTERM)
            time.sleep(0.05)
    except KeyboardInterrupt:
        for q in procs:
            q.send_signal(signal.SIGTERM)
        raise
    finally:
        for q in procs:
            try:
                q.wait(30)
            except subprocess.TimeoutExpired:
                q.kill()
    return rc


def node_ready_gpu_side(sysfs: str = "/sys/") -> dict:
    """Times the node agent's phases that need no privileges, against the real sysfs of the
    box: GPU<->NIC PCIe-affinity discovery, KFD xGMI mesh check, GPUDirect RDMA detection,
    and the RCCL artifacts (rccl.env + NCCL_TOPO_FILE XML) and NFD label written to a scratch
    directory.  A component of node-ready latency, not the metric: link-up, LLDP and the netlink
    writes need NET_ADMIN/NET_RAW and run in the netns harness (``--node-ready``)."""
    import tempfile

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
    out["gpus"] = len(d["gpus"])
    out["nics_paired"] = len(d["pairs"])
    out["xgmi_pairs"] = f"{x['pairs_connected']}/{x['pairs_expected']}"
    out["gpudirect_rdma"] = g["mode"]
    return out


_LAUNCH_ENV = ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK", "ROLE_WORLD_SIZE",
               "MASTER_ADDR", "MASTER_PORT")


def torch_env_probe(world: int, nbytes: int, budget_s: float, device: str = "cuda", variants=None,
                    steps: int = 5) -> list:
    """busbw of the timed loop itself (torch.distributed, this torch's RCCL, bf16, `nbytes`) under
    each RCCL knob variant of ``rccl_bench.ENV_PROBES``: bench.py runs again in a fresh set of
    `world` rank processes per variant, with the variant in its environment and every extra
    measurement off.  Variants not started within `budget_s` are reported as skipped.  A hung
    variant is killed with its whole process group (its ranks hold GPUs)."""
    import signal
    import subprocess

    from network_operator_amd.parallel import rccl_bench

    base = {k: v for k, v in os.environ.items() if k not in _LAUNCH_ENV and not k.startswith("TORCHELASTIC_")}
    out = []
    t0 = time.monotonic()
    for extra in (variants if variants is not None else rccl_bench.ENV_PROBES):
        left = budget_s - (time.monotonic() - t0)
        if left <= 0:
            out.append({"env": extra, "skipped": "time budget spent"})
            continue
        cmd = [sys.executable, os.path.abspath(__file__), "--gpus", str(world), "--steps", str(steps), "--warmup", "2",
               "--bytes", str(nbytes), "--sweep", "", "--collectives", "", "--node-ready", "off", "--xgmi-probe", "0",
               "--native-rccl", "0", "--xgmi-allreduce", "0", "--rccl-autotune", "0", "--gpu-side", "0",
               "--device", device]
        p = subprocess.Popen(cmd, env=dict(base, **extra), stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                             start_new_session=True)
        try:
            so, se = p.communicate(timeout=left + 30)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.communicate()
            out.append({"env": extra, "error": "timed out"})
            continue
        lines = [x for x in so.splitlines() if x.startswith("{")]
        if p.returncode != 0 or not lines:
            out.append({"env": extra, "error": f"rc={p.returncode}: {se[-300:]}"})
            continue
        j = json.loads(lines[-1])
        out.append({"env": extra, "busbw_GBps": j["busbw_GBps"], "time_us": j["ms_per_step"] * 1e3})
    return out


def autotune_file() -> str:
    return f"/tmp/netop-rccl-autotune-{os.environ.get('MASTER_PORT', '0')}-{os.getppid()}.json"


def _rccl_autotune(rank: int, world: int, nbytes: int, budget_s: float = 120.0,
                   started: float = time.time(), device: str = "cuda", variants=None) -> dict:
    """RCCL reads its parameters once per process, at communicator creation, so they must be
    chosen before init_process_group.

    Rank 0 measures the knob variants of ``rccl_bench.ENV_PROBES`` with bench.py itself
    (``torch_env_probe``: the same torch, RCCL build, dtype and message as the timed loop) over
    the node's first `world` GPUs.  Each variant runs in fresh processes, and all of them must
    fit in ``budget_s``.  Rank 0 publishes the winner through a file in /tmp keyed by the
    rendezvous port, and every rank exports it.  A variant must beat the defaults by >= 3 %
    (``rccl_bench.choose_env``).  (The validation Job tunes a node's ``rccl.env`` the same way
    with the native harness, ``validate.py --tune-rccl``.)  It is still RCCL: only its documented
    environment changes."""
    # Keyed by the launcher's pid as well as the port: every rank of one run shares its parent
    # (torchrun's agent or _spawn_ranks), so a file left by an earlier run on the same port
    # (the driver's N = 2, 4, 8 runs back to back) can never hand this run another world's knobs.
    path = autotune_file()
    if rank == 0:
        try:
            from network_operator_amd.parallel import rccl_bench

            probes = torch_env_probe(world, nbytes, budget_s, device=device, variants=variants)
            doc = dict(rccl_bench.choose_env(probes), probes=probes)
        except Exception as e:  # never leave the other ranks waiting: defaults, and say why
            doc = {"chosen": {}, "error": str(e)[-300:]}
        doc["created"] = time.time()
        tmp = path + f".{os.getpid()}"
        with open(tmp, "w") as f:
            json.dump(doc, f)
        os.replace(tmp, path)
    else:
        deadline = time.time() + budget_s + 300
        doc = None
        while time.time() < deadline:
            try:
                with open(path) as f:
                    d = json.load(f)
                if d.get("created", 0) >= started - 30:  # not a stale file from an earlier run
                    doc = d
                    break
            except (OSError, ValueError):
                pass
            time.sleep(0.2)
        if doc is None:
            return {"error": "rank 0 published no autotune result", "chosen": {}}
    for k, v in doc["chosen"].items():
        os.environ[k] = v
    return doc


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--bytes", type=int, default=1 << 30, help="all-reduce message size per rank")
    ap.add_argument("--sweep", default="4096,1048576,67108864", help="extra sizes (bytes) reported alongside")
    ap.add_argument("--node-ready", choices=["auto", "on", "off"], default="auto")
    ap.add_argument("--node-ready-runs", type=int, default=5)
    ap.add_argument("--collectives", default="all_gather,reduce_scatter,all_to_all",
                    help="other collectives reported at --bytes (n > 1 only)")
    ap.add_argument("--xgmi-probe", type=int, default=1, help="run the HIP xGMI link probe on rank 0 (n > 1)")
    ap.add_argument("--native-rccl", type=int, default=1, help="also run the native netop-rccl-bench harness on rank 0")
    ap.add_argument("--rccl-env-probe", type=int, default=0,
                    help="n > 1: also measure the 1 GiB busbw under RCCL knob variants (a fresh process each)")
    ap.add_argument("--extras-budget", type=float, default=150.0,
                    help="seconds rank 0 may spend on the diagnostics after the timed loop (probe, native "
                         "harness, knob probe, direct all-reduce); later ones are skipped once it is spent")
    ap.add_argument("--rccl-autotune", type=int, default=1,
                    help="n > 1: before RCCL starts, rank 0 measures RCCL knob variants by running this bench "
                         "again per variant (within --rccl-autotune-budget s) and every rank uses the fastest "
                         "(>= 3%% better than the defaults) for the run; 0 = RCCL defaults")
    ap.add_argument("--rccl-autotune-budget", type=float, default=120.0)
    ap.add_argument("--gpu-side", type=int, default=1, help="rank 0: time the agent's unprivileged phases on this box")
    # CPU rehearsal of the autotune plumbing (tests): run it with gloo too, on the first K variants.
    ap.add_argument("--autotune-cpu-variants", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--xgmi-allreduce", type=int, default=1,
                    help="also run the direct two-shot xGMI all-reduce on rank 0 (n > 1)")
    # CPU rehearsal of the multi-rank path (tests): gloo backend, fp32 on the host.
    ap.add_argument("--device", choices=["cuda", "cpu"], default="cuda", help=argparse.SUPPRESS)
    raw_argv = list(sys.argv[1:] if argv is None else argv)
    args = ap.parse_args(raw_argv)
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return _spawn_ranks(args.gpus, raw_argv, args.device)

    import torch
    import torch.distributed as dist

    from network_operator_amd.parallel import collectives as C

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus={args.gpus} but the launcher started WORLD_SIZE={world} ranks", file=sys.stderr)
        return 2
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(_free_port()))
    tuned = None
    if args.device == "cpu":
        device, dtype = torch.device("cpu"), torch.float32
        if args.autotune_cpu_variants and world > 1:
            from network_operator_amd.parallel import rccl_bench

            tuned = _rccl_autotune(rank, world, args.bytes, args.rccl_autotune_budget, device="cpu",
                                   variants=rccl_bench.ENV_PROBES[:args.autotune_cpu_variants])
        dist.init_process_group("gloo", rank=rank, world_size=world)
    else:
        if not torch.cuda.is_available():
            print("bench.py needs an MI355X GPU (torch.cuda.is_available() is False)", file=sys.stderr)
            return 2
        torch.cuda.set_device(local_rank)
        device, dtype = torch.device("cuda", local_rank), torch.bfloat16
        tuned = (_rccl_autotune(rank, world, args.bytes, args.rccl_autotune_budget)
                 if args.rccl_autotune and world > 1 else None)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=device)
    # Host-side group for waiting while rank 0 runs its extra GPU tools: an RCCL barrier would
    # leave a spinning kernel on every other GPU and disturb what those tools measure.
    host_pg = dist.new_group(backend="gloo") if args.device == "cuda" else None
    esize = torch.tensor([], dtype=dtype).element_size()

    # 1. Correctness of the collective path (exact, HIP pattern kernels on the GPU).
    verified, errors = C.verify_all_reduce(min(args.bytes // 2, 64 << 20), device)

    # 2. Headline: K timed all-reduce steps of --bytes per rank.
    numel = (args.bytes // esize) // 8 * 8
    buf = torch.zeros(numel, dtype=dtype, device=device)
    for _ in range(args.warmup):
        dist.all_reduce(buf)
    smi_before, smi_note = None, None
    if rank == 0 and args.device == "cuda":  # xGMI counters (amd-smi), outside the timed region
        try:
            from network_operator_amd.ops import smi

            smi_before = smi.snapshot()
        except Exception as e:
            smi_note = f"amd-smi counters unavailable: {e}"
    dist.barrier()
    C.sync(device)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        dist.all_reduce(buf)
    C.sync(device)
    dt = time.perf_counter() - t0
    dist.barrier()
    xgmi_traffic = None
    if rank == 0 and smi_before is not None:
        try:
            xgmi_traffic = smi.traffic(smi_before, smi.snapshot())
        except Exception as e:
            smi_note = f"amd-smi counters unavailable: {e}"
    t = torch.tensor([dt], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    per_step = dt / max(args.steps, 1)
    nbytes = numel * esize
    algbw, busbw = C.bandwidths("all_reduce", nbytes, world, per_step)
    del buf

    # 3. Size sweep (latency / medium messages), same definitions.
    sweep = []
    sizes = [int(s) for s in args.sweep.split(",") if s.strip()]
    if sizes:
        for r in C.run_sweep("all_reduce", sizes, iters=max(args.steps, 10), warmup=max(args.warmup, 3), device=device,
                             dtype=dtype):
            sweep.append({"bytes": r.bytes, "time_us": r.time_s * 1e6, "algbw_GBps": r.algbw_GBps,
                          "busbw_GBps": r.busbw_GBps})

    # 4. The other collectives RCCL runs over the same links (rccl-tests definitions), n > 1.
    others = []
    if world > 1:
        for op in [o.strip() for o in args.collectives.split(",") if o.strip()]:
            r = C.run_sweep(op, [nbytes], iters=max(args.steps // 2, 5), warmup=2, device=device, dtype=dtype)[0]
            others.append({"op": op, "bytes": r.bytes, "time_us": r.time_s * 1e6, "algbw_GBps": r.algbw_GBps,
                           "busbw_GBps": r.busbw_GBps})

    # 5. xGMI link probe (rank 0, single process over every GPU it can see): per-link pull
    #    bandwidth and all-peers-concurrent aggregate, byte-exact.  Runs after the timed loop.
    probe = None
    t_extras = time.monotonic()

    def budget_left() -> bool:
        return time.monotonic() - t_extras < args.extras_budget

    #    In a child process: this rank holds an RCCL communicator and must survive to print.
    if rank == 0 and world > 1 and args.device == "cuda" and args.xgmi_probe:
        try:
            from network_operator_amd.ops import hip as H

            r = H.xgmi_probe_isolated(64 << 20, iters=5, max_gpus=world, timeout=120)
            links = sorted(x for d, row in enumerate(r["link_GBps"]) for p, x in enumerate(row) if p != d)
            probe = {"gpus": r["gpus"], "errors": r["errors"] + r["push_errors"],
                     "link_GBps": {"min": links[0], "median": links[len(links) // 2], "max": links[-1]} if links else None,
                     "aggregate_GBps": {"min": min(r["aggregate_GBps"]), "max": max(r["aggregate_GBps"])},
                     "push_aggregate_GBps": {"min": min(r["push_aggregate_GBps"]), "max": max(r["push_aggregate_GBps"])}}
        except Exception as e:
            probe = {"error": str(e)[-500:]}

    # 6. Native RCCL harness (rank 0, one process over the first `world` GPUs, RCCL linked
    #    directly, every size checked exactly): a second opinion on the same links that does not
    #    go through torch.distributed.  Runs after the timed loop; failures are reported, not fatal.
    native = None
    if rank == 0 and args.device == "cuda" and args.native_rccl and budget_left():
        try:
            from network_operator_amd.parallel import rccl_bench

            rows = rccl_bench.run(op="all_reduce", gpus=world, min_bytes=1 << 20, max_bytes=1 << 30, factor=32,
                                  iters=20, warmup=5, timeout=120)
            native = {"rows": [{"bytes": r.bytes, "time_us": r.time_us, "algbw_GBps": r.algbw_GBps,
                                "busbw_GBps": r.busbw_GBps, "wrong": r.wrong} for r in rows],
                      "peak_busbw_GBps": max((r.busbw_GBps for r in rows), default=0.0)}
            if world > 1 and args.rccl_env_probe and budget_left():  # knob sensitivity (diagnostic only)
                native["env_probe"] = rccl_bench.env_probe(world, 1 << 30)
        except Exception as e:
            native = {"error": str(e)[-500:]}

    # 7. Direct two-shot xGMI all-reduce (hand-written HIP, all 7 links at once, pull and push),
    #    rank 0 over the first `world` GPUs, exact check of three seeds per size (n > 1).
    direct = None
    if rank == 0 and world > 1 and args.device == "cuda" and args.xgmi_allreduce and budget_left():
        try:
            from network_operator_amd.parallel import xgmi_allreduce as XA

            direct = XA.run(ranks=world, min_bytes=nbytes, max_bytes=nbytes, iters=10, warmup=3, timeout=120)
        except Exception as e:
            direct = {"error": str(e)[-500:]}

    # 8. The same algorithm the way jobs run it: one process per GPU, HIP IPC symmetric buffers,
    #    host-ordered phases (parallel/xgmi_comm.py), in its own process group so a failure there
    #    cannot take this run down.  Exact check of three seeds per size, both algorithms.
    direct_mp = None
    if rank == 0 and world > 1 and args.device == "cuda" and args.xgmi_allreduce and budget_left():
        try:
            from network_operator_amd.parallel import xgmi_comm

            direct_mp = xgmi_comm.run(world, nbytes=nbytes, min_bytes=1 << 20, iters=10, warmup=3, timeout=120)
        except Exception as e:
            direct_mp = {"error": str(e)[-500:]}

    gpu_side = None
    if rank == 0 and args.gpu_side:
        try:
            gpu_side = node_ready_gpu_side()
        except Exception as e:
            gpu_side = {"error": str(e)[-300:]}

    node_ready = None
    node_ready_note = None
    if rank == 0 and args.node_ready != "off":
        try:
            from network_operator_amd.testing import netns

            ok, why = netns.available()
            if ok:
                node_ready = netns.node_ready_bench(n_nics=max(world, 1), runs=args.node_ready_runs, legacy=False)
            else:
                node_ready_note = why
                if args.node_ready == "on":
                    raise RuntimeError(why)
        except Exception as e:  # the collective result stands on its own
            node_ready_note = f"node-ready harness unavailable: {e}"

    dist.barrier(group=host_pg)
    ceiling = C.xgmi_busbw_ceiling_GBps(world)
    # A single-rank in-place all-reduce moves no bytes (RCCL returns at once): bytes/time would be
    # a number with no meaning (round 1 printed 93 TB/s, 12x HBM peak).  Report null and why.
    algbw_note = None
    if world == 1:
        algbw = None
        algbw_note = ("n=1: the timed in-place all-reduce is a no-op in RCCL (no peer, no copy), so algbw is "
                      "not a bandwidth; ms_per_step is its launch latency. busbw is 0 by definition")
        for row in sweep:
            row["algbw_GBps"] = None
    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(busbw, 3),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": per_step * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16" if args.device == "cuda" else "fp32",
            "data": "synthetic (zeros for the timed loop; exact pattern check before timing)",
            "config": {"model": config_name(world), "global_batch": None, "seq_len": None,
                       "parallelism": f"dp{world}", "gpus": world, "message_bytes_per_rank": nbytes,
                       "op": "all_reduce(sum)",
                       "backend": ("torch.distributed nccl (RCCL)" if args.device == "cuda"
                                   else "torch.distributed gloo (CPU rehearsal)")},
            "collectives": others,
            "xgmi_probe": probe,
            "native_rccl": native,
            "rccl_autotune": tuned,
            "xgmi_allreduce": direct,
            "xgmi_allreduce_multiprocess": direct_mp,
            "algbw_GBps": algbw,
            "algbw_note": algbw_note,
            "busbw_GBps": busbw,
            # rccl-tests busbw is per rank; the whole job moves n times that over the links.
            "aggregate_busbw_GBps": busbw * world,
            "busbw_ceiling_GBps": ceiling,
            "busbw_vs_ceiling": (busbw / ceiling) if ceiling else None,
            "verified": verified,
            "verify_errors": errors,
            "sweep": sweep,
            "node_ready": node_ready,
            "node_ready_gpu_side": gpu_side,
            "xgmi_traffic": ({"links_up": xgmi_traffic["links_up"],
                              "links_with_traffic": xgmi_traffic["links_with_traffic"],
                              "GB_per_gpu": [round(sum(g["bytes_per_link"]) / 1e9, 3) for g in xgmi_traffic["gpus"]]}
                             if xgmi_traffic else None),
            "notes": (("n=1: busbw is 0 by definition (rccl-tests factor 2(n-1)/n); " if world == 1 else "")
                      + "reference publishes no numbers (BASELINE.md) so vs_baseline is null") + (f"; {node_ready_note}" if node_ready_note else "")
                     + (f"; {smi_note}" if smi_note else ""),
            "rccl_version": (".".join(str(x) for x in torch.cuda.nccl.version())
                             if args.device == "cuda" and hasattr(torch.cuda, "nccl") else None),
        }
        print(json.dumps(line), flush=True)
    dist.destroy_process_group()
    if rank == 0 and tuned is not None:
        try:
            os.unlink(autotune_file())
        except OSError:
            pass
    return 0 if verified else 1


if __name__ == "__main__":
    sys.exit(main())

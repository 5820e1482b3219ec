"""bench.py driver contract and the multi-rank collective path, rehearsed on the CPU with gloo
(world size 2 and 4) — the N-GPU path is the same code with backend nccl (RCCL)."""

import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
REQUIRED = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config"}


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("n", [2, 4, 8])
def test_bench_torchrun_cpu_rehearsal(n, tmp_path, node_sysfs):
    """The driver's launcher path: torchrun's agent store carries the agent's artifacts to the
    ranks before any communicator exists."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), str(ROOT / "bench.py"), "--gpus", str(n), "--steps", "4",
           "--warmup", "1", "--device", "cpu", "--bytes", str(1 << 20), "--sweep", "4096", "--node-ready", "off",
           "--sysfs-root", node_sysfs]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=tmp_path,
                       env=dict(os.environ, OMP_NUM_THREADS="1"))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    j = json.loads(lines[0])
    assert REQUIRED <= set(j)
    assert j["n_gpus"] == n and j["steps"] == 4 and j["warmup"] == 1
    assert j["verified"] is True and j["verify_errors"] == 0
    assert j["busbw_GBps"] == pytest.approx(j["algbw_GBps"] * 2 * (n - 1) / n, abs=1e-3)
    assert j["value"] == pytest.approx(j["busbw_GBps"] * n, abs=1e-2) == pytest.approx(j["aggregate_busbw_GBps"], abs=1e-2)
    assert j["config"]["parallelism"] == f"dp{n}"
    assert {c["op"] for c in j["collectives"]} == {"all_gather", "reduce_scatter", "all_to_all"}
    assert j["busbw_ceiling_GBps"] == pytest.approx((n - 1) * 76.0)
    a = j["agent_artifacts"]
    assert a["applied"] is True and a["ranks_applied"] == n and a["ranks_same_file"] is True
    assert j["busbw_rccl_defaults_GBps"] > 0


def _bench_line(r):
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [4, 8])
def test_bench_spawns_ranks_without_launcher(n, tmp_path):
    """The driver's per-N runs may call ``python bench.py --gpus N`` with no launcher: bench.py
    must start N ranks itself (round 1 silently measured one)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", str(n), "--steps", "3", "--warmup", "1", "--device", "cpu",
           "--bytes", str(1 << 18), "--sweep", "", "--collectives", "all_gather", "--node-ready", "off"]
    j = _bench_line(subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=tmp_path,
                                   env=dict(env, OMP_NUM_THREADS="1")))
    assert j["n_gpus"] == n and j["config"]["gpus"] == n and j["config"]["parallelism"] == f"dp{n}"
    assert f"{n}xMI355X" in j["config"]["model"]
    assert j["verified"] is True and j["verify_errors"] == 0
    assert j["value"] > 0 and j["busbw_GBps"] == pytest.approx(j["algbw_GBps"] * 2 * (n - 1) / n, abs=1e-3)
    assert j["value"] == pytest.approx(j["busbw_GBps"] * n, abs=1e-2)
    assert j["aggregate_busbw_GBps"] == pytest.approx(j["busbw_GBps"] * n)


def test_bench_single_rank_reports_no_fake_bandwidth(tmp_path):
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "1", "--steps", "3", "--warmup", "1", "--device", "cpu",
           "--bytes", str(1 << 18), "--sweep", "4096", "--node-ready", "off"]
    j = _bench_line(subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=tmp_path))
    assert j["n_gpus"] == 1 and j["value"] == 0.0
    # No netns harness ran (--node-ready off): the line must not claim BASELINE configs[1]
    # (LLDP + NIC up + label), only what did run.
    import bench

    assert j["config"]["model"] != bench.CONFIG_1 and "node-ready not run: --node-ready off" in j["config"]["model"]
    assert j["config"]["model"].startswith("gloo (CPU rehearsal) all-reduce")
    assert j["config"]["skipped"] == ["lldp", "nic_up", "label"] and "rccl_all_reduce" in j["config"]["ran"]
    assert j["algbw_GBps"] is None and "no-op" in j["algbw_note"]
    assert all(row["algbw_GBps"] is None for row in j["sweep"])
    side = j["node_ready_gpu_side"]
    assert set(side["phases_ms"]) >= {"discover", "xgmi", "gdr", "label"} and side["total_ms"] >= 0
    binary = side["agent_binary"]  # the real discover binary, 10 dry runs with the operator's flags
    if "error" in binary:  # a machine without GPUs and NICs (this container): said, not fatal
        assert "No interfaces found" in binary["stderr"], binary
    else:
        assert binary["runs"] == 10 and binary["process_wall_ms"]["p50"] > 0 and "discover" in binary["phases_ms"], binary


def test_bench_rejects_world_mismatch(tmp_path):
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_free_port()))
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "4", "--device", "cpu"], capture_output=True,
                       text=True, timeout=120, cwd=tmp_path, env=env)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    sys.path.insert(0, str(ROOT))
    from network_operator_amd.parallel import collectives as C

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ok, err = C.verify_all_reduce(4096, torch.device("cpu"))
    # a rank that contributes the wrong pattern must be detected on every rank
    buf = C.pattern_reference(4096, 2024, rank if rank else 99)
    dist.all_reduce(buf)
    want = sum(C.pattern_reference(4096, 2024, r) for r in range(world))
    bad = int((buf != want).sum())
    res = C.run_sweep("all_gather", [1 << 16], iters=2, warmup=1, device=torch.device("cpu"), dtype=torch.float32)[0]
    q.put((rank, ok, err, bad, res.bytes, res.n_ranks))
    dist.destroy_process_group()


def test_collectives_gloo_world2():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(60)
    for rank, ok, err, bad, nbytes, n in out:
        assert ok and err == 0
        assert bad > 0
        assert nbytes == 1 << 16 and n == 2


def test_bus_factors_and_ceiling():
    from network_operator_amd.parallel import collectives as C

    assert C.bus_factor("all_reduce", 8) == pytest.approx(1.75)
    assert C.bus_factor("all_gather", 8) == pytest.approx(0.875)
    assert C.bus_factor("all_reduce", 1) == 0
    algbw, busbw = C.bandwidths("all_reduce", 1 << 30, 8, 0.01)
    assert algbw == pytest.approx((1 << 30) / 0.01 / 1e9) and busbw == pytest.approx(algbw * 1.75)
    assert C.xgmi_busbw_ceiling_GBps(8) == pytest.approx(532.0)
    assert C.xgmi_busbw_ceiling_GBps(1) == 0
    assert C.sweep_sizes(8, 64) == [16, 32, 64]


def test_rccl_knob_choice_needs_a_real_gain():
    from network_operator_amd.parallel import rccl_bench as R

    probes = [{"env": {}, "busbw_GBps": 300.0}, {"env": {"NCCL_MIN_NCHANNELS": "64"}, "busbw_GBps": 305.0},
              {"env": {"NCCL_ALGO": "Ring"}, "error": "boom"}, {"env": {"X": "1"}, "skipped": "time budget spent"}]
    assert R.choose_env(probes)["chosen"] == {}  # +1.7 % is noise
    probes.append({"env": {"NCCL_MIN_NCHANNELS": "112"}, "busbw_GBps": 330.0})
    pick = R.choose_env(probes)
    assert pick["chosen"] == {"NCCL_MIN_NCHANNELS": "112"} and pick["baseline_busbw_GBps"] == 300.0
    assert R.choose_env([{"env": {"A": "1"}, "busbw_GBps": 1.0}])["chosen"] == {}  # no baseline, no choice


def test_autotune_measures_variants_with_bench_itself(tmp_path, node_sysfs):
    """The RCCL knob autotune runs bench.py again per variant (fresh rank processes with the
    variant in their environment, on top of the same agent artifacts as the timed loop) and
    publishes the choice to every rank before init."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1", "--device", "cpu",
           "--bytes", str(1 << 18), "--sweep", "", "--collectives", "", "--node-ready", "off",
           "--autotune-cpu-variants", "2", "--rccl-autotune-budget", "120", "--sysfs-root", node_sysfs]
    j = _bench_line(subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=tmp_path,
                                   env=dict(env, OMP_NUM_THREADS="1")))
    t = j["rccl_autotune"]
    assert [p["env"] for p in t["probes"]] == [{}, {"NCCL_MIN_NCHANNELS": "64"}]
    assert all(p.get("busbw_GBps", 0) > 0 for p in t["probes"]), t["probes"]
    assert t["baseline_busbw_GBps"] == t["probes"][0]["busbw_GBps"]
    assert isinstance(t["chosen"], dict)
    assert all(p["artifacts_applied"] for p in t["probes"]), t["probes"]
    assert j["verified"] is True


def test_autotune_budget_skips_late_variants(tmp_path):
    sys.path.insert(0, str(ROOT))
    import bench

    out = bench.torch_env_probe(2, 1 << 16, budget_s=0.0, device="cpu", variants=[{}, {"A": "1"}])
    assert out == [{"env": {}, "skipped": "time budget spent"}, {"env": {"A": "1"}, "skipped": "time budget spent"}]


@pytest.mark.gpu
def test_autotune_probe_runs_the_cuda_bench():
    """The variant runner's command line is accepted by the cuda path (n = 1 on the box: busbw 0)."""
    sys.path.insert(0, str(ROOT))
    import bench

    out = bench.torch_env_probe(1, 1 << 20, budget_s=90, device="cuda", variants=[{}, {"NCCL_MIN_NCHANNELS": "64"}])
    assert [o.get("error") for o in out] == [None, None], out
    assert all(o["busbw_GBps"] == 0.0 and o["time_us"] > 0 for o in out)


def test_autotune_handoff_through_the_rendezvous_store():
    """Rank 0 publishes the knob choice through the run's own rendezvous store (the driver's
    back-to-back N = 2, 4, 8 runs each have theirs), every rank exports it before RCCL starts."""
    import torch.distributed as dist

    sys.path.insert(0, str(ROOT))
    import bench

    store = dist.HashStore()
    store.set(bench.AUTOTUNE_KEY, json.dumps({"chosen": {"NCCL_ALGO": "Ring"}, "probes": []}))
    os.environ.pop("NCCL_ALGO", None)
    try:
        got = bench._rccl_autotune(store, 1, 2, 1 << 20)
        assert got["chosen"] == {"NCCL_ALGO": "Ring"} and os.environ["NCCL_ALGO"] == "Ring"
    finally:
        os.environ.pop("NCCL_ALGO", None)


# ------------------------------------------------------------------------------------------
# The operator's artifacts applied to the timed loop (VERDICT r2 "measure the configured fabric")
# ------------------------------------------------------------------------------------------
def _spawn_env(**extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    return dict(env, OMP_NUM_THREADS="1", **extra)


@pytest.fixture(scope="module")
def node_sysfs(tmp_path_factory):
    from network_operator_amd.testing import fakesysfs

    root = tmp_path_factory.mktemp("sys")
    fakesysfs.build_mi355x_node(root)
    return str(root) + "/"


@pytest.mark.parametrize("n", [2, 4, 8])
def test_bench_applies_agent_artifacts_on_every_rank(n, tmp_path, node_sysfs):
    """Rank 0 runs the agent (discover --dry-run) on the node's sysfs before RCCL starts; every
    rank exports the same NCCL_TOPO_FILE from its rccl.env; a fresh-process run without them is
    the A/B."""
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", str(n), "--steps", "3", "--warmup", "1", "--device", "cpu",
           "--bytes", str(1 << 16), "--sweep", "", "--collectives", "", "--node-ready", "off",
           "--sysfs-root", node_sysfs]
    j = _bench_line(subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=tmp_path, env=_spawn_env()))
    a = j["agent_artifacts"]
    assert a["applied"] is True, a
    assert a["ranks_applied"] == n and a["ranks_same_file"] is True
    assert a["topo_file_bytes"] > 1000 and a["env"] == {"NCCL_TOPO_FILE": a["topo_file"]}
    assert a["agent_status"]["xgmi_pairs"] == "28/28"
    assert [r["rank"] for r in a["per_rank"]] == list(range(n))
    assert {r["NCCL_TOPO_FILE"] for r in a["per_rank"]} == {a["topo_file"]}
    assert {r["topo_sha256"] for r in a["per_rank"]} == {a["topo_sha256"]}
    assert j["config"]["rccl_env"].startswith("agent artifacts")
    assert j["busbw_rccl_defaults_GBps"] > 0 and j["rccl_defaults"]["verified"] is True
    assert j["value"] > 0 and j["extras_log"][0]["extra"] == "rccl_defaults"
    assert not os.path.exists(a["dir"])  # scratch removed


def test_bench_applies_an_artifact_directory(tmp_path, node_sysfs):
    """--artifacts DIR: what a job on a configured node sources (rccl.env, then rccl-tuned.env)."""
    from network_operator_amd.parallel import fabric_artifacts as FA

    d = tmp_path / "scale-out"
    doc = FA.generate(str(d), sysfs_root=node_sysfs, env_extra="NCCL_MIN_NCHANNELS=32")
    assert "error" not in doc, doc
    (d / "rccl-tuned.env").write_text("# tuned\nNCCL_MIN_NCHANNELS=64\n")
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1", "--device", "cpu",
           "--bytes", str(1 << 16), "--sweep", "", "--collectives", "", "--node-ready", "off", "--rccl-defaults", "0",
           "--artifacts", str(d)]
    j = _bench_line(subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=tmp_path, env=_spawn_env()))
    a = j["agent_artifacts"]
    assert a["applied"] and a["env"] == {"NCCL_TOPO_FILE": str(d / "rccl-topo.xml"), "NCCL_MIN_NCHANNELS": "64"}
    assert a["ranks_applied"] == 2 and j["rccl_defaults"] is None
    assert (d / "rccl.env").exists()  # never removed: not the bench's scratch


def test_bench_hung_extra_still_prints_one_line(tmp_path, node_sysfs):
    """A diagnostic that hangs on first contact (here the RCCL-defaults A/B) is killed at the
    deadline with its whole process tree; the headline line still comes out, rc 0."""
    import time as _t

    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "4", "--steps", "3", "--warmup", "1", "--device", "cpu",
           "--bytes", str(1 << 16), "--sweep", "", "--collectives", "", "--node-ready", "off",
           "--sysfs-root", node_sysfs, "--deadline-s", "30"]
    t = _t.monotonic()
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120, cwd=tmp_path,
                       env=_spawn_env(NETOP_BENCH_HANG_EXTRA="rccl_defaults"))
    took = _t.monotonic() - t
    j = _bench_line(r)
    assert took < 30 + 15, took
    assert j["value"] > 0 and j["verified"] is True and j["agent_artifacts"]["applied"]
    assert j["rccl_defaults"]["error"] == "deadline" and j["rccl_defaults"]["timed_out"] is True
    assert j["busbw_rccl_defaults_GBps"] is None
    assert j["extras_log"] == [dict(j["rccl_defaults"], extra="rccl_defaults")]


def test_bench_watchdog_prints_when_rank0_hangs(tmp_path):
    """Rank 0 stuck after the timed loop: the deadline watchdog prints the measured line and every
    rank exits 0."""
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1", "--device", "cpu",
           "--bytes", str(1 << 16), "--sweep", "", "--collectives", "", "--node-ready", "off", "--deadline-s", "20"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120, cwd=tmp_path,
                       env=_spawn_env(NETOP_BENCH_HANG_EXTRA="rank0-after-headline"))
    j = _bench_line(r)
    assert j["value"] > 0 and j["n_gpus"] == 2 and "deadline" in r.stderr


def test_extras_runner_kills_the_whole_tree():
    import time as _t

    import psutil

    from network_operator_amd.parallel import bench_extras as E

    runner = E.Runner(_t.monotonic() + 60)
    # a child that starts a grandchild in a session of its own, then hangs
    code = ("import subprocess,sys,time; p=subprocess.Popen([sys.executable,'-c','import time; time.sleep(600)'],"
            "start_new_session=True); print(p.pid, flush=True); time.sleep(600)")
    before = {p.pid for p in psutil.process_iter()}
    got = runner.run("t", [sys.executable, "-c", code], cap_s=3)
    assert got["error"] == "timed out" and got["limit_s"] == 3
    _t.sleep(0.5)
    left = [p for p in psutil.process_iter(["cmdline"]) if p.pid not in before
            and "time.sleep(600)" in " ".join(p.info["cmdline"] or [])]
    assert not left, left
    assert runner.extra("sleep", 30, seconds=0.1) == {"slept": 0.1}
    late = E.Runner(_t.monotonic() + 1)
    assert late.extra("sleep", 30, seconds=0.1)["error"] == "deadline"


def _dump(gpus, links, nets=()):
    """An RCCL-style topology dump: gpus = [(busid, chain)], links = {busid: [targets]}."""
    body = []
    for b, chain in gpus:
        x = "".join(f'<xgmi target="{t}" count="1" tclass="0x038000"/>' for t in links.get(b, []))
        inner = f'<pci busid="{b}" class="0x120000"><gpu dev="0" rank="0" gcn="gfx950">{x}</gpu></pci>'
        for c in reversed(chain):
            inner = f'<pci busid="{c}" class="0x060400">{inner}</pci>'
        body.append(inner)
    n = "".join(f'<pci busid="{c}"><nic><net name="{nm}"/></nic></pci>' for nm, c in nets)
    return f'<system version="2"><cpu numaid="0">{"".join(body)}{n}</cpu></system>'


def test_rccl_view_counts_xgmi_links_and_compares_ancestry():
    from network_operator_amd.parallel import fabric_artifacts as FA

    g = [("0000:0a:00.0", ["0000:01:00.0"]), ("0000:23:00.0", ["0000:1c:00.0"]), ("0000:5a:00.0", ["0000:53:00.0"])]
    full = {a: [b for b, _ in g if b != a] + ["0000:f1:00.0"] for a, _ in g}  # + a GPU outside the job
    dump = _dump(g, full, nets=[("mlx5_1", "0000:05:00.0")])
    v = FA.rccl_view(dump, _dump(g, {}, nets=[("mlx5_1", "0000:05:00.0")]))
    assert v["gpus"] == 3 and v["min_xgmi_links"] == 2 and v["xgmi_elements"] == 9
    assert v["gpu_ancestry_equal"] and v["nic_ancestry_equal"] and v["nets_from_file"] == ["mlx5_1"]
    assert FA.links_verdict(3, v, None)["status"] == "ok"
    # the file moved one GPU under another switch
    moved = FA.rccl_view(dump, _dump([g[0], ("0000:23:00.0", ["0000:99:00.0"]), g[2]], {}))
    assert not moved["gpu_ancestry_equal"] and list(moved["gpu_ancestry_diff"]) == ["0000:23:00.0"]
    # one GPU lost a link under the file, while RCCL sees all of them without it: fail
    lost = dict(full, **{"0000:0a:00.0": ["0000:23:00.0"]})
    bad = FA.rccl_view(_dump(g, lost))
    verdict = FA.links_verdict(3, bad, v)
    assert verdict["status"] == "failed" and "costs links" in verdict["why"] and verdict["file_blamed"]
    # fewer than n-1 with nothing to compare: reported failed, but the file is not blamed (the
    # bench then keeps rc 0: its number is a real measurement of this fabric)
    alone = FA.links_verdict(3, bad, None)
    assert alone["status"] == "failed" and not alone.get("file_blamed")
    # the dump misses a GPU of the job
    assert FA.links_verdict(4, v, None)["status"] == "failed"
    # no <xgmi> elements at all, with and without the file: this RCCL records them elsewhere
    none = FA.rccl_view(_dump(g, {}))
    assert FA.links_verdict(3, none, none)["status"] == "unverifiable"
    assert FA.links_verdict(3, None, v)["status"] == "failed"
    assert FA.links_verdict(1, None, None)["status"] == "ok"


def test_env_file_parsing_keeps_exact_match_prefix(tmp_path):
    from network_operator_amd.parallel import fabric_artifacts as FA

    (tmp_path / "rccl.env").write_text("# c\nNCCL_IB_HCA==mlx5_0:1,mlx5_1:1\n\nexport NCCL_TOPO_FILE=/x.xml\nBAD\n")
    (tmp_path / "rccl-tuned.env").write_text("NCCL_MIN_NCHANNELS=64\n")
    assert FA.load_env_dir(str(tmp_path)) == {"NCCL_IB_HCA": "=mlx5_0:1,mlx5_1:1", "NCCL_TOPO_FILE": "/x.xml",
                                              "NCCL_MIN_NCHANNELS": "64"}
    env = {"NCCL_TOPO_FILE": "/x.xml", "NCCL_TOPO_DUMP_FILE": "/d", "PATH": "/bin"}
    assert FA.strip(env, ["NCCL_TOPO_FILE"]) == {"PATH": "/bin"}


@pytest.mark.parametrize("lost", [False, True])
def test_bench_fails_loudly_when_the_file_costs_xgmi_links(lost, tmp_path, node_sysfs):
    """n > 1: RCCL's dump under the agent's file must show n-1 xGMI peers per GPU.  Rehearsed on
    the CPU with prepared dumps standing in for RCCL's: the line is still printed, with the
    measurement, and the run exits 1 naming the cause."""
    g = [("0000:0a:00.0", ["0000:01:00.0"]), ("0000:23:00.0", ["0000:1c:00.0"])]
    full = {"0000:0a:00.0": ["0000:23:00.0"], "0000:23:00.0": ["0000:0a:00.0"]}
    (tmp_path / "with.xml").write_text(_dump(g, {} if lost else full))
    (tmp_path / "without.xml").write_text(_dump(g, full))
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1", "--device", "cpu",
           "--bytes", str(1 << 16), "--sweep", "", "--collectives", "", "--node-ready", "off",
           "--sysfs-root", node_sysfs]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=tmp_path,
                       env=_spawn_env(NETOP_BENCH_FAKE_RCCL_DUMP=str(tmp_path / "with.xml"),
                                      NETOP_BENCH_FAKE_RCCL_DUMP_DEFAULTS=str(tmp_path / "without.xml")))
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, (r.stdout, r.stderr[-2000:])
    j = json.loads(lines[0])
    chk = j["agent_artifacts"]["xgmi_links_check"]
    assert j["value"] > 0 and j["rccl_defaults"]["rccl_dump"]["min_xgmi_links"] == 1
    if lost:
        assert r.returncode == 1 and chk["status"] == "failed" and "costs links" in chk["why"]
        assert j["error"].startswith("agent artifacts check failed") and "costs links" in r.stderr
    else:
        assert r.returncode == 0 and chk["status"] == "ok" and chk["min_with_file"] == 1 and "error" not in j


def test_link_verdict_takes_the_hardware_counters_as_tie_breaker():
    """amd-smi's per-link counters around the timed loop are the hardware's account of what RCCL
    used: they settle a dump the parser cannot read.  Idle links are reported, not failed (which
    links a collective uses is RCCL's choice of rings)."""
    from network_operator_amd.parallel import fabric_artifacts as FA

    bdfs = ["0000:0a:00.0", "0000:23:00.0", "0000:5a:00.0"]

    def traffic(moved):
        return {"gpus": [{"bdf": b, "bytes_per_link": [moved.get((b, p), 0) for p in bdfs + ["0000:f1:00.0"]],
                          "peer_per_link": bdfs + ["0000:f1:00.0"]} for b in bdfs]}

    all_used = {(a, b): 5 << 30 for a in bdfs for b in bdfs if a != b}
    tv = FA.traffic_view(bdfs[:3], traffic(all_used))
    assert tv["min_links_with_traffic"] == 2 and tv["gpus"] == 3
    g = [(b, ["0000:01:00.0"]) for b in bdfs]
    no_xgmi = FA.rccl_view(_dump(g, {}))
    assert FA.links_verdict(3, no_xgmi, no_xgmi)["status"] == "unverifiable"
    v = FA.links_verdict(3, no_xgmi, no_xgmi, tv)
    assert v["status"] == "ok" and v["dump_status"] == "unverifiable" and "amd-smi" in v["why"]
    # the dump shows every link, but one pair never moved a byte: RCCL's rings chose so; reported only
    full = FA.rccl_view(_dump(g, {a: [b for b in bdfs if b != a] for a in bdfs}))
    idle = dict(all_used)
    idle.pop(("0000:0a:00.0", "0000:5a:00.0"))
    v = FA.links_verdict(3, full, None, FA.traffic_view(bdfs, traffic(idle)))
    assert v["status"] == "ok" and "1 of 2" in v["counters_note"]
    # no <xgmi> in the dump either way and an idle link: still unverifiable, never rescued
    v = FA.links_verdict(3, no_xgmi, no_xgmi, FA.traffic_view(bdfs, traffic(idle)))
    assert v["status"] == "unverifiable" and "counters_note" in v
    assert FA.traffic_view(bdfs, None) is None and FA.traffic_view(["0000:99:00.0"], traffic(all_used)) is None


def test_bench_reports_an_agent_that_cannot_run(tmp_path):
    """No GPU in the sysfs the agent reads: the artifacts are reported as not applied, with the
    agent's own error, the headline still comes out (RCCL defaults), and the other ranks were not
    left waiting for them."""
    (tmp_path / "empty-sys").mkdir()
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1", "--device", "cpu",
           "--bytes", str(1 << 16), "--sweep", "", "--collectives", "", "--node-ready", "off", "--rccl-defaults", "0",
           "--sysfs-root", str(tmp_path / "empty-sys") + "/"]
    j = _bench_line(subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=tmp_path, env=_spawn_env()))
    a = j["agent_artifacts"]
    assert a["applied"] is False and "No interfaces found" in a["error"] and a["ranks_applied"] == 0
    assert j["value"] > 0 and j["verified"] is True


def test_bench_applies_gpu_only_artifacts_on_a_node_without_scale_out_nics(tmp_path, node_sysfs):
    """A node whose GPUs have no scale-out NIC (a compute-only node in the driver's pool): the
    agent's dry run still writes the GPU / xGMI topology file and an intra-node rccl.env, so the
    measurement runs with the agent's artifacts instead of failing the strict check."""
    import shutil

    sysfs = tmp_path / "sys"
    shutil.copytree(node_sysfs, sysfs, symlinks=True)
    for d in (sysfs / "class" / "net").iterdir():
        shutil.rmtree(d) if d.is_dir() and not d.is_symlink() else d.unlink()
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1", "--device", "cpu",
           "--bytes", str(1 << 16), "--sweep", "", "--collectives", "", "--node-ready", "off", "--rccl-defaults", "0",
           "--sysfs-root", str(sysfs) + "/"]
    j = _bench_line(subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=tmp_path, env=_spawn_env()))
    a = j["agent_artifacts"]
    assert a["applied"] is True and a["ranks_applied"] == 2, a
    assert a["agent_status"]["xgmi_pairs"] == "28/28" and a["topo_file_bytes"] > 1000


def test_link_deficit_seen_without_the_file_too_is_not_blamed_on_it():
    from network_operator_amd.parallel import fabric_artifacts as FA

    view = {"gpus": 8, "xgmi_elements": 48, "min_xgmi_links": 6}
    v = FA.dump_verdict(8, view, dict(view))
    assert v["status"] == "degraded" and "with and without the agent's file" in v["why"]
    assert FA.dump_verdict(8, view, dict(view, min_xgmi_links=7))["status"] == "failed"  # the file costs a link
    assert FA.dump_verdict(8, dict(view, min_xgmi_links=7), dict(view, min_xgmi_links=7))["status"] == "ok"


def test_bench_claims_configs_1_only_when_its_node_ready_half_ran():
    """n = 1: the BASELINE.json configs[1] name (mock-switch LLDP -> NIC up -> NFD label) only with
    a node-ready result in the line; a box without the netns harness gets a name for what ran and
    the reason.  n = 2 / 4 keep their per-world-size names; n = 8 keeps configs[2]'s name and says
    what this run did instead of configuring the host RoCE links."""
    from types import SimpleNamespace

    import bench

    args = SimpleNamespace(node_ready="auto", device="cuda")
    ok = {"node_ready": {"fast_start_switch": {"p50_s": 0.009}}, "artifacts": {"applied": True}}
    model, ran, skipped = bench.run_config(args, 1, ok)
    assert model == bench.CONFIG_1 and skipped == [] and {"lldp", "nic_up", "label", "agent_artifacts"} <= set(ran)
    box = {"node_ready": None, "node_ready_note": "node-ready harness unavailable: unshare failed",
           "artifacts": {"applied": True}, "gpu_side": {"total_ms": 4.6}}
    model, ran, skipped = bench.run_config(args, 1, box)
    assert model == ("RCCL all-reduce with the agent's artifacts, 1xMI355X (node-ready not run: node-ready harness "
                     "unavailable: unshare failed)")
    assert skipped == ["lldp", "nic_up", "label"] and ran == ["rccl_all_reduce", "agent_artifacts",
                                                              "agent_gpu_side_phases"]
    for n in (2, 4):
        assert bench.run_config(args, n, box)[0] == bench.config_name(n)
    # n = 8: configs[2]'s name ("... host RoCE links configured ...") with what this run did
    model = bench.run_config(args, 8, box)[0]
    assert model.startswith(bench.config_name(8) + " [this run: RCCL all-reduce over xGMI with the agent's artifacts; "
                                                   "host RoCE links not configured by it (node-ready not run: ")
    assert bench.run_config(args, 8, ok)[0] == bench.config_name(8)


def test_only_the_all_gpu_run_plans_the_direct_xgmi_extras():
    """The driver runs N = 1, 2, 4, 8 back to back on an 8-GPU node: the direct xGMI all-reduces
    (first contact of the hand-written kernels with real peers) run only in the N = 8 run, after
    the RCCL A/B, the native harness and the link probe; a forced --xgmi-allreduce 1 runs them at
    any N > 1."""
    import argparse

    import bench

    def args(**kw):
        d = dict(rccl_defaults=1, artifacts="agent", native_rccl=1, xgmi_probe=1, xgmi_allreduce="auto",
                 node_ready="auto")
        d.update(kw)
        return argparse.Namespace(**d)
    plans = {n: bench.plan_extras(args(), n, gpu=True, device_count=8) for n in (1, 2, 4, 8)}
    assert plans[1] == ["rccl_defaults", "native_rccl", "node_ready"]
    assert plans[2] == plans[4] == ["rccl_defaults", "native_rccl", "xgmi_probe", "node_ready"]
    assert plans[8] == ["rccl_defaults", "native_rccl", "xgmi_probe", "xgmi_allreduce", "xgmi_comm", "node_ready"]
    assert "xgmi_allreduce" in bench.plan_extras(args(xgmi_allreduce="1"), 2, gpu=True, device_count=8)
    assert bench.plan_extras(args(), 8, gpu=False, device_count=0) == ["rccl_defaults", "node_ready"]


def _fake_smi_doc(bdfs, moved_bytes):
    """Two amd-smi snapshots (ops.smi.snapshot's shape): every GPU has its 7 xGMI links up (link 0
    is the self entry, 'X'), and moved `moved_bytes` over each between them."""
    def snap(kb):
        gpus = []
        for b in bdfs:
            peers = ["ffffffffffff:ff:1f.7"] + [p for p in bdfs if p != b]
            gpus.append({"bdf": b, "link_status": "X" + "U" * (len(peers) - 1), "xgmi_link_width": 16,
                         "xgmi_link_speed": 38, "xgmi_read_kb": [0] + [kb] * (len(peers) - 1),
                         "xgmi_write_kb": [0] + [kb] * (len(peers) - 1),
                         "links": [{"peer": p, "type": 2} for p in peers]})
        return {"gpus": gpus}
    return {"before": snap(1000), "after": snap(1000 + moved_bytes // 2048)}


def test_bench_n8_line_is_what_the_scaling_run_will_be_judged_on(tmp_path, node_sysfs):
    """the first real 8-GPU run, rehearsed on the CPU (gloo, 8 ranks) with a
    fake RCCL topology dump (8 GPUs, 7 xGMI peers each, with and without the agent's file) and
    fake amd-smi counters (7 links per GPU, all moving data):

    * ``value`` is the job aggregate, busbw_GBps x 8; busbw_GBps is rccl-tests' per-GPU busbw;
    * ``busbw_ceiling_GBps`` is (n-1) x 76 GB/s = 532 and busbw_vs_ceiling divides by it;
    * the link check passes from the dump and the counters (7 of 7);
    * autotune + headline + extras fit inside --deadline-s: the extras run in their planned order,
      the direct xGMI ones only because N equals the node's GPU count, and the one that would
      overrun is killed at the deadline and the next one never starts -- one line, rc 0."""
    import bench

    n = 8
    bdfs = bench.FAKE_BDFS[:n]
    chains = [(b, [f"0000:{int(b[5:7], 16) - 7:02x}:00.0"]) for b in bdfs]
    full = {b: [p for p in bdfs if p != b] for b in bdfs}
    (tmp_path / "dump.xml").write_text(_dump(chains, full))
    (tmp_path / "smi.json").write_text(json.dumps(_fake_smi_doc(bdfs, 64 << 20)))
    deadline = 75
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", str(n), "--steps", "3", "--warmup", "1", "--device", "cpu",
           "--bytes", str(1 << 18), "--sweep", "", "--collectives", "", "--node-ready", "off",
           "--sysfs-root", node_sysfs, "--deadline-s", str(deadline), "--autotune-cpu-variants", "1",
           "--rccl-autotune-budget", "60"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=deadline + 60, cwd=tmp_path, env=_spawn_env(
        NETOP_BENCH_FAKE_GPUS=str(n), NETOP_BENCH_FAKE_SMI=str(tmp_path / "smi.json"),
        NETOP_BENCH_FAKE_RCCL_DUMP=str(tmp_path / "dump.xml"),
        NETOP_BENCH_FAKE_RCCL_DUMP_DEFAULTS=str(tmp_path / "dump.xml"),
        NETOP_BENCH_FAKE_EXTRA_S="native_rccl=0.2,xgmi_probe=0.2,xgmi_allreduce=3600,xgmi_comm=0.2"))
    j = _bench_line(r)
    assert j["n_gpus"] == n and j["config"]["parallelism"] == "dp8" and "8xMI355X" in j["config"]["model"]
    # per-GPU vs aggregate
    assert j["busbw_GBps"] == pytest.approx(j["algbw_GBps"] * 2 * (n - 1) / n, abs=1e-3)
    assert j["value"] == pytest.approx(j["busbw_GBps"] * n, abs=1e-2) == pytest.approx(j["aggregate_busbw_GBps"], abs=1e-2)
    assert j["aggregate_busbw_rccl_defaults_GBps"] == pytest.approx(j["busbw_rccl_defaults_GBps"] * n, abs=1e-2)
    assert j["busbw_basis"].startswith("per GPU")
    assert j["busbw_ceiling_GBps"] == pytest.approx(7 * 76.0)
    assert j["busbw_vs_ceiling"] == pytest.approx(j["busbw_GBps"] / 532.0)
    # the link check: RCCL's (fake) dump and the (fake) counters both see 7 links per GPU
    chk = j["agent_artifacts"]["xgmi_links_check"]
    assert chk["status"] == "ok" and chk["min_with_file"] == 7 and chk["min_links_with_traffic"] == 7, chk
    assert j["xgmi_traffic"]["job"] == {"gpus": 8, "links_with_traffic_per_gpu": {b: 7 for b in bdfs},
                                        "min_links_with_traffic": 7}
    # autotune ran (one variant) and was folded in before the headline
    assert j["rccl_autotune"]["probes"] and j["rccl_autotune"]["baseline_busbw_GBps"] > 0
    # the extras, in order, within the deadline
    names = [e["extra"] for e in j["extras_log"]]
    assert names == ["rccl_defaults", "native_rccl", "xgmi_probe", "xgmi_allreduce"], j["extras_log"]
    assert j["native_rccl"]["fake"] and j["xgmi_probe"]["fake"]
    assert j["xgmi_allreduce"]["error"] == "deadline" and j["xgmi_allreduce"]["timed_out"]
    assert j["xgmi_allreduce_multiprocess"]["error"] == "deadline"  # never started
    assert "not started" in j["xgmi_allreduce_multiprocess"]["detail"]
    assert j["elapsed_s"] <= deadline + 5
    assert r.returncode == 0


def test_node_ready_unavailable_reason_is_structured_not_the_last_stderr_line(tmp_path):
    """VERDICT r5 weak #7 / do #7: under rocprofv3 the config name carried the profiler's exit log
    line ("... [rocprofv3] tool finalization ...") because the reason was the probe's last stderr
    line.  The reason is now structured ({"code", "why"}) and taken from unshare's own message.
    Here a stand-in unshare fails like the box's and more noise follows it."""
    fake = tmp_path / "bin"
    fake.mkdir()
    (fake / "unshare").write_text(
        "#!/bin/sh\n"
        "echo 'unshare: unshare failed: No space left on device' >&2\n"
        "echo 'W20261018 10:40:26.881727 5014 tool.cpp:98] [rocprofv3] tool finalization :: 0.000368 sec' >&2\n"
        "exit 1\n")
    (fake / "unshare").chmod(0o755)
    env = dict(os.environ, PATH=f"{fake}:{os.environ['PATH']}")
    from network_operator_amd.testing import netns

    old = os.environ["PATH"]
    os.environ["PATH"] = env["PATH"]
    try:
        assert netns.unavailable() == {"code": "unshare", "why": "unshare: unshare failed: No space left on device"}
    finally:
        os.environ["PATH"] = old
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "1", "--steps", "2", "--warmup", "1", "--device", "cpu",
           "--bytes", str(1 << 16), "--sweep", "4096", "--node-ready", "auto"]
    j = _bench_line(subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=tmp_path, env=env))
    model = j["config"]["model"]
    assert model.endswith("(node-ready not run: node-ready harness unavailable: unshare: unshare failed: "
                          "No space left on device)"), model
    assert "rocprofv3" not in json.dumps(j["config"]), j["config"]
    assert j["node_ready_unavailable"] == {"code": "unshare", "why": "unshare: unshare failed: No space left on device"}

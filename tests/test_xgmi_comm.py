"""Multi-process direct xGMI all-reduce (network_operator_amd/parallel/xgmi_comm.py).

CPU: the node-local shared-memory barrier that orders the phases, across real processes
(tests/xgmi_barrier_worker.py).  GPU: the full IPC all-reduce with several rank processes
mapped onto the one GPU of the test box ("virtual ranks"), exact against the pattern sum for
three seeds on reused buffers, both algorithms, and a non-power-of-two rank count."""

import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
WORKER = Path(__file__).resolve().parent / "xgmi_barrier_worker.py"


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _ranks(world, args, limit_s=100, **extra):
    """Runs `world` worker ranks; a rank still running after `limit_s` (each dumps its stacks at
    90 s) is killed and the test fails with every rank's stderr, never by the pytest timeout."""
    import tempfile
    import time

    init = tempfile.NamedTemporaryFile(prefix="netop-store-", delete=False)
    init.close()
    os.unlink(init.name)  # FileStore creates it; a stale file from an earlier run would confuse it
    env = dict(os.environ, **extra, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()), WORLD_SIZE=str(world),
               PYTHONPATH=str(ROOT), NETOP_INIT_FILE=init.name)
    # Output to files, not pipes: waiting on rank 0 while rank 1 fills its pipe (64 KiB of
    # warnings) would block rank 1 in write() and with it every rank's next barrier.
    files = [(tempfile.TemporaryFile(mode="w+"), tempfile.TemporaryFile(mode="w+")) for _ in range(world)]
    procs = [subprocess.Popen([sys.executable, str(WORKER), *args], env=dict(env, RANK=str(r)),
                              stdout=files[r][0], stderr=files[r][1], text=True) for r in range(world)]
    deadline = time.monotonic() + limit_s
    hung = []
    for r, p in enumerate(procs):
        try:
            p.wait(timeout=max(deadline - time.monotonic(), 1))
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
            hung.append(r)
    outs = []
    for fo, fe in files:
        fo.seek(0)
        fe.seek(0)
        outs.append((fo.read(), fe.read()))
        fo.close()
        fe.close()
    try:
        os.unlink(init.name)
    except OSError:
        pass
    report = "\n".join(f"--- rank {r} (rc {p.returncode}) stderr:\n{err[-3000:]}" for r, (p, (_, err)) in
                       enumerate(zip(procs, outs)))
    assert not hung, f"rank(s) {hung} still running after {limit_s} s\n{report}"
    for p, (_, err) in zip(procs, outs):
        assert p.returncode == 0, report
    # each rank's "RESULT ..." line (gloo logs to stdout as well)
    return [next((ln[len("RESULT "):] for ln in o.splitlines() if ln.startswith("RESULT ")), "") for o, _ in outs]


def test_shm_barrier_orders_phases_across_processes(tmp_path):
    outs = _ranks(4, ["order", str(tmp_path)])
    assert all(o.startswith("ok") for o in outs)
    name = outs[0].split()[1]
    assert not Path("/dev/shm" + name).exists()  # unlinked once every rank had mapped it


def test_shm_barrier_times_out_instead_of_hanging():
    word, secs = _ranks(2, ["timeout"])[0].split()
    assert word == "timeout" and 0.4 <= float(secs) < 5


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_xgmi_allreduce_multiprocess_virtual_ranks(cuda_device, world):
    from network_operator_amd.parallel import xgmi_comm

    r = xgmi_comm.run(world, nbytes=16 << 20, min_bytes=1 << 12, iters=3, warmup=1,
                      devices=",".join(["0"] * world), timeout=110)
    assert r["ranks"] == world and r["gpus"] == [0]
    assert r["wrong"] == 0, json.dumps(r)
    assert {x["algo"] for x in r["rows"]} == {"two_shot", "two_shot_push", "one_shot"}
    assert all(x["time_us"] > 0 for x in r["rows"])
    assert [c["op"] for c in r["collectives"]] == ["reduce_scatter", "all_gather"]
    assert all(c["wrong"] == 0 and c["time_us"] > 0 for c in r["collectives"])


@pytest.mark.gpu
def test_xgmi_allreduce_multiprocess_soak_every_call_exact(cuda_device):
    """150 all-reduces over 4 rank processes on the one GPU, each on a fresh pattern and checked
    exactly: the three algorithms in turn, random sizes, every third call straight after the
    previous one (its input refilled while peers may still be reading the last one's)."""
    from network_operator_amd.parallel import xgmi_comm

    r = xgmi_comm.run(4, nbytes=4 << 20, devices="0,0,0,0", timeout=110, soak=150)
    assert r["soak"] == 150 and sum(r["calls"].values()) == 150, json.dumps(r)
    assert r["wrong"] == 0, json.dumps(r)


@pytest.mark.gpu
def test_single_process_xgmi_allreduce_virtual_ranks_exact(cuda_device):
    """netop-xgmi-allreduce (the single-process two-shot bench.py runs on the whole-node run):
    four ranks mapped onto the one GPU run the full algorithm, pull and push, with every chunk,
    cross-stream event and reused buffer; every size exact for three seeds (rc 0, wrong 0)."""
    from network_operator_amd.parallel import xgmi_allreduce

    rows = xgmi_allreduce.run(timeout=110, ranks=4, min_bytes=1 << 20, max_bytes=16 << 20, factor=4, iters=3, warmup=1)
    assert {x["mode"] for x in rows} == {"pull", "push"} and len(rows) == 6
    assert all(x["wrong"] == 0 and x["ranks"] == 4 and x["gpus"] == 1 and x["time_us"] > 0 for x in rows), rows


@pytest.mark.gpu
def test_single_process_xgmi_allreduce_soak_every_call_exact(cuda_device):
    """netop-xgmi-allreduce --soak: 300 calls over 4 ranks on the one GPU, random sizes, pull and
    push in turn, every call on fresh data and checked exactly (rc 3 on any wrong element)."""
    import subprocess

    from network_operator_amd.utils.paths import native_bin

    r = subprocess.run([str(native_bin("netop-xgmi-allreduce")), "--ranks", "4", "-e", str(8 << 20), "--mode", "both",
                        "--soak", "300"], capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    doc = json.loads(r.stdout.strip().splitlines()[-1])
    assert doc["calls"] == {"pull": 150, "push": 150} and doc["wrong"] == {"pull": 0, "push": 0}, doc


@pytest.mark.gpu
def test_xgmi_allreduce_small_buffers_share_one_ipc_segment(cuda_device):
    """64 KiB symmetric buffers come from one caching-allocator segment, so both have the same
    IPC handle: each peer maps it once and addresses both buffers inside it."""
    from network_operator_amd.parallel import xgmi_comm

    r = xgmi_comm.run(2, nbytes=64 << 10, min_bytes=1 << 12, iters=2, warmup=1, devices="0,0", timeout=100)
    assert r["wrong"] == 0, json.dumps(r)


@pytest.mark.gpu
def test_xgmi_allreduce_spawned_from_inside_a_torchrun_job(cuda_device):
    """bench.py's n > 1 path: a torchrun-launched rank starts the multi-process all-reduce in
    its own process group; the launcher's RANK / MASTER_PORT / TORCHELASTIC_* must not leak."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), str(WORKER), "nested"]
    r = subprocess.run(cmd, env=dict(os.environ, PYTHONPATH=str(ROOT)), capture_output=True, text=True, timeout=140)
    assert r.returncode == 0, r.stderr[-2000:]
    line = next(ln for ln in r.stdout.splitlines() if ln.startswith("RESULT "))
    res = json.loads(line[len("RESULT "):])
    assert res == {"launcher_rank": "0", "wrong": 0, "ranks": 2}


def test_algorithm_choice_and_alignment():
    from network_operator_amd.parallel.xgmi_comm import ONE_SHOT_MAX_BYTES, choose_algo

    assert choose_algo(64, 8) == "one_shot"
    assert choose_algo(ONE_SHOT_MAX_BYTES // 2, 8) == "one_shot"
    assert choose_algo(ONE_SHOT_MAX_BYTES, 8) == "two_shot"
    assert choose_algo(ONE_SHOT_MAX_BYTES + 8, 8) == "one_shot"  # does not split into 8 whole chunks
    assert choose_algo(72, 8, "one_shot") == "one_shot"
    with pytest.raises(ValueError, match="algo must be one of"):
        choose_algo(64, 8, "ring")
    with pytest.raises(ValueError, match="multiple of 64"):
        choose_algo(72, 8, "two_shot_push")
    with pytest.raises(ValueError, match="multiple of 8"):
        choose_algo(12, 8, "one_shot")


@pytest.mark.gpu
def test_ddp_hook_trains_like_the_default_allreduce(cuda_device):
    """DDP with the xGMI hook (2 ranks on the box's GPU): parameters after three SGD steps match
    DDP's default fp32 all-reduce within bf16 compression error and are identical on both ranks."""
    res = json.loads(_ranks(2, ["ddp"])[0])
    assert res["ranks_identical"] and res["overlapped_equals_sync"], res
    assert res["max_abs_diff"] < 5e-3, res


@pytest.mark.gpu
def test_reduce_scatter_and_all_gather_exact(cuda_device):
    for res in (json.loads(r) for r in _ranks(3, ["collectives"])):
        assert res == {"reduce_scatter": 0, "all_gather": 0}, res


def test_rail_groups_split_a_two_node_job():
    """node_and_rail_groups for 4 ranks laid out as 2 nodes x 2: node groups {0,1},{2,3}; rail
    groups {0,2},{1,3}; the node group's shm barrier works although its rank 0 is global rank 2."""
    outs = [json.loads(o) for o in _ranks(4, ["rail_groups"], LOCAL_WORLD_SIZE="2")]
    for r, o in enumerate(outs):
        base = 2 * (r // 2)
        assert o == {"node": base + base + 1, "node_size": 2, "rail": (r % 2) + (r % 2 + 2), "rail_size": 2}, (r, o)


@pytest.mark.gpu
def test_rail_allreduce_two_virtual_nodes_exact(cuda_device):
    for res in (json.loads(r) for r in _ranks(4, ["rail"], LOCAL_WORLD_SIZE="2")):
        assert res == {"wrong": 0, "hook_ok": True}, res


def test_rail_segments_stay_vector_aligned():
    from types import SimpleNamespace

    from network_operator_amd.parallel.rail import RailAllReduce

    r = RailAllReduce.__new__(RailAllReduce)
    r.intra, r.segments, r.min_segment_bytes = SimpleNamespace(world=8), 4, 4 << 20
    assert r.segments_for(64 << 20) == 4           # 128 MiB of bf16
    assert r.segments_for(3 << 20) == 1            # 6 MiB: two 3 MiB segments would be under the minimum
    assert r.segments_for((8 << 20) + 128) == 2    # 4 or 3 segments would not split into whole vectors
    assert r.segments_for(192 * 65537) == 3
    r.segments = 1
    assert r.segments_for(64 << 20) == 1


def test_rail_env_pins_each_gpu_to_its_own_nic(tmp_path):
    """rail_env reads the agent's artifacts: NCCL_IB_HCA narrowed to the GPU's paired NIC, by PCI
    address first (HIP order is not PCI order), by the agent's GPU index as a fallback."""
    from network_operator_amd.parallel.rail import rail_env

    entries = [{"NIC_MAC": "02:00:00:00:00:0%d" % i, "NIC_IP": "10.0.%d.1" % i, "SUBNET_MASK": "255.255.255.252",
                "GATEWAY_MAC": "02:00:00:00:01:0%d" % i, "NIC_NAME": "ens%d" % i, "GPU_BDF": bdf, "GPU_INDEX": i,
                "RDMA_DEV": "rdma%d" % i, "RDMA_PORT": 1, "GID_INDEX": 3}
               for i, bdf in enumerate(["0000:05:00.0", "0000:26:00.0", "0000:75:00.0"])]
    (tmp_path / "rccl-net.json").write_text(json.dumps({"NIC_NET_CONFIG": entries}))
    (tmp_path / "rccl.env").write_text("# generated\nNCCL_IB_HCA==rdma0:1,rdma1:1,rdma2:1\nNCCL_IB_GID_INDEX=3\n"
                                       "NCCL_IB_DISABLE=0\nNCCL_IB_TC=106\n")
    env = rail_env("0000:75:00.0", artifact_dir=str(tmp_path))
    assert env == {"NCCL_IB_HCA": "=rdma2:1", "NCCL_IB_GID_INDEX": "3", "NCCL_IB_DISABLE": "0", "NCCL_IB_TC": "106"}
    assert rail_env(None, gpu_index=1, artifact_dir=str(tmp_path))["NCCL_IB_HCA"] == "=rdma1:1"
    with pytest.raises(LookupError):
        rail_env("0000:dc:00.0", artifact_dir=str(tmp_path), sysfs_root=str(tmp_path / "no-sysfs") + "/")


def test_rail_env_without_rccl_net_uses_the_node_topology(tmp_path):
    """L2 mode writes rccl.env but no rccl-net.json: the GPU's rail NIC then comes from the node
    topology (models/topology.NodeTopology over sysfs), i.e. the agent's own GPU<->NIC pairing."""
    from network_operator_amd.models.topology import NodeTopology
    from network_operator_amd.parallel.rail import rail_env
    from network_operator_amd.testing import fakesysfs

    sysfs = tmp_path / "sys"
    fakesysfs.build_mi355x_node(sysfs)
    art = tmp_path / "art"
    art.mkdir()
    (art / "rccl.env").write_text("NCCL_IB_HCA==mlx5_1:1,mlx5_3:1\nNCCL_IB_GID_INDEX=1\n")
    topo = NodeTopology.discover(str(sysfs) + "/")
    assert topo.xgmi.full_mesh and not topo.unpaired_gpus and len(topo.pairs) == 8
    gpu = topo.gpus[3]
    dev, port = topo.rdma_for_gpu(gpu)
    env = rail_env(gpu, artifact_dir=str(art), sysfs_root=str(sysfs) + "/")
    assert env["NCCL_IB_HCA"] == f"={dev}:{port}" and env["NCCL_IB_GID_INDEX"] == "1"


@pytest.mark.gpu
def test_device_bdf_names_the_gpu(cuda_device):
    import re

    from network_operator_amd.parallel.rail import device_bdf

    bdf = device_bdf(0)
    assert re.fullmatch(r"[0-9a-f]{4}:[0-9a-f]{2}:[0-9a-f]{2}\.0", bdf), bdf
    assert os.path.exists(f"/sys/bus/pci/devices/{bdf}")


@pytest.mark.gpu
def test_ipc_open_refuses_a_gpu_it_cannot_reach_before_mapping(cuda_device):
    """netop_ipc_open checks peer access to the exporter's GPU (its PCI bus id,
    published beside the handle) before mapping anything, like the single-process probe.  A GPU
    that is not visible here (or a pair without peer access) is refused with
    hipErrorPeerAccessUnsupported and nothing is mapped; the exporter's own bus id is the GPU's."""
    import ctypes

    import torch

    from network_operator_amd.ops import hip as H
    from network_operator_amd.parallel.rail import device_bdf

    L = H.lib()
    t = torch.empty(1 << 20, dtype=torch.uint8, device=cuda_device)
    h = ctypes.create_string_buffer(L.netop_ipc_handle_size())
    off = ctypes.c_uint64()
    H._check(L.netop_ipc_export(ctypes.c_void_p(t.data_ptr()), h, ctypes.byref(off)), "netop_ipc_export")
    bus = ctypes.create_string_buffer(32)
    H._check(L.netop_ipc_device_bus_id(ctypes.c_void_p(t.data_ptr()), bus, 32), "netop_ipc_device_bus_id")
    assert bus.value.decode().lower() == device_bdf(cuda_device.index or 0), bus.value
    ptr, base = ctypes.c_void_p(), ctypes.c_void_p()
    for unreachable in (b"0000:ff:1f.7", b"not-a-bus-id"):
        rc = L.netop_ipc_open(h.raw, 0, unreachable, ctypes.byref(ptr), ctypes.byref(base))
        assert rc == 217, rc  # hipErrorPeerAccessUnsupported
        assert ptr.value is None and base.value is None  # nothing mapped
    assert L.netop_ipc_open(h.raw, 0, None, ctypes.byref(ptr), ctypes.byref(base)) == 1  # hipErrorInvalidValue
    torch.cuda.synchronize()  # no sticky error left behind


def _pipe_write_blocked(pid):
    """True / False from the kernel's wait channel; None where it does not say (no wchan, or a
    sleeping process without one).  A running process has none: not blocked (yet)."""
    try:
        w = Path(f"/proc/{pid}/wchan").read_text().strip()
        state = Path(f"/proc/{pid}/stat").read_text().rsplit(")", 1)[1].split()[0]
    except (OSError, IndexError):
        return None
    if w in ("", "0"):
        return False if state == "R" else None
    return "pipe_write" in w


def _old_harness(world, args, limit_s, blocked_ranks=()):
    """The harness shape of round 3 before its fix: ranks' stdout and stderr through pipes, read
    one rank at a time (communicate() on rank 0, then rank 1, ...).  Returns (hung ranks, bytes
    each rank managed to write to stderr).  `blocked_ranks`: the limit starts once these are
    blocked writing their pipes (the kernel's wait channel says so), not at the spawn: on a
    loaded machine the ranks' own start (import torch) can take longer than the limit."""
    import time

    store = Path(os.environ.get("TMPDIR", "/tmp")) / f"netop-old-harness-{os.getpid()}"
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()), WORLD_SIZE=str(world),
               PYTHONPATH=str(ROOT), NETOP_INIT_FILE=str(store))
    procs = [subprocess.Popen([sys.executable, str(WORKER), *args], env=dict(env, RANK=str(r)),
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE) for r in range(world)]
    t_start = time.monotonic()
    # (a kernel that never names the wait channel costs this loop's 60 s, not a wrong verdict)
    while blocked_ranks and time.monotonic() < t_start + 60 and all(p.poll() is None for p in procs):
        if all(_pipe_write_blocked(procs[r].pid) for r in blocked_ranks):
            break
        time.sleep(0.05)
    deadline = time.monotonic() + limit_s
    hung = []
    try:
        for r, p in enumerate(procs):
            try:
                p.communicate(timeout=max(deadline - time.monotonic(), 0.1))
            except subprocess.TimeoutExpired:
                hung.append(r)
                break  # the harness never gets past this rank
    finally:
        written = []
        for p in procs:
            p.kill()
        for p in procs:
            _, err = p.communicate()
            written.append(len(err))
        store.unlink(missing_ok=True)
    return hung, written


def test_round3_hang_reproduced_pipes_read_rank_by_rank_deadlock():
    """VERDICT r3 weak #7, pinned on the CPU: ranks 1 and 2 write 256 KiB to stderr before a
    gloo barrier.  Read through pipes rank by rank, rank 0 waits at the barrier for rank 1,
    rank 1 is blocked in write() on its full pipe (exactly the pipe's 64 KiB got through), and
    the harness waits on rank 0: nothing moves until the limit kills it."""
    hung, written = _old_harness(3, ["chatty", str(256 << 10)], limit_s=3, blocked_ranks=(1, 2))
    assert hung == [0], (hung, written)
    assert written[1] == written[2] == 65536, written  # the pipe's capacity, then blocked


def test_round3_hang_does_not_happen_with_the_file_based_harnesses():
    """The same scenario through the harnesses in use now: the test's `_ranks` and
    `xgmi_comm.spawn_ranks` (behind xgmi_comm.run and the bench extras) write rank output to
    files, so every rank finishes."""
    from network_operator_amd.parallel import xgmi_comm

    assert _ranks(3, ["chatty", str(256 << 10)], limit_s=60) == ["ok"] * 3
    procs, outs = xgmi_comm.spawn_ranks(3, [sys.executable, str(WORKER), "chatty", str(256 << 10)], timeout=60)
    assert [p.returncode for p in procs] == [0, 0, 0]
    assert all("RESULT ok" in o for o in outs)
    assert all(o.count("w") >= 256 << 10 for o in outs[1:])  # nothing lost on the way

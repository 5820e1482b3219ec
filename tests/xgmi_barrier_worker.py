"""Rank process for tests/test_xgmi_comm.py: exercises the shared-memory phase barrier.

    RANK=r WORLD_SIZE=n MASTER_ADDR=... MASTER_PORT=... python xgmi_barrier_worker.py order DIR
    ... python xgmi_barrier_worker.py timeout
"""

import faulthandler
import os
import random
import sys
import time

import torch.distributed as dist

from network_operator_amd.parallel.xgmi_comm import ShmBarrier


# A rank that hangs prints every thread's stack and exits, well before the test's own limit, so
# the failure says where it hung (tests/test_xgmi_comm.py::_ranks shows each rank's stderr).
faulthandler.dump_traceback_later(float(os.environ.get("NETOP_RANK_HANG_S", "90")), exit=True)


def _init(rank: int, world: int) -> None:
    """gloo over a FileStore when the test gives one (no TCP port that another process on the
    box could take between the test picking it and rank 0 binding it), else env://."""
    f = os.environ.get("NETOP_INIT_FILE")
    if f:
        dist.init_process_group("gloo", init_method=f"file://{f}", rank=rank, world_size=world)
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)


def main() -> None:
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    _init(rank, world)
    bar = ShmBarrier(rank, world, None)
    if sys.argv[1] == "order":
        # Every rank's marker for phase k must exist once anyone is past barrier k.
        d = sys.argv[2]
        for k in range(60):
            if random.random() < 0.2:
                time.sleep(0.002)
            open(os.path.join(d, f"{k}.{rank}"), "w").close()
            bar.wait(20)
            missing = [r for r in range(world) if not os.path.exists(os.path.join(d, f"{k}.{r}"))]
            assert not missing, (k, missing)
        print("RESULT ok", bar.name, flush=True)
    elif rank == 0:  # "timeout": rank 1 never arrives
        t0 = time.monotonic()
        try:
            bar.wait(0.5)
            print("RESULT no-timeout", flush=True)
        except TimeoutError:
            print("RESULT timeout", round(time.monotonic() - t0, 2), flush=True)
    bar.close()
    dist.barrier()
    dist.destroy_process_group()


def chatty() -> None:
    """The round-3 hang's shape: every rank but 0 writes `NBYTES` (argv[2]) to stderr -- a page of
    warnings -- before a gloo barrier.  Read through pipes one rank at a time, that write blocks
    once the pipe is full and the barrier never completes."""
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    _init(rank, world)
    if rank:
        sys.stderr.write("w" * int(sys.argv[2]))
        sys.stderr.flush()
    dist.barrier()
    print("RESULT ok", flush=True)
    dist.destroy_process_group()


def nested() -> None:
    """Inside a torchrun-launched rank (as bench.py rank 0 does): spawn a 2-rank virtual
    all-reduce on GPU 0 with its own rendezvous, untouched by this job's launcher variables."""
    import json

    from network_operator_amd.parallel import xgmi_comm

    r = xgmi_comm.run(2, nbytes=4 << 20, min_bytes=4 << 20, iters=2, warmup=1, devices="0,0", timeout=100)
    print("RESULT " + json.dumps({"launcher_rank": os.environ.get("RANK"), "wrong": r["wrong"], "ranks": r["ranks"]}),
          flush=True)


def ddp() -> None:
    """Two data-parallel ranks on GPU 0: three SGD steps with DDP reducing gradients through the
    xGMI hook (bf16 on the wire) vs DDP's default all-reduce (fp32 over gloo)."""
    import json

    import torch
    from torch.nn.parallel import DistributedDataParallel as DDP

    from network_operator_amd.parallel.ddp_hooks import (XgmiOverlapState, xgmi_bf16_allreduce_hook,
                                                         xgmi_bf16_allreduce_hook_overlapped)
    from network_operator_amd.parallel.xgmi_comm import XgmiAllReduce

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    _init(rank, world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    params = {}
    for mode in ("reference", "xgmi", "xgmi_overlapped"):
        torch.manual_seed(0)
        net = torch.nn.Sequential(torch.nn.Linear(64, 256), torch.nn.ReLU(), torch.nn.Linear(256, 8)).to(dev)
        model = DDP(net)
        comm = state = None
        if mode == "xgmi":
            comm = XgmiAllReduce(1 << 20, device=dev)
            model.register_comm_hook(comm, xgmi_bf16_allreduce_hook)
        elif mode == "xgmi_overlapped":
            comm = XgmiAllReduce(1 << 20, device=dev)
            state = XgmiOverlapState(comm)
            model.register_comm_hook(state, xgmi_bf16_allreduce_hook_overlapped)
        opt = torch.optim.SGD(model.parameters(), lr=0.1)
        g = torch.Generator().manual_seed(100 + rank)  # different data per rank
        for _ in range(3):
            x, y = torch.randn(32, 64, generator=g).to(dev), torch.randn(32, 8, generator=g).to(dev)
            opt.zero_grad()
            ((model(x) - y) ** 2).mean().backward()
            opt.step()
        params[mode] = torch.cat([p.detach().flatten() for p in model.parameters()]).cpu()
        if state is not None:
            state.close()
        if comm is not None:
            comm.close()
    gathered = [torch.zeros_like(params["xgmi"]) for _ in range(world)]
    dist.all_gather(gathered, params["xgmi"])
    print("RESULT " + json.dumps({"max_abs_diff": float((params["xgmi"] - params["reference"]).abs().max()),
                                  "overlapped_equals_sync": bool(torch.equal(params["xgmi"], params["xgmi_overlapped"])),
                                  "ranks_identical": all(torch.equal(gathered[0], t) for t in gathered)}), flush=True)
    dist.destroy_process_group()


def collectives() -> None:
    """reduce_scatter and all_gather of XgmiAllReduce, two ranks on GPU 0, checked exactly with
    the offset-aware pattern kernels over three seeds on reused buffers."""
    import json

    import torch

    from network_operator_amd.ops import hip as H
    from network_operator_amd.parallel.xgmi_comm import XgmiAllReduce

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    _init(rank, world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    comm = XgmiAllReduce(8 << 20, device=dev)
    wrong = {"reduce_scatter": 0, "all_gather": 0}
    for numel in (8 * world, 4096 * world, (1 << 20) * world):
        chunk = numel // world
        for seed in (21, 22, 23):
            H.fill_pattern(comm.input(numel), seed, rank)
            mine = comm.reduce_scatter(numel)
            wrong["reduce_scatter"] += H.verify_pattern_at(mine, seed, 0, world, rank * chunk)
            H.fill_pattern_at(comm.input(chunk), seed, rank, 1, rank * chunk)
            out = comm.all_gather(chunk)
            for p in range(world):
                wrong["all_gather"] += H.verify_pattern_at(out[p * chunk:(p + 1) * chunk], seed, p, 1, p * chunk)
    comm.close()
    print("RESULT " + json.dumps(wrong), flush=True)
    dist.destroy_process_group()


def rail_groups() -> None:
    """node_and_rail_groups on gloo (CPU): with LOCAL_WORLD_SIZE=2 and 4 ranks, the node group
    of rank r is {2*(r//2), 2*(r//2)+1} and its rail group {r%2, r%2+2}; report each group's
    sum of member ranks."""
    import json

    import torch

    from network_operator_amd.parallel.rail import node_and_rail_groups

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    _init(rank, world)
    node, rail = node_and_rail_groups()
    sums = {}
    for name, g in (("node", node), ("rail", rail)):
        t = torch.tensor([float(rank)])
        dist.all_reduce(t, group=g)
        sums[name] = int(t.item())
        sums[name + "_size"] = dist.get_world_size(g)
    # the shared-memory barrier of a node group whose rank 0 is not global rank 0
    bar = ShmBarrier(dist.get_rank(node), dist.get_world_size(node), node)
    for _ in range(20):
        bar.wait(20)
    bar.close()
    print("RESULT " + json.dumps(sums), flush=True)
    dist.destroy_process_group()


def rail() -> None:
    """RailAllReduce, 4 ranks on GPU 0 laid out as 2 "nodes" x 2 local ranks (gloo carries the
    cross-node step): the result equals the pattern sum over all 4 ranks, three seeds."""
    import json

    import torch

    from network_operator_amd.ops import hip as H
    from network_operator_amd.parallel.rail import RailAllReduce, node_and_rail_groups

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    _init(rank, world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    node, rail_g = node_and_rail_groups()
    comm = RailAllReduce(8 << 20, node, rail_g, device=dev, segments=4, min_segment_bytes=1 << 12)
    wrong = 0
    # 256 elements: one segment; 48048: 3 segments (4 would not split into whole vectors per
    # local rank); 8 MiB: 4 pipelined segments
    for numel in (64 * world, 48048, (1 << 20) * world):
        for seed in (31, 32, 33):
            H.fill_pattern(comm.input(numel), seed, rank)
            wrong += H.verify_pattern_at(comm.all_reduce(numel), seed, 0, world, 0)
    # the DDP hook takes the rail all-reduce too: fp32 bucket of (rank + 1) averages to 2.5
    from network_operator_amd.parallel.ddp_hooks import xgmi_bf16_allreduce_hook

    class Bucket:
        def __init__(self, t):
            self.t = t

        def buffer(self):
            return self.t

    grads = torch.full((1000,), float(rank + 1), device=dev)
    out = xgmi_bf16_allreduce_hook(comm, Bucket(grads)).wait()
    hook_ok = bool(torch.all(out == (world + 1) / 2).item())
    comm.close()
    print("RESULT " + json.dumps({"wrong": wrong, "hook_ok": hook_ok}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    {"chatty": chatty, "nested": nested, "ddp": ddp, "collectives": collectives, "rail_groups": rail_groups, "rail": rail}.get(sys.argv[1] if len(sys.argv) > 1 else "", main)()

"""Direct xGMI all-reduce for one-process-per-GPU jobs (the way torch.distributed runs).

An MI355X node is a full mesh: every GPU has its own xGMI link to each of its 7 peers.  A
two-shot all-reduce in which every GPU reads from every peer at once loads all 7 links by
construction (ring algorithms need many concurrent rings to do the same):

    reduce-scatter  rank d sums chunk d of all n inputs, read straight from the peers' input
                    buffers over xGMI (peer pointers, fp32 accumulation, bf16 RNE);
    all-gather      rank d pulls every other reduced chunk from the rank that owns it.

``two_shot_push`` does the all-gather with remote stores instead (rank d writes its reduced
chunk into every peer's output): xGMI read and write bandwidth differ, so both are measured.
``one_shot`` instead has every rank sum the whole message from all inputs (one phase, n-1 times
the link traffic): the better choice for small messages, where phase overhead dominates.

Each rank owns two *symmetric* buffers (input, output) allocated once, exported with HIP IPC
and mapped by every peer (``native/hip/xgmi_comm.hip``).  Callers write the message into
``comm.input(numel)`` and read the result from the returned ``comm.output(numel)`` view, as
with symmetric-memory collectives.  Phases are ordered on the host — stream synchronize, a
node-local shared-memory barrier, next launch — so no kernel spins on a peer's flag: a rank
that dies costs its peers a barrier timeout (an exception), not a hung GPU.

Bootstrap needs only a host process group (gloo) for the handle exchange; RCCL is not used.
Reference counterpart: none — the reference only writes the collective library's config
(reference cmd/discover/gaudinet.go); this is the MI355X-side proof that the fabric the
operator verified carries collectives at link speed.

    python -m network_operator_amd.parallel.xgmi_comm --world 8 --bytes 1073741824
    python -m network_operator_amd.parallel.xgmi_comm --world 2 --devices 0,0   # virtual ranks
"""

from __future__ import annotations

import argparse
import ctypes
import json
import os
import shutil
import socket
import subprocess
import sys
import tempfile
import time
import uuid
from typing import List, Optional

from ..ops import hip as H

ALGOS = ("two_shot", "two_shot_push", "one_shot")
# Below this size one phase beats two: one_shot moves (n-1)x the bytes but pays one barrier
# less (virtual-rank measurements on MI355X: one_shot wins up to 16 MiB, two_shot from 64 MiB,
# profiles/r1_xgmi_comm_virtual8_n1gpu.json).  Over real xGMI links the crossover is lower.
ONE_SHOT_MAX_BYTES = 4 << 20
MAX_RANKS = 8


def choose_algo(numel: int, world: int, algo: str = "auto") -> str:
    """Validates (numel, algo) and resolves ``auto``: one_shot up to ONE_SHOT_MAX_BYTES (or when
    numel does not split into `world` chunks of whole 16-B vectors), two_shot above."""
    if algo == "auto":
        algo = "one_shot" if numel * 2 <= ONE_SHOT_MAX_BYTES or numel % (8 * world) else "two_shot"
    if algo not in ALGOS:
        raise ValueError(f"algo must be one of {ALGOS} or auto")
    align = 8 if algo == "one_shot" else 8 * world
    if numel % align:
        raise ValueError(f"numel must be a multiple of {align} for {algo}")
    return algo


class ShmBarrier:
    """Node-local sense-reversing barrier in POSIX shared memory (a few µs, vs ~100 µs for a
    gloo barrier).  Rank 0 creates the segment and unlinks its name once everyone mapped it."""

    def __init__(self, rank: int, world: int, group, name: Optional[str] = None):
        import torch.distributed as dist

        L = H.lib()
        names: List[Optional[str]] = [name or f"/netop-xgmi-{uuid.uuid4().hex[:16]}"]
        # `src` is a global rank: the group's rank 0 (a node's local group need not contain rank 0).
        dist.broadcast_object_list(names, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        self.name = names[0]
        self._h = None
        if rank == 0:
            self._h = L.netop_shm_barrier_open(self.name.encode(), world, 1)
            if not self._h:
                raise OSError(f"shm_open({self.name}) failed: cannot create the barrier segment in /dev/shm")
        dist.barrier(group=group)
        if rank != 0:
            self._h = L.netop_shm_barrier_open(self.name.encode(), world, 0)
        ok = [bool(self._h)]
        oks: List[Optional[List[bool]]] = [None] * world
        dist.all_gather_object(oks, ok, group=group)
        if rank == 0:
            L.netop_shm_unlink(self.name.encode())  # mappings stay; nothing is left in /dev/shm
        if not all(o[0] for o in oks):
            self.close()
            raise OSError(f"could not map the barrier segment {self.name} on every rank")

    def wait(self, timeout_s: float = 60.0) -> None:
        rc = H.lib().netop_shm_barrier_wait(self._h, int(timeout_s * 1000))
        if rc:
            raise TimeoutError(f"xGMI all-reduce barrier: a peer did not arrive within {timeout_s} s (rc {rc})")

    def close(self) -> None:
        if self._h:
            H.lib().netop_shm_barrier_close(self._h)
            self._h = None


class XgmiAllReduce:
    """Symmetric-buffer all-reduce over the node's xGMI mesh (bf16 sum)."""

    def __init__(self, capacity_bytes: int, group=None, device=None, timeout_s: float = 60.0, wg_per_cu: int = 4):
        import torch
        import torch.distributed as dist

        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        if not 1 <= self.world <= MAX_RANKS:
            raise ValueError(f"1..{MAX_RANKS} ranks (one node) supported, got {self.world}")
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.timeout_s = timeout_s
        self.wg_per_cu = wg_per_cu
        self.capacity = (int(capacity_bytes) + 255) // 256 * 256
        L = H.lib()
        self.inp = torch.empty(self.capacity, dtype=torch.uint8, device=self.device)
        self.out = torch.empty(self.capacity, dtype=torch.uint8, device=self.device)
        hsz = L.netop_ipc_handle_size()
        mine = []
        for t in (self.inp, self.out):
            h = ctypes.create_string_buffer(hsz)
            off = ctypes.c_uint64()
            H._check(L.netop_ipc_export(ctypes.c_void_p(t.data_ptr()), h, ctypes.byref(off)), "netop_ipc_export")
            mine.append((h.raw, off.value))
        # The exporter's GPU, so every importer checks peer access to it before mapping.
        bus = ctypes.create_string_buffer(32)
        H._check(L.netop_ipc_device_bus_id(ctypes.c_void_p(self.inp.data_ptr()), bus, 32), "netop_ipc_device_bus_id")
        allh: List[Optional[list]] = [None] * self.world
        dist.all_gather_object(allh, {"bus_id": bus.value, "handles": mine}, group=group)
        self._opened: List[int] = []
        self.peer_in: List[int] = []
        self.peer_out: List[int] = []
        try:
            for p in range(self.world):
                if p == self.rank:
                    self.peer_in.append(self.inp.data_ptr())
                    self.peer_out.append(self.out.data_ptr())
                    continue
                # Small buffers can share one caching-allocator segment, i.e. one IPC handle:
                # map each distinct handle once and address both buffers inside it.
                bases = {}
                for (raw, off), dst in zip(allh[p]["handles"], (self.peer_in, self.peer_out)):
                    if raw not in bases:
                        ptr, base = ctypes.c_void_p(), ctypes.c_void_p()
                        H._check(L.netop_ipc_open(raw, 0, allh[p]["bus_id"], ctypes.byref(ptr), ctypes.byref(base)),
                                 f"netop_ipc_open (rank {p}'s GPU {allh[p]['bus_id'].decode()})")
                        self._opened.append(base.value)
                        bases[raw] = base.value
                    dst.append(bases[raw] + off)
            self.barrier = ShmBarrier(self.rank, self.world, group)
        except Exception:
            self._close_handles()
            raise

    # -- buffers ----------------------------------------------------------------------------------
    def _view(self, buf, numel: int):
        import torch

        if numel * 2 > self.capacity:
            raise ValueError(f"{numel} bf16 elements exceed the {self.capacity}-byte symmetric buffer")
        return buf[: numel * 2].view(torch.bfloat16)

    def input(self, numel: int):
        """This rank's contribution goes here (a bf16 view of the symmetric input buffer)."""
        return self._view(self.inp, numel)

    def output(self, numel: int):
        return self._view(self.out, numel)

    # -- collective -------------------------------------------------------------------------------
    def _sync_and_wait(self, stream) -> None:
        stream.synchronize()
        self.barrier.wait(self.timeout_s)

    def all_reduce(self, numel: int, algo: str = "auto"):
        """Sum of every rank's ``input(numel)``, returned as ``output(numel)`` on every rank
        (``algo``: see :func:`choose_algo`)."""
        import torch

        algo = choose_algo(numel, self.world, algo)
        n, d = self.world, self.rank
        self._view(self.inp, numel)  # capacity check
        L = H.lib()
        stream = torch.cuda.current_stream(self.device)
        s = ctypes.c_void_p(stream.cuda_stream)
        vp = ctypes.c_void_p
        self._sync_and_wait(stream)  # every input is complete
        if algo == "one_shot" or n == 1:
            srcs = (vp * n)(*[vp(p) for p in self.peer_in])
            H._check(L.netop_sum_bf16(srcs, n, vp(self.out.data_ptr()), numel, self.wg_per_cu, s), "netop_sum_bf16")
            self._sync_and_wait(stream)  # nobody reads my input any more
            return self.output(numel)
        chunk = numel // n
        cb = chunk * 2
        srcs = (vp * n)(*[vp(p + d * cb) for p in self.peer_in])
        H._check(L.netop_sum_bf16(srcs, n, vp(self.out.data_ptr() + d * cb), chunk, self.wg_per_cu, s),
                 "netop_sum_bf16")
        self._sync_and_wait(stream)  # every reduced chunk is complete
        peers = [p for p in range(n) if p != d]
        if algo == "two_shot":  # all-gather by remote loads: pull chunk p from its owner
            src = (vp * len(peers))(*[vp(self.peer_out[p] + p * cb) for p in peers])
            dst = (vp * len(peers))(*[vp(self.out.data_ptr() + p * cb) for p in peers])
        else:  # two_shot_push: remote stores of my reduced chunk into every peer's output
            src = (vp * len(peers))(*[vp(self.out.data_ptr() + d * cb) for _ in peers])
            dst = (vp * len(peers))(*[vp(self.peer_out[p] + d * cb) for p in peers])
        H._check(L.netop_multi_copy(src, dst, len(peers), cb, self.wg_per_cu, s), "netop_multi_copy")
        self._sync_and_wait(stream)  # every chunk has arrived; nobody touches my buffers any more
        return self.output(numel)

    def reduce_scatter(self, numel: int, offset: int = 0):
        """Rank d gets chunk d of the sum of every rank's ``input(offset + numel)[offset:]``
        (numel / n elements, the first phase of the two-shot all-reduce), as a view into its
        output buffer at ``output(...)[offset + d*chunk:]``.  ``offset`` (a multiple of 8
        elements) lets a caller reduce a long message segment by segment."""
        import torch

        choose_algo(numel, self.world, "two_shot")  # numel splits into n whole-vector chunks
        if offset % 8:
            raise ValueError("offset must be a multiple of 8 elements")
        self._view(self.inp, offset + numel)
        n, d = self.world, self.rank
        chunk = numel // n
        cb, ob = chunk * 2, offset * 2
        stream = torch.cuda.current_stream(self.device)
        vp = ctypes.c_void_p
        self._sync_and_wait(stream)
        srcs = (vp * n)(*[vp(p + ob + d * cb) for p in self.peer_in])
        H._check(H.lib().netop_sum_bf16(srcs, n, vp(self.out.data_ptr() + ob + d * cb), chunk, self.wg_per_cu,
                                        vp(stream.cuda_stream)), "netop_sum_bf16")
        self._sync_and_wait(stream)  # nobody reads my input any more
        return self.output(offset + numel)[offset + d * chunk:offset + (d + 1) * chunk]

    def all_gather(self, chunk: int):
        """Every rank's ``input(chunk)``, concatenated in rank order, on every rank (a view of
        ``output(n * chunk)``); each rank pulls the n-1 peer chunks over their own links."""
        import torch

        if chunk % 8:
            raise ValueError("chunk must be a multiple of 8 elements")
        n, d = self.world, self.rank
        self._view(self.out, n * chunk)
        cb = chunk * 2
        stream = torch.cuda.current_stream(self.device)
        vp = ctypes.c_void_p
        self._sync_and_wait(stream)  # every contribution is complete
        src = (vp * n)(*[vp(self.peer_in[p]) for p in range(n)])  # own chunk too: a local copy
        dst = (vp * n)(*[vp(self.out.data_ptr() + p * cb) for p in range(n)])
        H._check(H.lib().netop_multi_copy(src, dst, n, cb, self.wg_per_cu, vp(stream.cuda_stream)),
                 "netop_multi_copy")
        self._sync_and_wait(stream)  # nobody reads my input any more
        return self.output(n * chunk)

    def all_gather_inplace(self, numel: int, offset: int = 0):
        """Every rank p already holds chunk p of the message at ``output(...)[offset + p*chunk:]``
        (e.g. after :meth:`reduce_scatter` and a cross-node step on that chunk); fill in the
        other n-1 chunks from their owners — the second phase of the two-shot all-reduce.
        Returns the whole ``numel``-element message at ``offset``."""
        import torch

        choose_algo(numel, self.world, "two_shot")
        if offset % 8:
            raise ValueError("offset must be a multiple of 8 elements")
        self._view(self.out, offset + numel)
        n, d = self.world, self.rank
        cb, ob = numel // n * 2, offset * 2
        stream = torch.cuda.current_stream(self.device)
        vp = ctypes.c_void_p
        self._sync_and_wait(stream)  # every owned chunk is final
        peers = [p for p in range(n) if p != d]
        src = (vp * len(peers))(*[vp(self.peer_out[p] + ob + p * cb) for p in peers])
        dst = (vp * len(peers))(*[vp(self.out.data_ptr() + ob + p * cb) for p in peers])
        H._check(H.lib().netop_multi_copy(src, dst, len(peers), cb, self.wg_per_cu, vp(stream.cuda_stream)),
                 "netop_multi_copy")
        self._sync_and_wait(stream)
        return self.output(offset + numel)[offset:]

    # -- lifetime ---------------------------------------------------------------------------------
    def _close_handles(self) -> None:
        L = H.lib()
        for base in self._opened:
            L.netop_ipc_close(ctypes.c_void_p(base))
        self._opened = []

    def close(self) -> None:
        import torch.distributed as dist

        # Peers may still be mapped onto our buffers until they are past their last phase.
        dist.barrier(group=self.group)
        self._close_handles()
        if getattr(self, "barrier", None):
            self.barrier.close()


# ---------------------------------------------------------------------------------------------
# Benchmark / self-test: `--world N` spawns N ranks (env RANK / WORLD_SIZE, gloo bootstrap)
# ---------------------------------------------------------------------------------------------
def _worker(args) -> int:
    import torch
    import torch.distributed as dist

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    devices = [int(x) for x in args.devices.split(",")] if args.devices else list(range(world))
    dev = torch.device("cuda", devices[rank % len(devices)])
    torch.cuda.set_device(dev)
    store = os.environ.get("NETOP_INIT_FILE")  # run(): a FileStore, no TCP port to race for
    dist.init_process_group("gloo", init_method=f"file://{store}" if store else None, rank=rank, world_size=world)
    sizes = []
    b = args.min_bytes
    while b <= args.bytes:
        sizes.append(b)
        b *= 4
    if not sizes or sizes[-1] != args.bytes:
        sizes.append(args.bytes)
    comm = XgmiAllReduce(args.bytes, device=dev, timeout_s=args.timeout)
    if args.soak:
        return _soak(args, comm, rank, world)

    def measure(fn, check, nbytes: int, factor: float, **row) -> dict:
        """Three exact checks (seeds on reused buffers), warmup, `iters` timed calls; max time
        and summed mismatches over the ranks."""
        wrong = sum(check(seed) for seed in (11, 12, 13))
        for _ in range(args.warmup):
            fn()
        torch.cuda.synchronize(dev)
        comm.barrier.wait(args.timeout)
        t0 = time.perf_counter()
        for _ in range(args.iters):
            fn()
        torch.cuda.synchronize(dev)
        t = torch.tensor([(time.perf_counter() - t0) / args.iters], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        w = torch.tensor([wrong], dtype=torch.int64)
        dist.all_reduce(w, op=dist.ReduceOp.SUM)
        dt = float(t[0])
        algbw = nbytes / dt / 1e9
        return dict(row, bytes=nbytes, time_us=dt * 1e6, algbw_GBps=algbw, busbw_GBps=algbw * factor, wrong=int(w[0]))

    rows = []
    for nbytes in sizes:
        for algo in args.algos.split(","):
            align = 8 if algo == "one_shot" else 8 * world
            numel = max(align, nbytes // 2 // align * align)

            def check_ar(seed, numel=numel, algo=algo):
                H.fill_pattern(comm.input(numel), seed, rank)
                return H.verify_sum(comm.all_reduce(numel, algo), seed, world)

            rows.append(measure(lambda numel=numel, algo=algo: comm.all_reduce(numel, algo), check_ar, numel * 2,
                                2 * (world - 1) / world, algo=algo))
    # The two phases as collectives of their own, at the largest size (rccl-tests sizes: the
    # full input of reduce_scatter, the full output of all_gather; bus factor (n-1)/n).
    numel = max(8 * world, args.bytes // 2 // (8 * world) * (8 * world))
    chunk = numel // world

    def check_rs(seed):
        H.fill_pattern(comm.input(numel), seed, rank)
        return H.verify_pattern_at(comm.reduce_scatter(numel), seed, 0, world, rank * chunk)

    def check_ag(seed):
        H.fill_pattern_at(comm.input(chunk), seed, rank, 1, rank * chunk)
        out = comm.all_gather(chunk)
        return sum(H.verify_pattern_at(out[p * chunk:(p + 1) * chunk], seed, p, 1, p * chunk) for p in range(world))

    collectives = [measure(lambda: comm.reduce_scatter(numel), check_rs, numel * 2, (world - 1) / world,
                           op="reduce_scatter"),
                   measure(lambda: comm.all_gather(chunk), check_ag, numel * 2, (world - 1) / world, op="all_gather")]
    comm.close()
    if rank == 0:
        devs = sorted({devices[r % len(devices)] for r in range(world)})
        print(json.dumps({"ranks": world, "gpus": devs, "rows": rows, "collectives": collectives,
                          "peak_busbw_GBps": max((r["busbw_GBps"] for r in rows), default=0.0),
                          "wrong": sum(r["wrong"] for r in rows + collectives)}), flush=True)
    dist.destroy_process_group()
    return 0


def _soak(args, comm, rank: int, world: int) -> int:
    """`--soak N`: N all-reduces, each on a fresh pattern and each checked exactly, cycling the
    algorithms over sizes drawn (same seed on every rank) from 4 KiB to --bytes, every third
    call straight after the previous one without a host round trip in between.  What a timed
    loop cannot show: a flag, barrier or buffer-reuse race that corrupts one call in hundreds."""
    import random

    import torch
    import torch.distributed as dist

    rng = random.Random(20261018)
    algos = args.algos.split(",")
    wrong = {a: 0 for a in algos}
    calls = {a: 0 for a in algos}
    t0 = time.perf_counter()
    for i in range(args.soak):
        algo = algos[i % len(algos)]
        align = 8 if algo == "one_shot" else 8 * world
        numel = max(align, rng.randrange(2048, args.bytes // 2 + 1) // align * align)
        seed = 1000 + i
        H.fill_pattern(comm.input(numel), seed, rank)
        out = comm.all_reduce(numel, algo)
        if i % 3 == 2:  # back to back: the next call's fill and exchange race this one's readers
            H.fill_pattern(comm.input(numel), seed + 7, rank)
            out = comm.all_reduce(numel, algo)
            seed += 7
        wrong[algo] += H.verify_sum(out, seed, world)
        calls[algo] += 1
    torch.cuda.synchronize()
    w = torch.tensor([wrong[a] for a in algos], dtype=torch.int64)
    dist.all_reduce(w, op=dist.ReduceOp.SUM)
    if rank == 0:
        print(json.dumps({"ranks": world, "soak": args.soak, "seconds": round(time.perf_counter() - t0, 2),
                          "calls": calls, "wrong_by_algo": {a: int(x) for a, x in zip(algos, w.tolist())},
                          "wrong": int(w.sum())}), flush=True)
    comm.close()
    dist.destroy_process_group()
    return 0


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


_LAUNCHER_ENV = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK", "ROLE_WORLD_SIZE",
                 "MASTER_ADDR", "MASTER_PORT", "GROUP_WORLD_SIZE", "ROLE_NAME")


def spawn_ranks(world: int, cmd: list, timeout: float, extra_env: Optional[dict] = None) -> tuple:
    """Starts `world` copies of `cmd` as ranks 0..world-1 with their own FileStore rendezvous and
    none of a parent launcher's variables; waits for all of them.  Returns (processes, outputs);
    raises TimeoutError (every rank killed) when they are not done within `timeout`.

    Output goes to temporary files, not pipes.  With pipes read one rank at a time, a rank that
    writes more than the pipe holds (64 KiB: a page of warnings) blocks in write() while the
    parent waits on another rank, and that rank waits for it at the next barrier: the round-3 GPU
    test hang, reproduced on the CPU by tests/test_xgmi_comm.py."""
    base = {k: v for k, v in os.environ.items() if k not in _LAUNCHER_ENV and not k.startswith("TORCHELASTIC_")}
    # Rendezvous over a FileStore: a free TCP port picked here could be taken by another process
    # before rank 0 binds it, and the other ranks would then wait for a store that never comes.
    store_dir = tempfile.mkdtemp(prefix="netop-xgmi-store-")
    base.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE=str(world),
                NETOP_INIT_FILE=os.path.join(store_dir, "store"), **(extra_env or {}))
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    base["PYTHONPATH"] = root + (os.pathsep + base["PYTHONPATH"] if base.get("PYTHONPATH") else "")
    logs = [tempfile.TemporaryFile(mode="w+") for _ in range(world)]
    procs = [subprocess.Popen(cmd, env=dict(base, RANK=str(r), LOCAL_RANK=str(r)), stdout=logs[r],
                              stderr=subprocess.STDOUT, text=True, cwd=root) for r in range(world)]
    deadline = time.monotonic() + timeout
    try:
        for p in procs:
            p.wait(timeout=max(1.0, deadline - time.monotonic()))
    except subprocess.TimeoutExpired:
        for p in procs:
            p.kill()
        for p in procs:
            p.wait()
        shutil.rmtree(store_dir, ignore_errors=True)
        raise TimeoutError(f"ranks did not finish within {timeout} s")
    outs = []
    for f in logs:
        f.seek(0)
        outs.append(f.read())
        f.close()
    shutil.rmtree(store_dir, ignore_errors=True)
    return procs, outs


def run(world: int, nbytes: int = 1 << 30, min_bytes: Optional[int] = None, iters: int = 10, warmup: int = 3,
        algos: str = ",".join(ALGOS), devices: Optional[str] = None, timeout: float = 120.0, soak: int = 0) -> dict:
    """Spawns `world` rank processes (one per GPU unless `devices` maps several onto one) and
    returns rank 0's result.  Safe to call from inside another distributed job: the children
    get their own rendezvous and none of the parent's launcher variables."""
    cmd = [sys.executable, "-m", "network_operator_amd.parallel.xgmi_comm", "--worker", "--bytes", str(nbytes),
           "--min-bytes", str(min_bytes or nbytes), "--iters", str(iters), "--warmup", str(warmup), "--algos", algos,
           "--timeout", str(min(timeout, 60.0))]
    if devices:
        cmd += ["--devices", devices]
    if soak:
        cmd += ["--soak", str(soak)]
    procs, outs = spawn_ranks(world, cmd, timeout)
    bad = [(r, p.returncode, o[-1500:]) for r, (p, o) in enumerate(zip(procs, outs)) if p.returncode != 0]
    if bad:
        raise RuntimeError(f"rank {bad[0][0]} exited {bad[0][1]}: {bad[0][2]}")
    line = [x for x in outs[0].splitlines() if x.startswith("{")]
    if not line:
        raise RuntimeError(f"no result from rank 0: {outs[0][-1500:]}")
    return json.loads(line[-1])


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m network_operator_amd.parallel.xgmi_comm")
    ap.add_argument("--world", type=int, default=0, help="spawn this many ranks (0: all visible GPUs)")
    ap.add_argument("--worker", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--bytes", type=int, default=1 << 30)
    ap.add_argument("--min-bytes", type=int, default=0)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--algos", default=",".join(ALGOS))
    ap.add_argument("--devices", default="", help="comma list of GPU ids per rank (repeats allowed: virtual ranks)")
    ap.add_argument("--timeout", type=float, default=120.0)
    ap.add_argument("--soak", type=int, default=0, help="instead of timing: this many all-reduces, each checked exactly")
    a = ap.parse_args(argv)
    if a.worker:
        if not a.min_bytes:
            a.min_bytes = a.bytes
        return _worker(a)
    world = a.world
    if world <= 0:
        import torch

        world = torch.cuda.device_count()
    print(json.dumps(run(world, a.bytes, a.min_bytes or None, a.iters, a.warmup, a.algos, a.devices or None,
                         a.timeout, a.soak)))
    return 0


if __name__ == "__main__":
    sys.exit(main())

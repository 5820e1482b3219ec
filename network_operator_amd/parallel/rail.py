"""Rail-aligned two-level all-reduce for multi-node jobs on MI355X nodes.

The operator gives every GPU its own scale-out NIC (the GPU-affine RoCE NIC behind the same
PCIe switch, ``rccl.env``'s ``NCCL_IB_HCA`` in GPU order) and routes each rail's /30s through
the switch's /16.  A data-parallel all-reduce over several such nodes then splits naturally:

1. **intra-node reduce-scatter over xGMI** (:class:`XgmiAllReduce`): local rank d ends up with
   chunk d of its node's sum, read from all 7 peers at once;
2. **inter-node all-reduce of chunk d on rail d**: only ranks with the same local rank talk
   across nodes (``torch.distributed`` group per rail, RCCL over that GPU's own NIC), so the 8
   NICs of a node carry 8 different chunks in parallel and no bytes cross PCIe to another GPU's NIC;
3. **intra-node all-gather over xGMI** of the final chunks.

Each NIC moves 2(N-1)/N of 1/8 of the message for N nodes — the bandwidth-optimal split for
8 rails — while xGMI does the rest.  Reference counterpart: none (the reference stops at
writing the collective library's configuration, cmd/discover/gaudinet.go).
"""

from __future__ import annotations

import json
import os
from typing import Dict, Optional, Tuple

from .xgmi_comm import XgmiAllReduce

ARTIFACT_DIR = "/etc/amd/scale-out"  # where the agent writes rccl-net.json / rccl.env on the host


def device_bdf(device_index: int) -> str:
    """PCI address (``dddd:bb:dd.f``) of HIP device ``device_index``.  HIP numbers GPUs in KFD
    order, which is not PCI order on MI355X nodes, so rails are matched by address."""
    import torch

    p = torch.cuda.get_device_properties(device_index)
    return f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"


def read_env_file(path: str) -> Dict[str, str]:
    """``KEY=VALUE`` lines of an env file such as the agent's ``rccl.env`` (comments skipped)."""
    from .fabric_artifacts import parse_env_text

    with open(path) as f:
        return parse_env_text(f.read())


def rail_env(gpu_bdf: Optional[str] = None, gpu_index: Optional[int] = None,
             artifact_dir: str = ARTIFACT_DIR, sysfs_root: str = "/sys/") -> Dict[str, str]:
    """RCCL settings that pin this rank's cross-node traffic to its own rail: the node-wide
    ``rccl.env`` with ``NCCL_IB_HCA`` narrowed to the RDMA device of the NIC the agent paired
    with this GPU -- the ``rccl-net.json`` entry with the same ``GPU_BDF``, else ``GPU_INDEX`` (the
    agent's PCI-order index), else (no ``rccl-net.json``: L2 mode writes none) the node topology
    discovered from sysfs (``models.topology.NodeTopology``, the agent's own pairing).  Apply
    before the rail group's communicator is created, e.g.
    ``os.environ.update(rail_env(device_bdf(local_rank)))`` ahead of ``init_process_group``.
    The setting is per process, so the job-wide communicator also sends this GPU's traffic
    through its own NIC -- what RCCL's topology search picks for GPU-affine NICs anyway.
    Raises ``LookupError`` when no RDMA NIC belongs to this GPU."""
    env_path = os.path.join(artifact_dir, "rccl.env")
    env = read_env_file(env_path) if os.path.exists(env_path) else {}
    entries = []
    net_path = os.path.join(artifact_dir, "rccl-net.json")
    if os.path.exists(net_path):
        with open(net_path) as f:
            entries = json.load(f).get("NIC_NET_CONFIG", [])
    want = gpu_bdf.lower() if gpu_bdf else None
    mine = next((e for e in entries if want and e.get("GPU_BDF", "").lower() == want), None)
    if mine is None and gpu_index is not None:
        mine = next((e for e in entries if e.get("GPU_INDEX") == gpu_index), None)
    if mine is None and want:
        from ..models.topology import NodeTopology

        hit = NodeTopology.discover(sysfs_root, with_xgmi=False).rdma_for_gpu(want)
        if hit:
            mine = {"RDMA_DEV": hit[0], "RDMA_PORT": hit[1]}
    if mine is None or not mine.get("RDMA_DEV"):
        raise LookupError(f"no configured RDMA NIC for GPU {gpu_bdf or gpu_index} in {net_path} or {sysfs_root}")
    env["NCCL_IB_HCA"] = f"={mine['RDMA_DEV']}:{mine.get('RDMA_PORT', 1)}"  # '=': exact name match
    if "GID_INDEX" in mine:
        env["NCCL_IB_GID_INDEX"] = str(mine["GID_INDEX"])
    # NCCL_SOCKET_IFNAME stays as the agent wrote it: every node lists its rails in GPU order, so
    # bootstrap meets on rail 0, a network every node shares (different rails need not route to
    # each other).
    return env


def node_and_rail_groups(local_size: Optional[int] = None) -> Tuple[object, object]:
    """(this rank's node group, this rank's rail group) for a job laid out node-major
    (global rank = node * local_size + local_rank, as torchrun assigns).  Collective: every rank
    creates every group, in the same order."""
    import torch.distributed as dist

    world, rank = dist.get_world_size(), dist.get_rank()
    local_size = local_size or int(os.environ.get("LOCAL_WORLD_SIZE", world))
    if world % local_size:
        raise ValueError(f"world size {world} is not a multiple of the node size {local_size}")
    nodes = world // local_size
    node_group = rail_group = None
    for node in range(nodes):
        g = dist.new_group(list(range(node * local_size, (node + 1) * local_size)))
        if rank // local_size == node:
            node_group = g
    for lr in range(local_size):
        g = dist.new_group([node * local_size + lr for node in range(nodes)])
        if rank % local_size == lr:
            rail_group = g
    return node_group, rail_group


class RailAllReduce:
    """bf16 sum over every rank of a multi-node job: xGMI inside a node, one rail per chunk
    across nodes."""

    def __init__(self, capacity_bytes: int, node_group, rail_group, device=None, timeout_s: float = 60.0,
                 segments: int = 4, min_segment_bytes: int = 4 << 20):
        import torch.distributed as dist

        self.segments, self.min_segment_bytes = segments, min_segment_bytes
        self.intra = XgmiAllReduce(capacity_bytes, group=node_group, device=device, timeout_s=timeout_s)
        self.rail = rail_group
        # the same surface as XgmiAllReduce, so the DDP hooks (ddp_hooks.py) take either
        self.device = self.intra.device
        self.world = self.intra.world * dist.get_world_size(rail_group)

    def input(self, numel: int):
        return self.intra.input(numel)

    def segments_for(self, numel: int) -> int:
        """How many pipeline segments ``numel`` is cut into: up to ``self.segments``, each at
        least ``self.min_segment_bytes`` and splitting into whole 8-element vectors per local rank."""
        align = 8 * self.intra.world
        for k in range(max(self.segments, 1), 1, -1):
            if numel % (k * align) == 0 and numel * 2 // k >= self.min_segment_bytes:
                return k
        return 1

    def all_reduce(self, numel: int, algo: str = "two_shot"):
        """Sum over every rank of ``input(numel)``; ``numel`` must split into whole 8-element
        vectors per local rank.  ``algo`` is accepted for the hooks' sake; the split is always
        two-shot (the cross-node step needs the scattered chunks).

        Pipelined over :meth:`segments_for` segments: segment k's cross-node all-reduce is
        issued asynchronously (RCCL's own stream, the rail NIC) while the xGMI reduce-scatter of
        segment k+1 runs, and segment k's xGMI all-gather overlaps the later segments' rail
        traffic — the two fabrics work at the same time instead of taking turns."""
        import torch.distributed as dist

        k = self.segments_for(numel)
        seg = numel // k
        works = []
        for s in range(k):
            mine = self.intra.reduce_scatter(seg, offset=s * seg)  # chunk `local rank` of this node's sum
            works.append(dist.all_reduce(mine, group=self.rail, async_op=True))  # that chunk, this GPU's rail
        for s, w in enumerate(works):
            w.wait()  # the current stream orders after the rail step; the gather synchronises it
            self.intra.all_gather_inplace(seg, offset=s * seg)
        return self.intra.output(numel)

    def close(self) -> None:
        self.intra.close()

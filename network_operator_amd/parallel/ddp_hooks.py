"""DistributedDataParallel communication hook over the direct xGMI all-reduce.

On a node the operator labelled scale-out ready, a data-parallel job can reduce its gradient
buckets with :class:`~network_operator_amd.parallel.xgmi_comm.XgmiAllReduce` instead of RCCL:
each bucket is cast to bf16 into the rank's symmetric input buffer (the same compression as
PyTorch's ``bf16_compress_hook``), summed over the xGMI mesh, and written back averaged.

    comm = XgmiAllReduce(capacity_bytes=256 << 20)          # >= 2 bytes x largest bucket
    model = DistributedDataParallel(model, device_ids=[dev])
    model.register_comm_hook(comm, xgmi_bf16_allreduce_hook)

The hook completes before it returns (the all-reduce orders its phases on the host), so it
trades DDP's backward/communication overlap for the direct mesh path; it is meant for
intra-node data parallelism with large buckets.
"""

from __future__ import annotations

from .xgmi_comm import XgmiAllReduce


def xgmi_bf16_allreduce_hook(comm: XgmiAllReduce, bucket):
    import torch

    buf = bucket.buffer()
    n = buf.numel()
    align = 8 * comm.world
    padded = (n + align - 1) // align * align
    x = comm.input(padded)
    x[:n].copy_(buf)  # cast to bf16 (no-op for bf16 gradients)
    if padded > n:
        x[n:].zero_()
    y = comm.all_reduce(padded, "auto")
    buf.copy_(y[:n])
    buf.div_(comm.world)
    fut: torch.futures.Future = torch.futures.Future()
    fut.set_result(buf)
    return fut

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
intra-node data parallelism with large buckets.  Across nodes, pass a
:class:`~network_operator_amd.parallel.rail.RailAllReduce` instead (xGMI inside the node, one
RoCE rail per chunk between nodes); the hooks only use ``input`` / ``all_reduce`` / ``world`` /
``device``.
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


class XgmiOverlapState:
    """State for :func:`xgmi_bf16_allreduce_hook_overlapped`: one communication stream and one
    worker thread, so buckets are reduced in DDP's launch order (the same on every rank) while
    the autograd thread keeps computing the next gradients."""

    def __init__(self, comm: XgmiAllReduce):
        import concurrent.futures

        import torch

        self.comm = comm
        self.stream = torch.cuda.Stream(device=comm.device)
        self.pool = concurrent.futures.ThreadPoolExecutor(max_workers=1, thread_name_prefix="xgmi-ddp")

    def close(self) -> None:
        self.pool.shutdown(wait=True)


def xgmi_bf16_allreduce_hook_overlapped(state: XgmiOverlapState, bucket):
    """Like :func:`xgmi_bf16_allreduce_hook`, but the bucket's all-reduce runs on the state's
    stream from its worker thread and the hook returns at once: communication overlaps the rest
    of the backward pass, and DDP waits on the returned future only when it needs the result."""
    import torch

    buf = bucket.buffer()
    ready = torch.cuda.Event()
    ready.record(torch.cuda.current_stream(state.comm.device))  # the bucket's gradients are complete
    fut: torch.futures.Future = torch.futures.Future()

    def work() -> None:
        try:
            with torch.cuda.stream(state.stream):
                state.stream.wait_event(ready)
                xgmi_bf16_allreduce_hook(state.comm, bucket).wait()
                state.stream.synchronize()
            fut.set_result(buf)
        except BaseException as e:  # surfaces in DDP's wait, on the training thread
            fut.set_exception(e)

    state.pool.submit(work)
    return fut

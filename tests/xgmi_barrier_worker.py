"""Rank process for tests/test_xgmi_comm.py: exercises the shared-memory phase barrier.

    RANK=r WORLD_SIZE=n MASTER_ADDR=... MASTER_PORT=... python xgmi_barrier_worker.py order DIR
    ... python xgmi_barrier_worker.py timeout
"""

import os
import random
import sys
import time

import torch.distributed as dist

from network_operator_amd.parallel.xgmi_comm import ShmBarrier


def main() -> None:
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
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


def nested() -> None:
    """Inside a torchrun-launched rank (as bench.py rank 0 does): spawn a 2-rank virtual
    all-reduce on GPU 0 with its own rendezvous, untouched by this job's launcher variables."""
    import json

    from network_operator_amd.parallel import xgmi_comm

    r = xgmi_comm.run(2, nbytes=4 << 20, min_bytes=4 << 20, iters=2, warmup=1, devices="0,0", timeout=100)
    print("RESULT " + json.dumps({"launcher_rank": os.environ.get("RANK"), "wrong": r["wrong"], "ranks": r["ranks"]}),
          flush=True)


if __name__ == "__main__":
    nested() if sys.argv[1:] == ["nested"] else main()

import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run on the GPU box with -m gpu)")
    config.addinivalue_line("markers", "netns: needs root / user namespaces + AF_PACKET (veth harness)")
    config.addinivalue_line("markers", "slow: long-running")


def _netns_ok():
    try:
        from network_operator_amd.testing import netns

        return netns.available()
    except Exception as e:  # pragma: no cover
        return False, str(e)


def pytest_collection_modifyitems(config, items):
    ok, why = None, None
    for item in items:
        if "netns" in item.keywords:
            if ok is None:
                ok, why = _netns_ok()
            if not ok:
                item.add_marker(pytest.mark.skip(reason=f"netns harness unavailable: {why}"))


@pytest.fixture(scope="session")
def native():
    from network_operator_amd.agent import native as _n

    return _n()


@pytest.fixture(scope="session")
def cuda_device():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no GPU is visible")
    return torch.device("cuda", 0)


@pytest.fixture(scope="session")
def single_rank_pg(cuda_device):
    """A 1-rank RCCL process group for the whole GPU session (one init per process)."""
    import torch.distributed as dist

    import tempfile

    store = os.path.join(tempfile.mkdtemp(prefix="netop-pg-"), "store")  # a FileStore: no TCP port to collide on
    if not dist.is_initialized():
        dist.init_process_group("nccl", init_method=f"file://{store}", rank=0, world_size=1, device_id=cuda_device)
    yield
    if dist.is_initialized():
        dist.destroy_process_group()

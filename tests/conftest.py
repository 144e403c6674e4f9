import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    if os.environ.get("PYTEST_XDIST_WORKER"):
        # several test processes share the CPUs: one intra-op thread each (OpenMP
        # workers spin-waiting on oversubscribed cores made the small-op CPU tests
        # run ~20x slower)
        import torch

        torch.set_num_threads(1)
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) to run")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def _has_gpu():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _has_gpu():
        return
    skip = pytest.mark.skip(reason="no HIP device")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture
def rccl_loopback():
    """A one-rank RCCL process group on cuda:0: the collectives and point-to-point
    calls of ``parallel.comm.Comm`` then run through RCCL kernels on a one-GPU box
    (``Comm.loopback`` for the all-to-alls; p2p to the own rank)."""
    import torch
    import torch.distributed as dist
    from dist_utils import free_port

    if dist.is_initialized():
        pytest.skip("a process group is already initialised")
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{free_port()}", rank=0, world_size=1,
                            device_id=dev)
    try:
        yield
    finally:
        import gc

        gc.collect()  # captured graphs that reference the communicator go first
        torch.cuda.synchronize()
        dist.destroy_process_group()

"""``Comm.shutdown``: every rank leaves the process group together (the benches end with it;
a rank leaving while a peer still held the gloo group aborted with ``terminate called
without an active exception``)."""
from tests.dist_utils import run_ranks


def _job(rank, world):
    import torch
    import torch.distributed as dist

    from flink_parameter_server_1_amd.parallel.comm import Comm

    comm = Comm(device=torch.device("cpu"))
    total = comm.sum_over_ranks(float(rank + 1))
    comm.shutdown()
    after = dist.is_initialized()
    comm.shutdown()  # a second call (no group any more) is a no-op
    return total, after


def test_shutdown_leaves_the_group_on_every_rank():
    res = run_ranks(_job, 2)
    assert res == [(3.0, False), (3.0, False)]


def test_shutdown_single_process_is_a_no_op():
    import torch

    from flink_parameter_server_1_amd.parallel.comm import Comm

    Comm(device=torch.device("cpu"), local=True).shutdown()

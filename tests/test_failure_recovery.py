"""Failure recovery: a job killed after its last snapshot resumes from it
and ends bit-identical to an uninterrupted run (deterministic CPU path, gloo ranks)."""
import os

import pytest
import torch

from dist_utils import run_ranks


def _job(rank, world, ckpt_dir, start_from_ckpt, stop_at, exchange, neg=0):
    from flink_parameter_server_1_amd.models.mf.fast import DistributedMF, MFConfig, SyntheticRatings
    from flink_parameter_server_1_amd.parallel.comm import Comm
    from flink_parameter_server_1_amd.utils.io import Checkpointer

    comm = Comm()
    cfg = MFConfig(num_users=500, num_items=300, dim=16, learning_rate=0.1, range_min=0.0, range_max=0.3,
                   exchange=exchange, negative_sample_rate=neg, user_memory=8)
    m = DistributedMF(cfg, comm)
    data = SyntheticRatings(500, 300, 400 * 12, rank, world, seed=21, truth_dim=4)
    ck = Checkpointer(ckpt_dir, {"users": m.users, "items": m.items}, comm, every_steps=5,
                      before_save=m.flush, aux=m) if ckpt_dir else None
    start = 0
    if start_from_ckpt:
        start = ck.restore_latest()["step"]
    for s in range(start, stop_at):
        m.step(*data.batch(s, 400))
        if ck:
            ck.maybe_save(s + 1)
    m.flush()
    return m.users.weight.clone(), m.items.weight.clone(), start


@pytest.mark.parametrize("exchange,neg", [("rotate", 0), ("ps", 0), ("rotate", 2), ("ps", 2)])
def test_resume_after_kill_matches_uninterrupted(tmp_path, exchange, neg):
    """``neg > 0``: the negative-sampling rings and RNG counter are aux state; a
    resume that restarted them empty would diverge."""
    # the uninterrupted run snapshots too: a snapshot flushes the in-flight micro-batch
    # (bounded-staleness pipeline), which is part of the schedule being reproduced
    full = run_ranks(_job, 2, str(tmp_path / "ck_full"), False, 10, exchange, neg)
    d = str(tmp_path / "ck")
    run_ranks(_job, 2, d, False, 7, exchange, neg)          # "killed" after step 7 (snapshot at 5)
    assert sorted(os.listdir(d)) == ["step_000000005"]
    resumed = run_ranks(_job, 2, d, True, 10, exchange, neg)  # restart: restore step 5, replay 6..10
    for a, b in zip(full, resumed):
        assert b[2] == 5
        assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])

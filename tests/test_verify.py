"""``parallel/verify.py`` (``bench.py --verify``) on CPU gloo process groups: the rotation
of a real multi-process world equals the sequential replay, and broken exchanges
(a wrong buffer on the wire, blocks never sent home) are reported on EVERY rank."""
import pytest
import torch

from dist_utils import run_ranks


def _check(rank, world, schedule, mutant, exchange="rotate", pipeline=True):
    from flink_parameter_server_1_amd.parallel.comm import Comm
    from flink_parameter_server_1_amd.parallel import verify
    from flink_parameter_server_1_amd.parallel.verify import rotation_check

    cls = None if mutant is None else verify.mutant_rotation(mutant)
    return rotation_check(Comm(device=torch.device("cpu")), schedule=schedule, rotation_cls=cls, exchange=exchange,
                          pipeline=pipeline)


@pytest.mark.parametrize("world,schedule", [(2, "bidir"), (3, "ring"), (3, "bidir")])
def test_rotation_check_passes_on_a_correct_world(world, schedule):
    res = run_ranks(_check, world, schedule, None)
    assert all(r["verify_ok"] for r in res)
    assert res[0]["verify_max_abs_err_items"] < 1e-5 and res[0]["verify_ref_moved"] > 1e-3
    assert all(r["verify_world"] == world for r in res)


@pytest.mark.parametrize("world,pipeline", [(2, True), (2, False), (3, True)])
def test_ps_check_matches_the_staleness_replay(world, pipeline):
    res = run_ranks(_check, world, "bidir", None, "ps", pipeline)
    assert all(r["verify_ok"] for r in res), res[0]
    assert res[0]["verify_exchange"] == "ps" and res[0]["verify_max_abs_err_items"] < 1e-5


@pytest.mark.parametrize("mutant", ["wrong_buffer", "no_home"])
def test_rotation_check_fails_on_every_rank_when_the_exchange_is_broken(mutant):
    res = run_ranks(_check, 2, "bidir", mutant)
    assert not any(r["verify_ok"] for r in res)


def test_replay_schedule_covers_every_block_once_per_step():
    from flink_parameter_server_1_amd.parallel.verify import active_blocks

    for world in (1, 2, 3, 8):
        for schedule, nblk in (("bidir", 4 * world), ("ring", 2 * world)):
            K = 2 * world
            for r in range(world):  # every rank's users meet every block exactly once per micro-batch
                seen = [b for t in range(K) for b in active_blocks(r, t, world, schedule)]
                assert sorted(seen) == list(range(nblk))
            for t in range(K):  # no block is held by two ranks in one sub-step
                held = [b for r in range(world) for b in active_blocks(r, t, world, schedule)]
                assert len(held) == len(set(held))


def _collision(rank, world, user_update):
    from flink_parameter_server_1_amd.parallel.comm import Comm
    from flink_parameter_server_1_amd.parallel.verify import rotation_check

    return rotation_check(Comm(device=torch.device("cpu")), schedule="bidir", user_update=user_update,
                          repeated_users=True)


@pytest.mark.parametrize("world", [2, 4])
def test_collision_check_passes_exact_user_rows_and_fails_hogwild(world):
    """The collision regime (every user rated 8 times per step): the exact user-row mode
    sums every delta and passes at the measured second-order tolerance; the Hogwild
    ``store`` mode (last writer wins on the CPU twin) loses 7 of 8 deltas and fails on every rank."""
    ok = run_ranks(_collision, world, "atomic")
    assert all(r["verify_ok"] for r in ok), ok[0]
    assert ok[0]["verify_repeated_users"] and ok[0]["verify_user_update"] == "atomic"
    assert ok[0]["verify_lost_update_err"] > 2 * ok[0]["verify_tol_users"]
    bad = run_ranks(_collision, world, "store")
    assert not any(r["verify_ok"] for r in bad)
    assert bad[0]["verify_max_abs_err_users"] > bad[0]["verify_tol_users"]


def test_occurrence_rounds_are_a_sequential_schedule():
    from flink_parameter_server_1_amd.parallel.verify import _occurrence_rounds

    u = torch.tensor([5, 3, 5, 5, 7, 3, 9])
    assert _occurrence_rounds(u).tolist() == [0, 0, 1, 2, 0, 1, 0]

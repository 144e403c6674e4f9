"""Model formats, checkpoint/resume with re-sharding, data readers, evaluators, host-native store."""
import os

import numpy as np
import pytest
import torch

from dist_utils import run_ranks
from flink_parameter_server_1_amd.utils import io, metrics, native_host


def test_host_library_built():
    assert native_host.available()


def test_id_value_text_roundtrip(tmp_path):
    p = str(tmp_path / "items.map")
    ids = np.array([3, 1, 7])
    vals = np.random.default_rng(0).normal(size=(3, 5)).astype(np.float32)
    io.write_factors_text(p, ids, vals)
    lines = open(p).read().splitlines()
    assert len(lines) == 15 and lines[0].startswith("3;")
    back = io.read_factors_text(p)
    assert sorted(back) == [1, 3, 7]
    np.testing.assert_allclose(back[7], vals[2], rtol=1e-6)
    # model stream feeds transform_with_model_load
    assert dict(io.model_stream_from_text(p)).keys() == back.keys()


def test_read_ratings(tmp_path):
    p = str(tmp_path / "log")
    with open(p, "w") as f:
        f.write("100 5 7\n101,6,8,0.5\n102\t7\t9\t2\n")
    ts, u, i, r = io.read_ratings(p)
    assert ts.tolist() == [100, 101, 102] and u.tolist() == [5, 6, 7] and i.tolist() == [7, 8, 9]
    np.testing.assert_allclose(r, [1.0, 0.5, 2.0])


def test_synthetic_host_generator_deterministic():
    a = io.synthetic_ratings_host(10000, 100, 50, seed=3)
    b = io.synthetic_ratings_host(10000, 100, 50, seed=3)
    assert all(np.array_equal(x, y) for x, y in zip(a, b))
    assert a[0].max() < 100 and a[1].max() < 50 and 0 <= a[2].min() and a[2].max() < 1


def test_snapshot_roundtrip_and_reshard(tmp_path):
    from flink_parameter_server_1_amd.parallel.table import ShardedTable

    N, D = 1000, 6
    full = ShardedTable(N, D, 0, 1, "hash", ("uniform", -1, 1), seed=4)
    full.weight += torch.arange(N, dtype=torch.float32)[:, None]
    # write as 3 shards
    for r in range(3):
        t = ShardedTable(N, D, r, 3, "hash", ("zeros",))
        t.load(torch.arange(N), full.weight)
        io.save_table(t, str(tmp_path / f"t.shard{r}-of-3.bin"))
    # restore at 2 shards (re-shard)
    for r in range(2):
        t = ShardedTable(N, D, r, 2, "range", ("zeros",))
        n = io.restore_table(t, str(tmp_path / "t.shard*-of-3.bin"))
        assert n == t.n_local
        ids, vals = t.dump(only_touched=False)
        torch.testing.assert_close(vals, full.weight[ids])


def _ckpt(rank, world, d):
    from flink_parameter_server_1_amd.models.mf.fast import DistributedMF, MFConfig, SyntheticRatings
    from flink_parameter_server_1_amd.parallel.comm import Comm

    comm = Comm()
    m = DistributedMF(MFConfig(num_users=200, num_items=100, dim=4), comm)
    data = SyntheticRatings(200, 100, 4000, rank, world)
    ck = io.Checkpointer(d, {"users": m.users, "items": m.items}, comm, every_steps=5, before_save=m.flush)
    for s in range(1, 11):
        m.step(*data.batch(s, 200))
        ck.maybe_save(s)
    ids, w = m.item_vectors(False)  # flushes (rotating blocks home)
    # fresh model, restore
    m2 = DistributedMF(MFConfig(num_users=200, num_items=100, dim=4, seed=9), comm)
    man = io.Checkpointer(d, {"users": m2.users, "items": m2.items}, comm).restore_latest()
    ids2, w2 = m2.items.dump(False)
    return man["step"], torch.equal(ids, ids2) and torch.allclose(w, w2)


def test_checkpoint_resume_distributed(tmp_path):
    res = run_ranks(_ckpt, 2, str(tmp_path / "ck"))
    assert all(step == 10 and ok for step, ok in res)
    assert len([p for p in os.listdir(tmp_path / "ck") if p.startswith("step_")]) == 2  # keep=2


def test_hash_store_semantics():
    hs = native_host.HashStore(3, -1.0, 1.0, seed=5)
    v = hs.pull([10, 11, 10])
    assert np.array_equal(v[0], v[2]) and len(hs) == 2
    from flink_parameter_server_1_amd.ops import reference as R

    np.testing.assert_allclose(v[0], R.init_values(torch.tensor([10]), 3, -1.0, 1.0, 5)[0].numpy(), rtol=1e-6)
    hs.push([10], [[1, 1, 1]])
    np.testing.assert_allclose(hs.pull([10])[0], v[0] + 1, rtol=1e-6)
    hs.push([99], [[2, 2, 2]])  # unseen key takes the delta (SimplePSLogic)
    np.testing.assert_allclose(hs.pull([99])[0], [2, 2, 2])
    k, vals = hs.dump()
    assert sorted(k.tolist()) == [10, 11, 99]


def test_ndcg_and_recall():
    assert metrics.ndcg_at_k([5, 6, 7], 5) == pytest.approx(1.0)
    assert metrics.ndcg_at_k([5, 6, 7], 7) == pytest.approx(np.log(2) / np.log(4))
    assert metrics.ndcg_at_k([5, 6], 9) == 0.0
    agg = metrics.NDCGAggregator(period_length=10)
    agg.add_stream([(1, 5, 3, [(0.9, 5), (0.1, 2)]), (1, 2, 4, [(0.9, 5), (0.1, 2)]), (1, 8, 15, [(0.9, 1)])])
    per = agg.periods()
    assert per[0][0] == 0 and per[0][3] == 2 and per[1][1] == 0.0
    rec, prec = metrics.recall_precision_at_k({1: [1, 2, 3, 4, 5]}, {1: {2, 9}}, 5)
    assert rec == 0.5 and prec == pytest.approx(0.2)


def test_prediction_log_format():
    lines = io.write_prediction_log([({3: 0.5, 1: 2.0}, 1)])
    assert lines == ["###PS###t;1;[1 -> 2.0,3 -> 0.5]"]

"""The ``transform`` contract on the MI355X: user PS rules, custom partitioners
and sparse int32 ids through the HIP dedup / hash-table / gather kernels
(fp64 rows: exact parity with the per-record engine)."""
import numpy as np
import pytest
import torch

import test_tensor_contract as T
from flink_parameter_server_1_amd import ops
from flink_parameter_server_1_amd.parallel.hash_table import HashShardTable

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


@pytest.mark.parametrize("rule", [T.clip_add, T.vmax])
def test_user_rule_custom_partitioner_gpu(rule):
    recs = T._records(1, 150, seed=21)
    ref = T._per_record(recs, 1, rule, T.custom_part, coef=0.1)
    got = T._tensor(recs, 1, rule, num_ids=40, partitioner=T.custom_part, device=DEV, coef=0.1)
    assert set(got) == set(ref)
    for k in ref:
        assert got[k] == pytest.approx(ref[k], abs=1e-12), k


@pytest.mark.parametrize("combine,mb", [("sum", 1), ("sequential", 16)])
def test_sparse_ids_gpu(combine, mb):
    recs = T._records(1, 300, seed=22, sparse=True)
    coef = 0.1 if mb == 1 else 0.0
    ref = T._per_record(recs, 1, T.clip_add, coef=coef)
    got = T._tensor(recs, 1, T.clip_add, combine=combine, mb=mb, device=DEV, coef=coef)
    assert set(got) == set(ref)
    for k in ref:
        assert got[k] == pytest.approx(ref[k], abs=1e-12), k


def test_hash_table_kernel_matches_cpu_semantics():
    """ht_lookup on the GPU vs the CPU twin: same key -> row bijection (rows in
    insert order may differ), one fresh request per new key, hash-uniform init of
    the fresh rows keyed by the id, lookups of absent keys give -1, growth keeps
    every row."""
    g = torch.Generator().manual_seed(1)
    keys = torch.randint(-2 ** 31, 2 ** 31 - 1, (20000,), generator=g, dtype=torch.int64)
    keys = torch.cat([keys, keys[:5000], torch.tensor([-2 ** 31, 2 ** 31 - 1, 0, -1])])
    tabs = {d: HashShardTable(8, init=("uniform", -1.0, 1.0), seed=5, device=d, capacity=64) for d in ("cpu", DEV)}
    out = {}
    for d, t in tabs.items():
        rows = []
        for s in range(0, keys.numel(), 4096):
            r, fresh = t.rows_for(keys[s:s + 4096].to(d))
            rows.append((r.cpu(), fresh.cpu()))
        out[d] = rows
    for d, t in tabs.items():
        r = torch.cat([x for x, _ in out[d]]).long()
        f = torch.cat([y for _, y in out[d]])
        assert bool((r >= 0).all())
        assert torch.equal(t.rowkey.cpu()[r].long(), keys)  # every request maps to its own key's row
        assert int(f.sum()) == torch.unique(keys).numel()   # exactly one inserter per key
        assert int(t.count) == torch.unique(keys).numel()   # rows are compact: [0, count) all used
        assert torch.unique(r).numel() == int(t.count)
        assert t.stats()["overflow"] == 0 and t.stats()["load_factor"] <= 0.5
        assert t.grow_events > 0
    # the same id gets the same init values on both devices (hash RNG by id)
    ids_c, vals_c = tabs["cpu"].dump()
    ids_g, vals_g = tabs[DEV].dump()
    oc, og = torch.argsort(ids_c), torch.argsort(ids_g.cpu())
    assert torch.equal(ids_c[oc], ids_g.cpu()[og])
    torch.testing.assert_close(vals_c[oc], vals_g.cpu()[og], rtol=0, atol=0)
    miss = torch.tensor([12345, -777], dtype=torch.int32)
    present = set(keys.tolist())
    for d, t in tabs.items():
        r, _ = t.rows_for(miss.to(d), insert=False)
        exp = [(-1 if int(k) not in present else int(r[i])) for i, k in enumerate(miss.tolist())]
        assert r.cpu().tolist() == exp
    assert ops.native_available()

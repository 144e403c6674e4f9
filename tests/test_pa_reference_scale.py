"""PassiveAggressiveParameterServerTest at the reference's own scale (500k dims,
~10k nnz per vector, 80 training vectors, 3 workers / 3 PS, range partitioning,
accuracy >= 80 % on the first 20 training vectors: T/passive/aggressive/
PassiveAggressiveParameterServerTest.scala:16-19,52-60,90) on the per-record
engine and on the tensor engine, plus exact per-example parity of the batched
PA step with the per-record transform."""
import numpy as np
import pytest
import torch

from dist_utils import run_ranks
from flink_parameter_server_1_amd.core.messages import Left
from flink_parameter_server_1_amd.models.pa.algorithms import PassiveAggressiveBinaryAlgorithm
from flink_parameter_server_1_amd.models.pa.server import binary_accuracy, transform_binary
from test_pa import _model_from_stream, reference_data

F_REF, NNZ_REF = 500_000, 10_000


@pytest.fixture(scope="module")
def ref_train():
    return reference_data(F_REF, nnz=NNZ_REF)


def test_per_record_pa_at_reference_scale(ref_train):
    out = transform_binary(None, input_source=[Left(x) for x in ref_train], worker_parallelism=3, ps_parallelism=3,
                           passive_aggressive_method=PassiveAggressiveBinaryAlgorithm.build_pa(), pull_limit=10000,
                           feature_count=F_REF, range_partitioning=True)
    w = _model_from_stream(out, F_REF)
    assert binary_accuracy(w, ref_train[:20], PassiveAggressiveBinaryAlgorithm.build_pa()) >= 80


def _csr(examples, labels=True):
    indptr = [0]
    idx, val, lab = [], [], []
    for v, y in examples:
        idx += v.indices.tolist()
        val += v.values.tolist()
        indptr.append(len(idx))
        lab.append((1 if y else -1) if labels else 0)
    return (torch.tensor(indptr, dtype=torch.int64), torch.tensor(idx, dtype=torch.int32),
            torch.tensor(val, dtype=torch.float32), torch.tensor(lab, dtype=torch.int8))


def _tensor_pa(rank, world, train, mb):
    from flink_parameter_server_1_amd.core.tensor_engine import fold_outputs
    from flink_parameter_server_1_amd.models.pa.batched import transform_pa_tensor
    from flink_parameter_server_1_amd.parallel.comm import Comm

    mine = train[rank::world]  # rebalance: round-robin over the workers
    batches = [_csr(mine[s:s + mb]) for s in range(0, len(mine), mb)]
    out = transform_pa_tensor(batches, F_REF, "binary", variant="PA", range_partitioning=True, comm=Comm())
    return fold_outputs(out)[1]


@pytest.mark.parametrize("world", [1, 3])
def test_tensor_pa_at_reference_scale(ref_train, world):
    res = run_ranks(_tensor_pa, world, ref_train, 4) if world > 1 else [_tensor_pa(0, 1, ref_train, 4)]
    w = np.zeros(F_REF)
    for dump in res:
        for k, v in dump.items():
            w[k] = v[0]
    acc = binary_accuracy(w, ref_train[:20], PassiveAggressiveBinaryAlgorithm.build_pa())
    assert acc >= 80, acc


@pytest.mark.parametrize("variant,build", [("PA", PassiveAggressiveBinaryAlgorithm.build_pa),
                                           ("PA-I", lambda: PassiveAggressiveBinaryAlgorithm.build_pai(0.3)),
                                           ("PA-II", lambda: PassiveAggressiveBinaryAlgorithm.build_paii(0.3))])
def test_distributed_pa_equals_per_record_transform(variant, build):
    """One example per micro-batch (``DistributedPA``, fp32) == per-record
    ``transform_binary`` with pullLimit 1 (fp64, sequential): same final model."""
    from flink_parameter_server_1_amd.models.pa.fast import DistributedPA, PAConfig

    train = reference_data(2000, nnz=12, n_train=60, seed=7)
    out = transform_binary(None, input_source=[Left(x) for x in train], worker_parallelism=1, ps_parallelism=1,
                           passive_aggressive_method=build(), pull_limit=1, feature_count=2000,
                           range_partitioning=True)
    w_ref = _model_from_stream(out, 2000)
    m = DistributedPA(PAConfig(feature_count=2000, kind="binary", variant=variant, aggressiveness=0.3,
                               local_direct=False))
    for x in train:
        m.train_step(*_csr([x]))
    ids, vals = m.dump(only_touched=False)
    w = np.zeros(2000)
    w[ids.numpy()] = vals.reshape(-1).numpy()
    np.testing.assert_allclose(w, w_ref, rtol=1e-4, atol=1e-6)
    assert int((w != 0).sum()) == int((w_ref != 0).sum())

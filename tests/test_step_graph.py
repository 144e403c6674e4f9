"""CPU side of the hipGraph step replay: eligibility is checked when the runtime starts."""
import pytest
import torch

from flink_parameter_server_1_amd.api.batched import FunctionBatchedWorkerLogic
from flink_parameter_server_1_amd.core.step_graph import _flatten, _rebuild
from flink_parameter_server_1_amd.core.tensor_engine import TensorRuntime
from flink_parameter_server_1_amd.parallel.comm import Comm
from flink_parameter_server_1_amd.ps.device_logics import DeviceSimplePSLogic


def test_graph_mode_refused_off_gpu():
    w = FunctionBatchedWorkerLogic(lambda b, ps: ps.pull(b), lambda p, ps: None, graph_safe=True)
    with pytest.raises(ValueError, match="not on a GPU"):
        TensorRuntime(Comm(device=torch.device("cpu")), graph=True).start(w, DeviceSimplePSLogic(100, 4))


def test_batch_signature_roundtrip():
    b = {"k": torch.zeros(3, dtype=torch.int64), "x": (torch.ones(2, 2), 5, [torch.zeros(1)])}
    leaves = []
    sig = _flatten(b, leaves)
    assert len(leaves) == 3
    r = _rebuild(sig, iter(leaves))
    assert r["x"][1] == 5 and r["k"] is b["k"] and r["x"][2][0] is b["x"][2][0]
    other = []
    assert _flatten({"k": torch.zeros(4, dtype=torch.int64), "x": (torch.ones(2, 2), 5, [torch.zeros(1)])},
                    other) != sig  # a shape change is a new signature
    assert _flatten(object(), []) is None

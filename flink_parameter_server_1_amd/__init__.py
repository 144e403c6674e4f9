"""flink_parameter_server_1_amd — an MI355X-native parameter server.

Same capabilities and API surface as the Flink parameter server
(``lucaRadicalbit/flink-parameter-server-1``): ``WorkerLogic`` /
``ParameterServerLogic`` callbacks, ``transform`` and model-load entry
points, hash/range/custom partitioning, pull limiting, message combining,
and the MF / LEMP top-K / Passive-Aggressive model library (+ word2vec).

Two execution paths share that API:

* the per-record *compat* engine (``core.engine``, ``core.dist_engine``) —
  exact reference semantics, CPU, gloo multi-process;
* the *tensor* engine (``parallel``) — HBM-resident PS shards on MI355X,
  RCCL all-to-all over xGMI for pull/push, hand-written gfx950 HIP kernels
  (``ops``) for gather / fused SGD / apply / top-K / SGNS / PA.
"""
from .api import *  # noqa: F401,F403
from .core import (Either, FlinkParameterServer, HashPartitioner, Left, LocalRuntime, LogicFactory,
                   PartitionedInput, Partitioner, RangePartitioner, Right, transform,
                   transform_with_double_model_load, transform_with_model_load)
from .ps import (LockPSLogicA, LockPSLogicB, RangePSLogicWithClose, SimplePSLogic, SimplePSLogicWithClose)

__version__ = "0.1.0"

"""Device PS logics: the built-in ``ParameterServerLogic``s as HBM shard tables.

The tensor engine (``core.tensor_engine``) never calls Python per key on the
PS side: a device logic describes the shard (size, row width, init, partition)
and its push rule, and the engine runs gather (K2) / apply (K3) kernels over
whole micro-batches.  Semantics of the reference logics:

* ``DeviceSimplePSLogic`` -- ``SimplePSLogic`` (``M/server/SimplePSLogic.scala:7-26``):
  init on first touch (here: deterministic per-id hash init of the dense
  shard, the same value whenever the row is first read), push =
  ``update(old, delta)``, ``(id, new value)`` emitted on every push.
* ``DeviceSimplePSLogicWithClose`` -- ``SimplePSLogicWithClose``
  (``M/server/SimplePSLogicWithClose.scala:7-32``): no per-push output, the
  touched rows of the shard are dumped at close.
* ``DeviceRangePSLogicWithClose`` -- ``RangePSLogicWithClose``
  (``M/server/RangePSLogicWithClose.scala:7-62``) with ``rangePartitionerPS``
  (``M/passive/aggressive/PassiveAggressiveParameterServer.scala:372-384``):
  contiguous ``ceil(F/P)`` id ranges per shard, dump at close.
* ``DeviceLockPSLogic`` -- ``LockPSLogicA``/``B`` (``M/server/LockPSLogicA.scala:13-46``):
  a pull locks the key until the puller pushes; contended keys are granted to
  one worker per round, the others are answered in later rounds with the
  updated value (``parallel.locked_ps``).

Update rules (``op``): ``add`` (vector sum, the MF / PA rule), ``set``
(overwrite, ``PSTopKGenerator``'s user store, ``M/matrix/factorization/PSTopKGenerator.scala:74-76``),
``sgd`` (``w -= lr * g``), ``adagrad`` and ``add_renorm`` (vector sum + length
recompute, ``psOnlineLearnerAndGenerator``'s ``LengthAndVector`` store,
``M/matrix/factorization/PSOnlineMatrixFactorizationAndTopKGenerator.scala:81-84``).
"""
from __future__ import annotations

from typing import Any, List, Optional, Tuple

import torch

from ..parallel.comm import Comm
from ..parallel.table import ShardedTable
from ..parallel.tensor_ps import TensorPS

#: wire dtypes of pull answers / pushed deltas ("fp64": CPU parity runs against
#: the per-record engine's double arithmetic)
_WIRE = {"fp32": torch.float32, "bf16": torch.bfloat16, "fp64": torch.float64}
OPS = ("add", "set", "sgd", "adagrad", "add_renorm")


class DevicePSLogic:
    """Base: one HBM shard per rank, hash (``|id| % P``) or range partitioned."""

    #: "push": ``(ids, rows)`` after every push; "close": shard dump at close; "none"
    emit = "none"
    locking = False

    def __init__(self, num_ids: int, dim: int = 1, *, op: str = "add", init: Tuple = ("zeros",), seed: int = 0,
                 partition: str = "hash", wire_dtype: str = "fp32", lr: float = 0.0, dtype=torch.float32,
                 track_touched: bool = True, table: Optional[ShardedTable] = None, ps: Optional[TensorPS] = None):
        """``table`` / ``ps``: serve an existing shard (and its PS front) instead of
        allocating one at ``open`` -- how the model classes (``DistributedMF``,
        ``DistributedPA``) run their PS path through this engine."""
        if op not in OPS:
            raise ValueError(f"op must be one of {OPS}, not {op!r}")
        self._given = (table, ps)
        self.num_ids, self.dim, self.op, self.init, self.seed = int(num_ids), int(dim), op, init, seed
        self.partition, self.wire_dtype, self.lr, self.dtype = partition, _WIRE[wire_dtype], lr, dtype
        self.track_touched = track_touched
        self.table: Optional[ShardedTable] = None
        self.ps: Optional[TensorPS] = None

    # ------------------------------------------------------------- lifecycle
    def open(self, comm: Comm) -> None:
        """Allocate this rank's shard (``ParameterServerLogic.open``)."""
        table, ps = self._given
        if table is not None:
            self.table = table
        else:
            self.table = ShardedTable(self.num_ids, self.dim, comm.rank, comm.world, self.partition, self.init,
                                      self.seed, comm.device, optimizer=self.op,
                                      track_touched=self.track_touched or self.emit == "close", dtype=self.dtype)
        self.ps = ps if ps is not None else TensorPS(self.table, comm, self.wire_dtype)
        # set-rules and per-push outputs must tell pushed keys from merely pulled ones
        self.ps.masked_push = self.op == "set" or self.emit == "push"

    @property
    def needs_mask(self) -> bool:
        return self.ps.masked_push

    def after_push(self, updated) -> List[Any]:
        """PS outputs of one applied push: ``(global ids, new rows)`` on this shard."""
        if self.emit == "push" and updated is not None and updated[0].numel():
            return [updated]
        return []

    def close(self) -> List[Any]:
        """Close-time outputs (``ParameterServerLogic.close``)."""
        if self.emit == "close":
            return [self.table.dump(only_touched=True)]
        return []

    def lengths(self, ids_local: torch.Tensor) -> torch.Tensor:
        return self.table.lengths(ids_local)


class DeviceSimplePSLogic(DevicePSLogic):
    emit = "push"


class DeviceSimplePSLogicWithClose(DevicePSLogic):
    emit = "close"


class DeviceRangePSLogicWithClose(DevicePSLogic):
    emit = "close"

    def __init__(self, feature_count: int, dim: int = 1, **kw):
        kw.setdefault("init", ("zeros",))
        super().__init__(feature_count, dim, partition="range", **kw)


class DeviceLockPSLogic(DevicePSLogic):
    """Per-key exclusive read-modify-write.  ``op`` is what the holder's push
    does: ``add`` (delta) or ``set`` (new value)."""

    emit = "push"
    locking = True

    def __init__(self, num_ids: int, dim: int = 1, **kw):
        kw.setdefault("op", "add")
        if kw["op"] not in ("add", "set"):
            raise ValueError("DeviceLockPSLogic supports op 'add' or 'set'")
        super().__init__(num_ids, dim, **kw)

    def open(self, comm: Comm) -> None:
        from ..parallel.locked_ps import LockedTensorPS

        super().open(comm)
        self.ps.masked_push = False  # a holder's release always carries its row
        self.locked = LockedTensorPS(self.table, comm, self.wire_dtype, ps=self.ps)

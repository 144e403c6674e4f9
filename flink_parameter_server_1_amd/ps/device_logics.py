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

* ``DeviceFunctionPSLogic`` -- ``SimplePSLogic`` with USER rules, the
  ``paramInit`` / ``paramUpdate`` closures of ``transform`` overload (a)
  (``M/FlinkParameterServer.scala:62-77``): ``init_fn(ids) -> rows`` and
  ``update_fn(old_rows, deltas[, ids]) -> new_rows``, vectorised torch callables
  run on the owner after the push all-to-all.  ``combine`` says how several
  pushes of one key inside one micro-batch meet: ``sum`` (pre-reduced on the
  worker, exact for additive rules), ``max`` / ``min`` / ``last``, or
  ``sequential`` (one push round per repeat, the reference's order).

Update rules (``op``): ``add`` (vector sum, the MF / PA rule), ``set``
(overwrite, ``PSTopKGenerator``'s user store, ``M/matrix/factorization/PSTopKGenerator.scala:74-76``),
``sgd`` (``w -= lr * g``), ``adagrad``, ``add_renorm`` (vector sum + length
recompute, ``psOnlineLearnerAndGenerator``'s ``LengthAndVector`` store,
``M/matrix/factorization/PSOnlineMatrixFactorizationAndTopKGenerator.scala:81-84``)
and ``fn`` (the user's ``update_fn``).

Shards: dense over ``[0, num_ids)`` (``ShardedTable``), partitioned by
``partition="hash"`` (``|id| % P``), ``"range"``, or a custom partitioner -- a
vectorised callable ``ids -> shard`` or an ``owner[num_ids]`` tensor (P2c,
the ``paramPartitioner`` of overload (c), ``M/FlinkParameterServer.scala:198-199``);
or ``sparse=True``: a device hash table over the whole int32 id space
(``parallel.hash_table.HashShardTable``; the reference's ``HashMap[Integer, P]``).
"""
from __future__ import annotations

from typing import Any, Callable, List, Optional, Tuple, Union

import torch

from ..parallel.comm import Comm
from ..parallel.hash_table import HashShardTable
from ..parallel.table import ShardedTable
from ..parallel.tensor_ps import TensorPS

#: wire dtypes of pull answers / pushed deltas ("fp64": CPU parity runs against
#: the per-record engine's double arithmetic)
_WIRE = {"fp32": torch.float32, "bf16": torch.bfloat16, "fp64": torch.float64}
OPS = ("add", "set", "sgd", "adagrad", "add_renorm", "fn")
COMBINE = ("sum", "last", "max", "min", "sequential")


def owner_table(partition: Union[Callable, torch.Tensor], num_ids: int, world: int) -> torch.Tensor:
    """``owner[num_ids]`` of a custom partitioner (callable over an id tensor, or
    the table itself); entries must lie in ``[0, world)``."""
    if callable(partition):
        owner = torch.as_tensor(partition(torch.arange(num_ids, dtype=torch.int64)))
    else:
        owner = torch.as_tensor(partition)
    owner = owner.to(torch.int64).reshape(-1).cpu()
    if owner.numel() != num_ids:
        raise ValueError(f"custom partitioner gave {owner.numel()} owners for {num_ids} ids")
    if num_ids and (int(owner.min()) < 0 or int(owner.max()) >= world):
        raise ValueError(f"custom partitioner returned shards outside [0, {world})")
    return owner


class DevicePSLogic:
    """Base: one HBM shard per rank, hash (``|id| % P``) or range partitioned."""

    #: "push": ``(ids, rows)`` after every push; "close": shard dump at close; "none"
    emit = "none"
    locking = False

    def __init__(self, num_ids: Optional[int], dim: int = 1, *, op: str = "add", init: Tuple = ("zeros",),
                 seed: int = 0, partition: Union[str, Callable, torch.Tensor] = "hash", wire_dtype: str = "fp32",
                 lr: float = 0.0, dtype=torch.float32, track_touched: bool = True,
                 table: Optional[ShardedTable] = None, ps: Optional[TensorPS] = None, sparse: bool = False,
                 capacity: int = 1 << 14, init_fn: Optional[Callable] = None, update_fn: Optional[Callable] = None,
                 combine: str = "sum", dedup: Optional[bool] = None, ps_parallelism: Optional[int] = None):
        """``table`` / ``ps``: serve an existing shard (and its PS front) instead of
        allocating one at ``open`` -- how the model classes (``DistributedMF``,
        ``DistributedPA``) run their PS path through this engine.  ``sparse``: a
        device hash-table shard (``num_ids`` may be None, ``capacity`` = initial
        rows per shard; it grows).  ``dedup``: de-duplicate each micro-batch's pulled
        keys (True), ship every request (False), or let the PS decide by batch size
        (None, ``TensorPS.dedups``); additive rules only ship requests.
        ``ps_parallelism``: shards P <= ranks (default: one per rank); shard s lives on
        rank s, the owner of an id is ``|id| % P`` (hash) or ``|id| // ceil(F/P)``
        (range), computed on the device -- no host owner table."""
        if op not in OPS:
            raise ValueError(f"op must be one of {OPS}, not {op!r}")
        if combine not in COMBINE:
            raise ValueError(f"combine must be one of {COMBINE}, not {combine!r}")
        if op == "fn" and update_fn is None:
            raise ValueError("op='fn' needs update_fn")
        if combine != "sum" and op in ("set",):
            raise ValueError("op='set' already keeps the last push of a key")
        if num_ids is None and not sparse:
            raise ValueError("a dense shard needs num_ids (or pass sparse=True)")
        if sparse and not (isinstance(partition, str) and partition == "hash"):
            raise ValueError("sparse shards are hash partitioned (|id| % P)")
        self._given = (table, ps)
        self.num_ids = int(num_ids) if num_ids is not None else 0
        self.dim, self.op, self.init, self.seed = int(dim), op, init, seed
        self.partition, self.wire_dtype, self.lr, self.dtype = partition, _WIRE[wire_dtype], lr, dtype
        self.track_touched = track_touched
        self.sparse, self.capacity = bool(sparse), int(capacity)
        self.init_fn, self.update_fn, self.combine = init_fn, update_fn, combine
        self.dedup = dedup
        self.ps_parallelism = ps_parallelism
        self.table: Optional[ShardedTable] = None
        self.ps: Optional[TensorPS] = None

    # ------------------------------------------------------------- lifecycle
    def open(self, comm: Comm) -> None:
        """Allocate this rank's shard (``ParameterServerLogic.open``)."""
        table, ps = self._given
        P = int(self.ps_parallelism or comm.world)
        if not 1 <= P <= comm.world:
            raise ValueError(f"ps_parallelism={P} on {comm.world} ranks: need 1 <= P <= ranks")
        if P != comm.world and (self.sparse or self.locking or table is not None):
            raise ValueError("ps_parallelism < ranks needs a dense, non-locking shard allocated by the logic")
        if table is not None:
            self.table = table
        elif self.sparse:
            self.table = HashShardTable(self.dim, comm.rank, comm.world, self.init, self.seed, comm.device,
                                        optimizer=self.op, capacity=self.capacity, dtype=self.dtype,
                                        init_fn=self.init_fn, update_fn=self.update_fn, num_ids=self.num_ids)
        else:
            partition, owner = self.partition, None
            if not isinstance(partition, str):
                owner, partition = owner_table(partition, self.num_ids, P), "lookup"
            track = self.track_touched or self.emit == "close" or self.op == "fn"
            # zero-init additive fp32 shards track touched rows by the -0.0 sentinel
            # (ShardedTable touch_sentinel: no byte-mark pass per micro-batch)
            sentinel = (track and tuple(self.init) == ("zeros",) and self.op in ("add", "sgd")
                        and self.dtype == torch.float32 and partition != "lookup" and self.init_fn is None)
            self.table = ShardedTable(self.num_ids, self.dim, comm.rank, P, partition, self.init,
                                      self.seed, comm.device, optimizer=self.op, track_touched=track,
                                      dtype=self.dtype, owner=owner, init_fn=self.init_fn, update_fn=self.update_fn,
                                      touch_sentinel=sentinel)
        self.ps = ps if ps is not None else TensorPS(self.table, comm, self.wire_dtype)
        # set-rules, user rules and per-push outputs must tell pushed keys from
        # merely pulled ones (a user rule need not map a zero delta to a no-op)
        self.ps.masked_push = self.op in ("set", "fn") or self.emit == "push" or self.combine != "sum"
        if self.dedup is not None:
            self.ps.dedup_mode = self.dedup

    @property
    def needs_mask(self) -> bool:
        return self.ps.masked_push

    def after_push(self, updated) -> List[Any]:
        """PS outputs of one applied push: ``(global ids, new rows)`` on this shard."""
        if self.emit == "push" and updated is not None:
            return [updated]  # (ids, rows) or a MaskedPair; no emptiness test (that would sync)
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


class DeviceFunctionPSLogic(DevicePSLogic):
    """``SimplePSLogic(paramInit, paramUpdate)`` with vectorised user rules:
    ``init_fn(ids int64[n]) -> [n, dim]`` (default zeros), ``update_fn(old [n, dim],
    delta [n, dim][, ids int64[n]]) -> [n, dim]``.  ``num_ids=None`` -> a sparse
    hash-table shard over the whole int32 id space (the reference's HashMap);
    ``emit="push"`` outputs ``(ids, new rows)`` after every push, ``"close"``
    dumps the shard at close (``SimplePSLogicWithClose``)."""

    def __init__(self, dim: int = 1, init_fn: Optional[Callable] = None, update_fn: Optional[Callable] = None,
                 num_ids: Optional[int] = None, *, emit: str = "push", combine: str = "sum", **kw):
        if update_fn is None:
            raise ValueError("DeviceFunctionPSLogic needs update_fn")
        if emit not in ("push", "close", "none"):
            raise ValueError(emit)
        self.emit = emit
        kw.setdefault("sparse", num_ids is None)
        super().__init__(num_ids, dim, op="fn", init_fn=init_fn, update_fn=update_fn, combine=combine, **kw)


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
        if kw.get("sparse"):
            raise ValueError("DeviceLockPSLogic needs a dense shard")
        super().__init__(num_ids, dim, **kw)

    def open(self, comm: Comm) -> None:
        from ..parallel.locked_ps import LockedTensorPS

        super().open(comm)
        self.ps.masked_push = False  # a holder's release always carries its row
        self.locked = LockedTensorPS(self.table, comm, self.wire_dtype, ps=self.ps)

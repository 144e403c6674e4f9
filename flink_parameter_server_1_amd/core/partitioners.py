"""Key -> shard partitioning (kernel K1).

* ``hash_partition(id, P) = |id| % P`` — the reference default
  ``Math.abs(id.hashCode) % psParallelism`` (``M/FlinkParameterServer.scala:126-138``,
  ``M/matrix/factorization/utils/Utils.scala:51-65``); for Int keys the
  hashCode is the value itself.  Kept bit-identical so model dumps shard the
  same way.  ``Math.abs(Int.MinValue)`` is negative in the JVM;
  here the modulo is always non-negative.
* ``range_partition(id, F, P) = |id| // ceil(F/P)`` — ``rangePartitionerPS``
  (``M/passive/aggressive/PassiveAggressiveParameterServer.scala:372-384``),
  paired with ``RangePSLogicWithClose``.

The tensor versions (``*_tensor``) are what the GPU engine uses; the HIP
bucketize kernel (``ops.bucketize``) computes the same function plus the
per-shard counts and stable positions that lay out the all-to-all.
"""
from __future__ import annotations

import math
from typing import Callable

import torch

from .messages import PSToWorker, WorkerToPS


def hash_partition(param_id: int, n: int) -> int:
    return abs(int(param_id)) % n


def range_block(feature_count: int, n: int) -> int:
    return int(math.ceil(feature_count / n))


def range_partition(param_id: int, feature_count: int, n: int) -> int:
    return min(abs(int(param_id)) // range_block(feature_count, n), n - 1)


def hash_partition_tensor(ids: torch.Tensor, n: int) -> torch.Tensor:
    return torch.remainder(ids.abs(), n)


def range_partition_tensor(ids: torch.Tensor, feature_count: int, n: int) -> torch.Tensor:
    return torch.clamp(ids.abs() // range_block(feature_count, n), max=n - 1)


class Partitioner:
    """A shard function over integer ids with its local-index mapping."""

    kind = "custom"

    def __init__(self, n: int, fn: Callable[[int], int] = None):
        self.n = n
        self.fn = fn

    def shard(self, param_id: int) -> int:
        return self.fn(param_id) % self.n

    def shard_tensor(self, ids: torch.Tensor) -> torch.Tensor:
        return torch.tensor([self.shard(int(i)) for i in ids.tolist()], dtype=torch.int64, device=ids.device)

    # message-level partitioner as used by ``transform`` overload (c)
    def for_worker_msgs(self) -> Callable[[WorkerToPS], int]:
        return lambda m: self.shard(m.msg.value.param_id)

    def __call__(self, param_id: int) -> int:
        return self.shard(param_id)


class HashPartitioner(Partitioner):
    kind = "hash"

    def __init__(self, n: int):
        super().__init__(n)

    def shard(self, param_id):
        return abs(int(param_id)) % self.n

    def shard_tensor(self, ids):
        return hash_partition_tensor(ids, self.n)

    def local_index(self, ids):
        return ids.abs() // self.n

    def shard_size(self, num_ids: int, shard: int) -> int:
        return max(0, (num_ids - shard + self.n - 1) // self.n)

    def global_ids(self, shard: int, num_ids: int) -> torch.Tensor:
        return torch.arange(shard, num_ids, self.n, dtype=torch.int64)


class RangePartitioner(Partitioner):
    kind = "range"

    def __init__(self, n: int, feature_count: int):
        super().__init__(n)
        self.feature_count = feature_count
        self.block = range_block(feature_count, n)

    def shard(self, param_id):
        return min(abs(int(param_id)) // self.block, self.n - 1)

    def shard_tensor(self, ids):
        return range_partition_tensor(ids, self.feature_count, self.n)

    def local_index(self, ids):
        return ids.abs() - self.shard_tensor(ids) * self.block

    def shard_size(self, num_ids: int, shard: int) -> int:
        lo = shard * self.block
        hi = min(num_ids, lo + self.block) if shard < self.n - 1 else num_ids
        return max(0, hi - lo)

    def global_ids(self, shard: int, num_ids: int) -> torch.Tensor:
        lo = shard * self.block
        return torch.arange(lo, lo + self.shard_size(num_ids, shard), dtype=torch.int64)


class LookupPartitioner(Partitioner):
    """Arbitrary id -> shard assignment given as a table (P2c: the reference's
    custom ``WorkerToPS => Int`` partitioners, ``M/FlinkParameterServer.scala:198-199``,
    on the device path).  ``owner[i]`` is the shard of id ``i``; a shard stores its
    ids densely in id order.  The tensor engine addresses it through *virtual keys*
    ``vkey = owner * block + local`` (``block`` = largest shard), i.e. as a range
    partition of the virtual key space, so every dedup / all-to-all / gather kernel
    is reused unchanged."""

    kind = "lookup"

    def __init__(self, n: int, owner):
        super().__init__(n)
        owner = torch.as_tensor(owner, dtype=torch.int64).cpu()
        if owner.numel() and (int(owner.min()) < 0 or int(owner.max()) >= n):
            raise ValueError("owner entries must lie in [0, n)")
        self.owner = owner
        counts = torch.bincount(owner, minlength=n)
        self.counts = counts
        self.block = max(1, int(counts.max())) if owner.numel() else 1
        order = torch.argsort(owner, stable=True)
        starts = torch.zeros(n + 1, dtype=torch.int64)
        starts[1:] = torch.cumsum(counts, 0)
        local = torch.empty_like(owner)
        local[order] = torch.arange(owner.numel()) - starts[owner[order]]
        self.local = local
        if n * self.block >= (1 << 31):
            raise ValueError("virtual key space exceeds int32")

    def shard(self, param_id):
        return int(self.owner[abs(int(param_id))])

    def shard_tensor(self, ids):
        return self.owner.to(ids.device)[ids.abs()]

    def local_index(self, ids):
        return self.local.to(ids.device)[ids.abs()]

    def shard_size(self, num_ids: int, shard: int) -> int:
        return int(self.counts[shard])

    def global_ids(self, shard: int, num_ids: int) -> torch.Tensor:
        return torch.nonzero(self.owner == shard).flatten()

    def vkeys(self) -> torch.Tensor:
        """``owner * block + local`` per id (int32)."""
        return (self.owner * self.block + self.local).to(torch.int32)


def range_partitioner_ps(feature_count: int):
    """``rangePartitionerPS(featureCount)(psParallelism)`` as a WorkerToPS partitioner."""

    def make(ps_parallelism: int):
        block = range_block(feature_count, ps_parallelism)
        return lambda msg: abs(msg.msg.value.param_id) // block

    return make


def worker_index_partitioner(msg: PSToWorker) -> int:
    return msg.worker_partition_index

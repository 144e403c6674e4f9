"""HBM-resident PS shard tables.

A ``ShardedTable`` is the device counterpart of the PS logics in
``ps/logics.py``: each rank owns one shard of a ``[num_ids, dim]`` parameter
table, laid out densely in HBM (288 GB per MI355X -- a 100B-parameter fp32
table is ~50 GB per GPU over 8).  Lazy "init on first pull" of the reference
(``M/server/SimplePSLogic.scala:13-14``) becomes a deterministic init of
every row keyed by its *global* id (hash RNG, ``ops.init_rows``), which
yields the same value whenever the row is first touched and whichever shard
holds it.  A ``touched`` byte per row reproduces the close-time dump of only
the touched parameters (``SimplePSLogicWithClose`` / ``RangePSLogicWithClose``).

Partitioning: ``hash`` (``|id| % P``, the reference default) or ``range``
(``|id| // ceil(F/P)``, ``rangePartitionerPS``).  Local row of an id:
hash -> ``id // P``; range -> ``id - shard * block``.
"""
from __future__ import annotations

import inspect
from typing import Callable, Optional, Tuple

import torch

from .. import ops
from ..core.partitioners import HashPartitioner, LookupPartitioner, RangePartitioner


def _arity(fn: Callable) -> int:
    try:
        ps = inspect.signature(fn).parameters.values()
    except (TypeError, ValueError):
        return 2
    if any(p.kind == p.VAR_POSITIONAL for p in ps):
        return 3
    return sum(p.kind in (p.POSITIONAL_ONLY, p.POSITIONAL_OR_KEYWORD) for p in ps)


def fn_init_values(init_fn: Callable, gids: torch.Tensor, dim: int, dtype, device) -> torch.Tensor:
    """``init_fn(global ids int64[n]) -> [n, dim]`` rows (a scalar row broadcasts)."""
    v = torch.as_tensor(init_fn(gids), device=device)
    return v.to(dtype).reshape(gids.numel(), -1).expand(gids.numel(), dim).contiguous() if v.numel() else \
        torch.zeros((0, dim), dtype=dtype, device=device)


def fn_apply(store: torch.Tensor, scratch: int, rows: torch.Tensor, deltas: torch.Tensor, update_fn: Callable,
             global_ids: Callable, fresh: Optional[torch.Tensor] = None) -> None:
    """User push rule on the owner (the ``paramUpdate: (P, P) => P`` of
    ``transform`` overload (a), ``M/FlinkParameterServer.scala:62-77``):
    ``store[r] = update_fn(store[r], delta[, ids])`` for every valid row
    (``rows >= 0``; rows unique within the call), ``delta`` itself where the id
    was absent (``fresh``: ``SimplePSLogic``'s ``None => delta``,
    ``M/server/SimplePSLogic.scala:16-22``).  Masked entries go to the scratch
    row, so nothing here needs a host sync."""
    if rows.numel() == 0:
        return
    valid = rows >= 0
    r = torch.where(valid, rows.long(), torch.full_like(rows.long(), scratch))
    old = store[r]
    d = deltas.reshape(old.shape).to(old.dtype)
    if _arity(update_fn) >= 3:
        new = update_fn(old, d, global_ids(r.clamp_max(scratch - 1)))
    else:
        new = update_fn(old, d)
    new = torch.as_tensor(new, device=old.device).to(old.dtype).reshape(old.shape)
    if fresh is not None:
        new = torch.where(fresh.bool().view(-1, 1), d, new)
    store.index_put_((r,), new)


class ShardedTable:
    PART_KIND = {"hash": 0, "range": 1, "lookup": 1}

    def __init__(self, num_ids: int, dim: int, rank: int = 0, world: int = 1, partition: str = "hash",
                 init: Tuple = ("uniform", -0.01, 0.01), seed: int = 0, device="cpu", optimizer: str = "add",
                 track_touched: bool = True, dtype=torch.float32, owner: Optional[torch.Tensor] = None,
                 init_fn: Optional[Callable] = None, update_fn: Optional[Callable] = None,
                 touch_sentinel: bool = False):
        """``partition="lookup"`` takes ``owner[num_ids]`` (id -> shard): an arbitrary
        assignment, addressed through virtual keys (``LookupPartitioner``).
        ``optimizer="fn"``: user rules -- ``init_fn(global ids) -> rows`` (applied to
        the whole shard at construction: deterministic-by-id rules then equal
        init-on-first-pull) and ``update_fn(old, delta[, ids]) -> new`` (``fn_apply``).

        ``touch_sentinel`` (zero init, additive rule, fp32): instead of a byte of
        "touched" marks per row, untouched rows hold -0.0 (which reads as zero); the
        first serve of a row, and any push to it, leave +0.0 or a value there
        (``csrc/kernels/table_ops.hip``), so the close-time dump keeps exactly the rows
        that were pulled or pushed without a mark pass per micro-batch (PA's 1B-feature
        shards: ~100 us of random byte stores per 4M requests, and 1 GB of marks)."""
        if partition not in self.PART_KIND:
            raise ValueError(partition)
        self.num_ids, self.dim, self.rank, self.world = int(num_ids), int(dim), rank, world
        self.partition = partition
        self.part_kind = self.PART_KIND[partition]
        self.device = torch.device(device)
        if partition == "lookup":
            if owner is None or len(owner) != self.num_ids:
                raise ValueError("partition='lookup' needs owner[num_ids]")
            self.part = LookupPartitioner(world, owner)
            self._vkey = self.part.vkeys().to(self.device)
            self._gids = self.part.global_ids(rank, self.num_ids).to(self.device)
        else:
            self.part = HashPartitioner(world) if partition == "hash" else RangePartitioner(world, num_ids)
        self.block = 1 if partition == "hash" else self.part.block
        # rank >= world: a rank of a larger job holding no shard (ps_parallelism < ranks)
        self.n_local = self.part.shard_size(self.num_ids, rank) if rank < world else 0
        self.optimizer = optimizer
        self.seed = seed
        self.init_spec = init
        self.init_fn, self.update_fn = init_fn, update_fn
        if optimizer == "fn" and update_fn is None:
            raise ValueError("optimizer='fn' needs update_fn")
        self.sentinel = bool(touch_sentinel)
        if self.sentinel and (init[0] != "zeros" or optimizer not in ("add", "sgd") or dtype != torch.float32
                              or partition == "lookup"):
            raise ValueError("touch_sentinel needs zero init, an additive rule (add / sgd), fp32 rows and a "
                             "hash / range partition")
        if self.sentinel:
            track_touched = False
        # function rules get one scratch row past the shard (masked apply entries)
        self._store = torch.empty((self.n_local + (optimizer == "fn"), self.dim), dtype=dtype, device=self.device)
        self.weight = self._store[:self.n_local]
        self.reset_parameters()
        # optimizer state: Adagrad accumulators [n, D]; add_renorm keeps each row's
        # euclidean length [n] next to it (LengthAndVector, K3 add+renorm)
        if optimizer == "adagrad":
            self.state = torch.zeros_like(self.weight)
        elif optimizer == "add_renorm":
            self.state = self.weight.norm(dim=1).to(torch.float32)
        else:
            self.state = None
        self._touched_store = torch.zeros(self.n_local + (optimizer == "fn"), dtype=torch.uint8,
                                          device=self.device) if track_touched else None
        self.touched = self._touched_store[:self.n_local] if track_touched else None

    sparse = False

    # ----------------------------------------------------------- id mapping
    @property
    def id_base(self) -> int:
        return self.rank if self.partition == "hash" else self.rank * self.block

    @property
    def id_stride(self) -> int:
        return self.world if self.partition == "hash" else 1

    @property
    def key_space(self) -> int:
        """Size of the key space the tensor PS dedups / routes (virtual keys for lookup)."""
        return self.world * self.block if self.partition == "lookup" else self.num_ids

    def route_keys(self, ids: torch.Tensor) -> torch.Tensor:
        """Global ids -> routing keys (identity, or virtual keys for ``lookup``)."""
        if self.partition == "lookup":
            return self._vkey[ids.long()]
        return ids

    def global_ids(self, local: torch.Tensor) -> torch.Tensor:
        if self.partition == "lookup":
            return self._gids[local.long()]
        return self.id_base + local.long() * self.id_stride

    def local_of(self, ids: torch.Tensor) -> torch.Tensor:
        return self.part.local_index(ids.long())

    # ----------------------------------------------------------- lifecycle
    def reset_parameters(self):
        kind = self.init_spec[0]
        if self.init_fn is not None:
            chunk = 1 << 20
            for s in range(0, self.n_local, chunk):
                loc = torch.arange(s, min(s + chunk, self.n_local), device=self.device)
                self.weight[s:s + loc.numel()] = fn_init_values(self.init_fn, self.global_ids(loc), self.dim,
                                                                self.weight.dtype, self.device)
        elif kind == "uniform" and self.partition == "lookup":
            _, lo, hi = self.init_spec  # ids are not an arithmetic progression: init by explicit id
            from ..ops import reference as R

            j = torch.arange(self.dim, dtype=torch.int64, device=self.device).view(1, -1)
            vals = float(lo) + (float(hi) - float(lo)) * R.hash_uniform(self.seed, self._gids.view(-1, 1), j)
            self.weight.copy_(vals)
        elif kind == "uniform":
            _, lo, hi = self.init_spec
            ops.init_rows(self.weight, self.id_base, self.id_stride, float(lo), float(hi), self.seed)
        elif kind == "zeros":
            self.weight.fill_(-0.0 if getattr(self, "sentinel", False) else 0.0)
        elif kind == "const":
            self.weight.fill_(float(self.init_spec[1]))
        else:
            raise ValueError(f"unknown init {kind}")

    # ----------------------------------------------------------- PS side
    @property
    def scratch_row(self) -> int:
        return self.n_local

    def rows_for(self, local_keys: torch.Tensor, insert: bool = True, push: bool = False):
        """``(rows, fresh)``: dense shards store local key k at row k; ``fresh``
        (function rules only, on a push) marks rows never touched before."""
        fresh = None
        if push and self.optimizer == "fn" and self.touched is not None and local_keys.numel():
            fresh = self.touched[local_keys.long().clamp_min(0)] == 0
        return local_keys, fresh

    def serve_rows(self, rows: torch.Tensor, wire_dtype=torch.float32, mark: bool = True) -> torch.Tensor:
        """Pull serve (K2); ``mark``: the served rows count as touched (close-time dump).
        The marks are a separate pass: fused into the narrow-row gather, the random byte
        stores cost 170 us per 3.8M rows of a 1B-row table, on their own 63 us
        (``bench/probe_sorted_gather.py``)."""
        out = ops.gather_rows(self.weight, rows, out_dtype=wire_dtype, flip=mark and self.sentinel)
        if mark and self.touched is not None:
            ops.mark_rows(self.touched, rows)
        return out

    def serve(self, local_keys: torch.Tensor, wire_dtype=torch.float32) -> torch.Tensor:
        """Pull serve (K2): rows for the requested local keys."""
        return self.serve_rows(local_keys, wire_dtype)

    def apply_rows(self, rows: torch.Tensor, deltas: torch.Tensor, lr: float = 0.0, op: Optional[str] = None,
                   fresh: Optional[torch.Tensor] = None, mark: bool = True) -> None:
        """Push apply (K3).  ``mark = False``: the rows are known to be touched already
        (served by the same plan), so the apply skips the byte stores."""
        op = op or self.optimizer
        if op == "fn":
            fn_apply(self._store, self.scratch_row, rows, deltas, self.update_fn, self.global_ids, fresh)
            if self.touched is not None:  # masked entries mark the scratch byte
                r = torch.where(rows >= 0, rows.long(), torch.full_like(rows.long(), self.scratch_row))
                self._touched_store[r] = 1
            return
        ops.apply_rows(self.weight, rows, deltas, op, lr=lr, state=self.state, touched=self.touched if mark else None)

    def apply(self, local_keys: torch.Tensor, deltas: torch.Tensor, lr: float = 0.0, op: Optional[str] = None):
        """Push apply (K3) with the table's update rule."""
        rows, fresh = self.rows_for(local_keys, push=True)
        self.apply_rows(rows, deltas, lr, op, fresh=fresh)
        if op == "set" and self.optimizer == "add_renorm":  # model load: lengths of the written rows
            k = local_keys.long()
            k = k[k >= 0]
            self.state[k] = self.weight[k].norm(dim=1).to(self.state.dtype)

    def lengths(self, local_keys: torch.Tensor) -> torch.Tensor:
        """Row lengths kept by an ``add_renorm`` table."""
        if self.optimizer != "add_renorm":
            raise ValueError("lengths() needs optimizer='add_renorm'")
        return self.state[local_keys.long()]

    def load(self, ids: torch.Tensor, values: torch.Tensor):
        """Model load (``transformWithModelLoad``): set rows owned by this shard."""
        ids = ids.to(self.device).long()
        mine = self.part.shard_tensor(ids) == self.rank
        loc = self.local_of(ids[mine]).to(torch.int32)
        vals = values.to(self.device)[mine].to(torch.float32).contiguous()
        if self.sentinel:  # raw copy: a snapshot's untouched rows keep their -0.0 sentinel
            self.weight[loc.long()] = vals.reshape(loc.numel(), self.dim)
            return
        ops.apply_rows(self.weight, loc, vals, "set", touched=self.touched)

    def dump(self, only_touched: bool = True, raw: bool = False):
        """(global ids, values) of this shard -- the close-time model output.  ``raw``:
        values exactly as stored (snapshots keep the -0.0 untouched sentinel so a restore
        keeps the touched set; model outputs print +0.0)."""
        if only_touched and self.sentinel:
            loc = torch.nonzero(self.touched_mask(), as_tuple=False).flatten()
        elif only_touched and self.touched is not None:
            loc = torch.nonzero(self.touched, as_tuple=False).flatten()
        else:
            loc = torch.arange(self.n_local, device=self.device)
        vals = self.weight[loc]
        if self.sentinel and not raw:  # model outputs never carry the sentinel: untouched entries print 0.0, not -0.0
            vals = vals + 0.0
        return self.global_ids(loc), vals

    def touched_mask(self) -> Optional[torch.Tensor]:
        """bool[n_local]: rows pulled or pushed so far (None: not tracked)."""
        if self.sentinel:
            return (self.weight.view(torch.int32) != -(1 << 31)).any(dim=1)
        return None if self.touched is None else self.touched.bool()

    def nbytes(self) -> int:
        n = self.weight.numel() * self.weight.element_size()
        if self.state is not None:
            n += self.state.numel() * self.state.element_size()
        return n

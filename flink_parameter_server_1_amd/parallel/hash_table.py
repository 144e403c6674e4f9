"""Sparse-id PS shard: a persistent open-addressing hash table in HBM.

The reference's ``SimplePSLogic`` keeps a ``HashMap[Integer, P]`` over the full
signed 32-bit id space and initialises a parameter on its first pull
(``M/server/SimplePSLogic.scala:7-26``); ids can be anything -- negative, huge,
sparse.  ``ShardedTable`` covers dense ``[0, num_ids)`` spaces (MF, PA); this
table covers the rest:

* shard of an id: ``|id| % P`` computed in 64 bits (no ``Math.abs(Int.MinValue)``
  overflow) -- ``part_kind`` 2 of the dedup / bucketize kernels;
* the owner maps an id to a row through ``kernels/hash_table.hip``: ``tab``
  (linear probing, CAS insert), ``rowmap`` (slot -> row), ``rowkey``
  (row -> id) and a COMPACT row pool ``[rows, D]`` filled in first-insert
  order.  Growing the pool or rehashing ``tab`` never moves a row, so row
  indices cached by in-flight plans stay valid;
* a pull inserts absent ids and initialises them (``init`` spec or a user
  ``init_fn``) -- lazy init on first touch; a push to an id never pulled
  inserts it with a zero row, so ``add`` / ``set`` store the delta itself and
  a function rule sees ``fresh`` (``None => delta`` of ``SimplePSLogic.onPushRecv``);
* capacity is kept ahead of the inserts without a per-call host sync: the
  row counter is copied to pinned memory asynchronously after every insert
  and the host tracks an upper bound (last seen count + keys sent since); only
  when that bound would exceed the reserve does the host read the exact count
  and grow (``tab`` to >= 2x the rows, power of two; pool by doubling).

``stats()`` reports the load factor, probe-free capacity and growth events.
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import torch

from .. import ops
from .table import fn_apply, fn_init_values


def _pow2_at_least(n: int) -> int:
    return 1 << max(10, (max(int(n), 1) - 1).bit_length())


class HashShardTable:
    """Drop-in for ``ShardedTable`` on the tensor PS path (``TensorPS`` /
    device PS logics) for arbitrary int32 ids."""

    sparse = True
    part_kind = 2
    block = 1
    partition = "hash"

    def __init__(self, dim: int, rank: int = 0, world: int = 1, init: Tuple = ("zeros",), seed: int = 0,
                 device="cpu", optimizer: str = "add", capacity: int = 1 << 14, dtype=torch.float32,
                 init_fn: Optional[Callable] = None, update_fn: Optional[Callable] = None, num_ids: int = 0,
                 max_load: float = 0.5):
        self.dim, self.rank, self.world = int(dim), rank, world
        self.device = torch.device(device)
        self.optimizer, self.seed, self.init_spec = optimizer, seed, tuple(init)
        self.init_fn, self.update_fn = init_fn, update_fn
        self.num_ids = int(num_ids)  # informational (0 = the whole int32 space)
        self.max_load = float(max_load)
        self.dtype = dtype
        if init_fn is None and self.init_spec[0] not in ops._HT_INIT:
            raise ValueError(f"unknown init {self.init_spec[0]}")
        cap = _pow2_at_least(int(capacity / self.max_load) + 1)
        self.tab = torch.zeros(cap, dtype=torch.int64, device=self.device)
        self.rowmap = torch.full((cap,), -1, dtype=torch.int32, device=self.device)
        rcap = max(int(capacity), 16)
        self.rowkey = torch.zeros(rcap, dtype=torch.int32, device=self.device)
        # +1: a scratch row that absorbs masked entries of the function-rule apply
        self._store = torch.zeros((rcap + 1, self.dim), dtype=dtype, device=self.device)
        self.state = self._new_state(rcap + 1)
        self.count = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.overflow = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.touched = None  # every stored row was touched (inserted by a pull or a push)
        self._ub = 0          # host upper bound of count
        self._since = 0       # keys reserved since the pending async count copy started
        self._pending = None  # (event, pinned count) of the last async copy
        self.grow_events = 0
        self.host_syncs = 0

    # ----------------------------------------------------------------- layout
    def _new_state(self, n):
        if self.optimizer == "adagrad":
            return torch.zeros((n, self.dim), dtype=torch.float32, device=self.device)
        if self.optimizer == "add_renorm":
            return torch.zeros(n, dtype=torch.float32, device=self.device)
        return None

    @property
    def rcap(self) -> int:
        return self.rowkey.numel()

    @property
    def weight(self) -> torch.Tensor:
        """The row pool (rows beyond ``count`` are unused)."""
        return self._store[:self.rcap]

    @property
    def scratch_row(self) -> int:
        return self.rcap

    @property
    def key_space(self) -> int:
        return 1 << 32

    @property
    def n_local(self) -> int:
        """Rows stored on this shard (host sync)."""
        return int(self.count[0])

    # ---------------------------------------------------------------- capacity
    def reserve(self, n_new: int) -> None:
        """Make room for up to ``n_new`` inserts before a lookup-insert launch."""
        if self._pending is not None and (self._pending[0] is None or self._pending[0].query()):
            self._ub = int(self._pending[1][0]) + self._since
            self._pending = None
        need = self._ub + int(n_new)
        if need <= self.rcap and need <= self.max_load * self.tab.numel():
            self._ub = need
            self._since += int(n_new)
            return
        exact = int(self.count[0])  # host sync: rare (only when the bound runs out)
        self.host_syncs += 1
        if int(self.overflow[0]):
            raise RuntimeError("device hash table overflow")
        need = exact + int(n_new)
        if need > self.rcap:
            self._grow_rows(max(2 * self.rcap, need + need // 2))
        if need > self.max_load * self.tab.numel():
            self._rehash(_pow2_at_least(int(2 * need / self.max_load)), exact)
        self._ub = need
        self._since = int(n_new)
        self._pending = None

    def _grow_rows(self, rcap: int) -> None:
        old_n = self.rcap
        store = torch.zeros((rcap + 1, self.dim), dtype=self.dtype, device=self.device)
        store[:old_n] = self._store[:old_n]
        self._store = store
        rk = torch.zeros(rcap, dtype=torch.int32, device=self.device)
        rk[:old_n] = self.rowkey
        self.rowkey = rk
        if self.state is not None:
            st = self._new_state(rcap + 1)
            st[:old_n] = self.state[:old_n]
            self.state = st
        self.grow_events += 1

    def _rehash(self, cap: int, count: int) -> None:
        self.tab = torch.zeros(cap, dtype=torch.int64, device=self.device)
        self.rowmap = torch.full((cap,), -1, dtype=torch.int32, device=self.device)
        ops.ht_rehash(self.rowkey, count, self.tab, self.rowmap, self.overflow)
        self.grow_events += 1

    def _after_insert(self) -> None:
        if self._pending is not None:
            return
        if self.device.type == "cuda":
            host = torch.empty(1, dtype=torch.int32, pin_memory=True)
            host.copy_(self.count, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            self._pending = (ev, host)
        else:
            self._pending = (None, self.count.clone())
        self._since = 0

    # ------------------------------------------------------------ id mapping
    def route_keys(self, ids: torch.Tensor) -> torch.Tensor:
        return ids

    def global_ids(self, rows: torch.Tensor) -> torch.Tensor:
        return self.rowkey[rows.long()].long()

    def rows_for(self, keys: torch.Tensor, insert: bool = True, push: bool = False):
        """``(rows int32, fresh uint8)`` of ``keys`` (int32 ids); inserts absent ids
        (pull: initialised; push: zero rows) unless ``insert`` is False (absent -> -1)."""
        keys = keys.to(device=self.device, dtype=torch.int32).contiguous()
        n = keys.numel()
        if insert:
            self.reserve(n)
        if push or not insert:
            init = ("zeros",)
        elif self.init_fn is not None:
            init = ("zeros",)
        else:
            init = self.init_spec
        kernel_init = insert and self._store.dtype == torch.float32  # the init kernel writes fp32 rows
        rows, fresh = ops.ht_lookup(keys, self.tab, self.rowmap, self.rowkey, self.count, self.overflow, insert,
                                    self._store if kernel_init else None, init, self.seed)
        if insert:
            self._after_insert()
            torch_init = self.init_fn is not None or (not kernel_init and init[0] != "zeros")
            if torch_init and not push and n:
                r = torch.where(rows >= 0, rows.long(), torch.full_like(rows.long(), self.scratch_row))
                if self.init_fn is not None:
                    vals = fn_init_values(self.init_fn, keys.long(), self.dim, self.dtype, self.device)
                elif init[0] == "const":
                    vals = torch.full((n, self.dim), float(init[1]), dtype=self.dtype, device=self.device)
                else:
                    from ..ops import reference as R

                    vals = R.init_values(keys, self.dim, float(init[1]), float(init[2]), self.seed).to(
                        device=self.device, dtype=self.dtype)
                # fresh rows are still zero: accumulating init * fresh writes each
                # fresh row exactly once and adds 0 to every other request's row
                self._store.index_put_((r,), vals * fresh.view(-1, 1).to(vals.dtype), accumulate=True)
            if self.optimizer == "add_renorm" and not push and n:  # lengths of the fresh rows
                r = torch.where(rows >= 0, rows.long(), torch.full_like(rows.long(), self.scratch_row))
                self.state[r] = torch.where(fresh.bool(), self._store[r].norm(dim=1).float(), self.state[r])
        return rows, fresh

    def local_of(self, ids: torch.Tensor) -> torch.Tensor:
        return self.rows_for(ids, insert=False)[0]

    # ----------------------------------------------------------------- PS side
    def serve_rows(self, rows: torch.Tensor, wire_dtype=torch.float32, mark: bool = True) -> torch.Tensor:
        return ops.gather_rows(self._store, rows.clamp_min(0), out_dtype=wire_dtype)

    def serve(self, keys: torch.Tensor, wire_dtype=torch.float32) -> torch.Tensor:
        return self.serve_rows(self.rows_for(keys)[0], wire_dtype)

    def apply_rows(self, rows: torch.Tensor, deltas: torch.Tensor, lr: float = 0.0, op: Optional[str] = None,
                   fresh: Optional[torch.Tensor] = None, mark: bool = True) -> None:
        op = op or self.optimizer
        if op == "fn":
            fn_apply(self._store, self.scratch_row, rows, deltas, self.update_fn, self.global_ids, fresh)
            return
        ops.apply_rows(self._store, rows, deltas, op, lr=lr, state=self.state)

    def apply(self, keys: torch.Tensor, deltas: torch.Tensor, lr: float = 0.0, op: Optional[str] = None):
        rows, fresh = self.rows_for(keys, push=True)
        self.apply_rows(rows, deltas, lr, op, fresh=fresh)

    def lengths(self, rows: torch.Tensor) -> torch.Tensor:
        if self.optimizer != "add_renorm":
            raise ValueError("lengths() needs optimizer='add_renorm'")
        return self.state[rows.long()]

    def load(self, ids: torch.Tensor, values: torch.Tensor):
        """Set rows of the ids this shard owns (model load)."""
        ids = ids.to(self.device).long()
        mine = (ids.abs() % self.world) == self.rank
        rows, _ = self.rows_for(ids[mine], push=True)
        ops.apply_rows(self._store, rows, values.to(self.device)[mine].to(torch.float32).contiguous(), "set")
        if self.optimizer == "add_renorm":
            self.state[rows.long()] = self._store[rows.long()].norm(dim=1).float()

    def dump(self, only_touched: bool = True, raw: bool = False):
        """``(ids, rows)`` of every stored id (exactly the inserted ones)."""
        n = self.n_local
        return self.rowkey[:n].long(), self._store[:n]

    def nbytes(self) -> int:
        n = self._store.numel() * self._store.element_size() + self.tab.numel() * 12 + self.rowkey.numel() * 4
        if self.state is not None:
            n += self.state.numel() * self.state.element_size()
        return n

    def stats(self) -> dict:
        n = self.n_local
        return {"rows": n, "row_capacity": self.rcap, "slots": self.tab.numel(),
                "load_factor": n / self.tab.numel(), "grow_events": self.grow_events,
                "host_syncs": self.host_syncs, "overflow": int(self.overflow[0])}

    def probe_lengths(self) -> torch.Tensor:
        """Probe length (distance from home slot) of every stored id -- a diagnostic."""
        occ = torch.nonzero(self.tab != 0).flatten()
        keys = (self.tab[occ] & 0xFFFFFFFF)
        from ..ops import reference as R

        home = R.fmix32(keys.cpu() ^ R.HT_SALT) & (self.tab.numel() - 1)
        return (occ.cpu() - home) % self.tab.numel()

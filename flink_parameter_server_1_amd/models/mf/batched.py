"""MF workers for the tensor engine (``core.tensor_engine``): the reference's MF
applications expressed through the public batched ``WorkerLogic`` API.

* ``OnlineMFWorker`` -- ``PSOnlineMatrixFactorizationWorker``
  (``M/matrix/factorization/workers/PSOnlineMatrixFactorizationWorker.scala:41-89``):
  user vectors resident in the worker (rows ``u // W`` of a hash-sharded user
  table, ratings partitioned by ``user % W``), item vectors on the PS
  (``DeviceSimplePSLogic(op="add")``: ``SimplePSLogic`` with ``vectorSum``,
  ``M/matrix/factorization/PSOnlineMatrixFactorization.scala:58-60``).  One
  pull per micro-batch of ratings; the fused SGD kernel (K4,
  ``ops.mf_sgd_pulled``) updates the user rows in place and accumulates one
  delta per unique item, which is pushed as is (``push_unique``).  Outputs
  ``Left((user ids, user rows))`` per micro-batch; the PS emits
  ``Right((item ids, item rows))`` per push.
* ``OfflineMFWorker`` -- ``PSOfflineMatrixFactorizationWorker``
  (``M/matrix/factorization/workers/PSOfflineMatrixFactorizationWorker.scala:64-146``):
  buffers its ratings on the device until the end of input (``on_eof``, the
  ``FlinkEOF`` barrier), then replays ``iterations`` epochs, each a fresh
  device permutation (the reference discards its shuffle, SURVEY B2 -- fixed).

``ps_online_mf_tensor`` / ``ps_offline_mf_tensor`` wire them up like
``psOnlineMF`` / ``psOfflineMF`` (same parameter names and defaults).
"""
from __future__ import annotations

from typing import Iterable, Optional

import torch

from ... import ops
from ...api.batched import BatchedWorkerLogic
from ...core.tensor_engine import TensorRuntime
from ...parallel.comm import Comm
from ...parallel.table import ShardedTable
from ...ps.device_logics import DeviceSimplePSLogic
from .core import USER_SEED_XOR


class OnlineMFWorker(BatchedWorkerLogic):
    """Batches are ``(user, item, rating)`` tensors holding this rank's ratings
    (``user % W == rank``; global ids)."""

    def __init__(self, num_users: int, num_factors: int = 10, learning_rate: float = 0.01, lam: float = 0.0,
                 range_min: float = -0.01, range_max: float = 0.01, seed: int = 0, emit_users: bool = True,
                 dtype=torch.float32):
        self.num_users, self.dim, self.lr, self.lam = int(num_users), int(num_factors), learning_rate, lam
        self.range = (range_min, range_max)
        self.seed, self.emit_users, self.dtype = seed, emit_users, dtype
        self.users: Optional[ShardedTable] = None

    def open(self, ctx):
        self.W, self.r = ctx.number_of_parallel_subtasks, ctx.index_of_this_subtask
        self.device = torch.device(ctx.device)
        # lazy per-user init of the reference = deterministic hash init by global id
        self.users = ShardedTable(self.num_users, self.dim, self.r, self.W, "hash",
                                  ("uniform", self.range[0], self.range[1]), (self.seed ^ USER_SEED_XOR) & 0xFFFFFFFF,
                                  self.device, track_touched=False, dtype=self.dtype)

    def update_model_batch(self, ids, values):
        """Worker-resident model load (users of this rank)."""
        mine = (ids.long().abs() % self.W) == self.r
        self.users.weight[(ids[mine].long() // self.W)] = values[mine].to(self.users.weight.dtype)

    def on_recv_batch(self, batch, ps):
        user, item, rating = batch
        user = user.to(self.device)
        local = (user.long() // self.W).to(torch.int32).contiguous()
        ps.pull(item.to(self.device), (local, user, rating.to(device=self.device, dtype=self.dtype).contiguous()))

    def on_pull_recv_batch(self, pulled, ps):
        local, user, rating = pulled.payload
        U = self.users.weight
        delta = torch.zeros((pulled.n_unique, self.dim), dtype=U.dtype, device=U.device)
        rows = pulled.rows if pulled.rows.dtype == U.dtype or pulled.rows.dtype == torch.bfloat16 else \
            pulled.rows.to(U.dtype)
        ops.mf_sgd_pulled(U, local, rating, rows.contiguous(), pulled.pos, delta, self.lr, self.lam)
        ps.push_unique(delta)
        if self.emit_users:
            ps.output((user, U[local.long()]))

    def user_vectors(self):
        ids = self.users.global_ids(torch.arange(self.users.n_local, device=self.device))
        return ids, self.users.weight


class OfflineMFWorker(OnlineMFWorker):
    """Multi-epoch MF: buffer until end of input, then ``iterations`` shuffled epochs."""

    def __init__(self, num_users: int, num_factors: int = 10, learning_rate: float = 0.01, iterations: int = 1,
                 micro_batch: int = 1024, shuffle: bool = True, **kw):
        super().__init__(num_users, num_factors, learning_rate, **kw)
        self.iterations, self.micro_batch, self.shuffle = int(iterations), int(micro_batch), shuffle
        self._buf = []
        self._replaying = False
        self._done = False

    def on_recv_batch(self, batch, ps):
        if self._replaying:
            return super().on_recv_batch(batch, ps)
        self._buf.append(tuple(t.to(self.device) for t in batch))  # no pulls before EOF

    def on_eof(self, ps) -> Optional[Iterable]:
        if self._done:
            return None
        self._done = True
        self._replaying = True
        if not self._buf:
            return ()
        u, i, r = (torch.cat(c) for c in zip(*self._buf))
        self._buf = []
        g = torch.Generator(device=self.device)
        g.manual_seed(self.seed * 7919 + self.r)

        def epochs():
            n, mb = u.numel(), self.micro_batch
            for _ in range(self.iterations):
                perm = torch.randperm(n, generator=g, device=self.device) if self.shuffle else \
                    torch.arange(n, device=self.device)
                for s in range(0, n, mb):
                    p = perm[s:s + mb]
                    yield u[p], i[p], r[p]

        return epochs()


def _item_logic(num_items, num_factors, range_min, range_max, seed, dtype, wire):
    return DeviceSimplePSLogic(num_items, num_factors, op="add", init=("uniform", range_min, range_max),
                               seed=seed, wire_dtype=wire, dtype=dtype)


def ps_online_mf_tensor(batches: Iterable, num_users: int, num_items: int, num_factors: int = 10,
                        range_min: float = -0.01, range_max: float = 0.01, learning_rate: float = 0.01,
                        lam: float = 0.0, staleness: int = 0, seed: int = 0, comm: Optional[Comm] = None,
                        output_sink=None, dtype=torch.float32, wire: str = "fp32",
                        iteration_wait_time: Optional[float] = None):
    """``psOnlineMF`` on the tensor engine; ``batches`` = this rank's ``(user, item,
    rating)`` micro-batches (users with ``user % W == rank``).  Returns the outputs."""
    worker = OnlineMFWorker(num_users, num_factors, learning_rate, lam, range_min, range_max, seed, dtype=dtype)
    rt = TensorRuntime(comm, staleness, iteration_wait_time, output_sink)
    return rt.execute(batches, worker, _item_logic(num_items, num_factors, range_min, range_max, seed, dtype, wire))


def ps_offline_mf_tensor(batches: Iterable, num_users: int, num_items: int, num_factors: int = 10,
                         range_min: float = -0.01, range_max: float = 0.01, learning_rate: float = 0.01,
                         iterations: int = 1, micro_batch: int = 1024, staleness: int = 0, seed: int = 0,
                         comm: Optional[Comm] = None, output_sink=None, dtype=torch.float32):
    """``psOfflineMF`` on the tensor engine (epochs start at the global end of input)."""
    worker = OfflineMFWorker(num_users, num_factors, learning_rate, iterations=iterations, micro_batch=micro_batch,
                             range_min=range_min, range_max=range_max, seed=seed, dtype=dtype)
    rt = TensorRuntime(comm, staleness, None, output_sink)
    return rt.execute(batches, worker, _item_logic(num_items, num_factors, range_min, range_max, seed, dtype, "fp32"))

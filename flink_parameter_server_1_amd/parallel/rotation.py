"""Item-block rotation over the xGMI ring: stratified MF-SGD without a pull/push round trip.

In ``psOnlineMF`` every rating pulls its item vector from the PS shard and
pushes a delta back (``M/matrix/factorization/workers/PSOnlineMatrixFactorizationWorker.scala:41-55``).
On a node of fully connected GPUs with 288 GB each, the item table (1M x 64
fp32 = 256 MB) is tiny next to the rating stream, so instead of moving rows to
the ratings, the *item shards move to the ratings* (stratified SGD, Gemulla et
al. 2011): the PS shards travel around the ring while each worker updates only
the block it currently holds.

Schedule (K = 2W item blocks, block ``2q+h`` = half ``h`` of PS shard ``q``):

* at rest rank ``r`` holds its home blocks ``2r`` and ``2r+1`` (its PS shard);
* in sub-step ``s`` rank ``r`` updates block ``(2r+s) % K`` with the ratings of
  its users that fall in it; blocks of opposite parity are idle and travel:
* during sub-step ``s >= 1`` rank ``r`` sends block ``2r+s-1`` (finished in
  ``s-1``) to rank ``r-1`` and receives block ``2r+s+1`` from rank ``r+1`` --
  exactly the block it needs next, so the transfer hides behind the compute;
* one micro-batch = K sub-steps = every block once; the schedule is periodic,
  so consecutive micro-batches continue it without a barrier.

Every item block is owned by exactly one GPU at any time and every user row
by its worker, so no parameter is ever updated concurrently by two GPUs and no
update is stale: the result equals a sequential schedule of the sub-steps
(serializable), unlike the bounded-staleness PS path.

``home()`` returns every block to its PS shard (``ShardedTable`` rows) for
evaluation, dumps and checkpoints.
"""
from __future__ import annotations

from typing import List, Optional

import torch

from .comm import Comm


def shard_halves(num_ids: int, world: int) -> List[int]:
    """``half[q]`` = rows of block ``2q`` (the first half of hash shard ``q``)."""
    out = []
    for q in range(world):
        n_local = (num_ids - q + world - 1) // world
        out.append((n_local + 1) // 2)
    return out


def block_rows(num_ids: int, world: int) -> List[int]:
    rows = []
    for q, h in enumerate(shard_halves(num_ids, world)):
        n_local = (num_ids - q + world - 1) // world
        rows += [h, n_local - h]
    return rows


class RingRotation:
    def __init__(self, comm: Comm, home: torch.Tensor, num_ids: int):
        """``home``: this rank's PS shard ``[n_local, D]`` (hash layout ``i % W``)."""
        self.comm = comm
        self.W, self.r = comm.world, comm.rank
        self.K = 2 * self.W
        self.home_t = home
        self.half = shard_halves(num_ids, self.W)
        self.rows = block_rows(num_ids, self.W)
        cap = max(self.rows)
        self.buf = [torch.empty((cap, home.shape[1]), dtype=home.dtype, device=home.device) for _ in range(3)]
        self.at_rest = True
        self.s = 0
        self._A = self._P = self._F = self._N = None
        self._works: Optional[list] = None
        self.bytes_sent = 0

    # --------------------------------------------------------------- blocks
    def _home_slice(self, h: int) -> torch.Tensor:
        hq = self.half[self.r]
        return self.home_t[:hq] if h == 0 else self.home_t[hq:]

    def active_block(self) -> int:
        return (2 * self.r + self.s) % self.K

    def active(self) -> torch.Tensor:
        return self.buf[self._A][: self.rows[self.active_block()]]

    def _peer(self, d: int) -> int:
        return (self.r + d) % self.W

    # --------------------------------------------------------------- schedule
    def _leave_rest(self):
        self.buf[0][: self.rows[2 * self.r]].copy_(self._home_slice(0))
        self.buf[1][: self.rows[2 * self.r + 1]].copy_(self._home_slice(1))
        self._A, self._N, self._F, self._P = 0, 1, 2, None
        self.s = 0
        self.at_rest = False

    def begin(self):
        """Start sub-step ``s``: issue the transfers that overlap its compute."""
        if self.at_rest:
            self._leave_rest()
        if self.W == 1 or self._P is None:  # both blocks resident (W = 1) / next block already home
            return
        out_b = (2 * self.r + self.s - 1) % self.K
        in_b = (2 * self.r + self.s + 1) % self.K
        self._works = self.comm.p2p([(self.buf[self._P][: self.rows[out_b]], self._peer(-1))],
                                    [(self.buf[self._F][: self.rows[in_b]], self._peer(+1))])
        self.bytes_sent += self.buf[self._P][: self.rows[out_b]].numel() * self.buf[0].element_size()

    def end(self):
        """Finish sub-step ``s`` (after its compute was enqueued) and rotate roles."""
        if self.W == 1:  # no peers: the two blocks alternate in place
            self._A, self._N = self._N, self._A
        elif self._P is None:
            self._A, self._P, self._F, self._N = self._N, self._A, self._F, None
        else:
            for w in self._works or []:
                w.wait()
            self._works = None
            self._A, self._P, self._F = self._F, self._A, self._P
        self.s += 1

    # --------------------------------------------------------------- homing
    def home(self):
        """Send every block back to its PS shard (between sub-steps)."""
        if self.at_rest:
            return
        s = self.s  # blocks held: A = 2r+s, P = 2r+s-1 (or N = 2r+1 right after rest)
        if self.W == 1:
            held = {s % 2: self._A, (s + 1) % 2: self._N}
        elif self._P is None:  # still at s == 0 layout: A = 2r, N = 2r+1 -- all home
            held = {2 * self.r: self._A, 2 * self.r + 1: self._N}
        else:
            held = {(2 * self.r + s) % self.K: self._A, (2 * self.r + s - 1) % self.K: self._P}

        def holder(b: int) -> int:
            if self.W == 1 or self._P is None:
                return b // 2
            d = (b - s) % self.K
            return d // 2 if d % 2 == 0 else ((b - s + 1) % self.K) // 2

        # messages between one pair are matched in posting order: post sends and
        # receives in ascending block id on both sides
        sends, recvs = [], []
        for b, bi in sorted(held.items()):
            dst = b // 2
            if dst != self.r:
                sends.append((self.buf[bi][: self.rows[b]], dst))
        for h in (0, 1):
            b = 2 * self.r + h
            src = holder(b)
            if src != self.r:
                recvs.append((self._home_slice(h), src))
        works = self.comm.p2p(sends, recvs)
        for b, bi in held.items():
            if b // 2 == self.r:
                self._home_slice(b % 2).copy_(self.buf[bi][: self.rows[b]])
        for w in works:
            w.wait()
        self.at_rest = True
        self.s = 0
        self._A = self._P = self._F = self._N = None

"""Item-block rotation over xGMI: stratified MF-SGD without a pull/push round trip.

In ``psOnlineMF`` every rating pulls its item vector from the PS shard and
pushes a delta back (``M/matrix/factorization/workers/PSOnlineMatrixFactorizationWorker.scala:41-55``).
On a node of fully connected GPUs with 288 GB each, the item table (1M x 64
fp32 = 256 MB) is tiny next to the rating stream, so instead of moving rows to
the ratings, the *item shards move to the ratings* (stratified SGD, Gemulla et
al. 2011): the PS shards travel between the GPUs while each worker updates only
the blocks it currently holds.

One ring (``_Ring``) of ``K = 2W`` blocks, two per rank at rest:

* in sub-step ``s`` rank ``r`` updates ring block ``(2r + s) % K`` (direction
  +1) or ``(2r + 1 - s) % K`` (direction -1); blocks of the other parity are idle
  and travel:
* during sub-step ``s >= 1`` rank ``r`` sends the block it finished in ``s-1`` to
  the neighbour that needs it next (``r - d``) and receives the block it needs
  in ``s+1`` from ``r + d`` -- the transfer hides behind the compute;
* one micro-batch = K sub-steps = every block once; the schedule is periodic,
  so consecutive micro-batches continue it without a barrier.

Schedules:

* ``"bidir"`` (default): each PS shard is split into two *virtual* hash shards
  (``i % 2W``: shard ``r`` and ``r + W`` of rank ``r``), giving two rings of
  quarter-shard blocks that rotate in OPPOSITE directions.  Every sub-step a
  rank updates one block of each ring (one launch, ``ops.mf_sgd_tiled_pair``)
  and each link direction to both ring neighbours carries a quarter-shard: per
  link direction and sub-step half the bytes of one ring, on both directions
  of two xGMI links instead of one direction of one link.
* ``"ring"``: one ring of half-shard blocks, direction +1.

Every item block is owned by exactly one GPU at any time and every user row by
its worker, so no parameter is ever updated concurrently by two GPUs and no
update is stale: the result equals a sequential schedule of the sub-steps
(serializable), unlike the bounded-staleness PS path.

``EmulatedRotation`` runs rank 0's schedule of an N-rank job on ONE GPU with
every block resident (no transfers): the per-GPU compute of an N-GPU step
(``bench/bench_emulate_world.py``).

``home()`` returns every block to its PS shard (``ShardedTable`` rows) for
evaluation, dumps and checkpoints.  ``wait_ms()`` is the time the compute stream
spent waiting for transfers (HIP events around each wait).
"""
from __future__ import annotations

from typing import List, Optional, Tuple

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


def layout_world(world: int, schedule: str) -> int:
    """Hash shards of the block layout the partitioners bucket by: ``2W`` virtual
    shards for the bidirectional schedule, ``W`` for the single ring."""
    return 2 * world if schedule == "bidir" else world


def _mark(stream=None) -> "torch.cuda.Event":
    """A timing event recorded on ``stream`` (default: the current stream)."""
    e = torch.cuda.Event(enable_timing=True)
    e.record(stream)
    return e


def _exposed_ms(events) -> float:
    """Exposed transfer time of ``(e0, e1, ec)`` records: ``e0`` / ``e1`` bracket the
    wait on the stream of the next sub-step, ``ec`` (or None) marks where the other
    compute stream stood (the previous sub-step, still running).  With one compute
    stream the exposure is the wait itself; with two, only the part of it after the
    other stream's sub-step ended left the GPU without a sub-step to run."""
    ms = 0.0
    for e0, e1, ec in events:
        d = e0.elapsed_time(e1)
        if ec is not None:
            d = min(d, ec.elapsed_time(e1))
        ms += max(0.0, d)
    return ms


class _Ring:
    """One ring of ``2W`` blocks (see the module docstring)."""

    def __init__(self, W: int, r: int, home: List[torch.Tensor], rows: List[int], direction: int, base: int,
                 like: torch.Tensor):
        self.W, self.r, self.K, self.d, self.base = W, r, 2 * W, direction, base
        self.home_v = home          # this rank's two ring blocks (2r, 2r+1) in the PS shard (views)
        self.rows = rows            # rows of every ring block
        cap = max(rows) if rows else 0
        self.buf = [torch.empty((cap, like.shape[1]), dtype=like.dtype, device=like.device) for _ in range(3)]
        self.s = 0
        self.A = self.P = self.F = self.N = None

    def order(self, s: int, r: Optional[int] = None) -> int:
        r = self.r if r is None else r
        return (2 * r + s) % self.K if self.d > 0 else (2 * r + 1 - s) % self.K

    def _home_of(self, j: int) -> torch.Tensor:
        return self.home_v[j - 2 * self.r]

    def leave_rest(self) -> None:
        o0, o1 = self.order(0), self.order(1)
        self.buf[0][: self.rows[o0]].copy_(self._home_of(o0))
        self.buf[1][: self.rows[o1]].copy_(self._home_of(o1))
        self.A, self.N, self.F, self.P = 0, 1, 2, None
        self.s = 0

    def transfers(self):
        """``(send, recv)`` of sub-step ``s`` (None when nothing moves)."""
        if self.W == 1 or self.P is None:
            return None
        out_b, in_b = self.order(self.s - 1), self.order(self.s + 1)
        return ((self.buf[self.P][: self.rows[out_b]], (self.r - self.d) % self.W),
                (self.buf[self.F][: self.rows[in_b]], (self.r + self.d) % self.W))

    def rotate(self) -> None:
        if self.W == 1:  # no peers: the two blocks alternate in place
            self.A, self.N = self.N, self.A
        elif self.P is None:
            self.A, self.P, self.F, self.N = self.N, self.A, self.F, None
        else:
            self.A, self.P, self.F = self.F, self.A, self.P
        self.s += 1

    def active(self) -> Tuple[int, torch.Tensor]:
        j = self.order(self.s)
        return self.base + j, self.buf[self.A][: self.rows[j]]

    def held(self) -> dict:
        """ring block -> buffer index of the blocks this rank holds now."""
        s = self.s
        if self.W == 1:
            return {self.order(s): self.A, self.order(s + 1): self.N}
        if self.P is None:
            return {self.order(0): self.A, self.order(1): self.N}
        return {self.order(s): self.A, self.order(s - 1): self.P}

    def holder(self, j: int) -> int:
        s = self.s
        for x in range(self.W):
            if self.P is None or self.W == 1:
                if j in (self.order(0, x), self.order(1, x)):
                    return x
            elif j in (self.order(s, x), self.order(s - 1, x)):
                return x
        raise AssertionError(f"no holder for ring block {j}")

    def home_ops(self):
        """``(sends, recvs, local copies)`` that return every block home."""
        sends, recvs, local = [], [], []
        held = self.held()
        for j, bi in sorted(held.items()):
            dst = j // 2
            if dst != self.r:
                sends.append((self.buf[bi][: self.rows[j]], dst))
            else:
                local.append((self._home_of(j), self.buf[bi][: self.rows[j]]))
        for j in (2 * self.r, 2 * self.r + 1):
            src = self.holder(j)
            if src != self.r:
                recvs.append((self._home_of(j), src))
        return sends, recvs, local


class RingRotation:
    """The rotation of one rank: one ring (``schedule="ring"``) or two
    counter-rotating rings (``"bidir"``) over its PS shard ``home``
    (``[n_local, D]``, hash layout ``i % W``)."""

    def __init__(self, comm: Comm, home: torch.Tensor, num_ids: int, schedule: str = "bidir"):
        if schedule not in ("bidir", "ring"):
            raise ValueError(f"rotation schedule must be 'bidir' or 'ring', not {schedule!r}")
        self.comm = comm
        self.W, self.r = comm.world, comm.rank
        self.schedule = schedule
        self.K = 2 * self.W  # sub-steps per micro-batch
        self.home_t = home
        W, r = self.W, self.r
        if schedule == "ring":
            hq = shard_halves(num_ids, W)[r]
            self.rings = [_Ring(W, r, [home[:hq], home[hq:]], block_rows(num_ids, W), +1, 0, home)]
        else:
            halves, rows = shard_halves(num_ids, 2 * W), block_rows(num_ids, 2 * W)
            v0, v1 = home[0::2], home[1::2]  # virtual shards r and r + W of this rank
            hl, hr = halves[r], halves[r + W]
            self.rings = [_Ring(W, r, [v0[:hl], v0[hl:]], rows[: 2 * W], +1, 0, home),
                          _Ring(W, r, [v1[:hr], v1[hr:]], rows[2 * W:], -1, 2 * W, home)]
        self.at_rest = True
        self.s = 0
        self._works: Optional[list] = None
        self._events: List[tuple] = []
        self._host_wait_s = 0.0
        self.bytes_sent = 0

    # --------------------------------------------------------------- schedule
    def active_blocks(self) -> List[Tuple[int, torch.Tensor]]:
        """``(block id in the partition layout, resident rows)`` updated this sub-step."""
        return [ring.active() for ring in self.rings]

    def begin(self):
        """Start a sub-step: issue the transfers that overlap its compute."""
        if self.at_rest:
            for ring in self.rings:
                ring.leave_rest()
            self.at_rest = False
            self.s = 0
        sends, recvs = [], []
        for ring in self.rings:  # every rank posts ring by ring: matched order per peer pair
            t = ring.transfers()
            if t is not None:
                sends.append(t[0])
                recvs.append(t[1])
        if sends:
            self._works = self.comm.p2p(sends, recvs)
            self.bytes_sent += sum(x.numel() * x.element_size() for x, _ in sends)

    def end(self, also=()):
        """Finish a sub-step (after its compute was enqueued) and rotate roles: the
        current stream -- the one that reads the arriving blocks -- waits for this
        sub-step's transfers, and so does every stream in ``also`` (with sub-steps on
        alternating streams, the stream that posts the next transfers: its receives
        reuse the buffers these sends read)."""
        if self._works:
            cuda = self.home_t.is_cuda
            if cuda:
                ec = _mark(also[0]) if also else None  # where the other compute stream is now
                e0 = _mark()
            else:
                import time

                t0 = time.perf_counter()
            for w in self._works:
                w.wait()
            if cuda:
                self._events.append((e0, _mark(), ec))
                for st in also:
                    with torch.cuda.stream(st):
                        for w in self._works:
                            w.wait()
            else:
                self._host_wait_s += time.perf_counter() - t0
        self._works = None
        for ring in self.rings:
            ring.rotate()
        self.s += 1

    def wait_ms(self, reset: bool = True) -> float:
        """Milliseconds the compute streams waited for transfers with nothing else to
        run, since the last call (synchronises on the recorded events)."""
        ms = self._host_wait_s * 1e3 + _exposed_ms(self._events)
        if reset:
            self._events, self._host_wait_s = [], 0.0
        return ms

    # --------------------------------------------------------------- homing
    def home(self):
        """Send every block back to its PS shard (between sub-steps)."""
        if self.at_rest:
            return
        sends, recvs, local = [], [], []
        for ring in self.rings:  # ring by ring, ascending block ids: same posting order on both sides
            s_, r_, l_ = ring.home_ops()
            sends += s_
            recvs += r_
            local += l_
        # NCCL receives need contiguous buffers; the bidir rings' home views are strided
        staged = [(torch.empty(v.shape, dtype=v.dtype, device=v.device), v, p) for v, p in recvs]
        works = self.comm.p2p(sends, [(t, p) for t, _, p in staged])
        for dst, src in local:
            dst.copy_(src)
        for w in works:
            w.wait()
        for t, v, _ in staged:
            v.copy_(t)
        self.at_rest = True
        self.s = 0


import os as _os

#: A/B switch of the emulated link model (``FPS_EMU_LINK=serial``: sleep for the link
#: time, then copy -- the round-5 model; default: one fill kernel lasting the link time)
_SERIAL_LINK = _os.environ.get("FPS_EMU_LINK", "") == "serial"


class _SymmetricLinks:
    """Device-timed xGMI links of the emulated rank (``EmulatedRotation(link_gbps=...)``).

    In a rotation every rank runs the same schedule on equal work, so the block a
    rank receives in sub-step ``s`` is posted by its neighbour when the neighbour's
    sub-step ``s - 1`` ends -- the moment this rank's own ``s - 1`` ends.  A posted
    transfer waits for that compute-stream event on a high-priority link stream, then
    ONE segment-fill kernel moves the bytes of the sub-step's blocks (the send's HBM
    read and the receive's HBM write of this GPU: every ring's block size, read from
    the first block) and lasts at least ``latency + bytes / link_gbps`` (the two rings'
    blocks travel on two different links, in parallel).  RCCL's point-to-point kernels write the receive buffer chunk
    by chunk as the data crosses the link, so the write overlaps the link time (round 5
    slept, then copied: on a GPU busy with the SGD the copies took 0.1-0.3 ms and sat on
    every sub-step's critical path, ``profiles/r6_link_model.md``).  Everything is enqueued at
    post time, so waiting on a transfer is a pure stream wait, as on RCCL (no host
    thread, no host block).  Only the emulated rank computes, at the full speed of its
    GPU: the measured wait is the exposure of the real schedule under rank symmetry,
    not the skew of N ranks sharing one GPU (``parallel/vworld.py``)."""

    def __init__(self, device, link_gbps: float, latency_us: float):
        from .vworld import _Sleep

        self._sleep = _Sleep
        self.us_per_byte = 1e-3 / float(link_gbps)  # GB/s -> us per byte
        self.latency_us = float(latency_us)
        self.device = device
        self.stream = torch.cuda.Stream(device=device, priority=-1)
        self._scratch = None

    def post(self, after: "torch.cuda.Event", copies, link_bytes: int) -> "torch.cuda.Event":
        """``copies``: ``(dst, src)`` of the blocks sent / received this sub-step; their
        bytes are moved by one kernel (rows of every block, read from the first: the
        same HBM traffic) into a scratch buffer that nothing reads."""
        from .. import ops

        us = self.latency_us + link_bytes * self.us_per_byte
        srcs = [src for _, src in copies if src.shape[0]]
        self.stream.wait_event(after)
        with torch.cuda.stream(self.stream):
            if srcs and _SERIAL_LINK:  # A/B (FPS_EMU_LINK=serial): the round-5 model, sleep then copy
                self._sleep.us(self.device, us)
                rows = [x.shape[0] for x in srcs]
                if self._scratch is None or self._scratch.shape[0] < sum(rows):
                    self._scratch = torch.empty((sum(rows),) + tuple(srcs[0].shape[1:]), dtype=srcs[0].dtype,
                                                device=srcs[0].device)
                off = 0
                for x in srcs:
                    self._scratch[off:off + x.shape[0]].copy_(x, non_blocking=True)
                    off += x.shape[0]
            elif srcs:
                rows = [x.shape[0] for x in srcs]
                src = srcs[0]
                if (self._scratch is None or self._scratch.shape[0] < sum(rows)
                        or self._scratch.shape[1:] != src.shape[1:] or self._scratch.dtype != src.dtype):
                    self._scratch = torch.empty((sum(rows),) + tuple(src.shape[1:]), dtype=src.dtype,
                                                device=src.device)
                ops.segment_fill(src.contiguous(), rows, self._scratch[:sum(rows)], min_us=us)
            else:
                self._sleep.us(self.device, us)
            done = torch.cuda.Event()
            done.record(self.stream)
        return done

    def wait(self, done: "torch.cuda.Event") -> None:
        torch.cuda.current_stream().wait_event(done)

    def close(self) -> None:
        pass


class EmulatedRotation:
    """Rank 0's rotation schedule of a ``world``-rank job on one device with every
    block resident: the same launches per sub-step as one GPU of the real job
    (``item`` = the whole ``[num_ids, D]`` table).  Without ``link_gbps`` nothing
    moves; with it every sub-step's transfers are modelled by ``_SymmetricLinks``
    (the real schedule's timing under rank symmetry) and ``wait_ms`` reports how long
    the compute stream waited for them."""

    def __init__(self, items: torch.Tensor, num_ids: int, world: int, schedule: str = "bidir",
                 link_gbps: Optional[float] = None, latency_us: float = 5.0):
        self.items, self.W, self.schedule = items, world, schedule
        self.Wv = layout_world(world, schedule)
        self.K = 2 * world
        self.halves = shard_halves(num_ids, self.Wv)
        self.rows = block_rows(num_ids, self.Wv)
        self.ids = []
        for g in range(2 * self.Wv):
            q, h = g // 2, g % 2
            n_local = (num_ids - q + self.Wv - 1) // self.Wv
            lo, hi = (0, self.halves[q]) if h == 0 else (self.halves[q], n_local)
            self.ids.append((q + self.Wv * torch.arange(lo, hi, device=items.device)).long())
        self.blocks = None
        self.at_rest = True
        self.s = 0
        self.bytes_sent = 0
        self.links = _SymmetricLinks(items.device, link_gbps, latency_us) \
            if link_gbps and items.is_cuda and world > 1 else None
        self._inflight = None
        self._events: List[tuple] = []

    def _ring_blocks(self, s: int) -> List[int]:
        W = self.W
        if self.schedule == "ring":
            return [s % (2 * W)]
        return [s % (2 * W), 2 * W + (1 - s) % (2 * W)]

    def active_blocks(self):
        return [(b, self.blocks[b]) for b in self._ring_blocks(self.s)]

    def begin(self):
        if self.at_rest:
            self.blocks = [self.items[ids].contiguous() for ids in self.ids]
            self.at_rest = False
            self.s = 0
        if self.links is not None and self.s >= 1:
            # sub-step s: each ring sends the block it finished in s - 1 and receives the
            # block it needs in s + 1 (posted when s - 1 ended, as the neighbour's is)
            after = torch.cuda.Event()
            after.record()
            copies, link_bytes = [], 0
            for out_b, in_b in zip(self._ring_blocks(self.s - 1), self._ring_blocks(self.s + 1)):
                n = min(self.blocks[out_b].shape[0], self.blocks[in_b].shape[0])
                copies.append((None, self.blocks[out_b][:n]))  # the link's scratch receives the bytes
                nbytes = self.blocks[in_b].numel() * self.blocks[in_b].element_size()
                link_bytes = max(link_bytes, nbytes)  # the rings use different links: in parallel
                self.bytes_sent += self.blocks[out_b].numel() * self.blocks[out_b].element_size()
            self._inflight = self.links.post(after, copies, link_bytes)

    def end(self, also=()):
        if self._inflight is not None:
            ec = _mark(also[0]) if also else None
            e0 = _mark()
            self.links.wait(self._inflight)
            self._events.append((e0, _mark(), ec))
            for st in also:
                st.wait_event(self._inflight)
            self._inflight = None
        self.s += 1

    def wait_ms(self, reset: bool = True) -> float:
        ms = _exposed_ms(self._events)
        if reset:
            self._events = []
        return ms

    def home(self):
        if self.at_rest:
            return
        for ids, blk in zip(self.ids, self.blocks):
            self.items[ids] = blk
        self.blocks = None
        self.at_rest = True
        self.s = 0

    def close(self) -> None:
        if self.links is not None:
            self.links.close()

"""Rank-symmetric emulation of an N-rank PS job on ONE GPU (per-GPU step at N).

In a weak-scaled PS job every rank runs the same code on statistically identical
data (its own micro-batch, keys spread uniformly over the N shards).  Under that
symmetry what rank 0 RECEIVES from peer j in an all-to-all has the size and the
key distribution of what it SENDS to peer j.  ``SymmetricComm`` therefore runs
rank 0 of an N-rank job with every collective answered by rank 0's own send
buffer -- the owner-side serve / apply then touches the same number of rows with
the same access pattern as on the real job (local keys ``key // N`` are valid rows
of every shard) -- while each all-to-all's transfer is modelled on the device:

* a posted exchange waits (on a high-priority link stream) for the posting
  stream's event, then ONE segment-fill kernel writes the receive buffer on the device
  and lasts at least ``latency + bytes to the busiest peer / link_gbps`` (a fully
  connected xGMI node: one link per peer, all in parallel): RCCL's kernels write the
  receive chunk by chunk as the data crosses the links, so a transfer completes at
  max(link time, write time).  (Round 5 slept, then copied: the write sat on the
  critical path after the link time.  A second stream for the write ran past the 4
  hardware queues a process gets and serialised unrelated streams,
  ``profiles/r6_link_model.md``.);
* ``Work.wait()`` is a stream wait, as on RCCL; ``wait_ms()`` reports the time the
  compute stream waited with nothing else to run.

Counts / flags / reductions are the symmetric ones (``exchange_counts`` returns
what was sent, ``sum_over_ranks(x) = N x``).

**Hot-owner mode** (``hot_owner=True``, the default of the benches since round 6).
Rank symmetry holds for the WORKER side (every rank's micro-batch is drawn from
the same distribution) but not for the OWNER side when keys are skewed: under
range partitioning of Zipf features, shard 0 receives 71 / 50 / 35 % of all
requests at N = 2 / 4 / 8.  The job then runs at the pace of the hottest owner,
so the emulated rank ``rank`` plays an OWNER as every peer sees it: peer j sends
shard s what this rank sends shard s (the worker-side symmetry), hence this rank
receives ``split[rank]`` rows from EVERY peer -- ``N x split[rank]`` rows to
serve / apply -- and its busiest incoming link carries ``split[rank]``.  Each
received segment is this rank's own self-segment (keys of its shard, valid rows),
tiled or cut to the expected size; a link's time is the larger of its outgoing
and incoming bytes (full-duplex links, one per peer).  The benches pick the
hottest shard as ``rank`` (``bench/bench_pa.py --emulate-rank``; range: shard 0)
and report every shard's share of the keys.  Values computed from the exchanged
rows are NOT those of a real job (rank 0 serves its own shard for every peer): the
emulation is for timing (``bench/bench_pa.py`` / ``bench_w2v.py --emulate-world``),
like ``rotation.EmulatedRotation`` is for the MF rotation.  Real multi-rank
correctness is ``parallel/vworld.py``'s and ``tests/test_multigpu_nccl_gpu.py``'s.
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence

import torch

from .comm import Comm


#: A/B switch of the link model (``FPS_EMU_LINK=serial``: sleep for the link time, then
#: write the receive -- the round-5 model; default: one fill kernel lasting the link time)
_SERIAL_LINK = os.environ.get("FPS_EMU_LINK", "") == "serial"


class _LinkWork:
    def __init__(self, comm: "SymmetricComm", done, e_post):
        self.comm, self.done, self.e_post = comm, done, e_post

    def wait(self) -> None:
        self.comm._wait(self.done)

    def is_completed(self) -> bool:
        return self.done is None or self.done.query()


class SymmetricComm(Comm):
    """Rank 0 of a ``world``-rank job under rank symmetry (module docstring)."""

    def __init__(self, world: int, device=None, link_gbps: float = 50.0, latency_us: float = 5.0,
                 hot_owner: bool = False, rank: int = 0):
        super().__init__(device=device, local=True)
        if world < 1:
            raise ValueError("world must be >= 1")
        if not 0 <= rank < world:
            raise ValueError(f"rank {rank} outside a world of {world}")
        self.world, self.rank, self.backend = int(world), int(rank), "emulated"
        #: owner-side model: every peer sends this rank what it sends itself (module docstring)
        self.hot_owner = bool(hot_owner)
        #: rows received over all all-to-alls (the owner-side load the model produced)
        self.recv_rows_total = 0
        self.peer_bytes = [0] * self.world
        self.link_gbps, self.latency_us = float(link_gbps), float(latency_us)
        self.cuda = self.device.type == "cuda"
        self._link = torch.cuda.Stream(device=self.device, priority=-1) if self.cuda else None
        #: exposed waits are those of this (compute) stream; an owner stream waiting for a
        #: transfer (``TensorPS.owner_stream``) idles no compute
        self._main = torch.cuda.current_stream(self.device) if self.cuda else None
        self._events: List[tuple] = []  # (wait start, wait end) events of every exposed wait
        #: time the compute stream's waits (two timing events per wait: ~1/10 of a PA
        #: micro-batch's host time, which a real RCCL job does not spend -- a bench can
        #: time its steps with this off and measure the waits in a pass of their own)
        self.time_waits = True
        self.transfers = 0

    # ------------------------------------------------------------- link model
    def _fill(self, send: torch.Tensor, out: torch.Tensor, send_splits: Sequence[int],
              recv_splits: Sequence[int], min_us: float = 0.0, stream=None) -> bool:
        """The received buffer: this rank's own send buffer (symmetric), or every
        incoming segment = this rank's self-segment tiled / cut (hot owner).  On the GPU
        one segment-fill kernel (on ``stream``, else the current one) that also lasts
        ``min_us`` (the link time); returns whether it did (else the caller models the
        link time itself)."""
        from .. import ops

        if not self.hot_owner:
            n = int(sum(send_splits))
            if n and send.is_cuda:
                ops.segment_fill(send[:n].contiguous(), [n], out[:n], min_us=min_us, stream=stream)
                return True
            self._on(stream, lambda: out[:n].copy_(send[:n], non_blocking=True))
            return False
        a = int(sum(send_splits[: self.rank]))
        own = send[a: a + int(send_splits[self.rank])]
        rs = [int(m) for m in recv_splits]
        n_out = sum(rs)
        # one kernel per exchange (the transfer model must not cost more device time than
        # the real receive): every peer sends the self-segment (requests / pushes), or a
        # prefix of it (answers)
        if own.shape[0] and n_out and own.is_cuda:
            ops.segment_fill(own.contiguous(), rs, out[:n_out], min_us=min_us, stream=stream)
            return True
        self._on(stream, lambda: self._fill_torch(send, own, out, rs))
        return False

    @staticmethod
    def _on(stream, fn) -> None:
        if stream is None:
            fn()
        else:
            with torch.cuda.stream(stream):
                fn()

    @staticmethod
    def _fill_torch(send: torch.Tensor, own: torch.Tensor, out: torch.Tensor, rs: List[int]) -> None:
        """The hot-owner receive with torch ops (CPU, or nothing of this rank's own to mirror)."""
        n_out, k = sum(rs), own.shape[0]
        if k and n_out and all(m == k for m in rs):
            out[:n_out].view((len(rs),) + tuple(own.shape)).copy_(own.unsqueeze(0).expand((len(rs),) + tuple(own.shape)))
            return
        if k and n_out:
            src = own if max(rs) <= k else torch.cat([own] * -(-max(rs) // k))
            torch.cat([src[:m] for m in rs], out=out[:n_out])
            return
        off = 0
        for m in rs:
            if m:  # nothing to mirror: any valid rows of the send buffer (zeros without any)
                if send.shape[0]:
                    done = 0
                    while done < m:
                        c = min(m - done, send.shape[0])
                        out[off + done: off + done + c].copy_(send[:c], non_blocking=True)
                        done += c
                else:
                    out[off: off + m].zero_()
            off += m

    def _post(self, send: torch.Tensor, out: torch.Tensor, send_splits: Sequence[int],
              recv_splits: Optional[Sequence[int]] = None) -> Optional[object]:
        """Model one all-to-all: latency + busiest link's bytes / link rate, then the
        receive's device copy; returns the completion event (None on the CPU)."""
        if recv_splits is None:
            recv_splits = send_splits
        row_bytes = send.element_size() * (send[0].numel() if send.dim() > 1 and send.shape[0] else 1)
        peer = [int(n) * row_bytes for j, n in enumerate(send_splits) if j != self.rank]
        if self.hot_owner:  # full-duplex links: the busier direction of each
            peer += [int(n) * row_bytes for j, n in enumerate(recv_splits) if j != self.rank]
        self._count(send, send_splits)
        self.recv_rows_total += int(sum(recv_splits))
        if not self.cuda:
            self._fill(send, out, send_splits, recv_splits)
            return None
        from .vworld import _Sleep

        us = (self.latency_us + (max(peer) if peer else 0) * 1e-3 / self.link_gbps) if self.world > 1 else 0.0
        link = self._link
        ready = torch.cuda.Event()  # the send is ready in post order
        ready.record(torch.cuda.current_stream(self.device))
        link.wait_event(ready)
        if _SERIAL_LINK:  # A/B (FPS_EMU_LINK=serial): the round-5 model, sleep then write
            with torch.cuda.stream(link):
                _Sleep.us(self.device, us)
            self._fill(send, out, send_splits, recv_splits, stream=link)
        elif not self._fill(send, out, send_splits, recv_splits, min_us=us, stream=link):  # the write, during the link
            with torch.cuda.stream(link):
                _Sleep.us(self.device, us)
        done = torch.cuda.Event()
        done.record(link)
        send.record_stream(link)
        out.record_stream(link)
        self.transfers += 1
        return done

    def _wait(self, done) -> None:
        if done is None:
            return
        cur = torch.cuda.current_stream(self.device)
        if not self.time_waits or cur != self._main:
            cur.wait_event(done)
            return
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record(cur)
        cur.wait_event(done)
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record(cur)
        self._events.append((e0, e1))

    def wait_ms(self, reset: bool = True) -> float:
        """Milliseconds the waiting streams spent blocked on modelled transfers."""
        ms = sum(max(0.0, a.elapsed_time(b)) for a, b in self._events)
        if reset:
            self._events = []
        return ms

    # ------------------------------------------------------------- collectives
    def barrier(self):
        pass

    def exchange_counts_async(self, send_counts: torch.Tensor):
        return self.exchange_counts(send_counts), None

    def exchange_counts(self, send_counts: torch.Tensor) -> torch.Tensor:
        if self.hot_owner:  # every peer sends this rank what it sends itself
            return send_counts[self.rank: self.rank + 1].expand_as(send_counts).clone()
        return send_counts.clone()

    def all_to_all(self, send: torch.Tensor, send_splits: Sequence[int], recv_splits: Sequence[int],
                   out: Optional[torch.Tensor] = None) -> torch.Tensor:
        n_out = int(sum(recv_splits))
        if out is None:
            out = torch.empty((n_out,) + tuple(send.shape[1:]), dtype=send.dtype, device=send.device)
        self._wait(self._post(send, out, send_splits, recv_splits))
        return out

    def all_to_all_async(self, send: torch.Tensor, send_splits: Sequence[int], recv_splits: Sequence[int]):
        n_out = int(sum(recv_splits))
        out = torch.empty((n_out,) + tuple(send.shape[1:]), dtype=send.dtype, device=send.device)
        return out, _LinkWork(self, self._post(send, out, send_splits, recv_splits), None)

    def all_reduce(self, t: torch.Tensor, op=None) -> torch.Tensor:
        import torch.distributed as dist

        if op is None or op == dist.ReduceOp.SUM:
            t.mul_(self.world)
        return t  # MAX / MIN of equal values

    def all_gather(self, t: torch.Tensor) -> List[torch.Tensor]:
        return [t for _ in range(self.world)]

    def p2p(self, sends: Sequence, recvs: Sequence) -> list:
        raise NotImplementedError("SymmetricComm models all-to-alls; the rotation has rotation.EmulatedRotation")

    def max_over_ranks(self, x: float) -> float:
        return x

    def gather_floats(self, x: float) -> List[float]:
        return [float(x)] * self.world

    def sum_over_ranks(self, x: float) -> float:
        return x * self.world


def shard_shares(keys: torch.Tensor, partitioner, unique: bool = True) -> List[float]:
    """Each shard's share of ``keys`` (de-duplicated first, as a micro-batch's pull plan
    does) under ``partitioner`` (``core.partitioners``): the owner-side load split."""
    k = keys.reshape(-1).to(torch.int64)
    if unique:
        k = torch.unique(k)
    sh = partitioner.shard_tensor(k).to(torch.int64)
    c = torch.bincount(sh.cpu(), minlength=partitioner.n).double()
    tot = float(c.sum()) or 1.0
    return [float(x) / tot for x in c]


def hottest_shard(keys: torch.Tensor, partitioner) -> int:
    """The shard receiving the most de-duplicated keys: the owner a job waits for."""
    sh = shard_shares(keys, partitioner)
    return max(range(len(sh)), key=lambda j: sh[j])

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
  stream's event, spends ``latency + bytes to the busiest peer / link_gbps`` in a
  one-wave device sleep (a fully connected xGMI node: one link per peer, all in
  parallel), then copies the buffer on the device (the receive's HBM write);
* ``Work.wait()`` is a stream wait, as on RCCL; ``wait_ms()`` reports the time the
  compute stream waited with nothing else to run.

Counts / flags / reductions are the symmetric ones (``exchange_counts`` returns
what was sent, ``sum_over_ranks(x) = N x``).  Values computed from the exchanged
rows are NOT those of a real job (rank 0 serves its own shard for every peer): the
emulation is for timing (``bench/bench_pa.py`` / ``bench_w2v.py --emulate-world``),
like ``rotation.EmulatedRotation`` is for the MF rotation.  Real multi-rank
correctness is ``parallel/vworld.py``'s and ``tests/test_multigpu_nccl_gpu.py``'s.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch

from .comm import Comm


class _LinkWork:
    def __init__(self, comm: "SymmetricComm", done, e_post):
        self.comm, self.done, self.e_post = comm, done, e_post

    def wait(self) -> None:
        self.comm._wait(self.done)

    def is_completed(self) -> bool:
        return self.done is None or self.done.query()


class SymmetricComm(Comm):
    """Rank 0 of a ``world``-rank job under rank symmetry (module docstring)."""

    def __init__(self, world: int, device=None, link_gbps: float = 50.0, latency_us: float = 5.0):
        super().__init__(device=device, local=True)
        if world < 1:
            raise ValueError("world must be >= 1")
        self.world, self.rank, self.backend = int(world), 0, "emulated"
        self.peer_bytes = [0] * self.world
        self.link_gbps, self.latency_us = float(link_gbps), float(latency_us)
        self.cuda = self.device.type == "cuda"
        self._link = torch.cuda.Stream(device=self.device, priority=-1) if self.cuda else None
        self._events: List[tuple] = []  # (wait start, wait end) events of every exposed wait
        self.transfers = 0

    # ------------------------------------------------------------- link model
    def _post(self, send: torch.Tensor, out: torch.Tensor, send_splits: Sequence[int]) -> Optional[object]:
        """Model one all-to-all: latency + busiest peer's bytes / link rate, then the
        receive's device copy; returns the completion event (None on the CPU)."""
        row_bytes = send.element_size() * (send[0].numel() if send.dim() > 1 and send.shape[0] else 1)
        peer = [int(n) * row_bytes for j, n in enumerate(send_splits) if j != self.rank]
        self._count(send, send_splits)
        n = int(sum(send_splits))
        if not self.cuda:
            out[:n].copy_(send[:n])
            return None
        from .vworld import _Sleep

        us = (self.latency_us + (max(peer) if peer else 0) * 1e-3 / self.link_gbps) if self.world > 1 else 0.0
        posted = torch.cuda.Event()
        posted.record()
        self._link.wait_event(posted)
        with torch.cuda.stream(self._link):
            _Sleep.us(self.device, us)
            out[:n].copy_(send[:n], non_blocking=True)
            done = torch.cuda.Event()
            done.record(self._link)
        send.record_stream(self._link)
        out.record_stream(self._link)
        self.transfers += 1
        return done

    def _wait(self, done) -> None:
        if done is None:
            return
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
        torch.cuda.current_stream(self.device).wait_event(done)
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
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

    def exchange_counts(self, send_counts: torch.Tensor) -> torch.Tensor:
        return send_counts.clone()

    def all_to_all(self, send: torch.Tensor, send_splits: Sequence[int], recv_splits: Sequence[int],
                   out: Optional[torch.Tensor] = None) -> torch.Tensor:
        n_out = int(sum(recv_splits))
        if out is None:
            out = torch.empty((n_out,) + tuple(send.shape[1:]), dtype=send.dtype, device=send.device)
        self._wait(self._post(send, out, send_splits))
        return out

    def all_to_all_async(self, send: torch.Tensor, send_splits: Sequence[int], recv_splits: Sequence[int]):
        n_out = int(sum(recv_splits))
        out = torch.empty((n_out,) + tuple(send.shape[1:]), dtype=send.dtype, device=send.device)
        return out, _LinkWork(self, self._post(send, out, send_splits), None)

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

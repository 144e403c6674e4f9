"""Process-group plumbing of the tensor engine.

One process per GPU; ``torch.distributed`` with the ``nccl`` backend, which
on ROCm *is* RCCL over xGMI.  The PS traffic is any-worker -> any-shard, so
the primitive is the variable-split all-to-all (``all_to_all_single``): on a
fully connected 8-GPU xGMI mesh every rank pair has its own link and an
all-to-all drives all 7 links of a GPU at once, where a ring collective
would be bound by one link.  Three all-to-all phases per micro-batch:

  X1  keys   worker -> owner shard    (int32, deduplicated per step)
  X2  rows   owner -> worker          (same splits reversed; keys implicit
                                       because answers come back in request
                                       order -- the reference's FIFO property)
  X1' deltas worker -> owner shard    (fp32 or bf16 rows, pre-reduced per key)

Gloo provides the same calls on CPU (multi-process tests).  With gloo and
GPU tensors (several ranks sharing one GPU: the full device compute path with
a host transport -- rehearsal of the multi-GPU code on a one-GPU box) every
exchange is staged through host memory.  ``world == 1`` short-circuits every
exchange to a local copy.
"""
from __future__ import annotations

import datetime
import os
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist


class Comm:
    def __init__(self, group=None, device=None, local: bool = False):
        """``local``: a world of one even inside a process group (side computations)."""
        self.group = group
        if not local and dist.is_available() and dist.is_initialized():
            self.rank = dist.get_rank(group)
            self.world = dist.get_world_size(group)
            self.backend = dist.get_backend(group)
        else:
            self.rank, self.world, self.backend = 0, 1, "local"
        if device is None:
            if torch.cuda.is_available():
                device = torch.device("cuda", torch.cuda.current_device())
            else:
                device = torch.device("cpu")
        self.device = torch.device(device)
        self.bytes_sent = 0
        #: run the all-to-alls through the process group even at world 1 (a one-rank
        #: RCCL group on a one-GPU box: exercises captured RCCL collectives in tests)
        self.loopback = False
        #: bytes this rank put on the wire to each peer (all-to-alls + point-to-point)
        self.peer_bytes = [0] * self.world

    # ------------------------------------------------------------- set-up
    @staticmethod
    def init_from_env(backend: Optional[str] = None, timeout_s: Optional[float] = None) -> "Comm":
        """Initialise the default group from torchrun env vars (or world=1).
        ``timeout_s`` (default ``FPS_PG_TIMEOUT_S`` or 600): collective timeout;
        pair with ``utils.watchdog.Watchdog`` to fail faster than that."""
        if timeout_s is None:
            timeout_s = float(os.environ.get("FPS_PG_TIMEOUT_S", "600"))
        world = int(os.environ.get("WORLD_SIZE", "1"))
        rank = int(os.environ.get("RANK", "0"))
        local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        use_gpu = torch.cuda.is_available()
        # rehearsal of the multi-GPU launch on a one-GPU box: FPS_SHARE_GPU=1 puts
        # every rank on cuda:0 and defaults the backend to gloo (host-staged)
        share = os.environ.get("FPS_SHARE_GPU", "0") == "1"
        backend = backend or os.environ.get("FPS_DIST_BACKEND") or ("gloo" if share else None)
        if use_gpu:
            dev_index = 0 if share else local_rank
            torch.cuda.set_device(dev_index)
            device = torch.device("cuda", dev_index)
        else:
            device = torch.device("cpu")
        if world > 1 and not dist.is_initialized():
            backend = backend or ("nccl" if use_gpu else "gloo")
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            kw = dict(backend=backend, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
            if backend == "nccl":
                kw["device_id"] = device
            dist.init_process_group(**kw)
        return Comm(device=device)

    # ------------------------------------------------------------- staging
    def _staged(self, t: torch.Tensor) -> bool:
        """gloo cannot move device tensors: stage them through host memory."""
        return self.backend == "gloo" and t.is_cuda

    # ------------------------------------------------------------- collectives
    def barrier(self):
        if self.world > 1:
            if self.backend == "nccl":
                dist.barrier(group=self.group, device_ids=[self.device.index])
            else:
                dist.barrier(group=self.group)

    def exchange_counts(self, send_counts: torch.Tensor) -> torch.Tensor:
        """Every rank tells every other how many rows it will send it."""
        if self.world == 1:
            return send_counts.clone()
        if self._staged(send_counts):
            return self.exchange_counts(send_counts.cpu()).to(send_counts.device)
        recv = torch.empty_like(send_counts)
        dist.all_to_all_single(recv, send_counts, group=self.group)
        return recv

    def exchange_counts_async(self, send_counts: torch.Tensor):
        """``exchange_counts`` without blocking the caller's stream: ``(recv, work)``;
        ``work.wait()`` (None: already complete) orders a stream after the exchange.  A
        synchronous exchange would make the compute stream wait for every transfer
        queued on the communicator before it (one RCCL stream per rank)."""
        if self.world == 1 or self._staged(send_counts):
            return self.exchange_counts(send_counts), None
        recv = torch.empty_like(send_counts)
        work = dist.all_to_all_single(recv, send_counts, group=self.group, async_op=True)
        return recv, work

    def all_to_all(self, send: torch.Tensor, send_splits: Sequence[int], recv_splits: Sequence[int],
                   out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Variable-split all-to-all along dim 0 (rows of any trailing shape)."""
        n_out = int(sum(recv_splits))
        if self.world == 1 and not self.loopback:
            if out is None:  # nothing leaves the rank: hand the buffer through
                return send[:n_out]
            out[:n_out].copy_(send[:n_out])
            return out
        if out is None:
            out = torch.empty((n_out,) + tuple(send.shape[1:]), dtype=send.dtype, device=send.device)
        self._count(send, send_splits)
        if self._staged(send):
            host_out = torch.empty((n_out,) + tuple(send.shape[1:]), dtype=send.dtype)
            dist.all_to_all_single(host_out, send[: int(sum(send_splits))].cpu(), list(map(int, recv_splits)),
                                   list(map(int, send_splits)), group=self.group)
            out[:n_out].copy_(host_out)
            return out
        dist.all_to_all_single(out[:n_out], send[: int(sum(send_splits))], list(map(int, recv_splits)),
                               list(map(int, send_splits)), group=self.group)
        return out

    def all_to_all_async(self, send: torch.Tensor, send_splits: Sequence[int], recv_splits: Sequence[int]):
        """Non-blocking all-to-all: returns ``(out, work)``; ``work.wait()`` orders the
        caller's stream after the transfer (no host block).  ``work`` is None at world 1."""
        n_out = int(sum(recv_splits))
        if self.world == 1 and not self.loopback:
            return send[:n_out], None
        if self._staged(send):  # host-staged transport is synchronous
            return self.all_to_all(send, send_splits, recv_splits), None
        out = torch.empty((n_out,) + tuple(send.shape[1:]), dtype=send.dtype, device=send.device)
        self._count(send, send_splits)
        work = dist.all_to_all_single(out, send[: int(sum(send_splits))], list(map(int, recv_splits)),
                                      list(map(int, send_splits)), group=self.group, async_op=True)
        return out, work

    def _count(self, send: torch.Tensor, send_splits: Sequence[int]) -> None:
        row_bytes = send.element_size() * (send[0].numel() if send.dim() > 1 and send.shape[0] else 1)
        for j, n in enumerate(send_splits):
            if j != self.rank and n:
                self.peer_bytes[j] += int(n) * row_bytes
                self.bytes_sent += int(n) * row_bytes

    def all_reduce(self, t: torch.Tensor, op=None) -> torch.Tensor:
        if self.world > 1:
            if self._staged(t):
                h = t.cpu()
                dist.all_reduce(h, op=op or dist.ReduceOp.SUM, group=self.group)
                t.copy_(h)
            else:
                dist.all_reduce(t, op=op or dist.ReduceOp.SUM, group=self.group)
        return t

    def all_gather(self, t: torch.Tensor) -> List[torch.Tensor]:
        if self.world == 1:
            return [t]
        if self._staged(t):
            return [x.to(t.device) for x in self.all_gather(t.cpu())]
        outs = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(outs, t, group=self.group)
        return outs

    def p2p(self, sends: Sequence, recvs: Sequence) -> list:
        """Batched point-to-point: ``sends`` / ``recvs`` are ``(tensor, peer)`` pairs,
        posted as one group (no ordering deadlock between pairs of ranks).  Returns
        the works to wait on (empty when the transfer already completed: staged)."""
        for t, peer in sends:
            self.peer_bytes[peer] += t.numel() * t.element_size()
        if self.backend == "gloo" and any(t.is_cuda for t, _ in list(sends) + list(recvs)):
            host_recvs = [(torch.empty(t.shape, dtype=t.dtype), peer) for t, peer in recvs]
            ops = [dist.P2POp(dist.isend, t.cpu(), peer, group=self.group) for t, peer in sends]
            ops += [dist.P2POp(dist.irecv, h, peer, group=self.group) for h, peer in host_recvs]
            for w in (dist.batch_isend_irecv(ops) if ops else []):
                w.wait()
            for (t, _), (h, _) in zip(recvs, host_recvs):
                t.copy_(h)
            return []
        ops = [dist.P2POp(dist.isend, t, peer, group=self.group) for t, peer in sends]
        ops += [dist.P2POp(dist.irecv, t, peer, group=self.group) for t, peer in recvs]
        return dist.batch_isend_irecv(ops) if ops else []

    def max_over_ranks(self, x: float) -> float:
        if self.world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=self.device if self.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return float(t.item())

    def gather_floats(self, x: float) -> List[float]:
        """``[x of rank 0, x of rank 1, ...]`` on every rank."""
        if self.world == 1:
            return [float(x)]
        t = torch.tensor([x], dtype=torch.float64, device=self.device if self.backend == "nccl" else "cpu")
        return [float(v.item()) for v in self.all_gather(t)]

    def sum_over_ranks(self, x: float) -> float:
        if self.world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=self.device if self.backend == "nccl" else "cpu")
        dist.all_reduce(t, group=self.group)
        return float(t.item())

    def shutdown(self) -> None:
        """End of a job: every rank reaches a barrier, then the default process group
        is destroyed.  A rank that leaves while a peer still holds the group open
        tears the backend down under it (gloo aborted a rank with
        ``terminate called without an active exception`` at interpreter exit)."""
        if self.world > 1 and dist.is_initialized():
            self.barrier()
            dist.destroy_process_group()

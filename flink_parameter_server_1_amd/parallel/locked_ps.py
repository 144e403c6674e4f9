"""Device-mode LockPSLogic: exclusive read-modify-write of parameters across workers.

The reference's ``LockPSLogicA`` / ``LockPSLogicB`` (``M/server/LockPSLogicA.scala``,
``M/server/LockPSLogicB.scala``) lock a parameter on pull: the puller holds it
until it pushes, later pullers wait in a FIFO queue and get the *updated*
value (B additionally merges duplicate requests of one worker).  That turns
asynchronous pull/push into a per-parameter critical section.

Tensor form, one micro-batch of keys per worker per round:

``acquire(keys)``
    dedup per worker (B's merge), key all-to-all, then on every shard a lock
    table ``lock[row] = worker or -1`` is claimed segment by segment in rank
    order (``ops.lock_acquire``): the lowest requesting rank wins a contended
    row, a worker keeps rows it already holds.  Rows and grant flags go back.
``release(pull, values, mode)``
    the worker sends its new values (``set``) or deltas (``add``) for its
    unique keys; the shard applies only granted rows (denied rows are padding)
    and frees their locks.

A denied worker retries its key in a later round and then reads the value the
winner wrote -- the reference's queue, with rounds in place of FIFO
callbacks.  Both calls are collective over the workers.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from .. import ops
from .comm import Comm
from .table import ShardedTable
from .tensor_ps import PullPlan, TensorPS


@dataclass
class LockedPull:
    plan: PullPlan
    rows: torch.Tensor            # [U, D] values of this worker's unique keys (wire dtype)
    granted: torch.Tensor         # [U] bool: this worker holds the lock
    granted_recv: torch.Tensor    # shard side: grant flag per received key (uint8)

    def request_rows(self) -> torch.Tensor:
        return self.rows.float()[self.plan.pos.long()]

    def request_granted(self) -> torch.Tensor:
        return self.granted[self.plan.pos.long()]


class LockedTensorPS:
    def __init__(self, table: ShardedTable, comm: Comm, wire_dtype=torch.float32, ps: TensorPS = None):
        self.table, self.comm = table, comm
        self.ps = ps if ps is not None else TensorPS(table, comm, wire_dtype)
        self.lock = torch.full((table.n_local,), -1, dtype=torch.int32, device=table.device)

    def acquire(self, keys: torch.Tensor, flag: int = 0) -> LockedPull:
        """``flag`` reaches every peer with the counts (``plan.peer_flags``)."""
        plan = self.ps.plan(keys, flag=flag)
        n = plan.recv_keys.numel()
        granted_recv = torch.zeros(n, dtype=torch.uint8, device=self.table.device)
        off = 0
        for src, cnt in enumerate(plan.recv_splits):  # rank order: lowest rank wins a contended row
            if cnt:
                granted_recv[off:off + cnt] = ops.lock_acquire(self.lock, plan.recv_keys[off:off + cnt], src)
            off += cnt
        served = self.table.serve(plan.recv_keys, self.ps.wire_dtype)
        rows = self.comm.all_to_all(served, plan.recv_splits, plan.send_splits)
        granted = self.comm.all_to_all(granted_recv, plan.recv_splits, plan.send_splits)
        return LockedPull(plan, rows, granted[: plan.n_unique].bool(), granted_recv)

    def release(self, pull: LockedPull, values: torch.Tensor, mode: str = "set") -> None:
        """``values``: [U, D] per unique key of this worker (ignored where not granted)."""
        if mode not in ("set", "add"):
            raise ValueError(mode)
        plan = pull.plan
        wire = values.to(self.ps.wire_dtype).contiguous()
        recv = self.comm.all_to_all(wire, plan.send_splits, plan.recv_splits)
        # granted rows are exclusive across sources, so a plain set / RMW is safe
        idx = torch.where(pull.granted_recv.bool(), plan.recv_keys, torch.full_like(plan.recv_keys, -1))
        self.table.apply(idx, recv, op="set" if mode == "set" else "add_unique")
        ops.lock_release(self.lock, plan.recv_keys, pull.granted_recv)

    def held(self) -> int:
        """Locks currently held on this shard (0 between rounds)."""
        return int((self.lock >= 0).sum())

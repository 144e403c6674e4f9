"""The tensor-path parameter server: batched pull / push over RCCL all-to-all.

Replaces the reference's per-record Flink iteration
(``M/FlinkParameterServer.scala:215-335``) with a micro-batch protocol:

``pull(keys)``
    1. de-duplicate the batch's keys and group them by owning shard (K1,
       ``ops.DedupWorkspace``) -- the batch's own pre-reduction, the GPU
       analogue of the combining senders (``M/common/CombinationLogic.scala``);
    2. exchange per-shard counts (tiny all-to-all) and bring them to the host
       (the only host sync of a step: torch needs split sizes on the host);
    3. X1: all-to-all of the unique local keys to their owners;
    4. owners gather their rows (K2) into the wire dtype;
    5. X2: all-to-all of the rows back.  Rows return in request order, so
       ``rows[pos[b]]`` is request ``b``'s parameter (positional FIFO).
``push(plan, deltas)``
    6. X1': all-to-all of per-unique-key deltas (pre-reduced on the worker by
       the compute kernel's atomics) to the owners;
    7. owners apply them (K3: add / sgd / adagrad).

``world == 1`` keeps the same code path with local copies instead of RCCL.
Staleness: every request in a micro-batch reads the table as of step 3-4;
``push`` of step k may overlap ``pull`` of step k+1 (``max_inflight``), the
bounded-staleness analogue of ``pullLimit`` (``M/WorkerLogic.scala:176-225``).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List

import torch

from .. import ops
from ..utils.tracing import trace_range
from .comm import Comm
from .table import ShardedTable


@dataclass
class PullPlan:
    send_splits: List[int]   # unique keys this worker sends to each shard
    recv_splits: List[int]   # keys each worker sends to this shard
    recv_keys: torch.Tensor  # local keys this shard must serve / apply
    pos: torch.Tensor        # request -> row of the pulled/delta buffers
    n_unique: int


class TensorPS:
    def __init__(self, table: ShardedTable, comm: Comm, wire_dtype=torch.float32):
        self.table = table
        self.comm = comm
        self.wire_dtype = wire_dtype
        self.dedup = ops.DedupWorkspace(table.key_space, comm.world, table.part_kind, table.block, table.device)
        self.stats = {"pulls": 0, "unique": 0, "steps": 0}

    def plan(self, keys: torch.Tensor, persistent: bool = False) -> PullPlan:
        """Dedup + split exchange + key all-to-all.  ``persistent`` copies the
        request->row map out of the reusable dedup workspace, so the plan
        survives the next ``plan`` call (pipelined steps)."""
        keys = self.table.route_keys(keys.to(device=self.table.device)).to(torch.int32).contiguous()
        with trace_range("ps.dedup"):
            counts, prefix, uniq, pos = self.dedup.run(keys)
        recv_counts = self.comm.exchange_counts(counts)
        both = torch.cat([counts, recv_counts]).cpu().tolist()  # host sync (split sizes)
        W = self.comm.world
        send_splits, recv_splits = both[:W], both[W:]
        n_unique = int(sum(send_splits))
        recv_keys = self.comm.all_to_all(uniq[:n_unique], send_splits, recv_splits)
        if persistent:
            pos = pos.clone()
            if W == 1:
                recv_keys = recv_keys.clone()
        self.stats["pulls"] += keys.numel()
        self.stats["unique"] += n_unique
        self.stats["steps"] += 1
        return PullPlan(send_splits, recv_splits, recv_keys, pos, n_unique)

    def pull(self, keys: torch.Tensor):
        """Returns ``(rows[U, D] in wire dtype, plan)``; request b's row is ``rows[plan.pos[b]]``."""
        plan = self.plan(keys)
        with trace_range("ps.serve"):
            served = self.table.serve(plan.recv_keys, self.wire_dtype)
        with trace_range("ps.answer-a2a"):
            rows = self.comm.all_to_all(served, plan.recv_splits, plan.send_splits)
        return rows, plan

    def pull_async(self, keys: torch.Tensor):
        """Start a pull whose row all-to-all runs on the communicator's stream while
        the caller keeps computing; returns ``(rows, work, plan)`` -- wait on
        ``work`` (if not None) before reading ``rows``."""
        plan = self.plan(keys, persistent=True)
        served = self.table.serve(plan.recv_keys, self.wire_dtype)
        rows, work = self.comm.all_to_all_async(served, plan.recv_splits, plan.send_splits)
        return rows, work, plan

    def push(self, plan: PullPlan, deltas: torch.Tensor, lr: float = 0.0):
        """Send per-unique-key deltas ``[U, D]`` (fp32) to their owners and apply."""
        wire = deltas if deltas.dtype == self.wire_dtype else deltas.to(self.wire_dtype)
        with trace_range("ps.push-a2a"):
            recv = self.comm.all_to_all(wire, plan.send_splits, plan.recv_splits)
        opt = self.table.optimizer
        seg_add = opt == "add" and len(plan.recv_splits) <= 16
        if seg_add or opt in ("adagrad", "set"):
            # Keys are unique within each source's segment but may repeat across
            # sources; non-atomic rules (adagrad's accumulator RMW, set) must
            # therefore apply segment by segment.  ``add`` does the same with a
            # plain read-modify-write (add_unique) instead of one float atomic per
            # element (the atomic apply ran at ~1 TB/s: 480 us for 2M dim-64
            # rows, profiles/r1_capacity_kernel_stats.csv; narrow rows are worse).
            off = 0
            for n in plan.recv_splits:
                if n:
                    self.table.apply(plan.recv_keys[off:off + n], recv[off:off + n], lr=lr,
                                     op="add_unique" if seg_add else None)
                off += n
        else:
            self.table.apply(plan.recv_keys, recv, lr=lr)

    def pull_values(self, keys: torch.Tensor) -> torch.Tensor:
        """Convenience: fp32 ``[B, D]`` values for every request (expanded)."""
        rows, plan = self.pull(keys)
        return rows.float()[plan.pos.long()]

"""Multi-process runtime of the per-record engine over ``torch.distributed``.

One process per rank (``torchrun``); rank ``r`` hosts worker subtasks
``w % world == r`` and PS subtasks ``p % world == r`` -- the analogue of Flink
task slots spread over TaskManagers.  Each round a rank

1. runs its local subtasks until they are idle (or a message budget is hit);
   messages to subtasks on this rank are delivered directly, messages to
   other ranks go to a per-destination outbox;
2. exchanges outboxes with every rank: one all-to-all of message counts, then
   one all-to-all of the pickled payloads (gloo, CPU byte tensors).  Messages
   are appended in source order, so every (sender, receiver) channel stays
   FIFO -- the ordering the reference's workers rely on;
3. all-reduces its "busy" flag; a round in which no rank sent anything and
   every rank was idle is global quiescence -> every subtask is closed.

Outputs of all ranks are gathered (``all_gather_object``) so every rank
returns the same stream, in rank order.  Used for the CPU multi-rank tests
(gloo, world 2-4) and to run compat-path jobs across GPU hosts.
"""
from __future__ import annotations

import pickle
import time
from typing import Optional

import torch
import torch.distributed as dist

from .engine import LocalRuntime, split_input


class DistRuntime(LocalRuntime):
    #: messages handled locally between two exchanges (per subtask, per pass)
    passes_per_round = 8

    def __init__(self, group=None, iteration_wait_time: Optional[float] = None, output_sink=None,
                 gather_outputs: bool = True):
        super().__init__(iteration_wait_time, output_sink)
        if not dist.is_initialized():
            raise RuntimeError("DistRuntime needs an initialised torch.distributed process group")
        self.group = group
        if group is None and dist.get_backend() != "gloo":
            # payloads are host byte tensors: use a gloo side group on GPU jobs
            self.group = dist.new_group(backend="gloo")
        self.rank = dist.get_rank()
        self.world = dist.get_world_size()
        self.gather_outputs = gather_outputs
        self.rounds = 0

    # ------------------------------------------------------------ routing
    def _owner(self, subtask: int) -> int:
        return subtask % self.world

    def route_to_ps(self, msg):
        p = self.ps_index(msg)
        r = self._owner(p)
        if r == self.rank:
            self.servers[p].inbox.append(msg)
        else:
            self.outbox[r].append(("ps", p, msg))

    def route_to_worker(self, msg):
        w = self.worker_index(msg)
        r = self._owner(w)
        if r == self.rank:
            self.workers[w].answers.append(msg)
        else:
            self.outbox[r].append(("w", w, msg))

    # ------------------------------------------------------------ exchange
    def _exchange(self) -> int:
        payloads = [pickle.dumps(self.outbox[r], protocol=pickle.HIGHEST_PROTOCOL) if self.outbox[r] else b""
                    for r in range(self.world)]
        sent = sum(len(self.outbox[r]) for r in range(self.world))
        for r in range(self.world):
            self.outbox[r] = []
        send_sizes = torch.tensor([len(p) for p in payloads], dtype=torch.int64)
        recv_sizes = torch.empty_like(send_sizes)
        dist.all_to_all_single(recv_sizes, send_sizes, group=self.group)
        send = torch.frombuffer(bytearray(b"".join(payloads)), dtype=torch.uint8) if sum(map(len, payloads)) else \
            torch.empty(0, dtype=torch.uint8)
        recv = torch.empty(int(recv_sizes.sum()), dtype=torch.uint8)
        dist.all_to_all_single(recv, send, recv_sizes.tolist(), send_sizes.tolist(), group=self.group)
        buf = recv.numpy().tobytes()
        off = 0
        for r, n in enumerate(recv_sizes.tolist()):
            if n:
                for kind, idx, msg in pickle.loads(buf[off:off + n]):
                    if kind == "ps":
                        self.servers[idx].inbox.append(msg)
                    else:
                        self.workers[idx].answers.append(msg)
            off += n
        return sent

    def _all_sum(self, x: int) -> int:
        t = torch.tensor([x], dtype=torch.int64)
        dist.all_reduce(t, group=self.group)
        return int(t.item())

    # ------------------------------------------------------------ driver
    def execute(self, training_data, worker_logic, ps_logic, param_partitioner, w_in_partition, W, P,
                worker_receiver, worker_sender, ps_receiver, ps_sender, data_partitioner):
        parts = split_input(training_data, W, data_partitioner)
        local_w = [w for w in range(W) if self._owner(w) == self.rank]
        local_p = [p for p in range(P) if self._owner(p) == self.rank]
        self.outbox = {r: [] for r in range(self.world)}
        self.setup(parts, worker_logic, ps_logic, param_partitioner, w_in_partition, W, P, worker_receiver,
                   worker_sender, ps_receiver, ps_sender, local_workers=local_w, local_ps=local_p)
        self.open(self.rank, self.world)
        budget = self._wait_budget()
        last_busy = time.monotonic()
        while True:
            for _ in range(self.passes_per_round):
                if not self._step_local():
                    break
            sent = self._exchange()
            pending_buf = self._pending_buffers()
            busy = int(sent > 0 or not self._locally_idle())
            total_busy = self._all_sum(busy)
            if total_busy:
                last_busy = time.monotonic()
                self.rounds += 1
                continue
            # every decision below is collective so all ranks leave together
            if self._all_sum(pending_buf):
                self._flush_buffers()  # globally idle: combination buffers cannot fill further
                continue
            if budget > 0 and self._all_sum(int(time.monotonic() - last_busy >= budget)) < self.world:
                time.sleep(0.001)  # keep alive for user threads (iteration_wait_time)
                continue
            break
        self.close()
        if self.gather_outputs and self.output_sink is None:
            allout = [None] * self.world
            dist.all_gather_object(allout, self.outputs, group=self.group)
            return [e for part in allout for e in part]
        return self.outputs

"""Bounded-staleness pull/compute/push pipeline over a ``TensorPS``.

The reference bounds asynchrony per worker with ``pullLimit``: at most that many
pulls may be outstanding, later ones are queued (``M/WorkerLogic.scala:176-225``,
``PullLimitedWorkerLogic``).  Over micro-batches the same knob becomes a
*staleness bound*: with ``staleness = s`` the pull of micro-batch ``k`` is served
before the pushes of micro-batches ``k-s .. k-1`` are applied, never earlier ones.

* ``s = 0``: synchronous semantics (pull k sees every earlier push);
* ``s = 1``: the row all-to-all of batch ``k+1`` runs while batch ``k`` computes;
* ``s > 1``: deeper pipelines for slow links / large tables (config #5 stress).

Each micro-batch goes through three stages (``TensorPS``):

* **A** ``plan_begin`` -- dedup + count exchange, counts copied to the host
  asynchronously;
* **B** ``plan_end`` + serve + answer all-to-all (async) -- the pull;
* **C** compute + push.

``submit(k)`` enqueues A(k), then B(k-1) (``lookahead``, the default for
``s > 0``; B(k) without it), then C of every pulled batch beyond the bound.  B(k-1) therefore waits on counts that were enqueued one call
earlier: by then the device is busy with older work, so the host never idles
the device on split sizes.  Everything is stream-ordered on the device, so the
bound is exact: the gather of batch ``k`` is enqueued after the apply of batch
``k-s-1``.

Several tables: ``ps`` may be a list of ``TensorPS`` (SGNS pulls input and output
rows per micro-batch); ``submit`` then takes one key tensor per table, their
plans share ONE count exchange (``TensorPS.plan_begin_multi``), and ``compute``
receives / returns lists (rows, plans, deltas) in table order.

Owner stream (``owner_stream=True``, world > 1 on the GPU over RCCL / the virtual or
emulated world): the owner side -- the serve of every pull and the apply of every
push -- runs on a second stream, each after its all-to-all, and every exchange is
posted asynchronously.  The compute stream then waits only for the answer rows of
the batch it computes; the key, push and count transfers and the owner's random
gather / apply passes overlap the worker's compute (``TensorPS.owner_stream``).  The
enqueue order is unchanged, so the owner stream holds serve(k) behind apply(k-s-1):
the staleness bound is the same.  ``drain`` joins the owner stream.

Interleaved schedule (``interleave``, the default where an owner stream is not used
but the transport is asynchronous): everything stays on the compute stream, but
each ``submit(k)`` posts the key all-to-all of ``k-1``, computes and pushes (posted,
not applied) the oldest batch, THEN waits for the keys and serves ``k-1``, and only
then waits for the push and applies it -- the key transfer hides behind the compute
and the push transfer behind the serve, without a concurrent owner stream (whose
random-access apply slows the worker's latency-bound kernels: PA,
``profiles/r6_ps_paths_hot_owner.md``).  Serve ``k-1`` still lands after apply
``k-s-2`` and before apply ``k-s-1``: the same bound.

End of input: every ``submit`` carries a ``flag`` that reaches all peers with
the counts; ``all_flagged`` turns True on every rank at the same micro-batch once
every rank flagged it (the ``FlinkEOF`` barrier, ``M/utils/FlinkEOF.scala:97-107``,
without an extra collective).  Fixed-shape plans keep the flags on the device; they
reach the host one ``submit`` later (``poll_flags``), the same micro-batch on every rank.
"""
from __future__ import annotations

import os
from collections import deque
from typing import Any, Callable, List, Optional, Tuple

import torch

from .tensor_ps import PullPlan, TensorPS

#: compute(rows, plan, payload) -> (deltas [U, D] or None, result)
ComputeFn = Callable[[torch.Tensor, PullPlan, Any], Tuple[Optional[torch.Tensor], Any]]


class BoundedStalenessPipeline:
    def __init__(self, ps, compute: ComputeFn, staleness: int = 1, lr: float = 0.0,
                 lookahead: Optional[bool] = None, owner_stream: Optional[bool] = None,
                 interleave: Optional[bool] = None):
        """``lookahead`` (default: ``staleness > 0``): stage B of a batch waits for
        the next ``submit``, so its counts are never waited for on an idle device.
        Without it (the default of the synchronous ``staleness = 0`` mode) a
        batch is pulled, computed and pushed inside its own ``submit``.
        ``owner_stream`` (default: where it applies -- ``owner_stream_ok``; env
        ``FPS_OWNER_STREAM=0`` turns it off): serve / apply on a second stream."""
        if staleness < 0:
            raise ValueError("staleness must be >= 0")
        self.multi = isinstance(ps, (list, tuple))
        self.pss: List[TensorPS] = list(ps) if self.multi else [ps]
        env = os.environ.get("FPS_OWNER_STREAM")  # A/B override: "0" off, "1" on where it applies
        if env in ("0", "1"):
            owner_stream = env == "1"
        if owner_stream is None or owner_stream:
            owner_stream = owner_stream_ok(self.pss[0].comm, self.pss[0].table.device)
        self.owner = None
        if owner_stream:
            self.owner = torch.cuda.Stream(self.pss[0].table.device)
            for p in self.pss:  # one owner stream for every table of the pipeline
                p.owner_stream = self.owner
        self.lookahead = staleness > 0 if lookahead is None else bool(lookahead)
        if interleave is None:
            interleave = (self.owner is None and staleness > 0 and self.lookahead
                          and async_transport(self.pss[0].comm, self.pss[0].table.device))
        self.interleave = bool(interleave) and self.owner is None and staleness > 0 and self.lookahead
        if self.interleave:
            for p in self.pss:
                p.async_exchange = True
        self.ps, self.compute, self.staleness, self.lr = ps, compute, int(staleness), lr
        self.lookahead = staleness > 0 if lookahead is None else bool(lookahead)
        self._planned: deque = deque()  # (pending plan, payload) after stage A
        self._pulled: deque = deque()   # (rows, work, plan, payload) after stage B
        self.max_observed = 0  # pushes of earlier batches still pending when a pull was served
        self.all_flagged = False
        self.submitted = 0
        self._flags_dev: Optional[torch.Tensor] = None  # newest fixed plan's peer flags (device)
        self._flags_host = None  # (pinned copy, event) of the previous one

    def submit(self, keys: torch.Tensor, payload: Any = None, flag: int = 0, presence=None) -> List[Any]:
        """Begin the pull of a new micro-batch; finish (compute + push) every
        batch that would otherwise exceed the staleness bound.  Returns the
        results of the batches finished by this call, oldest first.  ``presence``:
        the single-table plan's key-presence hint (``TensorPS.plan_begin``)."""
        if self.multi:
            self._planned.append((TensorPS.plan_begin_multi(self.pss, keys, flag), payload))
        else:
            self._planned.append((self.ps.plan_begin(keys, flag, presence=presence), payload))
        self.submitted += 1
        out: List[Any] = []
        if self.interleave and self.staleness > 0 and self.lookahead:  # (a synchronous call drops to the plain path)
            # keys of the batches beyond the lookahead posted; the oldest pulled batches
            # computed and their pushes posted; then the new ones served; then the pushes
            # applied (module docstring: the same staleness bound)
            ready = []
            while len(self._planned) > 1:
                ready.append(self._plan_next())
            pend = []
            while len(self._pulled) + len(ready) > self.staleness and self._pulled:
                r, p = self._finish(self._pulled.popleft(), defer=True)
                out.append(r)
                pend.extend(p)
            for item in ready:
                self._serve(*item)
            for ps, pp in pend:
                ps.apply_pending(pp)
            self.poll_flags()
            return out
        while len(self._planned) > (1 if self.lookahead else 0):
            self._pull_next()
        while len(self._pulled) > self.staleness:
            out.append(self._finish(self._pulled.popleft()))
        self.poll_flags()
        return out

    def poll_flags(self) -> None:
        """Fixed-shape plans: read the previous pulled plan's peer flags (copied to
        pinned memory one ``submit`` ago: by now the device is past them) and start
        the copy of the newest.  Every rank reads the same plan's flags at the same
        ``submit``, so ``all_flagged`` turns on everywhere at once, one micro-batch
        after the flags were sent.  A replayed hipGraph step calls this itself."""
        dev = self._flags_dev
        if dev is None or (dev.is_cuda and torch.cuda.is_current_stream_capturing()):
            return
        if self._flags_host is not None:
            host, ev = self._flags_host
            if ev is not None:
                ev.synchronize()
            if all(int(f) != 0 for f in host.tolist()):
                self.all_flagged = True
        self._flags_dev = None
        if dev.is_cuda:
            host = torch.empty(tuple(dev.shape), dtype=dev.dtype, pin_memory=True)
            host.copy_(dev, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
        else:
            host, ev = dev.clone(), None
        self._flags_host = (host, ev)

    def reset_flags(self) -> None:
        """A new input phase: forget every flag seen so far."""
        self.all_flagged = False
        self._flags_dev, self._flags_host = None, None

    def drain(self) -> List[Any]:
        out = []
        while self._planned:
            self._pull_next()
            while len(self._pulled) > self.staleness:
                out.append(self._finish(self._pulled.popleft()))
        while self._pulled:
            out.append(self._finish(self._pulled.popleft()))
        if self.owner is not None:  # every apply done before the caller reads the tables
            self.pss[0].owner_sync()
        return out

    @property
    def in_flight(self) -> int:
        """Micro-batches pulled whose pushes are not applied yet (<= staleness
        between calls); the batch of the latest ``submit`` is only planned."""
        return len(self._pulled)

    @property
    def planned(self) -> int:
        return len(self._planned)

    def _plan_next(self):
        """Stage B's first half: the plan's sizes from the host, its key all-to-all posted."""
        pps, payload = self._planned.popleft()
        if not self.multi:
            pps = [pps]
        plans = [ps.plan_end(pp) for ps, pp in zip(self.pss, pps)]
        if plans[0].flags_dev is not None:
            self._flags_dev = plans[0].flags_dev
        elif plans[0].peer_flags and all(f != 0 for f in plans[0].peer_flags):
            self.all_flagged = True
        return plans, payload

    def _serve(self, plans, payload):
        """Stage B's second half: serve + answer all-to-all (async)."""
        pulled = [ps.pull_planned(plan, async_op=True) for ps, plan in zip(self.pss, plans)]
        self.max_observed = max(self.max_observed, len(self._pulled))
        self._pulled.append(([r for r, _ in pulled], [w for _, w in pulled], plans, payload))

    def _pull_next(self):
        self._serve(*self._plan_next())

    def _finish(self, item, defer: bool = False) -> Any:
        rows, works, plans, payload = item
        for w in works:
            if w is not None:
                w.wait()
        if self.owner is not None:  # answer rows allocated on the owner stream, read here
            cur = torch.cuda.current_stream(self.pss[0].table.device)
            for r in rows:
                if r is not None and r.is_cuda:
                    r.record_stream(cur)
        pend = []
        if defer:
            for ps in self.pss:  # the compute's own pushes (engine workers) are deferred too
                ps._defer_into = pend
        try:
            if self.multi:
                deltas, result = self.compute(rows, plans, payload)
                for ps, plan, d in zip(self.pss, plans, deltas or [None] * len(plans)):
                    if d is not None:
                        pp = ps.push(plan, d, lr=self.lr, defer=defer)
                        if pp is not None:
                            pend.append((ps, pp))
            else:
                deltas, result = self.compute(rows[0], plans[0], payload)
                if deltas is not None:
                    pp = self.ps.push(plans[0], deltas, lr=self.lr, defer=defer)
                    if pp is not None:
                        pend.append((self.ps, pp))
        finally:
            if defer:
                for ps in self.pss:
                    ps._defer_into = None
        return (result, pend) if defer else result


def async_transport(comm, device) -> bool:
    """World > 1 on the GPU over an asynchronous transport (RCCL, the virtual world, the
    emulated world) -- not gloo (host-staged, synchronous)."""
    return (torch.device(device).type == "cuda" and comm.world > 1
            and getattr(comm, "backend", "") in ("nccl", "virtual", "emulated"))


def owner_stream_ok(comm, device) -> bool:
    """Does an owner stream apply?  World > 1 on the GPU with an asynchronous transport
    (RCCL, the virtual world, the emulated world); not gloo (host-staged, synchronous)
    and not inside a graph capture."""
    dev = torch.device(device)
    return (dev.type == "cuda" and comm.world > 1 and getattr(comm, "backend", "") in ("nccl", "virtual", "emulated")
            and not torch.cuda.is_current_stream_capturing())

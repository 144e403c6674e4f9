"""hipGraph replay of the tensor engine's fixed-shape micro-batch step.

At small micro-batches the tensor engine is bound by its host control loop:
every ``submit`` runs the worker's Python callbacks, the dedup / gather /
apply launchers and ~15-25 kernel launches (~140 us per micro-batch,
``profiles/r2_engine_plumbing.json``).  The reference has no such cost to
amortise -- it processes one record per message (``M/FlinkParameterServer.scala:215-335``)
-- but a micro-batch engine serving small batches (online learning, top-K
queries) needs it gone.  With static world-1 plans (``TensorPS.static``) the
whole step -- plan, pull, the worker's ``on_pull_recv_batch``, push, apply --
has shapes fixed by the batch's shapes and issues no host sync, so it can be
captured once into a hipGraph and replayed.  At world > 1 the fixed-shape plans
of ``TensorPS.capacity`` do the same (every exchange has host-known, constant
splits), and the step's three RCCL all-to-alls are captured with it; the peers'
end-of-input flags are read from the replayed step's buffer one micro-batch
later (``BoundedStalenessPipeline.poll_flags``):

* the first ``warmup`` micro-batches of a new shape signature run eagerly
  (they size the workspaces); the next is captured on the capture stream
  with the batch copied into static input buffers, then replayed;
* later micro-batches of that signature copy their tensors into the static
  buffers and replay the graph -- one graph launch instead of the host loop;
* outputs the step emitted during capture (``Left`` / ``Right`` pairs) are
  re-emitted as clones after every replay, so sinks never see graph-owned
  memory; counters / PS stats advance by the captured step's increments;
* the claim map of the dedup is cleared after every step (``clear_after``),
  so the epoch baked into the graph stays valid.

Contract (why it is opt-in, ``TensorRuntime(graph=True)``): the worker's
callbacks must be a pure device function of the batch and of device state --
no host syncs, no Python-side state that changes per micro-batch (the
replayed step does not run Python).  Workers declare it with
``graph_safe = True``.  Anything that would make a captured step wrong makes
the runtime run eagerly instead: world > 1 without fixed-shape plans or over a
host-staged (gloo) transport, a non-static plan, staleness or
lookahead (the pipeline carries state across ``submit`` calls), locking or
sequential-combine PS logics, sparse (growing) shards, arbitrary pushes, a
stage timer or ``FPS_DEBUG``.  A capture that fails (a callback synced)
disables graphs for the runtime with a warning and runs the batch eagerly.
"""
from __future__ import annotations

import gc
import traceback
import warnings
from typing import Any, Dict, List, Optional, Tuple

import torch

from .. import ops
from ..api.batched import MaskedPair
from .messages import Left, Right


def _flatten(batch: Any, leaves: List[torch.Tensor]):
    """Structure signature of ``batch``; appends its tensors to ``leaves``.
    Returns None when the batch holds something a graph cannot take."""
    if torch.is_tensor(batch):
        leaves.append(batch)
        return ("T", tuple(batch.shape), batch.dtype, batch.device.type)
    if isinstance(batch, (tuple, list)):
        sub = []
        for x in batch:
            s = _flatten(x, leaves)
            if s is None:
                return None
            sub.append(s)
        return ("L" if isinstance(batch, list) else "U", tuple(sub))
    if isinstance(batch, dict):
        sub = []
        for k in sorted(batch):
            s = _flatten(batch[k], leaves)
            if s is None:
                return None
            sub.append((k, s))
        return ("D", tuple(sub))
    if isinstance(batch, (int, float, str, bool)) or batch is None:
        return ("C", batch)  # a constant: part of the signature, baked into the graph
    return None


def _rebuild(sig, it):
    kind = sig[0]
    if kind == "T":
        return next(it)
    if kind in ("L", "U"):
        xs = [_rebuild(s, it) for s in sig[1]]
        return xs if kind == "L" else tuple(xs)
    if kind == "D":
        return {k: _rebuild(s, it) for k, s in sig[1]}
    return sig[1]


def _clone_out(x: Any) -> Any:
    """A copy of an emitted value that does not alias graph-owned memory."""
    if torch.is_tensor(x):
        return x.clone()
    if isinstance(x, MaskedPair):
        if x._pair is not None:
            return tuple(t.clone() for t in x._pair)
        return MaskedPair(x._ids.clone(), x._values.clone(), x._mask.clone())
    if isinstance(x, Left):
        return Left(_clone_out(x.value))
    if isinstance(x, Right):
        return Right(_clone_out(x.value))
    if isinstance(x, tuple):
        return tuple(_clone_out(v) for v in x)
    if isinstance(x, list):
        return [_clone_out(v) for v in x]
    if isinstance(x, dict):
        return {k: _clone_out(v) for k, v in x.items()}
    return x


def _tensor_attrs(obj) -> Dict[str, torch.Tensor]:
    return {k: v for k, v in vars(obj).items() if torch.is_tensor(v)} if obj is not None else {}


class _Entry:
    __slots__ = ("graph", "inputs", "emits", "counters", "stats", "held", "flags")

    def __init__(self, graph, inputs, emits, counters, stats, held, flags=None):
        self.graph, self.inputs, self.emits = graph, inputs, emits
        self.counters, self.stats, self.held = counters, stats, held
        self.flags = flags  # fixed-shape plans: the peers' flags in the graph's receive buffer


class StepGraphs:
    """Per-runtime cache of captured micro-batch steps, keyed by batch signature."""

    def __init__(self, rt, warmup: int = 2, max_graphs: int = 8):
        self.rt = rt
        self.warmup, self.max_graphs = int(warmup), int(max_graphs)
        self.entries: Dict[Any, _Entry] = {}
        self.seen: Dict[Any, int] = {}
        self.disabled: Optional[str] = None
        self.disabled_trace: Optional[str] = None
        self.replays = 0
        self.captures = 0
        self.released = False  # after ``release``: every later step runs eagerly

    # ----------------------------------------------------------- eligibility
    def why_not(self) -> Optional[str]:
        """None if the runtime's configuration can run captured steps, else the reason."""
        rt = self.rt
        ps_logic, ps = rt.ps_logic, rt.ps_logic.ps if rt.ps_logic is not None else None
        if rt.device.type != "cuda":
            return "not on a GPU"
        collective = rt.comm.world != 1 or getattr(rt.comm, "loopback", False)
        if collective and not (ps is not None and ps.fixed()):
            return "world > 1 without fixed-shape plans (TensorRuntime(capacity=...)): split sizes are host-read"
        if collective and rt.comm.backend != "nccl":
            return "only RCCL collectives can be captured (gloo stages through host memory)"
        if ops.DEBUG:
            return "FPS_DEBUG range checks sync"
        if rt.pipe is None or ps_logic.locking:
            return "locking PS logic (per-round host decisions)"
        if rt.pipe.staleness != 0 or rt.pipe.lookahead:
            return "staleness / lookahead pipelines carry state across submits"
        if not (getattr(ps, "static", False) or ps.fixed()):
            return "plan is not static"
        if getattr(ps_logic.table, "sparse", False):
            return "sparse shards grow (reallocate) under a captured step"
        if ps_logic.combine == "sequential":
            return "sequential combine needs a host-side round count"
        if rt.worker_logic.arbitrary_pushes:
            return "arbitrary pushes plan a second, host-synced round"
        if rt.timer is not None:
            return "a stage timer records events per stage"
        if not getattr(rt.worker_logic, "graph_safe", False):
            return "the worker logic does not declare graph_safe = True"
        return None

    def release(self) -> None:
        """Destroy the captured graphs (their memory pools, and the RCCL work baked into
        them: a communicator is only torn down once no graph references it)."""
        self.entries.clear()
        self.seen.clear()
        self.released = True

    # --------------------------------------------------------------- running
    def _held(self) -> List[Tuple[Any, str, torch.Tensor]]:
        """(owner, attribute, tensor) of every persistent buffer a captured step may
        touch: kept alive by the entry, and re-checked before each replay."""
        ps = self.rt.ps_logic.ps
        owners = [ps, ps.dedup, ps.table, self.rt.worker_logic]
        return [(o, k, v) for o in owners for k, v in _tensor_attrs(o).items()]

    def _valid(self, e: _Entry) -> bool:
        return all(getattr(o, k, None) is v for o, k, v in e.held)

    def submit(self, batch: Any, flag: int) -> bool:
        """Run ``batch`` through a captured step if possible; False = run it eagerly."""
        if self.disabled is not None or self.released or batch is None or flag:
            return False
        leaves: List[torch.Tensor] = []
        sig = _flatten(batch, leaves)
        if sig is None:
            return False
        e = self.entries.get(sig)
        if e is not None and not self._valid(e):  # a workspace was reallocated: recapture
            self.entries.clear()
            self.seen.clear()
            e = None
        if e is None:
            n = self.seen.get(sig, 0)
            self.seen[sig] = n + 1
            if n < self.warmup or len(self.entries) >= self.max_graphs:
                return False
            e = self._capture(sig, leaves, flag)
            if e is None:
                return False
        self._replay(e, leaves)
        return True

    def _capture(self, sig, leaves, flag) -> Optional[_Entry]:
        rt = self.rt
        dev = rt.device
        inputs = [torch.empty_like(t, device=dev) for t in leaves]
        static_batch = _rebuild(sig, iter(inputs))
        emits: List[Any] = []
        c0 = dict(rt.counters.c)
        s0 = dict(rt.ps_logic.ps.stats)
        sub0 = rt.pipe.submitted
        g = torch.cuda.CUDAGraph()
        rt._capture_emits = emits
        # no automatic garbage collection while capturing: a collected pinned host tensor
        # or event of an earlier eager step would be freed on the capturing thread, and
        # the host allocator's stream bookkeeping is illegal there (process abort);
        # torch.cuda.graph collects once before the capture starts
        gc_was_enabled = gc.isenabled()
        gc.disable()
        try:
            # thread_local: only this thread's calls are checked (a helper thread of the
            # process, e.g. a watchdog, must not invalidate the capture)
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                rt._submit_eager(static_batch, flag)
        except Exception as ex:  # a callback synced or allocated host-side state: stay eager
            self.disabled = f"capture failed: {type(ex).__name__}: {ex}"
            self.disabled_trace = traceback.format_exc()
            warnings.warn(f"tensor engine: hipGraph capture disabled ({self.disabled}); running eagerly")
            rt.counters.c.clear()
            rt.counters.c.update(c0)
            rt.ps_logic.ps.stats.clear()
            rt.ps_logic.ps.stats.update(s0)
            rt.pipe.submitted = sub0
            rt.pipe._flags_dev = None
            return None
        finally:
            rt._capture_emits = None
            if gc_was_enabled:
                gc.enable()
        dc = {k: v - c0.get(k, 0.0) for k, v in rt.counters.c.items() if v != c0.get(k, 0.0)}
        ds = {k: v - s0.get(k, 0) for k, v in rt.ps_logic.ps.stats.items() if v != s0.get(k, 0)}
        # the capture itself executed nothing: undo its host-side increments (replay adds them)
        for k, v in dc.items():
            rt.counters.c[k] -= v
        for k, v in ds.items():
            rt.ps_logic.ps.stats[k] -= v
        rt.pipe.submitted = sub0
        flags, rt.pipe._flags_dev = rt.pipe._flags_dev, None  # the capture executed nothing
        e = _Entry(g, inputs, emits, dc, ds, self._held(), flags)
        self.entries[sig] = e
        self.captures += 1
        return e

    def _replay(self, e: _Entry, leaves: List[torch.Tensor]) -> None:
        rt = self.rt
        for dst, src in zip(e.inputs, leaves):
            dst.copy_(src, non_blocking=True)
        e.graph.replay()
        if e.flags is not None:
            rt.pipe._flags_dev = e.flags
            rt.pipe.poll_flags()
        for k, v in e.counters.items():
            rt.counters.c[k] += v
        st = rt.ps_logic.ps.stats
        for k, v in e.stats.items():
            st[k] += v
        rt.pipe.submitted += 1
        self.replays += 1
        for out in e.emits:
            rt._emit(_clone_out(out))

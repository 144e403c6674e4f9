"""A stream-faithful virtual N-rank world on ONE GPU: the RCCL transport, emulated.

Every multi-rank run on a one-GPU box used gloo with the ranks sharing the GPU.
Gloo moves device tensors through host memory, so each transfer has completed
before the call returns: a missing ``Work.wait()``, a buffer reused before its
send has read it, or a receive buffer still being read when the next message
lands can never show up there.  RCCL over xGMI has none of those guarantees --
the reference's whole engine is the cross-process shuffle with its feedback
edge (``M/FlinkParameterServer.scala:265-317,331-335``), and ours is the same
exchange on asynchronous device streams.

``VirtualWorld`` runs N rank THREADS in one process on one device.  Each rank
has its own compute stream (``run_virtual`` sets it current in the thread) and
its own model instance, and talks through a ``VirtualComm`` -- a drop-in
``parallel.comm.Comm`` -- whose operations follow RCCL's semantics:

* an operation is *posted* when a rank calls it: an event is recorded on the
  rank's current stream (the data it sends / the buffer it receives into are
  ready in that stream's order), and nothing blocks the host;
* point-to-point messages match FIFO per (sender, receiver) channel; a
  collective matches when every rank has posted its n-th collective -- a rank
  posting a different collective (or different split sizes) than its peers
  aborts the world with a desync report instead of hanging;
* a matched transfer runs on a dedicated LINK stream after waiting for both
  sides' post events, after an injectable delay that models the xGMI time of
  the message (``latency_us + bytes / link_gbps``, scaled by ``dilate``; one
  message at a time per link).  ``delay_model="host"`` (default): a link thread
  watches the post events and issues the copy once the data has been ready for
  the modelled time -- the delay occupies no compute unit, so it does not
  compete with the ranks' kernels; ``"kernel"``: a ``torch.cuda._sleep`` on the
  link stream before the copy (needs a free CU slot to start: under a
  GPU-filling grid it queues behind the compute, which overstates the exposed
  wait);
* ``Work.wait()`` makes the CALLER's current stream wait for the transfer's
  completion event (the host blocks only until the peer has posted its side,
  i.e. until the transfer exists) -- exactly ``ProcessGroupNCCL``'s contract:
  whatever the caller enqueues before ``wait()`` may overlap the transfer, and a
  send buffer may not be reused before the wait.

Nothing else orders the link streams: a rank's later message may overtake an
earlier one to a different peer, and a send buffer is read whenever the link
gets to it.  That is weaker than RCCL's (one communicator stream per rank), so a
schedule that is correct here is correct over RCCL, and a race the real
transport could expose -- reading a receive buffer before waiting, reusing a send
buffer early -- turns into wrong numbers here once the delay is long enough.

``mode="sync"`` is the host-synchronous reference (gloo's semantics on one
device): every call returns only once its transfers are done, and every
transfer synchronizes the device before and after its copy.

Timing: ranks share the GPU, so every rank's compute runs ~N x slower than on
its own GPU; ``dilate=N`` stretches the modelled transfer times by the same
factor, keeping the compute / transfer ratio of the real N-GPU job.
``RingRotation.wait_ms`` / the bench's ``comm_wait_ms_per_step`` then measure
how much of the transfer time the schedule leaves exposed.
"""
from __future__ import annotations

import threading
import time
from collections import defaultdict, deque
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from .comm import Comm


class VirtualWorldAborted(RuntimeError):
    """Raised in every rank thread once one rank failed (or the world desynced)."""


def _reduce_op_name(op) -> str:
    if op is None:
        return "sum"
    for name in ("SUM", "MAX", "MIN", "PRODUCT"):
        if op == getattr(dist.ReduceOp, name):
            return name.lower()
    raise ValueError(f"unsupported reduce op {op!r}")


class _Sleep:
    """Calibrated device sleep: ``torch.cuda._sleep`` spins for a number of shader
    clock cycles; the cycles per microsecond are measured once per process."""

    cycles_per_us: Optional[float] = None

    @classmethod
    def calibrate(cls, device) -> float:
        if cls.cycles_per_us is None:
            with torch.cuda.device(device):
                s = torch.cuda.Stream(device)
                with torch.cuda.stream(s):
                    torch.cuda._sleep(1000)  # load the kernel
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    n = 2_000_000
                    a.record(s)
                    torch.cuda._sleep(n)
                    b.record(s)
                s.synchronize()
                ms = max(a.elapsed_time(b), 1e-3)
            cls.cycles_per_us = n / (ms * 1e3)
        return cls.cycles_per_us

    @classmethod
    def us(cls, device, us: float) -> None:
        if us > 0:
            torch.cuda._sleep(max(1, int(us * cls.calibrate(device))))


class VWork:
    """The handle of a posted operation (``Work`` of ``ProcessGroupNCCL``)."""

    def __init__(self, world: "VirtualWorld", rank: int, what: str):
        self.world, self.rank, self.what = world, rank, what
        self.pending = 0          # transfers of this op not issued yet
        self.events: List[Any] = []  # completion events (device) of the issued transfers
        self.posted_at = time.perf_counter()

    def _done_issuing(self) -> bool:
        return self.pending == 0

    def wait(self, timeout: Optional[float] = None) -> bool:
        w = self.world
        with w.cv:
            ok = w.cv.wait_for(lambda: self._done_issuing() or w.error is not None,
                               timeout=timeout if timeout is not None else w.timeout_s)
            if w.error is not None:
                raise VirtualWorldAborted(f"rank {self.rank} waiting on {self.what}: {w.error}")
            if not ok:
                w._abort(f"rank {self.rank}: {self.what} never matched (a peer did not post its side)")
                raise VirtualWorldAborted(w.error)
            events = list(self.events)
        if w.cuda:
            cur = torch.cuda.current_stream(w.device)
            for ev in events:
                cur.wait_event(ev)
        return True

    def is_completed(self) -> bool:
        with self.world.cv:
            if not self._done_issuing():
                return False
            return all(ev.query() for ev in self.events) if self.world.cuda else True


class _Post:
    """One side of a message: the tensor, the rank's post event, the work to complete."""

    __slots__ = ("tensor", "event", "work", "rank")

    def __init__(self, tensor, event, work, rank):
        self.tensor, self.event, self.work, self.rank = tensor, event, work, rank


class VirtualWorld:
    """The shared transport of ``world`` rank threads on ``device``."""

    def __init__(self, world: int, device=None, mode: str = "async", link_gbps: float = 50.0,
                 latency_us: float = 5.0, dilate: float = 1.0, delay: bool = True, timeout_s: float = 300.0,
                 delay_model: str = "host"):
        if mode not in ("async", "sync"):
            raise ValueError("mode must be 'async' (RCCL semantics) or 'sync' (host-synchronous reference)")
        if delay_model not in ("host", "kernel"):
            raise ValueError("delay_model must be 'host' or 'kernel'")
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else \
                torch.device("cpu")
        self.world, self.device, self.mode = int(world), torch.device(device), mode
        self.cuda = self.device.type == "cuda"
        self.link_gbps, self.latency_us, self.dilate = float(link_gbps), float(latency_us), float(dilate)
        self.delay = bool(delay) and self.cuda and mode == "async"
        self.timeout_s = float(timeout_s)
        self.cv = threading.Condition()
        self.error: Optional[str] = None
        self._sends: Dict[Tuple[int, int], deque] = defaultdict(deque)
        self._recvs: Dict[Tuple[int, int], deque] = defaultdict(deque)
        self._coll_seq = [0] * self.world
        self._coll: Dict[int, Dict[int, tuple]] = {}
        self._host_seq = [0] * self.world
        self._host: Dict[int, Dict[int, Any]] = {}
        self._links: Dict[Tuple[int, int], Any] = {}
        self._link_pool: List[Any] = []
        #: modelled transfer microseconds and bytes, per (src, dst) link
        self.link_us: Dict[Tuple[int, int], float] = defaultdict(float)
        self.link_bytes: Dict[Tuple[int, int], int] = defaultdict(int)
        self.transfers = 0
        self.delay_model = delay_model
        self._pending: deque = deque()     # host-timed transfers not issued yet
        self._link_busy: Dict[Tuple[int, int], float] = defaultdict(float)
        self._link_thread: Optional[threading.Thread] = None
        self._closed = False
        if self.delay and delay_model == "kernel":
            _Sleep.calibrate(self.device)
        if self.delay and delay_model == "host":
            self._link_thread = threading.Thread(target=self._link_loop, name="vworld-links", daemon=True)
            self._link_thread.start()

    # ------------------------------------------------------------------ plumbing
    def comm(self, rank: int) -> "VirtualComm":
        return VirtualComm(self, rank)

    def _abort(self, msg: str) -> None:
        with self.cv:
            if self.error is None:
                self.error = msg
            self.cv.notify_all()

    def _check(self) -> None:
        if self.error is not None:
            raise VirtualWorldAborted(self.error)

    def _event(self):
        """Post event on the calling thread's current stream (None off-GPU)."""
        if not self.cuda:
            return None
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        return ev

    def _link(self, src: int, dst: int):
        """The stream of link ``src -> dst``: high-priority pool streams (the compute
        streams come from the normal pool), assigned round-robin in order of first
        use so the links of a ring schedule get distinct streams."""
        s = self._links.get((src, dst))
        if s is None:
            n_max = max(2 * self.world, 2)
            if len(self._link_pool) < n_max:
                self._link_pool.append(torch.cuda.Stream(self.device, priority=-1))
                s = self._link_pool[-1]
            else:
                s = self._link_pool[len(self._links) % n_max]
            self._links[(src, dst)] = s
        return s

    def _delay_us(self, nbytes: int) -> float:
        return (self.latency_us + nbytes / (self.link_gbps * 1e3)) * self.dilate

    def _copy(self, src_rank: int, dst_rank: int, dst: torch.Tensor, src: torch.Tensor, evs, works) -> None:
        """Issue one matched transfer (called with ``cv`` held)."""
        nbytes = src.numel() * src.element_size()
        self.link_bytes[(src_rank, dst_rank)] += nbytes
        self.transfers += 1
        if not self.cuda:
            if src.numel():
                dst.copy_(src.reshape(dst.shape))
            for w in works:
                w.pending -= 1
            return
        if self.mode == "sync":  # gloo on one device: everything before is done, the copy is done
            torch.cuda.synchronize(self.device)
            if src.numel():
                dst.copy_(src.reshape(dst.shape))
            torch.cuda.synchronize(self.device)
            for w in works:
                w.pending -= 1
            return
        if self.delay and self.delay_model == "host" and src_rank != dst_rank:
            us = self._delay_us(nbytes)
            self.link_us[(src_rank, dst_rank)] += us
            self._pending.append([src_rank, dst_rank, dst, src, evs, works, us, None])
            self.cv.notify_all()
            return
        self._issue(src_rank, dst_rank, dst, src, evs, works)

    def _issue(self, src_rank: int, dst_rank: int, dst: torch.Tensor, src: torch.Tensor, evs, works) -> None:
        """Enqueue the copy of a transfer on its link stream (called with ``cv`` held)."""
        nbytes = src.numel() * src.element_size()
        s = self._link(src_rank, dst_rank)
        with torch.cuda.stream(s):
            for ev in evs:
                if ev is not None:
                    s.wait_event(ev)
            if self.delay and self.delay_model == "kernel" and src_rank != dst_rank:
                us = self._delay_us(nbytes)
                self.link_us[(src_rank, dst_rank)] += us
                _Sleep.us(self.device, us)
            if src.numel():
                dst.copy_(src.reshape(dst.shape), non_blocking=True)
            done = torch.cuda.Event()
            done.record(s)
        # the caching allocator must not hand these blocks out before the link read them
        src.record_stream(s)
        dst.record_stream(s)
        for w in works:
            w.events.append(done)
            w.pending -= 1

    def _link_loop(self) -> None:
        """Host-timed links: a transfer starts when both sides' post events have
        completed (and its link finished the previous message), and is issued to the
        device once its modelled duration has passed."""
        torch.cuda.set_device(self.device)
        while True:
            with self.cv:
                if self._closed or self.error is not None:
                    return
                now = time.perf_counter()
                issued = False
                for item in list(self._pending):
                    src_rank, dst_rank, dst, src, evs, works, us, t_start = item
                    key = (src_rank, dst_rank)
                    if t_start is None:
                        if all(ev is None or ev.query() for ev in evs):
                            item[7] = t_start = max(now, self._link_busy[key])
                            self._link_busy[key] = t_start + us * 1e-6
                        continue
                    if now >= t_start + us * 1e-6:
                        self._pending.remove(item)
                        self._issue(src_rank, dst_rank, dst, src, evs, works)
                        issued = True
                if issued:
                    self.cv.notify_all()
                wait_s = 2e-5 if self._pending else 1e-3
                self.cv.wait(timeout=wait_s)

    def close(self) -> None:
        with self.cv:
            self._closed = True
            self.cv.notify_all()
        if self._link_thread is not None:
            self._link_thread.join(5.0)

    # ------------------------------------------------------------------ point-to-point
    def post_p2p(self, rank: int, sends: Sequence, recvs: Sequence) -> List[VWork]:
        self._check()
        ev = self._event()
        works = []
        with self.cv:
            for t, peer in sends:
                w = VWork(self, rank, f"send {rank}->{peer} {tuple(t.shape)}")
                w.pending = 1
                self._sends[(rank, int(peer))].append(_Post(t, ev, w, rank))
                works.append(w)
            for t, peer in recvs:
                w = VWork(self, rank, f"recv {peer}->{rank} {tuple(t.shape)}")
                w.pending = 1
                self._recvs[(int(peer), rank)].append(_Post(t, ev, w, rank))
                works.append(w)
            for key in {(rank, int(p)) for _, p in sends} | {(int(p), rank) for _, p in recvs}:
                self._match_p2p(key)
            self.cv.notify_all()
        if self.mode == "sync":  # gloo: the call returns once its transfers are done
            for w in works:
                w.wait()
        return works

    def _match_p2p(self, key) -> None:
        sq, rq = self._sends[key], self._recvs[key]
        while sq and rq:
            s, r = sq.popleft(), rq.popleft()
            if s.tensor.numel() != r.tensor.numel() or s.tensor.dtype != r.tensor.dtype:
                self._abort(f"p2p {key[0]}->{key[1]} mismatch: send {tuple(s.tensor.shape)} {s.tensor.dtype} vs "
                            f"recv {tuple(r.tensor.shape)} {r.tensor.dtype}")
                return
            self._copy(key[0], key[1], r.tensor, s.tensor, (s.event, r.event), (s.work, r.work))

    # ------------------------------------------------------------------ collectives
    def post_collective(self, rank: int, kind: str, sig: tuple, payload: dict) -> VWork:
        """Post this rank's next collective; issue it once every rank posted it."""
        self._check()
        ev = self._event()
        w = VWork(self, rank, kind)
        with self.cv:
            k = self._coll_seq[rank]
            self._coll_seq[rank] += 1
            slot = self._coll.setdefault(k, {})
            slot[rank] = (kind, sig, payload, ev, w)
            w.pending = 1
            if len(slot) == self.world:
                del self._coll[k]
                self._issue_collective(k, slot)
            self.cv.notify_all()
        if self.mode == "sync":
            w.wait()
        return w

    def _issue_collective(self, k: int, slot: dict) -> None:
        kinds = {r: (v[0], v[1]) for r, v in slot.items()}
        if len({kd for kd, _ in kinds.values()}) != 1:
            self._abort(f"collective #{k} desync: " + ", ".join(f"rank {r}: {kd}" for r, (kd, _) in
                                                              sorted(kinds.items())))
            return
        kind = slot[0][0]
        W = self.world
        if kind == "all_to_all":
            # send_splits of rank r [p] must equal recv_splits of rank p [r]
            for r in range(W):
                ss = slot[r][1][0]
                for p in range(W):
                    if int(ss[p]) != int(slot[p][1][1][r]):
                        self._abort(f"all_to_all #{k}: rank {r} sends {ss[p]} rows to rank {p}, which expects "
                                    f"{slot[p][1][1][r]}")
                        return
            for r in range(W):
                slot[r][4].pending = 0
            for r in range(W):
                send, ss = slot[r][2]["send"], slot[r][1][0]
                so = 0
                for p in range(W):
                    n = int(ss[p])
                    out, rs = slot[p][2]["out"], slot[p][1][1]
                    ro = int(sum(int(x) for x in rs[:r]))
                    if n:
                        ws = (slot[r][4], slot[p][4]) if r != p else (slot[r][4],)
                        for w in ws:
                            w.pending += 1
                        self._copy(r, p, out[ro:ro + n], send[so:so + n], (slot[r][3], slot[p][3]), ws)
                    so += n
            return
        if kind == "all_gather":
            for r in range(W):
                slot[r][4].pending = 0
            for r in range(W):
                for p in range(W):
                    ws = (slot[r][4],) if r == p else (slot[r][4], slot[p][4])
                    for w in ws:
                        w.pending += 1
                    self._copy(r, p, slot[p][2]["outs"][r], slot[r][2]["t"], (slot[r][3], slot[p][3]), ws)
            return
        if kind == "all_reduce":
            ts = [slot[r][2]["t"] for r in range(W)]
            op = slot[0][1][0]
            evs = [slot[r][3] for r in range(W)]
            self._reduce(ts, op, evs, [slot[r][4] for r in range(W)])
            return
        if kind == "barrier":
            for r in range(W):
                slot[r][4].pending = 0
            return
        self._abort(f"unknown collective {kind}")

    def _reduce(self, ts: List[torch.Tensor], op: str, evs, works) -> None:
        """In-place all-reduce: every input is read before any result is written."""
        fold = {"sum": torch.add, "max": torch.maximum, "min": torch.minimum, "product": torch.mul}[op]

        def run():
            acc = ts[0].clone()
            for t in ts[1:]:
                acc = fold(acc, t.to(acc.device))
            for t in ts:
                t.copy_(acc)
            return acc

        self.transfers += 1
        if not self.cuda or self.mode == "sync":
            if self.cuda:
                torch.cuda.synchronize(self.device)
            run()
            if self.cuda:
                torch.cuda.synchronize(self.device)
            for w in works:
                w.pending = 0
            return
        s = self._link(-1, -1)
        with torch.cuda.stream(s):
            for ev in evs:
                s.wait_event(ev)
            if self.delay and self.delay_model == "kernel":  # (host-timed links model point-to-point traffic)
                _Sleep.us(self.device, self._delay_us(ts[0].numel() * ts[0].element_size() * 2))
            run()
            done = torch.cuda.Event()
            done.record(s)
        for t in ts:
            t.record_stream(s)
        for w in works:
            w.events.append(done)
            w.pending = 0

    # ------------------------------------------------------------------ host values
    def host_allgather(self, rank: int, value: Any) -> List[Any]:
        """Every rank's ``value``, in rank order (a host-side collective)."""
        self._check()
        with self.cv:
            k = self._host_seq[rank]
            self._host_seq[rank] += 1
            slot = self._host.setdefault(k, {})
            slot[rank] = value
            self.cv.notify_all()
            ok = self.cv.wait_for(lambda: len(slot) == self.world or self.error is not None, timeout=self.timeout_s)
            if self.error is not None:
                raise VirtualWorldAborted(self.error)
            if not ok:
                self._abort(f"rank {rank}: host collective #{k} timed out")
                raise VirtualWorldAborted(self.error)
            return [slot[r] for r in range(self.world)]

    def modelled_link_ms(self) -> Dict[str, float]:
        return {f"{a}->{b}": us / 1e3 for (a, b), us in sorted(self.link_us.items())}


class VirtualComm(Comm):
    """``parallel.comm.Comm`` over a ``VirtualWorld`` (rank ``rank``)."""

    def __init__(self, vw: VirtualWorld, rank: int):
        self.vw = vw
        self.group = None
        self.rank, self.world = int(rank), vw.world
        self.backend = "virtual"
        self.device = vw.device
        self.bytes_sent = 0
        self.peer_bytes = [0] * self.world
        self.loopback = False  # Comm's world-1 all-to-all reads it (run_virtual(fn, 1))

    def _staged(self, t: torch.Tensor) -> bool:
        return False

    # ------------------------------------------------------------------ collectives
    def barrier(self):
        if self.vw.cuda:
            torch.cuda.current_stream(self.device).synchronize()
        self.vw.host_allgather(self.rank, None)

    def exchange_counts(self, send_counts: torch.Tensor) -> torch.Tensor:
        if self.world == 1:
            return send_counts.clone()
        recv = torch.empty_like(send_counts)
        W = self.world
        rows = send_counts.shape[0]
        if rows != W:
            raise ValueError("exchange_counts: one row per rank")
        self._a2a_post(send_counts.contiguous(), [1] * W, [1] * W, recv).wait()
        return recv

    def exchange_counts_async(self, send_counts: torch.Tensor):
        if self.world == 1:
            return send_counts.clone(), None
        recv = torch.empty_like(send_counts)
        W = self.world
        if send_counts.shape[0] != W:
            raise ValueError("exchange_counts: one row per rank")
        return recv, self._a2a_post(send_counts.contiguous(), [1] * W, [1] * W, recv)

    def _a2a_post(self, send, send_splits, recv_splits, out) -> VWork:
        ss = [int(x) for x in send_splits]
        rs = [int(x) for x in recv_splits]
        return self.vw.post_collective(self.rank, "all_to_all", (ss, rs), {"send": send, "out": out})

    def all_to_all(self, send: torch.Tensor, send_splits: Sequence[int], recv_splits: Sequence[int],
                   out: Optional[torch.Tensor] = None) -> torch.Tensor:
        n_out = int(sum(recv_splits))
        if self.world == 1:
            return super().all_to_all(send, send_splits, recv_splits, out)
        if out is None:
            out = torch.empty((n_out,) + tuple(send.shape[1:]), dtype=send.dtype, device=send.device)
        self._count(send, send_splits)
        self._a2a_post(send, send_splits, recv_splits, out[:n_out]).wait()
        return out

    def all_to_all_async(self, send: torch.Tensor, send_splits: Sequence[int], recv_splits: Sequence[int]):
        n_out = int(sum(recv_splits))
        if self.world == 1:
            return send[:n_out], None
        out = torch.empty((n_out,) + tuple(send.shape[1:]), dtype=send.dtype, device=send.device)
        self._count(send, send_splits)
        return out, self._a2a_post(send, send_splits, recv_splits, out)

    def all_reduce(self, t: torch.Tensor, op=None) -> torch.Tensor:
        if self.world > 1:
            self.vw.post_collective(self.rank, "all_reduce", (_reduce_op_name(op),), {"t": t}).wait()
        return t

    def all_gather(self, t: torch.Tensor) -> List[torch.Tensor]:
        if self.world == 1:
            return [t]
        outs = [torch.empty_like(t) for _ in range(self.world)]
        self.vw.post_collective(self.rank, "all_gather", (tuple(t.shape), str(t.dtype)),
                                {"t": t.contiguous(), "outs": outs}).wait()
        return outs

    def p2p(self, sends: Sequence, recvs: Sequence) -> list:
        for t, peer in sends:
            self.peer_bytes[peer] += t.numel() * t.element_size()
        if not sends and not recvs:
            return []
        return self.vw.post_p2p(self.rank, list(sends), list(recvs))

    # host-side values (no device round trip needed: the values live on the host)
    def max_over_ranks(self, x: float) -> float:
        return max(float(v) for v in self.vw.host_allgather(self.rank, float(x))) if self.world > 1 else x

    def gather_floats(self, x: float) -> List[float]:
        return [float(v) for v in self.vw.host_allgather(self.rank, float(x))] if self.world > 1 else [float(x)]

    def sum_over_ranks(self, x: float) -> float:
        return float(sum(self.vw.host_allgather(self.rank, float(x)))) if self.world > 1 else x


def run_virtual(fn: Callable[..., Any], world: int, *args, device=None, mode: str = "async",
                link_gbps: float = 50.0, latency_us: float = 5.0, dilate: float = 1.0, delay: bool = True,
                timeout_s: float = 300.0, return_world: bool = False, delay_model: str = "host", **kwargs):
    """Run ``fn(comm, *args, **kwargs)`` on ``world`` rank threads of one
    ``VirtualWorld``; each thread gets its own current stream.  Returns the list of
    results (and the world when ``return_world``); re-raises the first rank's error."""
    vw = VirtualWorld(world, device, mode=mode, link_gbps=link_gbps, latency_us=latency_us, dilate=dilate,
                      delay=delay, timeout_s=timeout_s, delay_model=delay_model)
    results: List[Any] = [None] * world
    errors: List[Optional[BaseException]] = [None] * world

    def body(r: int) -> None:
        try:
            if vw.cuda:
                torch.cuda.set_device(vw.device)
                s = torch.cuda.Stream(vw.device)
                with torch.cuda.stream(s):
                    results[r] = fn(vw.comm(r), *args, **kwargs)
                s.synchronize()
            else:
                results[r] = fn(vw.comm(r), *args, **kwargs)
        except BaseException as e:  # noqa: BLE001 - reported by the caller
            errors[r] = e
            vw._abort(f"rank {r} raised {type(e).__name__}: {e}")

    threads = [threading.Thread(target=body, args=(r,), name=f"vrank{r}", daemon=True) for r in range(world)]
    # N rank threads and the link thread share one interpreter: a short GIL switch
    # interval keeps a thread that just became runnable (a transfer to issue, a wait
    # that matched) from queueing behind the default 5 ms time slice of another
    import sys

    switch = sys.getswitchinterval()
    sys.setswitchinterval(5e-5)
    for t in threads:
        t.start()
    deadline = time.time() + timeout_s + 10.0  # past the waits' own timeout: they report what hung
    for t in threads:
        t.join(max(0.0, deadline - time.time()))
    vw.close()
    sys.setswitchinterval(switch)
    if any(t.is_alive() for t in threads):
        vw._abort("virtual world timed out")
        for t in threads:
            t.join(10.0)
        raise TimeoutError(f"virtual world of {world} ranks did not finish in {timeout_s} s")
    if vw.cuda:
        torch.cuda.synchronize(vw.device)
    first = next((e for e in errors if e is not None and not isinstance(e, VirtualWorldAborted)), None)
    first = first or next((e for e in errors if e is not None), None)
    if first is not None:
        raise first
    return (results, vw) if return_world else results

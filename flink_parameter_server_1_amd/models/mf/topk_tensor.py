"""Top-K recommendation apps on the tensor engine (SURVEY C34-C39 on MI355X).

* ``ps_top_k_generator_tensor`` -- ``psTopKGenerator``
  (``M/matrix/factorization/PSTopKGenerator.scala:47-107``): user vectors on the
  PS (``set`` rule; unloaded users are invalid, ``:62,74-76``), item vectors
  worker-resident (double model load, ``Right`` records), every query rating
  broadcast to all ranks (``:78-89``), partial top-``workerK`` lists gathered and
  merged with the user's seen items dropped (``CollectTopKFromEachWorker``,
  ``M/matrix/factorization/utils/CollectTopKFromEachWorker.scala:30-59``).
* ``ps_online_learner_and_generator_tensor`` -- ``psOnlineLearnerAndGenerator``
  (``M/matrix/factorization/PSOnlineMatrixFactorizationAndTopKGenerator.scala:50-100``,
  worker ``M/matrix/factorization/workers/PSOnlineMatrixFactorizationAndTopKGeneratorWorker.scala:59-166``):
  per broadcast rating the user is pulled, a top-K is served from the current
  item shards, then ONLY the rank owning the item (``item % W``) runs the SGD
  step on its local item (and negatives) and pushes the user delta to the PS,
  whose rule is ``attachLength(vectorSum(v, d))`` (``add_renorm``, K3).

Device pieces: LEMP scoring on MFMA (``LempTopK``, K8) with the pruning
strategies as candidate masks (``lemp_candidate_mask``), an ``all_gather`` of the
partial lists (X7), the merge kernel (``ops.topk_merge_cand``, K13) fed with
candidates from which the seen items were removed by a device seen store
(``SeenStore``).

Semantics inside a micro-batch: every rating of the batch is served from the
item vectors as of the batch start and the batch's SGD steps follow; with one
rating per micro-batch this is the reference's per-record order (the parity
tests run that way).
"""
from __future__ import annotations

from typing import Iterable, List, Optional

import torch

from ... import ops
from ...api.batched import BatchedWorkerLogic
from ...core.messages import Left
from ...core.tensor_engine import TensorRuntime
from ...parallel.comm import Comm
from ...ps.device_logics import DeviceSimplePSLogic
from ...utils.tracing import stage
from .core import USER_SEED_XOR
from .pruning import COORD, INCR, LC, LENGTH, LI
from .topk_fast import LempTopK


# ----------------------------------------------------------------- seen store
class SeenStore:
    """Per-user memory of the last ``memory`` recommended-for items
    (``CollectTopKFromEachWorker``'s ``seenSet`` / ``seenList``; ``memory = -1``:
    unbounded, 0: none).  Device-side: sorted ``(user << 32 | item)`` keys with
    the per-user sequence number of their latest insertion; an item is seen by a
    user iff that insertion is among the user's last ``memory`` ones.  (The
    reference drops an item from the set when its OLDEST list entry is evicted
    even if it was re-added since; here it stays excluded while any occurrence is
    inside the window -- documented deviation.)"""

    #: dense per-user rings when ``num_users * memory`` is at most this many slots
    RING_SLOTS = 1 << 28

    def __init__(self, memory: int, device, num_users: Optional[int] = None):
        """With ``num_users`` known and a small window, the store is a dense ring of
        the last ``memory`` items per user (``[num_users, memory]`` int32: O(1) add,
        O(memory) lookup -- the same window semantics); otherwise sorted keys."""
        self.memory = int(memory)
        self.device = torch.device(device)
        self.ring = None
        if num_users is not None and 0 < self.memory <= 256 and int(num_users) * self.memory <= self.RING_SLOTS:
            self.ring = torch.full((int(num_users), self.memory), -1, dtype=torch.int32, device=self.device)
            self.ring_cur = torch.zeros(int(num_users), dtype=torch.int64, device=self.device)
        self._adds = 0
        self._prune_at = 0
        self.keys = torch.zeros(0, dtype=torch.int64, device=self.device)
        self.seq = torch.zeros(0, dtype=torch.int64, device=self.device)
        self.ucount_keys = torch.zeros(0, dtype=torch.int64, device=self.device)
        self.ucount = torch.zeros(0, dtype=torch.int64, device=self.device)

    def _user_count(self, users: torch.Tensor) -> torch.Tensor:
        if self.ucount_keys.numel() == 0:
            return torch.zeros_like(users)
        i = torch.searchsorted(self.ucount_keys, users).clamp(max=self.ucount_keys.numel() - 1)
        return torch.where(self.ucount_keys[i] == users, self.ucount[i], torch.zeros_like(users))

    def contains(self, users: torch.Tensor, items: torch.Tensor) -> torch.Tensor:
        """``[B, M]`` bool: ``items[b, m]`` is in user ``users[b]``'s window."""
        if self.ring is not None:
            R = self.ring[users.long()]  # [B, memory]
            return (items.to(torch.int32).unsqueeze(2) == R.unsqueeze(1)).any(2) & (items >= 0)
        if self.memory == 0 or self.keys.numel() == 0:
            return torch.zeros(items.shape, dtype=torch.bool, device=items.device)
        u = users.long().view(-1, 1)
        key = (u << 32) | (items.long() & 0xFFFFFFFF)
        i = torch.searchsorted(self.keys, key).clamp(max=self.keys.numel() - 1)
        found = self.keys[i] == key
        if self.memory < 0:
            return found & (items >= 0)
        lo = self._user_count(users.long()).view(-1, 1) - self.memory
        return found & (self.seq[i] >= lo) & (items >= 0)

    def add(self, users: torch.Tensor, items: torch.Tensor) -> None:
        """Record one item per user, in order (users distinct within the call)."""
        if self.memory == 0 or users.numel() == 0:
            return
        users, items = users.long(), items.long()
        if self.ring is not None:
            c = self.ring_cur[users]
            self.ring[users, c % self.memory] = items.to(torch.int32)
            self.ring_cur[users] = c + 1
            return
        cnt = self._user_count(users)
        key = (users << 32) | (items & 0xFFFFFFFF)
        # keep the latest insertion of every key (keys are distinct within the call)
        self.keys, self.seq = _upsert_sorted(self.keys, self.seq, key, cnt)
        self.ucount_keys, self.ucount = _upsert_sorted(self.ucount_keys, self.ucount, users, cnt + 1)
        self._adds += users.numel()
        if self.memory > 0 and self.keys.numel() > 4096 and self._adds >= self._prune_at:
            # drop entries that left every window (now and then: O(store) each time)
            lo = self._user_count(self.keys >> 32) - self.memory
            keep = self.seq >= lo
            self.keys, self.seq = self.keys[keep], self.seq[keep]
            self._prune_at = self._adds + max(4096, self.keys.numel() // 2)


def _upsert_sorted(keys: torch.Tensor, vals: torch.Tensor, nk: torch.Tensor, nv: torch.Tensor):
    """Sorted unique ``keys`` (values ``vals``) updated with distinct keys ``nk`` ->
    values ``nv``: existing keys take the new value, new keys are merged in order.
    O(store + batch) (searchsorted + two scatters) instead of re-sorting the store."""
    o = torch.argsort(nk)
    nk, nv = nk[o], nv[o]
    N = keys.numel()
    if N:
        i = torch.searchsorted(keys, nk).clamp(max=N - 1)
        hit = keys[i] == nk
        vals = vals.clone()
        vals[i[hit]] = nv[hit]
        fresh = ~hit
        nk, nv = nk[fresh], nv[fresh]
    n = nk.numel()
    if n == 0:
        return keys, vals
    dev = nk.device
    out_k = torch.empty(N + n, dtype=nk.dtype, device=dev)
    out_v = torch.empty(N + n, dtype=nv.dtype, device=dev)
    if N:
        at = torch.arange(N, device=dev) + torch.searchsorted(nk, keys)
        out_k[at] = keys
        out_v[at] = vals
    at = torch.arange(n, device=dev) + torch.searchsorted(keys, nk)
    out_k[at] = nk
    out_v[at] = nv
    return out_k, out_v


def occurrence_rounds(users: torch.Tensor) -> torch.Tensor:
    """Round of every entry: 0 for a user's first entry in the batch, 1 for its
    second ... (rounds are processed in order, each holding a user at most once)."""
    order = torch.argsort(users, stable=True)
    su = users[order]
    start = torch.ones_like(su, dtype=torch.bool)
    if su.numel() > 1:
        start[1:] = su[1:] != su[:-1]
    idx = torch.arange(su.numel(), device=users.device)
    run_start = torch.cummax(torch.where(start, idx, torch.zeros_like(idx)), 0).values
    rnd = torch.empty_like(idx)
    rnd[order] = idx - run_start
    return rnd


class RoundPlan:
    """The occurrence rounds of a micro-batch's users, planned when the batch is
    RECEIVED: entries ordered by round (stable: batch order inside a round) and the
    per-round counts copied to pinned host memory behind an event.  By the time
    the batch's answer is served (one micro-batch later on a pipelined engine)
    the counts are on the host, so the merge loop over rounds issues no
    device->host sync -- the same trick as the PS count exchange
    (``parallel.tensor_ps``)."""

    def __init__(self, users: torch.Tensor, fused: bool = False):
        """``fused``: plan for the one-launch merge (``ops.topk_seen_merge``): per entry
        its round, its user's entry count and the position of the user's first entry in
        the user-sorted order -- no rounds, no host copy."""
        B = users.numel()
        self.fused = fused
        if fused and users.is_cuda and B <= (1 << 20):  # one kernel after the sort
            self.by_user, self.rnd, self.first, self.nu = ops.round_plan(users)
            return
        if fused:
            by_user = torch.argsort(users, stable=True)
            su = users[by_user]
            start = torch.ones(B, dtype=torch.bool, device=users.device)
            if B > 1:
                start[1:] = su[1:] != su[:-1]
            idx = torch.arange(B, device=users.device)
            run_start = torch.cummax(torch.where(start, idx, torch.zeros_like(idx)), 0).values
            run_id = torch.cumsum(start, 0) - 1
            run_len = torch.zeros(B, dtype=torch.int32, device=users.device)
            run_len.index_add_(0, run_id, torch.ones(B, dtype=torch.int32, device=users.device))
            self.by_user = by_user
            self.rnd = torch.empty(B, dtype=torch.int32, device=users.device)
            self.rnd[by_user] = (idx - run_start).to(torch.int32)
            self.first = torch.empty(B, dtype=torch.int32, device=users.device)
            self.first[by_user] = run_start.to(torch.int32)
            self.nu = torch.empty(B, dtype=torch.int32, device=users.device)
            self.nu[by_user] = run_len[run_id]
            return
        rnd = occurrence_rounds(users)
        self.order = torch.argsort(rnd, stable=True)
        cnt = torch.zeros(B + 1, dtype=torch.int32, device=users.device)
        cnt.index_add_(0, rnd, torch.ones_like(rnd, dtype=torch.int32))
        if users.is_cuda:
            self._host = torch.empty(B + 1, dtype=torch.int32, pin_memory=True)
            self._host.copy_(cnt, non_blocking=True)
            self._event = torch.cuda.Event()
            self._event.record()
        else:
            self._host, self._event = cnt, None

    def rounds(self) -> List[tuple]:
        """``[(start, n)]`` slices of ``order``, one per non-empty round, in order."""
        if self._event is not None:
            self._event.synchronize()
        out, a = [], 0
        for n in self._host.tolist():
            if n == 0:
                break  # rounds are dense: round r exists only if round r-1 does
            out.append((a, n))
            a += n
        return out


# ------------------------------------------------------------- LEMP pruning
def _theta(best_s: torch.Tensor) -> torch.Tensor:
    """k-th best so far; 0 while fewer than k candidates were kept (the reference's
    ``if (topK.length < K) 0.0 else topK.head._1``)."""
    t = best_s[:, -1]
    return torch.where(torch.isfinite(t), t, torch.zeros_like(t))


def lemp_candidate_mask(Q: torch.Tensor, qlen: torch.Tensor, theta: torch.Tensor, X: torch.Tensor,
                        xlen: torch.Tensor, strategy, reference_quirks: bool = False) -> torch.Tensor:
    """``[B, n]`` bool: candidates the LEMP strategy keeps for a length-sorted
    bucket ``X`` (``M/matrix/factorization/pruning/LEMPPruningFunctions.scala:20-89``,
    selection as ``M/matrix/factorization/workers/PSTopKGeneratorWorker.scala:72-96``).
    The bound is exact, so masking only skips work; the top-K is unchanged."""
    B, n = Q.shape[0], X.shape[0]
    head, last = float(xlen[0]), float(xlen[-1])
    if isinstance(strategy, (LC, LI)):
        use_len = head > last * strategy.algorithm_switch_threshold
        if use_len:
            strategy = LENGTH()
        else:
            strategy = COORD() if isinstance(strategy, LC) else INCR(strategy.num_focus_coordinates)
    if isinstance(strategy, LENGTH):
        mn = theta / qlen.clamp_min(1e-30)
        x2 = (xlen * xlen).view(1, -1)
        if reference_quirks:  # squared length vs the unsquared bound
            return x2 >= mn.view(-1, 1)
        bound = torch.where(mn > 0, mn * mn, torch.full_like(mn, float("-inf")))
        return x2 >= bound.view(-1, 1)
    if isinstance(strategy, COORD):
        denom = head * qlen
        tbq = torch.where(denom > 0, theta / denom.clamp_min(1e-30), torch.zeros_like(theta))
        f = torch.argmax(Q * Q, dim=1)
        qf = Q.gather(1, f.view(-1, 1)).view(-1)
        qbf = torch.where(qlen > 0, qf / qlen.clamp_min(1e-30), torch.zeros_like(qf))
        a = qbf * tbq
        b = torch.sqrt(torch.clamp((1 - tbq * tbq) * (1 - qbf * qbf), min=0.0))
        lfp, ufp = a - b, a + b
        ratio = torch.where(qbf != 0, tbq / torch.where(qbf != 0, qbf, torch.ones_like(qbf)),
                            torch.full_like(qbf, float("inf")))
        lf = torch.where((qbf >= 0) | (lfp > ratio), lfp, torch.full_like(lfp, -1.0))
        uf = torch.where((qbf <= 0) | (ufp < ratio), ufp, torch.full_like(ufp, 1.0))
        pf = X.t()[f]  # [B, n]: coordinate f of every item
        pbf = torch.where(xlen.view(1, -1) > 0, pf / xlen.clamp_min(1e-30).view(1, -1), torch.zeros_like(pf))
        return (lf.view(-1, 1) <= pbf) & (pbf <= uf.view(-1, 1))
    if isinstance(strategy, INCR):
        D = Q.shape[1]
        d = D - 1 if reference_quirks else D  # the reference skips the last coordinate
        nf = min(strategy.num_focus_coordinates, d)
        F = torch.argsort(-(Q[:, :d] * Q[:, :d]), dim=1, stable=True)[:, :nf]
        M = torch.zeros_like(Q).scatter_(1, F, 1.0)  # focus-set mask per query
        QF = Q * M
        q_mF_sqr = qlen * qlen - (QF * QF).sum(1)
        qFpF = QF @ X.t()                        # [B, n]
        pF_sqr = M @ (X * X).t()                 # [B, n]
        ub = theta.view(-1, 1) - qFpF
        return (ub < 0) | (q_mF_sqr.view(-1, 1) * ((xlen * xlen).view(1, -1) - pF_sqr) >= ub * ub)
    raise ValueError(f"unknown LEMP strategy {strategy!r}")


class PrunedLempTopK(LempTopK):
    """LEMP top-K with a pruning strategy (``M/matrix/factorization/workers/PSTopKGeneratorWorker.scala:35-114``).

    The reference prunes with ``theta = 0`` until a query holds ``workerK``
    candidates (``if (topK.length < K) 0.0 else topK.head._1``), which can drop
    negative-score items; once every query's k-th best is positive its bounds are
    exact.  So the scan runs the reference's bucket loop with the strategy's masks
    (torch, one host check per bucket) only until every query's k-th best is
    positive -- the first bucket on real data -- and continues with the device scan
    (``LempTopK(strategy=...)``): the length bound and, for COORD / LC, the
    focus-coordinate bound per block of 32 items inside the bf16 scorer, no host
    sync per bucket.  ``reference_quirks`` (inexact LENGTH / INCR bounds, SURVEY
    B6 / B7) keeps the mask loop for the whole scan (bit parity only).  ``pruned``
    / ``scored`` count the mask loop's candidates, ``coord_stats`` the device
    scan's (32 x 32) block pairs."""

    #: device scan segments (the reference's ``bucketSize`` is an algorithmic knob of
    #: its per-item loop; on MFMA tiles it only sizes the launches)
    DEVICE_BUCKET = 65536

    def __init__(self, item_ids, item_vecs, bucket_size: int = 4096, strategy=None, reference_quirks=False,
                 growth=None):
        super().__init__(item_ids, item_vecs, max(bucket_size, self.DEVICE_BUCKET), strategy=strategy, growth=growth)
        self.ref_bucket = int(bucket_size)
        self.strategy, self.quirks = strategy, reference_quirks
        self.pruned = 0
        self.scored = 0

    def query(self, Q: torch.Tensor, k: int, exclude=None, copy: bool = True):
        if self.strategy is None:
            return super().query(Q, k, copy=copy)
        Q = Q.float().contiguous()
        best_s, best_i, s0 = self._mask_scan(Q, k, settle=not self.quirks)
        if s0 < self.vecs.shape[0]:
            best_s, best_i = super().query(Q, k, start=s0, state=(best_s, best_i))
        best_i = torch.where(torch.isfinite(best_s), best_i, torch.full_like(best_i, -1))
        return best_s, best_i

    def _mask_scan(self, Q: torch.Tensor, k: int, settle: bool):
        """The reference's bucket loop with the strategy's masks; with ``settle`` it
        stops after the first bucket that leaves every query's k-th best positive.
        Returns ``(best_s, best_i, next item position)``."""
        B, dev = Q.shape[0], Q.device
        qlen = torch.linalg.vector_norm(Q, dim=1)
        best_s = torch.full((B, k), float("-inf"), device=dev)
        best_i = torch.full((B, k), -1, dtype=torch.long, device=dev)
        N = self.vecs.shape[0]
        for s in range(0, N, self.ref_bucket):
            e = min(N, s + self.ref_bucket)
            theta = _theta(best_s)
            full = torch.isfinite(best_s[:, -1])
            if s > 0 and bool((full & (qlen * self.lengths[s] <= theta)).all()):
                return best_s, best_i, N
            self.buckets_scanned += 1
            X, xl = self.vecs[s:e], self.lengths[s:e]
            S = ops.score_gemm(Q, X) if dev.type == "cuda" else Q @ X.t()
            keep = lemp_candidate_mask(Q, qlen, theta, X, xl, self.strategy, self.quirks)
            # queries already settled (reference: the bucket loop stopped) take nothing more
            live = ~(full & (qlen * self.lengths[s] <= theta))
            keep &= live.view(-1, 1)
            self.scored += int(keep.sum())
            self.pruned += int(keep.numel() - keep.sum())
            S = torch.where(keep, S, torch.full_like(S, float("-inf")))
            if dev.type == "cuda" and k <= ops.TOPK_MAX_K:
                ops.topk_merge(S.contiguous(), self.ids[s:e], best_s, best_i)
            else:
                cs = torch.cat([best_s, S], 1)
                ts, tj = torch.topk(cs, min(k, cs.shape[1]), dim=1)
                ci = torch.cat([best_i, self.ids[s:e].expand(B, e - s)], 1)
                best_s, best_i = ts, torch.gather(ci, 1, tj)
            if settle and bool((best_s[:, -1] > 0).all()):
                return best_s, best_i, e
        return best_s, best_i, N


# ------------------------------------------------------------------ merging
def _fkey(s: torch.Tensor) -> torch.Tensor:
    """Order-preserving float -> uint32 key (int32 storage), as ``fkey`` in topk.hip."""
    u = s.contiguous().view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    k = torch.where(u >= 0x80000000, (~u) & 0xFFFFFFFF, u | 0x80000000)
    return torch.where(k >= 0x80000000, k - (1 << 32), k).to(torch.int32)


def merge_partials(scores: torch.Tensor, ids: torch.Tensor, K: int, excluded: torch.Tensor):
    """Merge gathered partial lists ``[B, m]`` into the best ``K`` with ``excluded``
    entries (seen items, empty slots) removed (K13: ``ops.topk_merge_cand`` on the
    GPU -- the kept candidates are compacted to the front of each row first)."""
    B, m = scores.shape
    dev = scores.device
    if m < K:  # fewer candidates than K: pad (the list is shorter, as in the reference)
        pad = K - m
        scores = torch.cat([scores, torch.full((B, pad), float("-inf"), device=dev)], 1)
        ids = torch.cat([ids, torch.full((B, pad), -1, dtype=ids.dtype, device=dev)], 1)
        excluded = torch.cat([excluded, torch.ones((B, pad), dtype=torch.bool, device=dev)], 1)
        m = K
    keep = ~excluded & (ids >= 0) & torch.isfinite(scores)
    if dev.type == "cuda" and K <= ops.TOPK_MAX_K and m <= ops.TOPK_CAND_CAP:
        order = torch.argsort((~keep).to(torch.int8), dim=1, stable=True)  # kept candidates first
        ck = _fkey(torch.gather(scores, 1, order))
        ci = torch.gather(ids.long(), 1, order)
        cnt = keep.sum(1).to(torch.int32)
        best_s = torch.full((B, K), float("-inf"), device=dev)
        best_i = torch.full((B, K), -1, dtype=torch.long, device=dev)
        ops.topk_merge_cand(ck.contiguous(), ci.contiguous(), cnt, best_s, best_i)
    else:
        s = torch.where(keep, scores, torch.full_like(scores, float("-inf")))
        best_s, j = torch.topk(s, min(K, m), dim=1)
        best_i = torch.gather(ids.long(), 1, j)
    best_i = torch.where(torch.isfinite(best_s), best_i, torch.full_like(best_i, -1))
    return best_s, best_i


def _gather_partials(comm: Comm, s: torch.Tensor, i: torch.Tensor):
    if comm.world == 1:
        return s, i
    return torch.cat(comm.all_gather(s.contiguous()), 1), torch.cat(comm.all_gather(i.contiguous()), 1)


def as_reference_records(outputs) -> List[tuple]:
    """Rank 0's tensor outputs -> the reference's ``(user, item, ts, [(score, item)])``
    records (``CollectTopKFromEachWorker`` output order)."""
    recs = []
    for e in outputs:
        if not isinstance(e, Left) or not isinstance(e.value, tuple) or len(e.value) != 3:
            continue
        (u, it, ts), S, I = e.value
        S, I = S.cpu().tolist(), I.cpu().tolist()
        for b, (uu, ii, tt) in enumerate(zip(u.tolist(), it.tolist(), ts.tolist())):
            recs.append((uu, ii, tt, [(float(x), int(y)) for x, y in zip(S[b], I[b]) if y >= 0]))
    return recs


class _TopKServing:
    """Shared query path: partial LEMP top-K on the local items, gather, seen-aware merge."""

    def _fused_merge(self, ss: Optional[torch.Tensor] = None) -> bool:
        """The one-launch merge applies: dense ring seen store on the GPU, lists and K
        within the kernel's LDS capacity."""
        seen = getattr(self, "seen", None)
        if not getattr(self, "fused", True) or seen is None or seen.ring is None or not seen.ring.is_cuda or self.K > ops.TOPK_MAX_K \
                or seen.memory > ops.TOPK_MAX_K:
            return False
        return ss is None or ss.shape[1] <= ops.TOPK_CAND_CAP

    def _serve(self, Q, valid, users, items, ts, ps, plan: Optional[RoundPlan] = None):
        with stage("topk.score", None):
            if self.index is not None and self.index.vecs.shape[0] > 0:
                # the partial lists are consumed on the stream within this batch (merge,
                # seen merge), before the next replay of the scan rewrites them: no copies
                s, i = self.index.query(Q, self.worker_k, copy=False)
            else:
                s = torch.full((Q.shape[0], self.worker_k), float("-inf"), device=Q.device)
                i = torch.full((Q.shape[0], self.worker_k), -1, dtype=torch.long, device=Q.device)
            if valid is not None:  # None: every query row is valid
                s = torch.where(valid.view(-1, 1), s, torch.full_like(s, float("-inf")))
                i = torch.where(valid.view(-1, 1), i, torch.full_like(i, -1))
        with stage("topk.merge", None):
            ss, ii = _gather_partials(self.comm, s, i)
            if plan is not None and plan.fused and self._fused_merge(ss):
                # every round in one launch + the ring update (topk.hip seen_merge_kernel)
                best_s, best_i = ops.topk_seen_merge(ss.contiguous(), ii.long().contiguous(), self.K, users.long(),
                                                     items.long(), plan.rnd, plan.first, plan.nu, plan.by_user,
                                                     self.seen.ring, self.seen.ring_cur)
                if self.rank == 0:
                    ps.output(((users, items, ts), best_s, best_i))
                return
            plan = plan if plan is not None and not plan.fused else RoundPlan(users)
            best_s = torch.empty((users.numel(), self.K), device=Q.device)
            best_i = torch.empty((users.numel(), self.K), dtype=torch.long, device=Q.device)
            for a, n in plan.rounds():  # a user's later entries see its earlier ones as seen
                sel = plan.order[a:a + n]
                exc = self.seen.contains(users[sel], ii[sel])
                bs, bi = merge_partials(ss[sel], ii[sel], self.K, exc)
                best_s[sel], best_i[sel] = bs, bi
                self.seen.add(users[sel], items[sel])  # the rated item counts as seen afterwards
        if self.rank == 0:  # the merge of the reference runs at parallelism 1
            ps.output(((users, items, ts), best_s, best_i))


class TopKQueryWorker(BatchedWorkerLogic, _TopKServing):
    """``PSTopKGeneratorWorker`` + the gather/merge; batches are ``(user, item, ts)``
    tensors, identical on every rank (broadcast input)."""

    pushes = False

    def __init__(self, K: int = 100, worker_k: int = 75, memory: int = 0, bucket_size: int = 4096, pruning=None,
                 reference_quirks: bool = False, num_users: Optional[int] = None):
        self.K, self.worker_k, self.memory, self.num_users = K, worker_k, memory, num_users
        self.bucket_size, self.pruning, self.quirks = bucket_size, pruning, reference_quirks
        self._ids: List[torch.Tensor] = []
        self._vecs: List[torch.Tensor] = []
        self.index = None

    def open(self, ctx):
        self.rank, self.device = ctx.rank, torch.device(ctx.device)
        self.comm = getattr(ctx, "comm", None) or Comm(device=self.device)
        self.seen = SeenStore(self.memory, self.device, self.num_users)

    def update_model_batch(self, ids, values):
        """Worker-resident items ``(id, [vec..., len])`` or ``(id, vec)``."""
        self._ids.append(ids.to(self.device).long())
        self._vecs.append(values.to(self.device).float())
        self.index = None

    def _build(self, D):
        if self.index is None and self._ids:
            ids, vecs = torch.cat(self._ids), torch.cat(self._vecs)
            if vecs.shape[1] == D + 1:
                vecs = vecs[:, :D]
            self.index = PrunedLempTopK(ids, vecs, self.bucket_size, self.pruning, self.quirks)

    def on_recv_batch(self, batch, ps):
        users, items, ts = (t.to(self.device) for t in batch)
        ps.pull(users, (users, items, ts, RoundPlan(users, fused=self._fused_merge())))

    def on_pull_recv_batch(self, pulled, ps):
        users, items, ts, plan = pulled.payload
        rows = pulled.values()
        D = rows.shape[1] - 1
        valid = rows[:, D] >= 0  # (len, vec) stores; len -1 = invalid (never loaded)
        self._build(D)
        self._serve(rows[:, :D].contiguous(), valid, users, items, ts, ps, plan)


def ps_top_k_generator_tensor(queries: Iterable, ps_model, worker_model, num_users: int, num_factors: int = 10,
                              user_memory: int = 0, K: int = 100, worker_k: int = 75, bucket_size: int = 4096,
                              pruning_algorithm=None, comm: Optional[Comm] = None, reference_quirks: bool = False,
                              capacity: Optional[int] = None):
    """``psTopKGenerator`` on the tensor engine (this rank's part of the job).

    ``queries``: the broadcast ``(user, item, ts)`` micro-batches (the same on every
    rank); ``ps_model``: this rank's ``(user, [vec..., len])`` records (``Left``);
    ``worker_model``: this rank's ``(item, [vec..., len])`` records (``Right``).
    Returns rank 0's ``Left(((user, item, ts), scores [B, K], items [B, K]))``.
    ``capacity`` (the largest micro-batch): fixed-shape PS plans -- at W > 1 no
    micro-batch waits for a count exchange on the host."""
    worker = TopKQueryWorker(K, worker_k, user_memory, bucket_size, pruning_algorithm, reference_quirks, num_users)
    logic = DeviceSimplePSLogic(num_users, num_factors + 1, op="set", init=("const", -1.0), track_touched=False)
    logic.emit = "none"
    rt = TensorRuntime(comm, staleness=0, capacity=capacity)
    return rt.execute(queries, worker, logic, model=ps_model, worker_model=worker_model)


class OnlineMFTopKWorker(BatchedWorkerLogic, _TopKServing):
    """``PSOnlineMatrixFactorizationAndTopKGeneratorWorker`` on device tensors.

    Item ``i`` lives on rank ``i % W`` (local row ``i // W``), initialised on first
    use by its owner (deterministic hash init by id, so the value does not depend
    on when it is first touched).  Per micro-batch: serve top-K for every rating
    (current items), then the owned ratings' SGD: negatives drawn among this
    rank's initialised items (<= 32 rejections against the user's recent items on
    this rank), item rows updated in place, the summed user delta pushed.

    The LEMP index over the initialised items is built once and then kept current
    in place (``LempTopK.update_rows`` on the rows the SGD touched); it is rebuilt
    when new items were initialised and re-sorted every ``resort_every`` batches.
    Non-owned ratings ride through the SGD masked (no compaction, no host sync)."""

    def __init__(self, num_items: int, num_factors: int, learning_rate: float, K: int = 100, worker_k: int = 75,
                 memory: int = 65535, negative_sample_rate: int = 0, bucket_size: int = 4096, pruning=None,
                 range_min: float = -0.001, range_max: float = 0.001, seed: int = 0, neg_memory: int = 128,
                 reference_quirks: bool = False, prefill_items: bool = False, num_users: Optional[int] = None,
                 resort_every: int = 64):
        """``prefill_items``: every owned item counts as initialised from the start
        (a warm catalogue, e.g. a benchmark) instead of on its first rating.
        ``num_users`` (optional) lets the seen store use dense per-user rings."""
        self.num_items, self.dim, self.lr = int(num_items), int(num_factors), learning_rate
        self.K, self.worker_k, self.memory = K, worker_k, memory
        self.neg_rate, self.bucket_size, self.pruning, self.quirks = negative_sample_rate, bucket_size, pruning, \
            reference_quirks
        self.range, self.seed, self.neg_memory = (range_min, range_max), seed, int(neg_memory)
        self.prefill_items, self.num_users, self.resort_every = prefill_items, num_users, int(resort_every)
        self.served = 0
        #: GPU: one-launch seen-aware merge and one launch per SGD phase (``mf_online.hip``);
        #: False keeps the torch chains (the A/B and parity reference)
        self.fused = True
        self._trained = None  # device counter of SGD updates on this rank (ratings + drawn negatives)
        self.rebuilds = 0

    def open(self, ctx):
        from ...parallel.table import ShardedTable

        self.W, self.rank, self.device = ctx.world_size, ctx.rank, torch.device(ctx.device)
        self.comm = getattr(ctx, "comm", None) or Comm(device=self.device)
        self._trained = torch.zeros((), dtype=torch.int64, device=self.device)
        self.seen = SeenStore(self.memory, self.device, self.num_users)
        self.items = ShardedTable(self.num_items, self.dim, self.rank, self.W, "hash",
                                  ("uniform", self.range[0], self.range[1]), (self.seed ^ USER_SEED_XOR) & 0xFFFFFFFF,
                                  self.device, track_touched=False)
        n = self.items.n_local
        # one spare slot: masked writes of non-owned ratings land there
        self._valid_buf = torch.full((n + 1,), bool(self.prefill_items), dtype=torch.bool, device=self.device)
        self.valid = self._valid_buf[:n]
        self.index = None
        self._stale = True      # the index must be (re)built before the next query
        self._since_sort = 0
        if self.neg_rate > 0:
            n_u = 1 << 20  # per-user rings are keyed by user id modulo this (bounded state; a power of 2)
            self._ring_users = n_u
            self._ring = torch.full((n_u * self.neg_memory,), -1, dtype=torch.int32, device=self.device)
            self._ring_cur = torch.zeros(n_u, dtype=torch.int32, device=self.device)
            self._known_flag = torch.zeros(self.num_items, dtype=torch.int32, device=self.device)
            self._known = torch.zeros(self.num_items, dtype=torch.int32, device=self.device)
            self._known_cnt = torch.zeros(1, dtype=torch.int32, device=self.device)
            self._neg_counter = 0

    def on_recv_batch(self, batch, ps):
        users, items, ts, rating = (t.to(self.device) for t in batch)
        ps.pull(users, (users, items, ts, rating.float(), RoundPlan(users, fused=self._fused_merge())))

    @property
    def trained(self) -> int:
        """SGD updates applied on this rank so far (owned ratings + drawn negatives);
        reading it synchronises with the device."""
        return 0 if self._trained is None else int(self._trained.item())

    def _rebuild_index(self):
        loc = torch.nonzero(self.valid).flatten()
        ids = self.items.global_ids(loc)
        # growth 2: the index is updated in place every batch (refresh_from), its length order
        # goes stale, the bound cuts less, and doubling keeps the candidate lists short
        # (growth 4: 2.04-2.13e6 vs 2.19-2.21e6 q/s, profiles/r5_topk_growth_ab.txt)
        self.index = PrunedLempTopK(ids, self.items.weight[loc], self.bucket_size, self.pruning, self.quirks,
                                    growth=2) if loc.numel() else None
        self.rebuilds += 1
        self._stale = False
        self._since_sort = 0
        if self.index is not None:
            self._index_rows = loc[self.index.order]  # index position -> local row
            self._pos = torch.full((self.items.n_local,), -1, dtype=torch.long, device=self.device)
            self._pos[self._index_rows] = torch.arange(loc.numel(), device=self.device)

    def _refresh_index(self, rows: torch.Tensor):
        """Write the current vectors of local ``rows`` (initialised items; repeats and
        spurious rows are harmless: every write is the row's current value) into the index."""
        if self.index is None or self._stale:
            return
        if self.pruning is not None or self._since_sort >= self.resort_every:
            self._stale = True  # LEMP strategies read the sorted order: rebuild instead
            return
        if rows.is_cuda:
            self.index.refresh_from(rows.long(), self._pos, self.items.weight)
            return
        p = self._pos[rows]
        ok = p >= 0
        rows = torch.where(ok, rows, self._index_rows[0])
        p = torch.where(ok, p, torch.zeros_like(p))
        self.index.update_rows(p, self.items.weight[rows])

    def on_pull_recv_batch(self, pulled, ps):
        users, items, ts, rating, plan = pulled.payload
        U = pulled.values()  # [B, D] user vectors (length recomputed on the worker)
        self.served += users.numel()
        if self._stale or self.index is None:
            self._rebuild_index()
        self._since_sort += 1
        self._serve(U, None, users, items, ts, ps, plan)
        # learning: the owner of each rated item (non-owned rows masked, not compacted)
        n = self.items.n_local
        if self.W == 1:  # every item is local, row = id (no ownership mask: every row is pushed)
            own = None
            loc = items.long()
        else:
            own = (items.long() % self.W) == self.rank
            loc = torch.where(own, items.long() // self.W, torch.zeros_like(items, dtype=torch.long))
        if not self.prefill_items:
            # a first rating initialises the item: the index must take it in (one sync)
            fresh = ~self.valid[loc] if own is None else own & ~self.valid[loc]
            if bool(fresh.any()):
                self._stale = True
            self._valid_buf[loc if own is None else torch.where(own, loc, torch.full_like(loc, n))] = True
        du = torch.zeros_like(U)
        lr = self.lr
        W_ = self.items.weight
        touched = [loc]
        if self.fused and U.is_cuda and W_.dtype == torch.float32 and self.dim <= 256:
            self._learn_fused(U, users, items, rating, own, loc, du)
            ps.push(du, mask=own)  # None at W == 1: the engine's unmasked accumulate (fewer launches)
            return
        if own is None:
            own = torch.ones(items.shape, dtype=torch.bool, device=items.device)
        if self.neg_rate > 0:
            rows_own = torch.arange(users.numel(), device=U.device) if self.W == 1 else torch.nonzero(own).flatten()
            ou, oi = users[rows_own].to(torch.int32), items[rows_own].to(torch.int32)
            uring = ou & (self._ring_users - 1)  # user id mod 2^20 (ids >= 0): one op, not three
            ops.ring_push(self._ring, self._ring_cur, uring, oi, self.neg_memory)
            ops.known_append(self._known_flag, self._known, self._known_cnt, oi)
            negs = ops.sample_uniform_reject(ou.numel(), self.neg_rate, self.num_items, oi, uring, self._ring,
                                             self.neg_memory, seed=self.seed + 7 * self.rank,
                                             counter=self._neg_counter, device=self.device, known=self._known,
                                             known_count=self._known_cnt).view(-1, self.neg_rate)
            self._neg_counter += 1
            Ub = U[rows_own]
            for j in range(self.neg_rate):  # reference order: negatives first, then the rating
                ng = negs[:, j].long()
                okf = (ng >= 0).to(U.dtype).view(-1, 1)
                nl = torch.where(ng >= 0, ng // self.W, torch.zeros_like(ng))
                iv = W_[nl]
                e = 0.0 - (Ub * iv).sum(1, keepdim=True)
                du.index_add_(0, rows_own, lr * e * iv * okf)
                W_.index_add_(0, nl, lr * e * Ub * okf)
                touched.append(nl)
                self._trained += (ng >= 0).sum()
        ownf = own.to(U.dtype).view(-1, 1)
        iv = W_[loc]
        e = rating.view(-1, 1) - (U * iv).sum(1, keepdim=True)
        du += lr * e * iv * ownf
        W_.index_add_(0, loc, lr * e * U * ownf)
        self._refresh_index(torch.cat(touched))
        self._trained += own.sum()
        ps.push(du, mask=own)


    def _learn_fused(self, U, users, items, rating, own, loc, du):
        """The learning side on the GPU: one ``mf_online_phase`` launch per negative
        and one for the ratings (the torch chain's batch semantics: a phase reads the
        item rows as the previous phases left them), then one index refresh."""
        W_ = self.items.weight
        U = U.float().contiguous()
        touched = [loc]
        if self.neg_rate > 0:
            rows_own = None if self.W == 1 else torch.nonzero(own).flatten()
            ou = users if rows_own is None else users[rows_own]
            oi = items if rows_own is None else items[rows_own]
            ou, oi = ou.to(torch.int32), oi.to(torch.int32)
            uring = ou & (self._ring_users - 1)  # user id mod 2^20 (ids >= 0): one op, not three
            ops.ring_push(self._ring, self._ring_cur, uring, oi, self.neg_memory)
            ops.known_append(self._known_flag, self._known, self._known_cnt, oi)
            negs = ops.sample_uniform_reject(ou.numel(), self.neg_rate, self.num_items, oi, uring, self._ring,
                                             self.neg_memory, seed=self.seed + 7 * self.rank,
                                             counter=self._neg_counter, device=self.device, known=self._known,
                                             known_count=self._known_cnt).view(-1, self.neg_rate).long()
            self._neg_counter += 1
            # [n_own, neg_rate] local rows, -1 = no negative drawn
            nl = negs if self.W == 1 else torch.where(negs >= 0, negs // self.W, torch.full_like(negs, -1))
            nlt = nl.t().contiguous()  # phase-major
            for j in range(self.neg_rate):  # reference order: negatives first, then the rating
                ops.mf_online_phase(U, rows_own, nlt[j], None, self.lr, W_, du, self._trained)
            touched.append(nlt.view(-1))
        irow = loc if self.W == 1 else torch.where(own, loc, torch.full_like(loc, -1))
        ops.mf_online_phase(U, None, irow.contiguous(), rating, self.lr, W_, du, self._trained)
        self._refresh_index(torch.cat(touched))


def ps_online_learner_and_generator_tensor(batches: Iterable, num_users: int, num_items: int, num_factors: int = 10,
                                           range_min: float = -0.001, range_max: float = 0.001,
                                           learning_rate: float = 0.01, negative_sample_rate: int = 0,
                                           user_memory: int = 65535, K: int = 100, worker_k: int = 75,
                                           bucket_size: int = 4096, pruning_algorithm=None, seed: int = 0,
                                           comm: Optional[Comm] = None, output_sink=None,
                                           capacity: Optional[int] = None):
    """``psOnlineLearnerAndGenerator`` on the tensor engine (this rank's part):
    ``batches`` = the broadcast ``(user, item, ts, rating)`` micro-batches (same on
    every rank).  Outputs: rank 0's top-K records (``Left``) and every rank's PS
    user updates ``Right((users, vectors))`` (``SimplePSLogic`` emits on push).
    ``capacity`` (the largest micro-batch): fixed-shape PS plans (no per-batch count
    exchange read on the host at W > 1)."""
    worker = OnlineMFTopKWorker(num_items, num_factors, learning_rate, K, worker_k, user_memory,
                                negative_sample_rate, bucket_size, pruning_algorithm, range_min, range_max, seed,
                                num_users=num_users)
    logic = DeviceSimplePSLogic(num_users, num_factors, op="add_renorm", init=("uniform", range_min, range_max),
                                seed=seed)
    rt = TensorRuntime(comm, staleness=0, output_sink=output_sink, capacity=capacity)
    return rt.execute(batches, worker, logic)

"""Top-K recommendation on the GPU: LEMP bucket scan with MFMA scoring (K8) + merge (K13).

The reference's top-K worker (``M/matrix/factorization/workers/PSTopKGeneratorWorker.scala:35-114``)
scans length-sorted buckets of worker-resident item vectors per query user,
stops when ``|bucket head| * |u| <= k-th best score`` and filters candidates
with LEMP pruning (``M/matrix/factorization/pruning/LEMPPruningFunctions.scala``).
On MI355X a whole query *batch* is scored against a bucket with one MFMA GEMM
(``ops.score_gemm``), merged into the running top-K (``torch.topk`` on
``[B, k + bucket]``), and the LEMP length bound is applied per query at bucket
granularity: the scan stops once every query in the batch is settled.  The
result is exact (equal to brute force), which is what the CPU pruning
strategies also guarantee; they only change how much work is skipped.

On the GPU the fused scan runs on bf16 MFMA by default: ``ops.score_filter_bf16``
lists every item whose bf16 score is within a proven rounding margin of the
query's k-th best, ``ops.cand_rescore`` recomputes those candidates with the fp32
MFMA chain of the fp32 scorer (bit-identical keys), and the merge is unchanged --
the same top-K as the fp32 scan at ~2x the rate (``profiles/r2_bf16_topk.md``).

``DistributedTopK`` reproduces the scatter-gather of ``psTopKGenerator`` /
``psOnlineLearnerAndGenerator``: item vectors are sharded over the ranks
(worker-resident), every rank scores the same broadcast query batch against
its shard, partial top-Ks are ``all_gather``-ed and merged with the users'
seen items excluded (``CollectTopKFromEachWorker``, ``M/matrix/factorization/utils/CollectTopKFromEachWorker.scala:41-45``).
"""
from __future__ import annotations

import os
from typing import Optional

import torch

from ... import ops


def _row_norms(Q: torch.Tensor) -> torch.Tensor:
    """|q| per row.  ``torch.linalg.vector_norm`` over the rows of a [4096, 64] batch ran
    as a 60 us reduction kernel (``profiles/r4_mf_topk_fused_kernel_stats.csv``); the
    bounds that use it carry a relative slack, so the summation order is free."""
    return Q.square().sum(1).sqrt_()


class LempTopK:
    #: items scored unfused first (their merge sets every query's k-th best)
    seed_items = 4096
    #: largest fused segment (segments double from ``seed_items``)
    max_segment = 1 << 19

    def __init__(self, item_ids: torch.Tensor, item_vecs: torch.Tensor, bucket_size: int = 65536, strategy=None,
                 growth: Optional[int] = None):
        """``strategy`` (a ``pruning`` LEMP strategy; None = LENGTH): the bounds the
        device scan applies per block of 32 items before scoring.  LENGTH (and LI /
        INCR, whose incremental per-candidate bound has no work to skip on MFMA
        tiles): the length bound; COORD (and LC on buckets whose length spread is
        below its switch threshold): the length and the focus-coordinate bounds.
        Every bound is exact, so the top-K equals the unpruned scan's."""
        vecs = item_vecs.float().contiguous()
        lengths = torch.linalg.vector_norm(vecs, dim=1)
        order = torch.argsort(lengths, descending=True)
        #: index position -> row of ``item_vecs`` (incremental updates address rows by it)
        self.order = order
        self.vecs = vecs[order].contiguous()
        self.ids = item_ids.to(vecs.device).long()[order]
        self.lengths = lengths[order]
        self.bucket = bucket_size
        self.buckets_scanned = 0
        #: GPU: score the first ``seed_items`` items unfused (sets every query's k-th
        #: best), then fuse scoring with the threshold filter; ``sync_free``: the LEMP
        #: length bound applied per tile on the device (``ops.score_filter_lemp``) and
        #: overflow flagged on the device, instead of two host syncs per segment
        self.fused = True
        self.sync_free = os.environ.get("FPS_TOPK_SYNC_SCAN", "0") != "1"
        #: fused path: test "every query settled" on the host (one sync) only every
        #: ``break_check`` segments; the device tile bound skips settled work anyway
        self.break_check = int(os.environ.get("FPS_TOPK_BREAK_CHECK", "8"))
        #: fused path: segments double from ``seed_items`` up to ``max_segment`` items
        self.geometric = True
        #: fused path: each segment is ``growth - 1`` times the items scanned before it.  A
        #: segment passes ~k ln(growth) candidates per query that the length bound does not
        #: cut, and every segment costs a re-score + merge launch pair whatever its size: with
        #: long-tailed item lengths (the longest items 1.5x+ the median) the bound cuts the
        #: late segments and fewer, larger segments win (growth 4: LEMP 6.4 -> 6.8e6 q/s);
        #: with near-equal lengths (random-init factors) doubling keeps the candidate lists
        #: short (MF + top-K 2.2 vs 2.1e6; profiles/r5_topk_growth_ab.txt).  FPS_TOPK_GROWTH
        #: overrides.
        env_growth = os.environ.get("FPS_TOPK_GROWTH")
        if env_growth is not None:
            self.growth = int(env_growth)
        elif growth is not None:  # the caller knows its index (e.g. one updated in place: 2)
            self.growth = int(growth)
        else:
            n = self.lengths.numel()
            spread = 1.0
            if n > 2 * self.seed_items:
                pair = self.lengths[torch.tensor([self.seed_items, n // 2], device=self.lengths.device)].tolist()
                spread = pair[0] / max(pair[1], 1e-30)
            # (COORD / LC choose their bound per segment from its length spread, which the
            # short doubling segments keep small)
            from .pruning import COORD, LC
            coordish = isinstance(strategy, (COORD, LC))
            self.growth = 4 if spread > 1.5 and not coordish else 2
        self.overflows = 0
        self._suffix = None  # False once rows were updated out of order
        #: fused GPU scan on bf16 MFMA (``ops.score_filter_bf16``: candidates within a
        #: proven rounding margin) + exact fp32 re-score of the candidates
        #: (``ops.cand_rescore``, bit-identical keys): same result as the fp32 scan.
        #: ``FPS_TOPK_BF16=0`` keeps the fp32 scorer.
        self.bf16 = (vecs.is_cuda and vecs.shape[1] in ops.BF16_SCORE_DIMS
                     and os.environ.get("FPS_TOPK_BF16", "1") != "0")
        self.vecs_bf = self.vecs.bfloat16() if self.bf16 else None
        self.strategy = strategy
        self._cb = None          # LEMP COORD: per-32-item-block coordinate ranges (lazy)
        self._len_host = None    # lengths on the host (LC's per-bucket switch)
        #: (32 queries, 32 items) block pairs the COORD scans scored / skipped
        self.coord_stats = torch.zeros(2, dtype=torch.int32, device=vecs.device) if vecs.is_cuda else None
        #: device COORD gate of a scan (``ops.coord_gate``): on at the start of every query
        #: batch, off for 3 segments after a segment whose bound skipped < 1/4 of its block
        #: pairs, then probed again
        self._coord_gate = torch.ones(1, dtype=torch.int32, device=vecs.device) if vecs.is_cuda else None
        self._coord_prev = torch.zeros(2, dtype=torch.int32, device=vecs.device) if vecs.is_cuda else None
        #: COORD / LC self-disable across query batches: a batch whose COORD bound skipped
        #: less than ``COORD_MIN_SKIP`` of the block pairs it evaluated switches COORD off
        #: -- no query grouping, no bound inputs, no gate launches: the LENGTH scan --
        #: for the next ``COORD_REPROBE`` batches, then it is probed again.  Read with the
        #: scan's one end-of-batch sync.  (The device gate above only skips evaluating the
        #: bound inside a scan; the grouping and the per-segment launches stayed.)
        self.coord_off_batches = 0
        self.coord_batches = {"on": 0, "off": 0}
        #: GPU: fresh LENGTH scans replay one hipGraph per (batch size, k) (``_query_graph``);
        #: FPS_TOPK_GRAPH=0 keeps every scan eager
        self.graphs = vecs.is_cuda and os.environ.get("FPS_TOPK_GRAPH", "1") != "0"
        self._graph: dict = {}

    def update_rows(self, pos: torch.Tensor, vecs: torch.Tensor) -> None:
        """Rewrite the items at index positions ``pos`` (distinct, or repeated with equal
        values) with new vectors, in place: the length order is no longer exact, so the
        bucket bounds switch to the suffix maximum of the lengths (still exact)."""
        v = vecs.float()
        self.vecs[pos] = v
        if self.vecs_bf is not None:
            self.vecs_bf[pos] = v.bfloat16()
        self.lengths[pos] = torch.linalg.vector_norm(v, dim=1)
        self._suffix = False  # the order is stale: bounds take the max of the tail
        self._cb = self._len_host = None

    def refresh_from(self, rows: torch.Tensor, pos: torch.Tensor, table: torch.Tensor) -> None:
        """``update_rows`` from a table: the current ``table[rows]`` go to index positions
        ``pos[row]`` (rows with ``pos < 0`` are not indexed and skipped).  One kernel on the
        GPU (``ops.index_refresh``) instead of the gather / mask / scatter chain."""
        if self.vecs.is_cuda:
            ops.index_refresh(rows, pos, table, self.vecs, self.vecs_bf, self.lengths)
            self._suffix = False
            self._cb = self._len_host = None
            return
        p = pos[rows]
        ok = p >= 0
        self.update_rows(p[ok], table[rows[ok]])

    def _bound(self, s: int) -> torch.Tensor:
        """max |x| over index positions >= s (a 0-dim tensor)."""
        if self._suffix is None:
            return self.lengths[s]
        return self.lengths[s:].max()

    def query(self, Q: torch.Tensor, k: int, exclude: Optional[torch.Tensor] = None, start: int = 0,
              state=None, unfused: bool = False, copy: bool = True):
        """Exact top-``k`` inner products. ``exclude`` = bool mask [B, N_sorted-order-free] not supported;
        use ``exclude_ids`` in ``DistributedTopK`` for seen-item filtering.  ``copy=False``: a
        replayed scan may hand out its graph's own result buffers, valid until the next
        query of that shape is enqueued (a caller that consumes them on the stream before
        then saves two copies per batch).  ``start`` /
        ``state = (best_s, best_i)``: continue a scan whose items ``[0, start)`` are
        already merged into ``state``.  ``unfused``: the score-matrix scan (the rescan
        of a batch whose fused scan overflowed)."""
        Q = Q.float().contiguous()
        B = Q.shape[0]
        dev = Q.device
        N = self.vecs.shape[0]
        fused = self.fused and dev.type == "cuda" and k <= ops.TOPK_MAX_K and not unfused
        if fused and self.sync_free and N > max(self.seed_items, start) and state is None and start == 0 \
                and (Q.shape[0], int(k)) in self._graph and not self._coord_active() and not ops.DEBUG:
            if self._uses_coord():  # COORD switched off for this batch (the per-batch switch)
                self.coord_off_batches -= 1
                self.coord_batches["off"] += 1
            res = self._query_graph(Q, None, k, copy)  # the captured scan computes the norms itself
            if res is not None:
                return res
            self.overflows += 1
            fused = False
        qlen = _row_norms(Q)
        if fused and self.sync_free and N > max(self.seed_items, start):
            st = None if state is None else (state[0].clone(), state[1].clone())
            if self._uses_coord():
                if self.coord_off_batches > 0:
                    self.coord_off_batches -= 1
                    self.coord_batches["off"] += 1
                else:
                    self.coord_batches["on"] += 1
            perm = self._focus_order(Q) if self.bf16 else None
            if perm is not None:
                # the COORD bound is evaluated per 32-query block and skips a block pair only
                # when it holds for all 32 queries: queries grouped by focus coordinate share
                # one coordinate range per block (random order mixes ~32 coordinates in a
                # block, and a block pair almost never passes them all)
                res = self._query_fused(Q[perm], qlen[perm], k, start,
                                        None if st is None else (st[0][perm], st[1][perm]))
                if res is not None:
                    inv = torch.empty_like(perm)
                    inv[perm] = torch.arange(perm.numel(), device=perm.device)
                    res = (res[0][inv], res[1][inv])
            elif st is None and start == 0 and self.graphs and not self._coord_active() and not ops.DEBUG:
                res = self._query_graph(Q, qlen, k, copy)
            else:
                res = self._query_fused(Q, qlen, k, start, st)
            if res is not None:
                return res
            self.overflows += 1  # some query passed more than cap scores: rescan unfused
            fused = False
        if state is None:
            best_s = torch.full((B, k), float("-inf"), device=dev)
            best_i = torch.full((B, k), -1, dtype=torch.long, device=dev)
        else:
            best_s, best_i = state[0].clone(), state[1].clone()
        # segments: the first ``seed_items`` (longest) items, then the rest of each bucket
        seed = min(N, start + self.seed_items) if fused else start
        bounds = sorted({start, seed, *range(self.bucket, N, self.bucket), N} - {N}) + [N]
        bounds = [b for b in bounds if b >= start]
        S = None
        cand = None
        for s, e in zip(bounds[:-1], bounds[1:]):
            # LEMP bucket bound: no item of this or later buckets can beat the k-th best
            if s > 0 and bool((qlen * self._bound(s) <= best_s[:, -1]).all()):
                break
            n = e - s
            if s % self.bucket == 0:
                self.buckets_scanned += 1
            if fused and s > start:
                # scoring fused with the k-th-best filter: only the few passing scores
                # leave the kernel (no [B, n] score matrix)
                if cand is None:
                    cap = ops.TOPK_CAND_CAP
                    cand = (torch.empty((B, cap), dtype=torch.int32, device=dev),
                            torch.empty((B, cap), dtype=torch.long, device=dev),
                            torch.empty(B, dtype=torch.int32, device=dev))
                ck, ci, cnt = cand
                cnt.zero_()
                ops.score_filter(Q, self.vecs[s:e], self.ids[s:e], best_s, ck, ci, cnt)
                if int(cnt.max()) <= ck.shape[1]:
                    ops.topk_merge_cand(ck, ci, cnt, best_s, best_i)
                    continue
                self.overflows += 1  # some query passed more than cap scores: rescan unfused
            if S is None or S.shape[1] < n:
                S = torch.empty((B, max(n, self.bucket)), device=dev)
            ops.score_gemm(Q, self.vecs[s:e], S[:, :n])
            if dev.type == "cuda" and k <= ops.TOPK_MAX_K:
                ops.topk_merge(S[:, :n], self.ids[s:e], best_s, best_i)  # threshold filter + LDS sort
            else:
                cand_s = torch.cat([best_s, S[:, :n]], 1)
                top_s, top_j = torch.topk(cand_s, min(k, cand_s.shape[1]), dim=1)
                cand_i = torch.cat([best_i, self.ids[s:e].expand(B, n)], 1)
                best_s, best_i = top_s, torch.gather(cand_i, 1, top_j)
        return best_s, best_i

    def query_async(self, Q: torch.Tensor, k: int) -> "TopKFuture":
        """``query`` without the end-of-scan host sync: the scan of a fresh batch is
        replayed from its hipGraph, its result copied out on the device and its
        overflow flag copied to pinned host memory behind an event -- nothing waits.
        ``TopKFuture.result()`` reads the flag, so a caller that enqueues batch k + 1
        before asking for batch k's result never drains the device (an overflowed
        batch is rescanned then: ``query(..., unfused=True)``, the same exact top-K).
        ``Q`` must not be modified before ``result()``.  Batches the graph does not
        cover (first of a shape, COORD scans, continued scans, CPU) run ``query``."""
        Q = Q.float().contiguous()
        key = (Q.shape[0], int(k))
        if not (Q.is_cuda and self.fused and self.sync_free and self.graphs and k <= ops.TOPK_MAX_K
                and self.vecs.shape[0] > self.seed_items and key in self._graph and not self._coord_active()
                and not ops.DEBUG):
            return TopKFuture(value=self.query(Q, k))
        if self._uses_coord():  # COORD switched off for this batch (the per-batch switch)
            self.coord_off_batches -= 1
            self.coord_batches["off"] += 1
        graph, q_in, best_s, best_i, ovf, scanned = self._graph[key]
        q_in.copy_(Q)
        graph.replay()
        self.buckets_scanned += scanned
        flag = torch.empty(1, dtype=torch.int32, pin_memory=True)
        flag.copy_(ovf, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        # the graph's buffers are rewritten by the next replay: the result is a copy
        return TopKFuture(raw=(best_s.clone(), best_i.clone()), index=self, Q=Q, k=int(k), flag=flag, event=ev)

    def _query_graph(self, Q: torch.Tensor, qlen: torch.Tensor, k: int, copy: bool = True):
        """The fused scan of a fresh query batch as one hipGraph replay: the seed
        segment, every segment's zero / filter / re-score / merge chain and the norms
        (~35 launches at 1M items) from one host call -- the scan's launches had been
        issued at ~10 us of host time each (MF + top-K at 4096 queries per batch was
        host-bound, ``profiles/r4_mf_topk_kernel_stats.csv``).  One graph per (batch
        size, k), captured after the first batch of that shape (which runs eagerly);
        the graph reads the index tensors in place, so ``update_rows`` stays visible
        and a rebuilt index (a new object) captures its own.  The COORD scans (query
        grouping, gate, per-batch switch) and continued scans run eagerly."""
        key = (Q.shape[0], int(k))
        g = self._graph.get(key)
        if g is None:
            # this batch runs eagerly (it also warms the launches up); the capture that
            # follows executes nothing, so the next batch of this shape replays
            res = self._query_fused(Q, qlen, k)
            self._capture(Q, k)
            return res
        graph, q_in, best_s, best_i, ovf, scanned = g
        q_in.copy_(Q)
        graph.replay()
        self.buckets_scanned += scanned
        if int(ovf.item()):  # the scan's one sync, as the eager path's
            return None
        # the graph's buffers are rewritten by the next replay: hand out copies (unless the
        # caller consumes them before it)
        return (best_s.clone(), best_i.clone()) if copy else (best_s, best_i)

    def _capture(self, Q: torch.Tensor, k: int):
        import gc

        q_in = torch.empty_like(Q)
        q_in.copy_(Q)
        graph = torch.cuda.CUDAGraph()
        b0 = self.buckets_scanned
        enabled = gc.isenabled()
        gc.disable()  # a collection on this thread inside the capture could free a pinned buffer / event
        try:
            with torch.cuda.graph(graph):
                best_s, best_i, ovf = self._scan(q_in, None, k, capturing=True)[:3]
        except RuntimeError as e:  # a launch that cannot be captured: stay eager for this index
            import warnings

            warnings.warn(f"LempTopK: scan capture failed ({e}); eager scans")
            self.graphs = False
            return None
        finally:
            if enabled:
                gc.enable()
        scanned = self.buckets_scanned - b0
        self.buckets_scanned = b0
        g = (graph, q_in, best_s, best_i, ovf, scanned)
        self._graph[(Q.shape[0], int(k))] = g
        return g

    def _query_fused(self, Q, qlen, k, start: int = 0, state=None):
        """The fused scan (``_scan``) and its one host sync: the overflow flag (-> None:
        the caller rescans) and, with COORD, this batch's skip rate for the per-batch
        switch."""
        best_s, best_i, ovf, stats0 = self._scan(Q, qlen, k, start, state)
        if stats0 is not None:  # one sync: overflow flag + this batch's COORD block pairs
            o, scored, skipped = torch.cat([ovf, self.coord_stats - stats0]).tolist()
            if scored + skipped and skipped < self.COORD_MIN_SKIP * (scored + skipped):
                self.coord_off_batches = self.COORD_REPROBE
        elif ovf is not None:
            o = int(ovf.item())
        else:
            o = 0
        if o:
            return None
        return best_s, best_i

    def _scan(self, Q, qlen, k, start: int = 0, state=None, capturing: bool = False):
        """GPU scan without a host sync per segment: seed segment scored + merged,
        then per segment the fused 128 x 128 scorer (tiles that cannot beat any of
        their queries' k-th best skip themselves) and the candidate merge, which
        flags overflowing rows on the device.  One sync per ``break_check``
        segments (early exit) and one at the end (overflow -> ``None``: rescan).
        ``start`` / ``state``: continue from a partial scan (the seed segment then
        runs from ``start`` to the next 32-item boundary, or is skipped)."""
        B, dev = Q.shape[0], Q.device
        N = self.vecs.shape[0]
        # a fresh GPU scan's set-up (norms, bf16 queries, running lists, counts, flag) in
        # one launch instead of eight (ops.topk_scan_prep)
        prep = None
        if state is None and Q.is_cuda and Q.dtype == torch.float32 and k <= ops.TOPK_MAX_K:
            prep = ops.topk_scan_prep(Q, k, bf16=self.bf16)
            if qlen is None:
                qlen = prep[0]
        elif qlen is None:
            qlen = _row_norms(Q)
        if prep is not None:
            best_s, best_i = prep[2], prep[3]
            seed = self.seed_items
        elif state is None:
            best_s = torch.full((B, k), float("-inf"), device=dev)
            best_i = torch.full((B, k), -1, dtype=torch.long, device=dev)
            seed = self.seed_items
        else:
            best_s, best_i = state
            seed = min(N, -(-start // 32) * 32)  # fused segments start on 32-item blocks
        if seed > start:
            S = ops.score_gemm(Q, self.vecs[start:seed])
            ops.topk_merge(S, self.ids[start:seed], best_s, best_i, fresh=state is None)
            del S
            self.buckets_scanned += 1
        if seed >= N:
            return best_s, best_i, None, None
        # segments grow geometrically: a segment of n items after s scanned ones passes
        # ~k ln(1 + n / s) scores per query, so doubling keeps every merge on the small
        # rank path (one 4096 -> 65536 step passed ~1100) at log2(N / seed) segments
        # (8 for 1M items, against 19 when capped at 65536: 4 launches each).  LC keeps
        # the bucket as the largest segment while its COORD bound is on: it picks its
        # bound per segment from the segment's length spread, the reference's
        # per-bucket choice (switched off, it is the LENGTH scan).
        from .pruning import LC

        lc_buckets = isinstance(self.strategy, LC) and self._coord_active()
        cap_seg = self.bucket if lc_buckets else max(self.bucket, self.max_segment)
        cuts = {seed}
        c = max(seed, self.seed_items) if self.geometric else N
        if not self.geometric:
            cuts |= {b for b in range(self.bucket, N, self.bucket) if b > seed}
        while c < N:
            cuts.add(c)
            c += min(c * (self.growth - 1), cap_seg)
        bounds = sorted(cuts) + [N]
        cap = ops.TOPK_CAND_CAP
        ck = torch.empty((B, cap), dtype=torch.int32, device=dev)
        ci = torch.empty((B, cap), dtype=torch.long, device=dev)
        if prep is not None:  # counts and flag zeroed, bf16 queries written by the set-up launch
            Qb, cnt, ovf = prep[1], prep[4], prep[5]
        else:
            cnt = torch.empty(B, dtype=torch.int32, device=dev)
            ovf = torch.zeros(1, dtype=torch.int32, device=dev)
            Qb = Q.bfloat16() if self.bf16 else None
        # the longest item of every 32-item block (the scorer's per-block length bound),
        # recomputed per scan: update_rows / refresh_from change the lengths in place
        xbm = ops.block_max32(self.lengths) if self.bf16 else None
        coord = self._coord_inputs(Q, qlen, bounds) if self.bf16 else None
        if coord is not None:
            self._coord_gate.fill_(1)
            self._coord_prev.copy_(self.coord_stats)
            stats0 = self.coord_stats.clone()
        if prep is None:
            cnt.zero_()  # then zeroed by each segment's merge (reset_cnt)
        for j, (s, e) in enumerate(zip(bounds[:-1], bounds[1:])):
            if self.break_check and j and j % self.break_check == 0 and not capturing and \
                    bool((qlen * self._bound(s) <= best_s[:, -1]).all()):
                break
            self.buckets_scanned += len(range(-(-s // self.bucket) * self.bucket, e, self.bucket))
            if self.bf16:
                seg_coord = None
                if coord is not None and self._coord_segment(s, e):
                    qf, qbf = coord
                    seg_coord = (qf, qbf, self._cb[s // 32: -(-e // 32)])
                ops.score_filter_bf16(Qb, self.vecs_bf[s:e], best_s, ci, cnt, qlen, None,
                                      coord=seg_coord, stats=self.coord_stats if seg_coord is not None else None,
                                      gate=self._coord_gate if seg_coord is not None else None,
                                      xbm=xbm[s // 32: -(-e // 32)] if s % 32 == 0
                                      else ops.block_max32(self.lengths[s:e]))
                if seg_coord is not None:
                    ops.coord_gate(self.coord_stats, self._coord_prev, self._coord_gate)
                # (re-score fused into the rank merge, one query per workgroup: 59 us against
                # 22 + 27 us for the two kernels -- profiles/r2_bf16_topk.md)
                ops.cand_rescore(Q, self.vecs[s:e], self.ids[s:e], best_s, ck, ci, cnt)
            else:
                ops.score_filter_lemp(Q, self.vecs[s:e], self.ids[s:e], best_s, ck, ci, cnt, qlen,
                                      self.lengths[s:e])
            ops.topk_merge_cand(ck, ci, cnt, best_s, best_i, overflow=ovf, reset_cnt=True)
        return best_s, best_i, ovf, (stats0 if coord is not None else None)

    #: COORD self-disable (see ``coord_off_batches``)
    COORD_MIN_SKIP = 0.25
    COORD_REPROBE = 64

    def _uses_coord(self) -> bool:
        from .pruning import COORD, LC

        return isinstance(self.strategy, (COORD, LC))

    def _coord_active(self) -> bool:
        return self._uses_coord() and self.coord_off_batches == 0


    def _coord_inputs(self, Q, qlen, bounds):
        """``(focus coordinate int32[B], q_f / |q|)`` when the strategy uses COORD
        on some segment (segments start on 32-item blocks), else None."""
        if not self._coord_active() or any(b % 32 for b in bounds[:-1]):
            return None
        if self._cb is None:
            self._cb = ops.coord_block_bounds(self.vecs, self.lengths)
        f = torch.argmax(Q * Q, dim=1)
        qbf = Q.gather(1, f.view(-1, 1)).view(-1) / qlen.clamp_min(1e-30)
        return f.to(torch.int32).contiguous(), qbf.contiguous()

    def _focus_order(self, Q: torch.Tensor) -> Optional[torch.Tensor]:
        """Query order grouping equal focus coordinates (``argmax q_c^2``) when the
        strategy evaluates COORD on the device and the batch spans several 32-query
        blocks; None otherwise (the order does not change any result: each query's
        top-K is its own)."""
        if not self._coord_active() or Q.shape[0] <= 32:
            return None
        return torch.argsort(torch.argmax(Q * Q, dim=1), stable=True)

    def _coord_segment(self, s: int, e: int) -> bool:
        """COORD on this segment?  LC switches to LENGTH where the segment's lengths
        spread more than its threshold (``head > last * t``, the reference's choice
        per bucket, ``M/matrix/factorization/workers/PSTopKGeneratorWorker.scala:82-96``)."""
        from .pruning import LC

        if not isinstance(self.strategy, LC):
            return True
        if self._len_host is None:
            self._len_host = self.lengths.cpu()
        return not (float(self._len_host[s]) > float(self._len_host[e - 1]) * self.strategy.algorithm_switch_threshold)


class TopKFuture:
    """The top-K of one query batch, completed on the host only when asked
    (``LempTopK.query_async``): ``result()`` waits for the batch's event -- long
    done when later batches were enqueued first -- reads its overflow flag from
    pinned memory, rescans the batch if it overflowed, and applies ``finish``
    (the cross-shard merge) once."""

    def __init__(self, value=None, raw=None, index=None, Q=None, k: int = 0, flag=None, event=None, finish=None):
        self._value, self._raw, self._index, self._Q, self._k = value, raw, index, Q, k
        self._flag, self._event, self._finish = flag, event, finish
        if value is not None and finish is not None:
            self._value, self._finish = finish(value), None

    def then(self, finish) -> "TopKFuture":
        """Apply ``finish(best_s, best_i) -> result`` to the result (now if it is ready)."""
        if self._value is not None:
            self._value = finish(self._value)
        else:
            self._finish = finish
        return self

    def done(self) -> bool:
        return self._value is not None or self._event is None or self._event.query()

    def result(self):
        if self._value is None:
            self._event.synchronize()
            res = self._raw
            if int(self._flag[0]):  # some query passed more than the candidate cap: rescan
                self._index.overflows += 1
                res = self._index.query(self._Q, self._k, unfused=True)
            self._value = self._finish(res) if self._finish is not None else res
            self._raw = self._Q = self._index = None
        return self._value


def merge_top_k(scores: torch.Tensor, ids: torch.Tensor, k: int, exclude_ids: Optional[torch.Tensor] = None):
    """Merge partial top-K lists ``[B, m]`` into the best ``k``; ``exclude_ids`` [B, E]
    (padded with -1) are dropped first (K13).  No host sync."""
    s = scores.clone()
    if exclude_ids is not None and exclude_ids.numel():
        hit = (ids[:, :, None] == exclude_ids[:, None, :]).any(-1)
        s.masked_fill_(hit, float("-inf"))
    s.masked_fill_(ids < 0, float("-inf"))
    top_s, j = torch.topk(s, min(k, s.shape[1]), dim=1)
    return top_s, torch.gather(ids, 1, j)


class DistributedTopK:
    """Item shards per rank, broadcast queries, all-gather + merge."""

    def __init__(self, item_ids: torch.Tensor, item_vecs: torch.Tensor, comm=None, bucket_size: int = 65536,
                 strategy=None):
        from ...parallel.comm import Comm

        self.comm = comm or Comm()
        self.local = LempTopK(item_ids, item_vecs, bucket_size, strategy=strategy)

    def query(self, Q: torch.Tensor, K: int, worker_k: Optional[int] = None,
              exclude_ids: Optional[torch.Tensor] = None):
        wk = worker_k or K
        s, i = self.local.query(Q, wk)
        if self.comm.world == 1 and exclude_ids is None and wk == K:
            return s, i  # one shard, nothing to exclude: the local list is the answer (sorted, -inf pads)
        if self.comm.world > 1:
            ss = torch.cat(self.comm.all_gather(s.contiguous()), 1)
            ii = torch.cat(self.comm.all_gather(i.contiguous()), 1)
        else:
            ss, ii = s, i
        return merge_top_k(ss, ii, K, exclude_ids)

    def query_async(self, Q: torch.Tensor, K: int, worker_k: Optional[int] = None,
                    exclude_ids: Optional[torch.Tensor] = None) -> TopKFuture:
        """``query`` whose overflow check is deferred to ``result()`` (``LempTopK.query_async``):
        enqueue batch k + 1, then take batch k's result -- no host sync per batch on one
        rank.  Across ranks the partial lists are merged after every rank's flag is known,
        so world > 1 completes synchronously."""
        if self.comm.world > 1:
            return TopKFuture(value=self.query(Q, K, worker_k, exclude_ids))
        wk = worker_k or K
        if exclude_ids is None and wk == K:  # the local list is the answer (as ``query``)
            return self.local.query_async(Q, K)
        return self.local.query_async(Q, wk).then(lambda r: merge_top_k(r[0], r[1], K, exclude_ids))

"""Word2vec skip-gram with negative sampling on the parameter server (BASELINE config #3).

Not in the reference's model library; it is the north-star's third workload
("word2vec SGNS, 1M vocab, dim 300, 8 PS shards over xGMI") and has the same
shape as the MF worker loop (K4+K5 with a sigmoid loss).

Parameters: input vectors ``W_in[V, D]`` (init U[-0.5/D, 0.5/D)) and output
vectors ``W_out[V, D]`` (zeros), each a hash-sharded PS table.  One step on a
micro-batch of (center, context) pairs:

1. draw negatives from unigram^0.75 (alias table, K5): ``mode="standard"``
   (default) ``negatives`` independent ones per pair -- word2vec's objective;
   ``mode="shared"``: ``shared_negatives`` per block of 32 pairs (x ``neg_group``
   blocks), each weighted ``negatives / shared_negatives`` (Ji et al.'s
   block-shared negatives: the same expected gradient, ~10-40x fewer negative
   rows touched; a different estimator, reported separately);
2. pull the center rows from ``W_in`` and context + negative rows from
   ``W_out`` (deduplicated all-to-all, ``TensorPS``); both tables' plans share
   one count exchange, made one micro-batch ahead
   (``BoundedStalenessPipeline`` over both tables), so the host never waits
   for split sizes in steady state;
3. ``ops.sgns_standard`` (K6, ``sgns_std.hip``) / ``ops.sgns_step`` (MFMA,
   ``sgns.hip``) computes per-row deltas;
4. push both delta sets; the PS adds them.  At one rank the owner is the worker:
   ``fuse_local_push`` (default) has the kernel add the deltas straight into the
   tables (the pulled snapshot is still what it reads; the PS's add is the same
   sum), so the delta buffers, their zeroing and the apply pass go away.

With one rank (``local_direct``, default) steps 2 and 4 collapse: the kernel
reads the rows straight from the local tables and adds its deltas into them
with its float atomics -- no dedup, gather, delta buffers or apply pass (the
Hogwild update of the reference word2vec; the PS add is the same sum).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch

from ... import ops
from ...parallel.comm import Comm
from ...parallel.table import ShardedTable
from ...parallel.staleness import BoundedStalenessPipeline
from ...parallel.tensor_ps import TensorPS
from ...utils.tracing import stage

_WIRE = {"fp32": torch.float32, "bf16": torch.bfloat16}


@dataclass
class SGNSConfig:
    vocab_size: int = 1_000_000
    dim: int = 300
    window: int = 5
    negatives: int = 5            # per-pair negatives the shared block emulates
    learning_rate: float = 0.025
    unigram_power: float = 0.75
    seed: int = 0
    wire_dtype: str = "fp32"
    pipeline: bool = True         # PS path (any W, world 1 included): the pulls of batch k+1 overlap the SGNS step
                                  # of batch k, so each batch reads rows one batch stale (staleness 1); False =
                                  # synchronous pulls (staleness 0)
    shared_negatives: int = 16    # negatives shared by each block of 32 pairs (16: kernel v4, 32: v3)
    neg_group: int = 4            # v4: consecutive 32-pair blocks sharing one negative set (1, 2, 4):
                                  # 4 measured +6 % pairs/s at the same loss curve (profiles/r2_sgns.md)
    local_direct: bool = True     # W = 1: kernel reads / atomically updates the local tables in place
    fuse_local_push: bool = True  # W = 1 PS path: the kernel adds its pushes into the tables (no delta buffers)
    mode: str = "standard"        # "standard": `negatives` independent negatives per pair | "shared"


class DistributedSGNS:
    BLOCK = 32  # pairs per block (kernel constant); cfg.shared_negatives negatives per block

    def __init__(self, cfg: SGNSConfig, counts: Optional[torch.Tensor] = None, comm: Optional[Comm] = None):
        self.cfg = cfg
        self.comm = comm or Comm()
        W, r, dev = self.comm.world, self.comm.rank, self.comm.device
        D = cfg.dim
        self.w_in = ShardedTable(cfg.vocab_size, D, r, W, "hash", ("uniform", -0.5 / D, 0.5 / D), cfg.seed, dev)
        self.w_out = ShardedTable(cfg.vocab_size, D, r, W, "hash", ("zeros",), cfg.seed + 1, dev)
        wire = _WIRE[cfg.wire_dtype]
        self.ps_in = TensorPS(self.w_in, self.comm, wire)
        self.ps_out = TensorPS(self.w_out, self.comm, wire)
        # the kernels find "negative == context" and center runs by comparing plan
        # positions: request plans (one position per request) would silently break
        # both, so the SGNS tables always de-duplicate
        self.ps_in.dedup_mode = True
        self.ps_out.dedup_mode = True
        # PS path: both tables planned together (one count exchange per micro-batch),
        # one micro-batch ahead (lookahead): the host reads counts enqueued a step
        # earlier and never idles the device; staleness 1 when pipelined
        self.pipe = BoundedStalenessPipeline([self.ps_in, self.ps_out], self._compute,
                                             staleness=1 if cfg.pipeline else 0)
        if counts is None:  # Zipf-like default frequency profile
            counts = 1.0 / torch.arange(1, cfg.vocab_size + 1, dtype=torch.float64)
        prob, alias = ops.build_alias_table((counts.double() ** cfg.unigram_power).numpy())
        self.prob, self.alias = prob.to(dev), alias.to(dev)
        self.counter = 0
        self.pairs_seen = 0
        self.timer = None  # utils.metrics.StageTimer (optional)
        if cfg.mode not in ("standard", "shared"):
            raise ValueError(f"SGNS mode must be 'standard' or 'shared', not {cfg.mode!r}")
        self.standard = cfg.mode == "standard"

    def _n_negatives(self, P: int) -> int:
        c = self.cfg
        if self.standard:
            return P * c.negatives
        return ((P + self.BLOCK * c.neg_group - 1) // (self.BLOCK * c.neg_group)) * c.shared_negatives

    def step(self, centers: torch.Tensor, contexts: torch.Tensor, lr: Optional[float] = None,
             with_loss: bool = False):
        """One micro-batch of (center, context) pairs.  With ``pipeline`` at W > 1
        the pulls of this batch are issued and the previously pulled batch is
        computed and pushed (staleness: one micro-batch); ``flush()`` finishes the
        last one.  ``with_loss`` computes synchronously and returns the mean loss."""
        c = self.cfg
        lr = c.learning_rate if lr is None else lr
        if self._direct:
            return self._direct_step(centers, contexts, lr, with_loss)
        P = centers.numel()
        with stage("sgns.negatives", self.timer):
            negs = ops.sample_alias(self.prob, self.alias, self._n_negatives(P),
                                    seed=c.seed + 17 * self.comm.rank, counter=self.counter)
        self.counter += 1
        outs = torch.cat([contexts.to(device=negs.device, dtype=torch.int32), negs])
        keys = (centers, outs)
        if with_loss:  # synchronous: every earlier batch applied, this one computed now
            self.pipe.drain()
            st, la = self.pipe.staleness, self.pipe.lookahead
            self.pipe.staleness, self.pipe.lookahead = 0, False
            try:
                res = self.pipe.submit(keys, (P, lr, True))
            finally:
                self.pipe.staleness, self.pipe.lookahead = st, la
            return res[0]
        self.pipe.submit(keys, (P, lr, False))
        return None

    @property
    def _direct(self) -> bool:
        return (self.cfg.local_direct and self.comm.world == 1 and self.w_in.optimizer == "add"
                and self.w_out.optimizer == "add")

    def _direct_step(self, centers, contexts, lr, with_loss):
        """W = 1: rows of the local tables addressed by id (local row = id), deltas
        added in place by the kernel's atomics."""
        c = self.cfg
        P = centers.numel()
        dev = self.w_in.weight.device
        negs = ops.sample_alias(self.prob, self.alias, self._n_negatives(P), seed=c.seed + 17 * self.comm.rank,
                                counter=self.counter)
        self.counter += 1
        cen = centers.to(device=dev, dtype=torch.int32).contiguous()
        ctx = contexts.to(device=dev, dtype=torch.int32).contiguous()
        negs = negs.to(device=dev, dtype=torch.int32).contiguous()
        if self.w_in.touched is not None:  # close-time dumps cover exactly the touched rows
            ops.mark_rows(self.w_in.touched, cen)
        if self.w_out.touched is not None:
            ops.mark_rows(self.w_out.touched, ctx)
            ops.mark_rows(self.w_out.touched, negs)
        with stage("sgns.step", self.timer):
            if self.standard:
                loss = ops.sgns_standard(self.w_in.weight, self.w_out.weight, cen, ctx, negs, c.negatives, lr,
                                         self.w_in.weight, self.w_out.weight, with_loss=with_loss)
            else:
                loss = ops.sgns_step(self.w_in.weight, self.w_out.weight, cen, ctx, negs, lr,
                                     c.negatives / c.shared_negatives, self.w_in.weight, self.w_out.weight,
                                     with_loss=with_loss, neg_k=c.shared_negatives,
                                     neg_group=c.neg_group)
        self.pairs_seen += P
        if with_loss:
            return float(loss.item()) / max(P, 1)
        return None

    @property
    def _pipelined(self) -> bool:
        return self.cfg.pipeline and not self._direct

    def flush(self):
        self.pipe.drain()

    def _compute(self, rows, plans, payload):
        """The SGNS kernel on one micro-batch's pulled rows: per-unique-row deltas of
        both tables (pushed by the pipeline) and, on request, the summed loss."""
        c = self.cfg
        P, lr, with_loss = payload
        rows_in, rows_out = rows
        plan_in, plan_out = plans
        dev = rows_in.device
        fused = self._fused_push(plans)
        if fused:  # pulled row j of a table is its row recv_keys[j]: deltas go there, in place
            d_in, d_out = self.w_in.weight, self.w_out.weight
            wm_in, wm_out = plan_in.recv_keys, plan_out.recv_keys
        else:
            d_in = torch.zeros((plan_in.n_unique, c.dim), dtype=torch.float32, device=dev)
            wm_in = wm_out = None
        # bf16 wire: the output-row deltas leave the kernel in bf16 (the push's wire rows),
        # d_out is its scratch (no zero-fill, no narrowing pass: ops.sgns_standard)
        out_bf = None
        if not fused and self.standard and self.ps_out.wire_dtype == torch.bfloat16 and rows_out.is_cuda \
                and not plan_out.fixed and plan_out.valid is None:
            d_out = torch.empty((plan_out.n_unique, c.dim), dtype=torch.float32, device=dev)
            out_bf = torch.empty((plan_out.n_unique, c.dim), dtype=torch.bfloat16, device=dev)
        elif not fused:
            d_out = torch.zeros((plan_out.n_unique, c.dim), dtype=torch.float32, device=dev)
        pos_o = plan_out.pos[:P].contiguous()
        pos_neg = plan_out.pos[P:].contiguous()
        with stage("sgns.step", self.timer):
            if self.standard:
                # bf16 wire rows go to the kernels as pulled (read as bf16 pairs, widened in
                # registers: ops.sgns_standard); fp32 rows as they are
                loss = ops.sgns_standard(rows_in, rows_out, plan_in.pos.contiguous(), pos_o, pos_neg,
                                         c.negatives, lr, d_in, d_out, with_loss=with_loss, wmap_in=wm_in,
                                         wmap_out=wm_out, d_out_bf16=out_bf)
            else:
                loss = ops.sgns_step(rows_in, rows_out, plan_in.pos.contiguous(), pos_o, pos_neg, lr,
                                     c.negatives / c.shared_negatives, d_in, d_out, with_loss=with_loss,
                                     neg_k=c.shared_negatives, neg_group=c.neg_group)
        self.pairs_seen += P
        if fused:
            for ps, plan in zip((self.ps_in, self.ps_out), plans):
                ps.note_local_push(plan)
            return None, (float(loss.item()) / max(P, 1) if with_loss else None)
        return [d_in, d_out if out_bf is None else out_bf], (float(loss.item()) / max(P, 1) if with_loss else None)

    def _fused_push(self, plans) -> bool:
        """World 1, additive tables, de-duplicating plans: the owner is this rank and each
        pulled row maps to one table row, so the kernel can apply the push itself."""
        return (self.cfg.fuse_local_push and self.standard and self.comm.world == 1
                and self.w_in.optimizer == "add" and self.w_out.optimizer == "add"
                and all(p.unique and p.valid is None and not p.fixed for p in plans))

    def embeddings(self, only_touched: bool = True):
        self.flush()
        return self.w_in.dump(only_touched)


def skipgram_pairs(tokens: torch.Tensor, window: int, generator: Optional[torch.Generator] = None,
                   center_major: bool = True):
    """(center, context) pairs with word2vec's random reduced window b ~ U{1..window}.

    ``center_major`` orders the pairs by center position (word2vec's own order:
    a center's whole window, then the next center), so the pairs of one
    32-pair kernel block share few centers and the kernel sums their center
    gradients before the atomics (``sgns.hip``)."""
    T = tokens.numel()
    b = torch.randint(1, window + 1, (T,), generator=generator, device=tokens.device)
    cs, os_, ps = [], [], []
    for o in range(1, window + 1):
        idx = torch.arange(T - o, device=tokens.device)
        fwd = b[idx] >= o           # context t+o of center t
        bwd = b[idx + o] >= o       # context t of center t+o
        cs += [tokens[idx][fwd], tokens[idx + o][bwd]]
        os_ += [tokens[idx + o][fwd], tokens[idx][bwd]]
        ps += [idx[fwd], (idx + o)[bwd]]
    c, o_ = torch.cat(cs).to(torch.int32), torch.cat(os_).to(torch.int32)
    if center_major:
        order = torch.argsort(torch.cat(ps), stable=True)
        c, o_ = c[order], o_[order]
    return c, o_


def synthetic_corpus(n_tokens: int, vocab_size: int, n_topics: int = 64, topic_len: int = 50, seed: int = 0,
                     device="cpu") -> torch.Tensor:
    """Zipf-frequency tokens in topic runs: words co-occur with their topic's words,
    so embeddings have structure to learn."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    topic_of_word = torch.randint(0, n_topics, (vocab_size,), generator=g)
    order = torch.argsort(topic_of_word, stable=True)
    starts = torch.searchsorted(topic_of_word[order], torch.arange(n_topics))
    sizes = torch.bincount(topic_of_word, minlength=n_topics)
    n_runs = (n_tokens + topic_len - 1) // topic_len
    topics = torch.randint(0, n_topics, (n_runs,), generator=g).repeat_interleave(topic_len)[:n_tokens]
    # Zipf inside the topic via u^3 skew
    u = torch.rand(n_tokens, generator=g) ** 3
    rank = (u * sizes[topics].clamp(min=1)).long()
    return order[starts[topics] + rank].to(torch.int32).to(device)

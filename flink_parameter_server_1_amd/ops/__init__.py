"""Tensor ops of the fast path: gfx950 HIP kernels on device tensors, the
plain-PyTorch reference (``ops.reference``) on CPU tensors.

Dispatch is by the tensor's device.  A CUDA(HIP) tensor *always* goes to the
native kernel; if the library is missing that raises (no silent eager
fallback on a GPU box).
"""
from __future__ import annotations

import os
from typing import Optional

import torch

from . import _native as N
from . import reference as R

_OPS = {"add": 0, "set": 1, "sgd": 2, "adagrad": 3, "add_unique": 4, "add_renorm": 5}


def native_available() -> bool:
    return N.available()


def _on_gpu(t: torch.Tensor) -> bool:
    return t.is_cuda


#: debug mode: ``FPS_DEBUG=1`` range-checks every index tensor on
#: the host before a kernel launch (a device fault becomes a Python exception
#: naming the op) and lets models check their tables for NaN/inf after a step.
#: Costs a device sync per check; pair with ``HIP_LAUNCH_BLOCKING=1`` to pin a
#: fault to its launch.
DEBUG = os.environ.get("FPS_DEBUG", "0") == "1"


def check_index(idx: torch.Tensor, upper: int, what: str, allow_negative: bool = False) -> None:
    """Raise IndexError unless every entry lies in ``[0, upper)`` (negative allowed as padding)."""
    if idx.numel() == 0:
        return
    lo, hi = int(idx.min()), int(idx.max())
    if hi >= upper or (lo < 0 and not allow_negative):
        raise IndexError(f"{what}: index range [{lo}, {hi}] outside [0, {upper})")


def check_finite(t: torch.Tensor, what: str, exc=FloatingPointError) -> None:
    if not bool(torch.isfinite(t).all()):
        raise exc(f"{what}: non-finite values")


def _c(t):
    """Kernel operand check: every pointer handed to a gfx950 kernel must be a
    contiguous DEVICE tensor (a host pointer in a kernel faults the GPU)."""
    if not t.is_cuda:
        raise ValueError(f"kernel operand on {t.device}: expected a GPU tensor")
    if not t.is_contiguous():
        raise ValueError("kernel inputs must be contiguous")
    return t


def init_rows(table: torch.Tensor, id_base: int = 0, id_stride: int = 1, lo: float = 0.0, hi: float = 1.0,
              seed: int = 0) -> torch.Tensor:
    """Fill ``table[r] = U[lo,hi)`` keyed by global id ``id_base + r*id_stride`` (K9)."""
    n, d = table.shape
    if _on_gpu(table):
        lib = N.require()
        N.check(lib.fps_init_rows(_c(table).data_ptr(), n, d, id_base, id_stride, lo, hi, seed & 0xFFFFFFFF,
                                  N.stream_ptr(table.device)), "init_rows")
        return table
    return R.init_rows(table, id_base, id_stride, lo, hi, seed)


def static_plan(uniq: torch.Tensor, prefix: torch.Tensor, nb: int, pos: torch.Tensor):
    """The world-1 static de-duplicated plan: ``(gkeys[nb], valid[nb], pos copy,
    push_rows[nb])`` with slot ``j`` serving ``uniq[j]`` for ``j < U = prefix[1]`` and the
    real key ``uniq[j mod U]`` as padding after (``valid[j] = j < U``); ``push_rows`` =
    ``gkeys`` with -1 on the padding (the rows a push applies).  One launch on the GPU."""
    if _on_gpu(uniq) and uniq.dtype == torch.int32 and pos.dtype == torch.int32 and prefix.dtype == torch.int32:
        gkeys = torch.empty(nb, dtype=torch.int32, device=uniq.device)
        valid = torch.empty(nb, dtype=torch.bool, device=uniq.device)
        pos_c = torch.empty_like(pos)
        push_rows = torch.empty(nb, dtype=torch.int32, device=uniq.device)
        N.check(N.require().fps_static_plan(_c(uniq).data_ptr(), _c(prefix).data_ptr(), int(nb), _c(pos).data_ptr(),
                                            pos.numel(), gkeys.data_ptr(), valid.data_ptr(), pos_c.data_ptr(),
                                            push_rows.data_ptr(), N.stream_ptr(uniq.device)), "static_plan")
        return gkeys, valid, pos_c, push_rows
    j = torch.arange(nb, device=uniq.device)
    valid = j < prefix[1]
    gkeys = torch.where(valid, uniq[:nb], uniq[j % prefix[1].clamp_min(1)])
    return gkeys, valid, pos.clone(), torch.where(valid, gkeys, torch.full_like(gkeys, -1))


def mark_rows(touched: torch.Tensor, rows: torch.Tensor) -> None:
    """``touched[rows] = 1`` (uint8 flags, int32 rows): the dump bookkeeping of the
    in-place (``local_direct``) update paths, one byte store per request."""
    if _on_gpu(touched):
        N.check(N.require().fps_mark_rows(touched.data_ptr(), _c(rows.to(torch.int32)).data_ptr(), rows.numel(),
                                          N.stream_ptr(touched.device)), "mark_rows")
        return
    r = rows.long()
    touched[r[r >= 0]] = 1


def pack_counts(counts: torch.Tensor, W: int, request: bool, flag: int) -> torch.Tensor:
    """The count message of a dynamic PS plan, int32 ``[W, 2]``: row ``j`` =
    ``(2 counts[j] + request, flag)`` (``TensorPS._wire_counts`` + the flag column);
    one launch on the GPU."""
    if _on_gpu(counts) and counts.dtype == torch.int32 and counts.is_contiguous() and counts.numel() >= W:
        out = torch.empty((W, 2), dtype=torch.int32, device=counts.device)
        N.check(N.require().fps_pack_counts(counts.data_ptr(), int(W), int(bool(request)), int(flag), out.data_ptr(),
                                            N.stream_ptr(counts.device)), "pack_counts")
        return out
    c = counts[:W].view(W, 1).to(torch.int32) * 2 + int(bool(request))
    return torch.cat([c, torch.full((W, 1), int(flag), dtype=torch.int32, device=counts.device)], dim=1)


_FILL_KNOB = False


def segment_fill(src: torch.Tensor, rows, out: torch.Tensor, min_us: float = 0.0, stream=None) -> None:
    """``out`` = the concatenation over ``j`` of ``src``'s first ``rows[j]`` rows, ``src``
    tiled where ``rows[j] > len(src)`` (row ``i`` of segment ``j`` is ``src[i % len(src)]``):
    the emulated all-to-all's receive (``parallel/emulated.py``), one launch on the GPU.
    ``rows`` is a host sequence (<= 64 segments); ``out`` holds at least ``sum(rows)`` rows.
    ``min_us`` (GPU): the launch also lasts at least that long -- a modelled link
    transfer that writes its receive as the data arrives (done at max(link, write)).
    ``stream`` (GPU): launch there instead of on the current stream."""
    rows = [int(m) for m in rows]
    n_out, k = sum(rows), src.shape[0]
    if n_out == 0 and not (min_us > 0 and src.is_cuda):
        return
    if k == 0 and n_out:
        raise ValueError("segment_fill: nothing to tile (empty src)")
    if out.shape[0] < n_out or tuple(out.shape[1:]) != tuple(src.shape[1:]) or out.dtype != src.dtype:
        raise ValueError(f"segment_fill: out {tuple(out.shape)} {out.dtype} cannot take {n_out} rows of "
                         f"{tuple(src.shape[1:])} {src.dtype}")
    if _on_gpu(src):
        import ctypes

        global _FILL_KNOB
        if not _FILL_KNOB:  # A/B: FPS_FILL_LINK_WGS = workgroups of a link-timed fill (default 256)
            _FILL_KNOB = True
            if os.environ.get("FPS_FILL_LINK_WGS"):
                N.require().fps_segment_fill_set_link_wgs(int(os.environ["FPS_FILL_LINK_WGS"]))
        if len(rows) > 64:
            raise ValueError(f"segment_fill: {len(rows)} segments, the kernel takes <= 64")
        _c(src), _c(out)

        arr = (ctypes.c_int64 * len(rows))(*rows)
        row_bytes = src.element_size()
        for d in src.shape[1:]:
            row_bytes *= int(d)
        N.check(N.require().fps_segment_fill(src.data_ptr(), k, row_bytes, out.data_ptr(), ctypes.addressof(arr),
                                             len(rows), N.stream_ptr(src.device) if stream is None else
                                             stream.cuda_stream, float(min_us)),
                "segment_fill")
        return
    off = 0
    for m in rows:
        done = 0
        while done < m:
            c = min(m - done, k)
            out[off + done: off + done + c].copy_(src[:c], non_blocking=True)
            done += c
        off += m


def gather_rows(table: torch.Tensor, idx: torch.Tensor, out: torch.Tensor = None, out_dtype=torch.float32,
                touched: torch.Tensor = None, flip: bool = False) -> torch.Tensor:
    """Pull serve: ``out[r] = table[idx[r]]`` (optionally bf16 on the wire) (K2);
    ``idx[r] < 0`` (a padding slot of a fixed-shape plan) serves a zero row.
    The HIP kernel serves fp32 tables; fp64 tables (the bit-parity configuration
    against the per-record engine's doubles) take the torch twin on any device.
    ``flip``: served entries holding the untouched sentinel -0.0 become +0.0 in the
    table (``ShardedTable(touch_sentinel=True)``)."""
    n = idx.numel()
    if DEBUG:
        check_index(idx, table.shape[0], "gather_rows", allow_negative=True)
    d = table.shape[1]
    if out is None:
        out = torch.empty((n, d), dtype=out_dtype, device=table.device)
    if _on_gpu(table) and table.dtype == torch.float32 and out.dtype in (torch.float32, torch.bfloat16):
        lib = N.require()
        N.check(lib.fps_gather_rows(_c(table).data_ptr(), _c(idx).data_ptr(), int(idx.dtype == torch.int64), n, d,
                                    _c(out).data_ptr(), int(out.dtype == torch.bfloat16), N.ptr(touched), int(flip),
                                    N.stream_ptr(table.device)), "gather_rows")
        return out
    out.copy_(R.gather_rows(table, idx, out.dtype, touched))
    if flip:
        flip_sentinel(table, idx)
    return out


def apply_rows(table: torch.Tensor, idx: torch.Tensor, delta: torch.Tensor, op: str = "add", lr: float = 0.0,
               eps: float = 1e-10, state: torch.Tensor = None, touched: torch.Tensor = None) -> torch.Tensor:
    """Push apply (K3): ``add`` (atomic), ``set``, ``sgd`` (w -= lr*g, atomic),
    ``adagrad`` (unique idx; ``state`` = accumulators ``[n, D]``), ``add_renorm``
    (unique idx; w += g and ``state[row] = |w|``, ``state`` = lengths ``[n]``).
    ``idx < 0`` marks padding rows.  fp32 tables run the HIP kernel; fp64 tables
    (bit-parity runs) the torch twin on any device."""
    if DEBUG:
        check_index(idx, table.shape[0], "apply_rows", allow_negative=True)
        check_finite(delta.float(), "apply_rows delta")
    n = idx.numel()
    d = table.shape[1]
    if _on_gpu(table) and table.dtype == torch.float32:
        if idx.dtype != torch.int32:
            idx = idx.to(torch.int32)
        lib = N.require()
        N.check(lib.fps_apply_rows(_c(table).data_ptr(), N.ptr(state), _c(idx).data_ptr(), n, d, _c(delta).data_ptr(),
                                   int(delta.dtype == torch.bfloat16), _OPS[op], lr, eps, N.ptr(touched),
                                   N.stream_ptr(table.device)), "apply_rows")
        return table
    return R.apply_rows(table, idx, delta, op, lr, eps, state, touched)


_HT_INIT = {"zeros": 0, "const": 1, "uniform": 2}


def ht_lookup(keys: torch.Tensor, tab: torch.Tensor, rowmap: torch.Tensor, rowkey: torch.Tensor, count: torch.Tensor,
              overflow: torch.Tensor, insert: bool, rows: torch.Tensor = None, init=None, seed: int = 0):
    """Persistent device hash table (``kernels/hash_table.hip``): rows of int32
    ``keys`` (any value of the signed 32-bit range), inserting absent keys when
    ``insert`` (the fresh rows are initialised per ``init`` = ``("zeros",)`` /
    ``("const", v)`` / ``("uniform", lo, hi)``; ``None`` leaves them).  Returns
    ``(row int32[n], fresh uint8[n])``; ``row = -1``: absent (lookup) or a full
    table (``overflow[0]`` set).  The caller sizes ``tab`` / ``rowkey`` first
    (``parallel.hash_table.HashShardTable.reserve``)."""
    n = keys.numel()
    keys = keys.to(torch.int32).contiguous()
    kind, lo, hi = -1, 0.0, 0.0
    if init is not None:
        kind = _HT_INIT[init[0]]
        lo = float(init[1]) if len(init) > 1 else 0.0
        hi = float(init[2]) if len(init) > 2 else 0.0
    if _on_gpu(tab):
        row = torch.empty(n, dtype=torch.int32, device=tab.device)
        fresh = torch.zeros(n, dtype=torch.uint8, device=tab.device)
        if n == 0:
            return row, fresh
        slot = torch.empty(n, dtype=torch.int32, device=tab.device)
        d = rows.shape[1] if rows is not None else 0
        N.check(N.require().fps_ht_lookup(_c(keys).data_ptr(), n, _c(tab).data_ptr(), tab.numel(),
                                          _c(rowmap).data_ptr(), _c(rowkey).data_ptr(), _c(count).data_ptr(),
                                          rowkey.numel(), int(bool(insert)), slot.data_ptr(), fresh.data_ptr(),
                                          row.data_ptr(), _c(overflow).data_ptr(), N.ptr(rows), d, kind, lo, hi,
                                          seed & 0xFFFFFFFF, N.stream_ptr(tab.device)), "ht_lookup")
        return row, fresh
    row, fresh, ov = R.ht_lookup(keys, tab, rowmap, rowkey, count, insert, rows, kind, lo, hi, seed)
    if ov:
        overflow[0] = ov
    return row, fresh


def ht_rehash(rowkey: torch.Tensor, count: int, tab: torch.Tensor, rowmap: torch.Tensor,
              overflow: torch.Tensor) -> None:
    """Rebuild a zeroed ``tab`` / ``rowmap`` from the first ``count`` row keys."""
    if _on_gpu(tab):
        N.check(N.require().fps_ht_rehash(_c(rowkey).data_ptr(), int(count), _c(tab).data_ptr(), tab.numel(),
                                          _c(rowmap).data_ptr(), _c(overflow).data_ptr(), N.stream_ptr(tab.device)),
                "ht_rehash")
        return
    R.ht_rehash(rowkey, int(count), tab, rowmap)


class DedupWorkspace:
    """Per-step key de-duplication + shard grouping for one worker (K1).

    Dense path: ``map`` is an epoch-tagged ``uint64[num_ids]`` claim table
    (nothing is cleared between steps).  Hashed path (id spaces above
    ``DENSE_MAP_MAX_IDS``): a per-batch epoch-tagged open-addressing table of
    ~2x the batch whose inserting CAS also elects each key's owner.  ``run(keys)`` returns device tensors
    ``counts[W], prefix[W+1], uniq[U], pos[B]``: the unique *local* keys
    grouped by owning shard (contiguous, so they are directly the all-to-all
    send buffer with splits ``counts``) and each request's row in it.
    """

    #: id spaces above this use the hashed claim map (per-batch open-addressing
    #: table, ~32 B per request) instead of a dense ``uint64[num_ids]`` map
    #: (1B-feature PA tables would otherwise need an 8 GB map per worker)
    DENSE_MAP_MAX_IDS = 1 << 28
    #: dense id spaces at most this many times the batch use the flag dedup
    #: (flag store per request + one scan of the key space, no atomics):
    #: 64M MF item keys over 1M ids took 4.9 ms with the claim map
    FLAGS_MAX_RATIO = 8

    def __init__(self, num_ids: int, W: int, part_kind: int = 0, block: int = 1, device="cpu",
                 hashed: Optional[bool] = None, method: Optional[str] = None, out_world: Optional[int] = None):
        """``W`` = number of PS shards the keys route to (hash ``|id| % W``, range by
        ``block``); ``out_world`` (>= W, default W) = ranks of the all-to-all: the
        returned ``counts`` / ``prefix`` cover every rank, ranks >= W (no shard) get
        zero keys -- ``ps_parallelism < world`` without a host owner table."""
        self.num_ids, self.W, self.part_kind, self.block = num_ids, W, part_kind, block
        self.out_world = int(out_world or W)
        if self.out_world < W:
            raise ValueError(f"out_world {out_world} < shards {W}")
        self.method = method or os.environ.get("FPS_DEDUP")  # None = auto | "claim" | "flags"
        if self.method not in (None, "claim", "flags"):
            raise ValueError(f"dedup method must be 'claim' or 'flags', not {self.method!r}")
        self.flag = None
        #: empty every claimed entry after the step (``reset_claims``): set by a
        #: runtime that replays captured steps
        self.clear_after = False
        self.device = torch.device(device)
        self.epoch = 0
        self.cap = 0
        self.hash_cap = 0
        self.hashed = num_ids > self.DENSE_MAP_MAX_IDS if hashed is None else bool(hashed)
        if self.device.type == "cuda":
            if not self.hashed:
                self.map = torch.zeros(num_ids, dtype=torch.int64, device=device)
            self.counts = torch.zeros(W, dtype=torch.int32, device=device)
            self.prefix = torch.zeros(W + 1, dtype=torch.int32, device=device)

    def _grow(self, n):
        if n > self.cap:
            self.cap = max(n, int(self.cap * 1.25))
            self.owner_slot = torch.empty(self.cap, dtype=torch.int32, device=self.device)
            self.uniq = torch.empty(self.cap, dtype=torch.int32, device=self.device)
            self.pos = torch.empty(self.cap, dtype=torch.int32, device=self.device)
            if self.hashed:
                self.hslot = torch.empty(self.cap, dtype=torch.int32, device=self.device)
        if self.hashed and 2 * n > self.hash_cap:
            self.hash_cap = 1 << max(10, (2 * n - 1).bit_length())
            # fresh zeroed table: epoch 0 entries count as empty, epochs restart at 1;
            # owner slots are indexed by hash slot on this path
            self.tab = torch.zeros(self.hash_cap, dtype=torch.int64, device=self.device)
            self.owner_slot_h = torch.empty(self.hash_cap, dtype=torch.int32, device=self.device)
            self.epoch = 0

    def _outputs(self, n: int, fresh: bool):
        """(counts zeroed, prefix, uniq, pos) to write: the workspace's own, or -- ``fresh``
        -- new tensors the caller may keep while later batches reuse the workspace (no
        copy of ~2 x 4 B per request, ``TensorPS._pending``)."""
        if not fresh:
            self.counts.zero_()
            return self.counts, self.prefix, self.uniq, self.pos
        dev = self.device
        return (torch.zeros(self.W, dtype=torch.int32, device=dev), torch.empty(self.W + 1, dtype=torch.int32, device=dev),
                torch.empty(max(n, 1), dtype=torch.int32, device=dev), torch.empty(max(n, 1), dtype=torch.int32, device=dev))

    def run(self, keys: torch.Tensor, fresh: bool = False):
        """De-duplicate and group ``keys`` by owner: ``(counts, prefix, uniq, pos)``.
        ``fresh``: outputs in new tensors instead of the reused workspace."""
        if self.device.type != "cuda":
            c, p, u, q = R.dedup(keys, self.W, self.part_kind, self.block)
            return self._widen(c, p) + (u, q)
        n = keys.numel()
        self._grow(max(n, 1))
        self.epoch += 1
        if self.epoch >= 0xFFFFFFFF:  # wrap: clear the tags once every 4e9 steps
            self.epoch = 1
            (self.tab if self.hashed else self.map).zero_()
            if self.flag is not None:
                self.flag.zero_()
        counts, prefix, uniq, pos = self._outputs(n, fresh)
        lib = N.require()
        s = N.stream_ptr(self.device)
        use_flags = not self.hashed and (self.method == "flags" or
                                         (self.method is None and self.num_ids <= self.FLAGS_MAX_RATIO * n))
        if use_flags:
            if self.flag is None:
                self.flag = torch.zeros(self.num_ids, dtype=torch.int32, device=self.device)
                self.slot = torch.empty(self.num_ids, dtype=torch.int32, device=self.device)
                self.bsum = torch.empty(lib.fps_dedup_flags_ws_ints(self.num_ids, self.W), dtype=torch.int32,
                                        device=self.device)
            N.check(lib.fps_dedup_flags(_c(keys).data_ptr(), n, self.flag.data_ptr(), self.slot.data_ptr(),
                                        self.epoch, self.num_ids, self.W, self.part_kind, self.block,
                                        self.bsum.data_ptr(), counts.data_ptr(), prefix.data_ptr(),
                                        uniq.data_ptr(), pos.data_ptr(), s), "dedup_flags")
        elif self.hashed:
            N.check(lib.fps_dedup_hashed(_c(keys).data_ptr(), n, self.tab.data_ptr(), self.hash_cap, self.epoch,
                                         self.W, self.part_kind, self.block, counts.data_ptr(),
                                         prefix.data_ptr(), self.hslot.data_ptr(), self.owner_slot_h.data_ptr(),
                                         uniq.data_ptr(), pos.data_ptr(), s), "dedup_hashed")
        else:
            N.check(lib.fps_dedup(_c(keys).data_ptr(), n, self.map.data_ptr(), self.epoch, self.W,
                                  self.part_kind, self.block, counts.data_ptr(), prefix.data_ptr(),
                                  self.owner_slot.data_ptr(), uniq.data_ptr(), pos.data_ptr(), s), "dedup")
        return self._widen(counts, prefix) + (uniq, pos[:n])

    def _widen(self, counts, prefix):
        """``(counts[out_world], prefix[out_world + 1])``: the shards' counts, then zeros
        for the ranks without a shard (their prefix entries repeat the total)."""
        if self.out_world == self.W:
            return counts, prefix
        E = self.out_world - self.W
        counts = torch.cat([counts[:self.W], counts.new_zeros(E)])
        prefix = torch.cat([prefix[:self.W + 1], prefix[self.W:self.W + 1].expand(E)])
        return counts, prefix

    def route(self, keys: torch.Tensor, fresh: bool = False):
        """Like ``run`` but WITHOUT de-duplication: every request is its own entry of
        ``uniq`` (grouped by owning shard), ``pos`` a permutation of the requests.
        Same return layout as ``run``."""
        if self.device.type != "cuda":
            c, p, u, q = R.route(keys, self.W, self.part_kind, self.block)
            return self._widen(c, p) + (u, q)
        n = keys.numel()
        self._grow(max(n, 1))
        counts, prefix, uniq, pos = self._outputs(n, fresh)
        N.check(N.require().fps_route_requests(_c(keys).data_ptr(), n, self.W, self.part_kind, self.block,
                                               counts.data_ptr(), prefix.data_ptr(),
                                               self.owner_slot.data_ptr(), uniq.data_ptr(), pos.data_ptr(),
                                               N.stream_ptr(self.device)), "route_requests")
        return self._widen(counts, prefix) + (uniq, pos[:n])

    def reset_claims(self, keys: torch.Tensor) -> None:
        """Empty the claim entries of ``keys`` (the step's unique keys).  In
        ``clear_after`` mode every entry is empty between steps, so a constant
        epoch -- the one baked into a captured hipGraph step
        (``core.step_graph``) -- stays valid."""
        if self.device.type != "cuda":
            return
        if self.hashed:
            self.tab.zero_()
            return
        k = keys.long()
        self.map.index_fill_(0, k, 0)
        if self.flag is not None:
            self.flag.index_fill_(0, k, 0)


def lock_acquire(lock: torch.Tensor, rows: torch.Tensor, src: int) -> torch.Tensor:
    """Device-mode LockPS: try to lock ``rows`` for worker ``src``; uint8 granted flags."""
    if _on_gpu(lock):
        granted = torch.empty(rows.numel(), dtype=torch.uint8, device=lock.device)
        if DEBUG:
            check_index(rows, lock.numel(), "lock_acquire")
        N.check(N.require().fps_lock_acquire(_c(lock).data_ptr(), _c(rows).data_ptr(), rows.numel(), int(src),
                                             granted.data_ptr(), N.stream_ptr(lock.device)), "lock_acquire")
        return granted
    return R.lock_acquire(lock, rows, src)


def lock_release(lock: torch.Tensor, rows: torch.Tensor, granted: torch.Tensor) -> None:
    if _on_gpu(lock):
        N.check(N.require().fps_lock_release(_c(lock).data_ptr(), _c(rows).data_ptr(), rows.numel(),
                                             _c(granted).data_ptr(), N.stream_ptr(lock.device)), "lock_release")
        return
    R.lock_release(lock, rows, granted)


def bucketize(keys: torch.Tensor, W: int, part_kind: int = 0, block: int = 1):
    """Shard id per key and per-shard counts."""
    if _on_gpu(keys):
        shard = torch.empty(keys.numel(), dtype=torch.int32, device=keys.device)
        counts = torch.zeros(W, dtype=torch.int32, device=keys.device)
        lib = N.require()
        N.check(lib.fps_bucketize(_c(keys).data_ptr(), keys.numel(), W, part_kind, block, shard.data_ptr(),
                                  counts.data_ptr(), N.stream_ptr(keys.device)), "bucketize")
        return shard, counts
    return R.bucketize(keys, W, part_kind, block)


def mf_sgd_local(U, I, uid, iid, r, lr: float, lam: float = 0.0, user_atomic: bool = False):
    """Fused MF SGD step with the item shard local (pull = read, push = atomic add) (K4)."""
    if DEBUG:
        check_index(uid, U.shape[0], "mf_sgd_local uid")
        check_index(iid, I.shape[0], "mf_sgd_local iid")
    if _on_gpu(U):
        lib = N.require()
        N.check(lib.fps_mf_sgd_local(_c(U).data_ptr(), _c(I).data_ptr(), _c(uid).data_ptr(), _c(iid).data_ptr(),
                                     _c(r).data_ptr(), uid.numel(), U.shape[1], lr, lam, int(user_atomic),
                                     N.stream_ptr(U.device)), "mf_sgd_local")
        return
    R.mf_sgd_local(U, I, uid, iid, r, lr, lam, user_atomic)


def mf_sgd_pulled(U, uid, r, rows, pos, delta, lr: float, lam: float = 0.0, user_atomic: bool = False):
    """MF SGD on pulled item rows; item deltas accumulate into ``delta[pos]`` (K4)."""
    if DEBUG:
        check_index(uid, U.shape[0], "mf_sgd_pulled uid")
        check_index(pos, rows.shape[0], "mf_sgd_pulled pos")
    if _on_gpu(U):
        lib = N.require()
        N.check(lib.fps_mf_sgd_pulled(_c(U).data_ptr(), _c(uid).data_ptr(), _c(r).data_ptr(), _c(rows).data_ptr(),
                                      int(rows.dtype == torch.bfloat16), _c(pos).data_ptr(), _c(delta).data_ptr(),
                                      uid.numel(), U.shape[1], lr, lam, int(user_atomic), N.stream_ptr(U.device)),
                "mf_sgd_pulled")
        return
    R.mf_sgd_pulled(U, uid, r, rows, pos, delta, lr, lam, user_atomic)


def mf_sgd_local_seg(U, I, uid, iid, r, seg_ptr, seg: int, max_b: int, lr: float, lam: float = 0.0,
                     user_atomic: bool = False):
    """``mf_sgd_local`` on the ratings ``[ptr[seg], ptr[seg+1])``; on the GPU the
    bounds are read on the device (no host sync), ``max_b`` only sizes the grid."""
    if _on_gpu(U):
        lib = N.require()
        sp = _c(seg_ptr)
        N.check(lib.fps_mf_sgd_local_seg(_c(U).data_ptr(), _c(I).data_ptr(), _c(uid).data_ptr(), _c(iid).data_ptr(),
                                         _c(r).data_ptr(), sp.data_ptr() + 4 * seg, max(int(max_b), 1), U.shape[1],
                                         lr, lam, int(user_atomic), N.stream_ptr(U.device)), "mf_sgd_local_seg")
        return
    a, b = int(seg_ptr[seg]), int(seg_ptr[seg + 1])
    R.mf_sgd_local(U, I, uid[a:b], iid[a:b], r[a:b], lr, lam, user_atomic)


class RotationPartitioner:
    """Groups a worker's ratings by rotation item block (``rotate.hip``) with
    reusable device buffers; ``run`` returns ``(ptr[K+1], uid, row, rating)``
    (device tensors; nothing is synchronised to the host)."""

    def __init__(self, W: int, half: torch.Tensor, device):
        self.W, self.K = W, 2 * W
        self.device = torch.device(device)
        self.half = half.to(device=self.device, dtype=torch.int32).contiguous()
        self.cap = 0
        if self.device.type == "cuda":
            self.counts = torch.zeros(self.K, dtype=torch.int32, device=self.device)
            self.cursor = torch.zeros(self.K, dtype=torch.int32, device=self.device)
            self.ptr = torch.zeros(self.K + 1, dtype=torch.int32, device=self.device)

    def run(self, uid, iid, rating, seen: Optional[torch.Tensor] = None):
        """``seen`` (uint8[num_items], optional): set to 1 for every rated item."""
        if self.device.type != "cuda":
            if seen is not None:
                seen[iid.long()] = 1
            _, ptr, u, row, r = R.rot_partition(uid, iid, rating, self.W, self.half)
            return ptr, u, row, r
        n = uid.numel()
        if n > self.cap:
            self.cap = max(n, int(self.cap * 1.25))
            self.u_out = torch.empty(self.cap, dtype=torch.int32, device=self.device)
            self.row_out = torch.empty(self.cap, dtype=torch.int32, device=self.device)
            self.r_out = torch.empty(self.cap, dtype=torch.float32, device=self.device)
        self.counts.zero_()
        self.cursor.zero_()
        lib = N.require()
        N.check(lib.fps_rot_partition(_c(uid).data_ptr(), _c(iid).data_ptr(), _c(rating).data_ptr(), n, self.W,
                                      self.half.data_ptr(), self.counts.data_ptr(), self.ptr.data_ptr(),
                                      self.cursor.data_ptr(), self.u_out.data_ptr(), self.row_out.data_ptr(),
                                      self.r_out.data_ptr(), N.ptr(seen), N.stream_ptr(self.device)), "rot_partition")
        return self.ptr, self.u_out[:n], self.row_out[:n], self.r_out[:n]


#: dims the LDS-tiled MF kernel is instantiated for
TILED_DIMS = (16, 32, 64, 128, 256)


#: bucket counters a tile partition keeps in LDS (``TP_MAX_BUCKETS`` in mf_tiled.hip)
TILE_MAX_BUCKETS = 32768


def tile_rows_for(dim: int, block_rows: int, W: int = 1) -> Optional[int]:
    """Rows per tile for blocks of ``block_rows``: the largest power of two <= 256
    that still gives >= ~1k tiles (workgroups) per block, grown if the 2W*T tile
    buckets exceed the partition's LDS counters.  Large tiles shorten the
    partition (fewer buckets: longer scatter runs, smaller histograms; R = 256
    beat 128 and 64 at N = 1, 64M ratings per step); small blocks (rotation at
    N = 8) need small tiles to fill the GPU.  ``FPS_TILE_ROWS`` overrides.
    None if no tile size fits (then use the flat kernel)."""
    if dim not in TILED_DIMS:
        return None

    def kt(rr):
        return 2 * W * -(-block_rows // rr)

    env = os.environ.get("FPS_TILE_ROWS")
    if env:
        r = max(32, int(env))
    else:
        r = 256
        while r > 32 and -(-block_rows // r) < 960:
            r //= 2
    while kt(r) > TILE_MAX_BUCKETS and r < 256:
        r *= 2
    return r if kt(r) <= TILE_MAX_BUCKETS and r <= 256 else None


class TilePartitioner:
    """Buckets a micro-batch's ratings by (user phase, item block, tile of ``R``
    rows) for ``mf_sgd_tiled`` (``mf_tiled.hip``): a few kernels, nothing
    synchronised to the host.  ``run`` returns ``(ptr[P*2W*T+1], rec)`` with
    ``rec`` an int32 ``[n, 4]`` array of packed records {uid, row-in-block,
    rating bits, bucket} (``[n, 2]`` with ``rec8``) grouped by bucket (on CPU:
    the three columns as tensors).  Phase ``p`` = local users
    ``[p*upp, (p+1)*upp)``; bucket ``(p*2W + b)*T + t``.

    The partition is the two-level one with LDS-sorted batches (count, coarse
    scatter, bucket scatter); the single-level, atomic two-level and
    capacity-slot variants measured slower (``profiles/r1_mf_partition_levels.md``,
    ``profiles/r2_tp4.md``) and were removed."""

    def __init__(self, W: int, half, R: int, T: int, device, rec8: bool = False, phases: int = 1,
                 users_per_phase: Optional[int] = None, num_users: int = 0, num_items: int = 0):
        """``num_users`` (local rows of the user shard) / ``num_items``: ratings with an id
        outside are dropped by the partition instead of indexing past the bucket counters
        and the tables (0 = no bound beyond the phases' user range)."""
        self.W, self.R, self.T = W, int(R), int(T)
        self.nu, self.ni = int(num_users), int(num_items)
        self.P = max(1, int(phases))
        self.upp = int(users_per_phase) if (self.P > 1 and users_per_phase) else (1 << 30)
        if self.P > 1 and not users_per_phase:
            raise ValueError("phases > 1 needs users_per_phase")
        # 8-B records {uid | row_in_tile << 24, rating}: users < 2^24, R <= 256
        self.rec8 = bool(rec8) and self.R <= 256
        self.rec_cols = 2 if self.rec8 else 4
        self.KT = self.P * 2 * W * self.T
        if self.KT > TILE_MAX_BUCKETS:
            raise ValueError(f"{self.KT} tile buckets exceed the partition's {TILE_MAX_BUCKETS} LDS counters")
        self.device = torch.device(device)
        self.half = torch.as_tensor(half).to(device=self.device, dtype=torch.int32).contiguous()
        self.cap = 0
        if self.device.type == "cuda":
            self.ptr = torch.empty(self.KT + 1, dtype=torch.int32, device=self.device)

    def run(self, uid, iid, rating, seen: Optional[torch.Tensor] = None):
        if self.device.type != "cuda":
            nu = self.nu if self.nu > 0 else self.P * self.upp
            ni = self.ni if self.ni > 0 else (1 << 31) - 1
            keep = (uid >= 0) & (uid < nu) & (iid >= 0) & (iid < ni)  # as the kernels: drop, never index
            if not bool(keep.all()):
                uid, iid, rating = uid[keep], iid[keep], rating[keep]
            if seen is not None:
                seen[iid.long()] = 1
            ptr, u, row, r = R.tile_partition(uid, iid, rating, self.W, self.half, self.R, self.T, self.P,
                                              self.upp)
            return ptr, (u, row, r)
        lib = N.require()
        h16 = os.environ.get("FPS_TP_H16")  # A/B switch of the count kernel's counter width
        if h16 is not None:
            lib.fps_tile_partition_set_h16(int(h16))
        grid = os.environ.get("FPS_TP_GRID")  # A/B switch: most workgroups per partition launch
        if grid is not None:
            lib.fps_tile_partition_set_grid(int(grid))
        slim = os.environ.get("FPS_TP_SLIM")  # A/B switch: 256-thread partition kernels (mf_tiled.hip)
        if slim is not None:
            lib.fps_tile_partition_set_slim(int(slim))
        n = uid.numel()
        if n > self.cap:
            self.cap = max(n, int(self.cap * 1.25))
            self.rec = torch.empty((self.cap, self.rec_cols), dtype=torch.int32, device=self.device)
            self.tmp = torch.empty((self.cap, 4), dtype=torch.int32, device=self.device)
        if not hasattr(self, "ws"):
            self.ws = torch.empty(lib.fps_tile_partition_ws_ints(self.W, self.T, self.P), dtype=torch.int32,
                                  device=self.device)
        N.check(lib.fps_tile_partition(_c(uid).data_ptr(), _c(iid).data_ptr(), _c(rating).data_ptr(), n, self.W,
                                       self.half.data_ptr(), self.R, self.T, self.P, self.upp, self.nu, self.ni,
                                       self.ws.data_ptr(),
                                       self.tmp.data_ptr(), self.ptr.data_ptr(), self.rec.data_ptr(), int(self.rec8),
                                       N.ptr(seen), N.stream_ptr(self.device)), "tile_partition")
        return self.ptr, self.rec[:n]

    def unpack(self, rec, ptr=None):
        """(uid, row-in-block, rating) columns of packed records (tests / CPU);
        8-B records need ``ptr`` to recover the tile of every record."""
        if isinstance(rec, tuple):
            return rec
        if rec.shape[1] == 4:
            return rec[:, 0], rec[:, 1], rec[:, 2].contiguous().view(torch.float32)
        x = rec[:, 0]
        uid = x & 0xFFFFFF
        row_in_tile = (x.long() >> 24) & 0xFF
        counts = (ptr[1:] - ptr[:-1]).long()
        bucket = torch.repeat_interleave(torch.arange(counts.numel(), device=rec.device), counts)
        row = (bucket % self.T) * self.R + row_in_tile
        return uid, row.to(torch.int32), rec[:, 1].contiguous().view(torch.float32)


#: user-row modes of the tiled SGD (``mf_sgd_tiled(user_mode=...)``)
USER_MODES = {"store": 0, "sc1": 1, "atomic": 2}


def mf_sgd_tiled(U, I_block, rec, ptr, block: int, T: int, tile_rows: int, lr: float, lam: float = 0.0,
                 delta: Optional[torch.Tensor] = None, delta_init: bool = True, user_sc1: bool = False,
                 user_mode: int = 0):
    """MF SGD of the ratings of item block ``block`` (tiles ``ptr[block*T : (block+1)*T + 1]``,
    records from ``TilePartitioner``): one workgroup per tile, every item row owned
    by one lane group (registers), item deltas summed per row -- no item atomics.
    ``delta`` (same shape as ``I_block``): leave ``I_block`` unchanged and write
    every row's summed item delta there instead (the PS path's push);
    ``delta_init=False`` adds to the deltas of an earlier launch over the same rows
    (the rows then continue from ``I_block + delta``).  ``user_sc1``: user rows loaded /
    stored write-through (``sc1``; 8-B records, user table < 4 GiB) -- about half the
    Hogwild lost user updates of plain accesses (``profiles/r4_hogwild.md``).
    ``user_mode`` (``USER_MODES``): 0 plain (Hogwild), 1 = ``user_sc1``, 2 = exact: every
    user delta added with float atomics (no update lost; same constraints as sc1)."""
    user_mode = max(int(user_mode), 1 if user_sc1 else 0)
    if delta is not None and (delta.shape != I_block.shape or delta.dtype != torch.float32):
        raise ValueError("mf_sgd_tiled: delta must be an fp32 tensor shaped like the item block")
    if _on_gpu(U):
        lib = N.require()
        p0 = _c(ptr).data_ptr() + 4 * block * T
        N.check(lib.fps_mf_sgd_tiled(_c(U).data_ptr(), _c(I_block).data_ptr(), _c(rec).data_ptr(),
                                     int(rec.shape[1] == 2), p0, T, tile_rows, I_block.shape[0], None, None, 0, 1,
                                     U.shape[1], lr, lam, None if delta is None else _c(delta).data_ptr(),
                                     int(delta_init), U.numel() * 4, user_mode, N.stream_ptr(U.device)),
                "mf_sgd_tiled")
        return
    uid, row, r = rec
    a, b = int(ptr[block * T]), int(ptr[(block + 1) * T])
    if delta is None:
        R.mf_sgd_local(U, I_block, uid[a:b], row[a:b], r[a:b], lr, lam, user_atomic=user_mode == 2)
        return
    work = I_block.clone() if delta_init else I_block + delta
    R.mf_sgd_local(U, work, uid[a:b], row[a:b], r[a:b], lr, lam, user_atomic=user_mode == 2)
    torch.sub(work, I_block, out=delta)


def mf_sgd_tiled_pair(U, I0, I1, rec, ptr, block: int, T: int, tile_rows: int, lr: float, lam: float = 0.0,
                      block1: Optional[int] = None, user_sc1: bool = False, user_mode: int = 0):
    """``mf_sgd_tiled`` of item blocks ``block`` (rows ``I0``) and ``block1`` (default
    ``block + 1``; rows ``I1``) in one launch of 2T workgroups: the blocks share no
    item row, so they need no ordering, and one launch instead of two halves the
    tail of partly filled waves."""
    block1 = block + 1 if block1 is None else block1
    user_mode = max(int(user_mode), 1 if user_sc1 else 0)
    if _on_gpu(U):
        lib = N.require()
        base = _c(ptr).data_ptr()
        N.check(lib.fps_mf_sgd_tiled(_c(U).data_ptr(), _c(I0).data_ptr(), _c(rec).data_ptr(),
                                     int(rec.shape[1] == 2), base + 4 * block * T, T, tile_rows, I0.shape[0],
                                     _c(I1).data_ptr(), base + 4 * block1 * T, I1.shape[0], 2, U.shape[1], lr, lam,
                                     None, 1, U.numel() * 4, user_mode, N.stream_ptr(U.device)),
                "mf_sgd_tiled_pair")
        return
    mf_sgd_tiled(U, I0, rec, ptr, block, T, tile_rows, lr, lam, user_mode=user_mode)
    mf_sgd_tiled(U, I1, rec, ptr, block1, T, tile_rows, lr, lam, user_mode=user_mode)


PAIR_LOSSES = {"logistic": 0, "squared": 1}


def pair_sgd_pulled(rows, pa, pb, label, delta, lr: float, loss: str = "logistic", with_loss: bool = False):
    """Pairwise embedding SGD on pulled rows (both sides from one PS table):
    ``delta[pa] += lr*g*rows[pb]``, ``delta[pb] += lr*g*rows[pa]`` (config #5 compute).
    Returns the loss sum as a device/host scalar tensor when ``with_loss``."""
    kind = PAIR_LOSSES[loss]
    if _on_gpu(delta):
        out = torch.zeros(1, dtype=torch.float64, device=delta.device) if with_loss else None
        lib = N.require()
        N.check(lib.fps_pair_sgd_pulled(_c(rows).data_ptr(), int(rows.dtype == torch.bfloat16), _c(pa).data_ptr(),
                                        _c(pb).data_ptr(), _c(label).data_ptr(), _c(delta).data_ptr(), pa.numel(),
                                        delta.shape[1], lr, kind, out.data_ptr() if out is not None else None,
                                        N.stream_ptr(delta.device)), "pair_sgd_pulled")
        return out
    loss_v = R.pair_sgd_pulled(rows, pa, pb, label, delta, lr, kind)
    return torch.tensor([loss_v], dtype=torch.float64) if with_loss else None


class CSRGrouper:
    """Counting sort of request indices by key (``key`` in ``[0, n_groups)``) with
    reusable device buffers; returns ``(ptr[G+1] int32, order[B] int32)``."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.cap_g = 0
        self.cap_b = 0

    def run(self, keys: torch.Tensor, n_groups: int):
        if self.device.type != "cuda":
            return R.csr_group(keys, n_groups)
        n = keys.numel()
        if n_groups + 1 > self.cap_g:
            self.cap_g = max(n_groups + 1, int(self.cap_g * 1.25))
            self.cnt = torch.empty(self.cap_g, dtype=torch.int32, device=self.device)
            self.cursor = torch.empty(self.cap_g, dtype=torch.int32, device=self.device)
            self.ptr = torch.empty(self.cap_g, dtype=torch.int32, device=self.device)
        if n > self.cap_b:
            self.cap_b = max(n, int(self.cap_b * 1.25))
            self.order = torch.empty(self.cap_b, dtype=torch.int32, device=self.device)
        cnt = self.cnt[:n_groups]
        cnt.zero_()
        lib = N.require()
        s = N.stream_ptr(self.device)
        N.check(lib.fps_csr_count(_c(keys).data_ptr(), n, cnt.data_ptr(), s), "csr_count")
        ptr = self.ptr[: n_groups + 1]
        ptr[:1].zero_()
        torch.cumsum(cnt, 0, out=ptr[1:])
        cur = self.cursor[:n_groups]
        cur.zero_()
        N.check(lib.fps_csr_scatter(keys.data_ptr(), n, ptr.data_ptr(), cur.data_ptr(), self.order.data_ptr(), s),
                "csr_scatter")
        return ptr, self.order[:n]


def mf_sgd_grouped(U, I, uid, r, ptr, order, lr: float, lam: float = 0.0, delta: torch.Tensor = None):
    """Item-grouped MF SGD (K4, grouped form): group ``g`` = row ``g`` of ``I``; its
    ratings (``order[ptr[g]:ptr[g+1]]``) update the row sequentially in registers.
    ``delta`` given -> ``I`` is a pulled-rows buffer and ``delta[g] = final - pulled``;
    otherwise ``I`` (local shard) is updated in place."""
    G = ptr.numel() - 1
    if _on_gpu(U):
        mode = 0 if delta is None else (2 if I.dtype == torch.bfloat16 else 1)
        lib = N.require()
        N.check(lib.fps_mf_sgd_grouped(_c(U).data_ptr(), _c(I).data_ptr(), mode, _c(uid).data_ptr(),
                                       _c(r).data_ptr(), _c(ptr).data_ptr(), _c(order).data_ptr(), G, U.shape[1], lr,
                                       lam, N.ptr(delta), N.stream_ptr(U.device)), "mf_sgd_grouped")
        return
    R.mf_sgd_grouped(U, I, uid, r, ptr, order, lr, lam, delta)


def sample_uniform_reject(n: int, k: int, n_items: int, positive=None, user=None, ring=None, mem: int = 0,
                          seed: int = 0, counter: int = 0, device="cpu", known=None, known_count=None) -> torch.Tensor:
    """``k`` uniform negatives per row, avoiding the positive and the user's ring (K5).
    With ``known``/``known_count`` (device list + count) candidates come from the
    worker's known items, as in the reference worker."""
    device = torch.device(device)
    if device.type == "cuda":
        out = torch.empty(n * k, dtype=torch.int32, device=device)
        lib = N.require()
        N.check(lib.fps_sample_uniform_reject(n, k, n_items, N.ptr(positive), N.ptr(user), N.ptr(ring), mem,
                                              N.ptr(known), N.ptr(known_count), seed & 0xFFFFFFFF, counter,
                                              out.data_ptr(), N.stream_ptr(device)), "sample_uniform_reject")
        return out
    kc = int(known_count[0]) if known_count is not None else None
    return R.sample_uniform_reject(n, k, n_items, positive, user, ring, mem, seed, counter, known, kc)


def ring_push(ring, cursor, uid, iid, mem: int) -> None:
    """Append each rating's item to its user's ring of the last ``mem`` items."""
    if _on_gpu(ring):
        N.check(N.require().fps_ring_push(_c(ring).data_ptr(), _c(cursor).data_ptr(), _c(uid).data_ptr(),
                                          _c(iid).data_ptr(), uid.numel(), mem, N.stream_ptr(ring.device)),
                "ring_push")
        return
    R.ring_push(ring, cursor, uid, iid, mem)


def known_append(flag, lst, count, iid) -> None:
    """Append first-seen items to a known-item list (``count`` is a 1-element device counter)."""
    if _on_gpu(flag):
        N.check(N.require().fps_known_append(_c(flag).data_ptr(), _c(lst).data_ptr(), _c(count).data_ptr(),
                                             _c(iid).data_ptr(), iid.numel(), N.stream_ptr(flag.device)),
                "known_append")
        return
    R.known_append(flag, lst, count, iid)


def build_alias_table(weights):
    """Walker/Vose alias table of a discrete distribution -> (prob fp32, alias int32) on CPU."""
    import numpy as np

    w = np.asarray(weights, dtype=np.float64)
    V = w.size
    p = w * V / w.sum()
    prob = np.zeros(V)
    alias = np.zeros(V, dtype=np.int64)
    small = [i for i in range(V) if p[i] < 1.0]
    large = [i for i in range(V) if p[i] >= 1.0]
    while small and large:
        s, g = small.pop(), large.pop()
        prob[s], alias[s] = p[s], g
        p[g] -= 1.0 - p[s]
        (small if p[g] < 1.0 else large).append(g)
    for i in large + small:
        prob[i], alias[i] = 1.0, i
    return torch.from_numpy(prob.astype(np.float32)), torch.from_numpy(alias.astype(np.int32))


def sample_alias(prob: torch.Tensor, alias: torch.Tensor, n: int, seed: int = 0, counter: int = 0) -> torch.Tensor:
    if prob.is_cuda:
        out = torch.empty(n, dtype=torch.int32, device=prob.device)
        lib = N.require()
        N.check(lib.fps_sample_alias(_c(prob).data_ptr(), _c(alias).data_ptr(), prob.numel(), n, seed & 0xFFFFFFFF,
                                     counter, out.data_ptr(), N.stream_ptr(prob.device)), "sample_alias")
        return out
    return R.sample_alias(prob, alias, n, seed, counter)


#: shared negatives per block of 32 pairs the SGNS kernels take (v4: 16, v3: 32)
SGNS_NEG_K = (16, 32)


def sgns_step(rows_in, rows_out, pos_c, pos_o, pos_neg, lr: float, neg_weight: float, d_in, d_out,
              with_loss: bool = False, neg_k: int = 16, neg_group: int = 1):
    """Block-shared-negative skip-gram step on MFMA (K6); deltas accumulate into
    ``d_in`` / ``d_out`` (per pulled row).  ``pos_neg`` has ``neg_k`` rows per 32
    pairs: 16 runs kernel v4 (two 512-thread blocks per CU), 32 kernel v3.
    ``neg_group`` (1, 2 or 4; v4 only): that many consecutive blocks of 32 pairs share
    one set of ``neg_k`` negatives (``pos_neg`` holds ``neg_k`` rows per 32 * neg_group
    pairs); their negative-row gradients are summed on chip and pushed once.  (A
    loader / atomic wave-split variant, v5, measured slower than v4 and was removed in
    round 3: ``profiles/r1_w2v_v4.md``.)"""
    D = rows_in.shape[1]
    if neg_k not in SGNS_NEG_K:
        raise ValueError(f"sgns_step: neg_k must be one of {SGNS_NEG_K}")
    if neg_group not in (1, 2, 4) or (neg_group > 1 and neg_k != 16):
        raise ValueError("sgns_step: neg_group is 1, 2 or 4 (groups > 1 with neg_k = 16)")
    if pos_neg.numel() < neg_k * ((pos_c.numel() + 32 * neg_group - 1) // (32 * neg_group)):
        raise ValueError("sgns_step: pos_neg needs neg_k rows per 32 * neg_group pairs")
    if rows_in.is_cuda:
        loss = torch.zeros(1, dtype=torch.float32, device=rows_in.device) if with_loss else None
        lib = N.require()
        if neg_k == 16:
            N.check(lib.fps_sgns_step_v4g(
                _c(rows_in).data_ptr(), _c(rows_out).data_ptr(), int(rows_in.dtype == torch.bfloat16),
                _c(pos_c).data_ptr(), _c(pos_o).data_ptr(), _c(pos_neg).data_ptr(), pos_c.numel(), D, lr,
                neg_weight, _c(d_in).data_ptr(), _c(d_out).data_ptr(), N.ptr(loss), neg_group,
                N.stream_ptr(rows_in.device)), "sgns_step")
            return loss
        N.check(lib.fps_sgns_step(_c(rows_in).data_ptr(), _c(rows_out).data_ptr(),
                                  int(rows_in.dtype == torch.bfloat16), _c(pos_c).data_ptr(), _c(pos_o).data_ptr(),
                                  _c(pos_neg).data_ptr(), pos_c.numel(), D, lr, neg_weight, _c(d_in).data_ptr(),
                                  _c(d_out).data_ptr(), N.ptr(loss), N.stream_ptr(rows_in.device)), "sgns_step")
        return loss
    return torch.tensor([R.sgns_step(rows_in, rows_out, pos_c, pos_o, pos_neg, lr, neg_weight, d_in, d_out, neg_k,
                                     neg_group)])


SGNS_METHODS = ("sorted", "atomic")


def sgns_standard(rows_in, rows_out, pos_c, pos_o, pos_neg, k: int, lr: float, d_in, d_out,
                  with_loss: bool = False, method: Optional[str] = None, wmap_in=None, wmap_out=None,
                  d_out_bf16=None):
    """Standard skip-gram negative sampling (K6, ``kernels/sgns_std.hip``): ``k``
    independent negatives per pair (``pos_neg[P * k]``), word2vec's objective.
    ``d_in`` / ``d_out`` receive the deltas (the tables themselves on the local
    path).  ``wmap_in`` / ``wmap_out`` (int32, optional): the delta of row ``r`` goes
    to row ``wmap[r]`` of ``d_in`` / ``d_out`` (world-1 PS path: pushes added straight
    into the owner's tables).  Returns the summed loss (a device / host 1-element
    tensor) or None.

    GPU: one wave per 16 pairs, sequential inside a wave's center runs (the
    center's change is added once per run).  Output rows (context + negatives):

    * ``method="sorted"`` (default): the pass computes each pair's coefficients
      g_x against the output rows as of the call; the (row, entry) list is sorted
      by row and ``sgns_rows_kernel`` adds sum g_x * h per row, one plain
      read-modify-write per row run (float atomics only where a run straddles two
      waves).  ``h`` = the center rows after this call's center updates
      (``rows_in``; on the PS path the pulled rows).
    * ``method="atomic"``: Hogwild float atomics per pair and row, inside the pass.

    ``d_out_bf16`` (bf16, shaped as ``d_out``; the PS path's bf16 push): the output-row
    deltas are returned there in bf16 and ``d_out`` is scratch (its content on entry
    does not matter).  With bf16 rows and the sorted form on the GPU the rows kernel
    writes them directly (no zero-fill of ``d_out``, no widening pass after).

    CPU: the mini-batch form."""
    P = pos_c.numel()
    D = rows_in.shape[1]
    if pos_neg.numel() != P * k:
        raise ValueError("sgns_standard: pos_neg needs k rows per pair")
    if rows_in.is_cuda:
        for t in (d_in, d_out):
            if t.dtype != torch.float32:
                raise ValueError("sgns_standard: fp32 deltas")
        # rows: fp32, or bf16 (both tables; the PS path's wire rows as pulled, even D) read
        # directly by the kernels -- no widening pass over every pulled row
        bf = rows_in.dtype == torch.bfloat16 and rows_out.dtype == torch.bfloat16 and D % 2 == 0
        if not bf and (rows_in.dtype != torch.float32 or rows_out.dtype != torch.float32):
            rows_in, rows_out = rows_in.float(), rows_out.float()
        if D > 512:
            raise ValueError("sgns_standard: D <= 512")
        loss = torch.zeros(1, dtype=torch.float32, device=rows_in.device) if with_loss else None
        wmap_in = None if wmap_in is None else _c(wmap_in.to(torch.int32))
        wmap_out = None if wmap_out is None else _c(wmap_out.to(torch.int32))
        method = method or os.environ.get("FPS_SGNS_METHOD", "sorted")
        if method not in SGNS_METHODS:
            raise ValueError(f"sgns_standard: method must be one of {SGNS_METHODS}")
        ob = d_out_bf16 is not None
        if ob and (d_out_bf16.dtype != torch.bfloat16 or d_out_bf16.shape != d_out.shape):
            raise ValueError("sgns_standard: d_out_bf16 must be bf16 and shaped as d_out")
        direct_ob = ob and bf and method == "sorted" and wmap_out is None
        if ob and not direct_ob:  # d_out is scratch: the deltas accumulate from zero, then narrow
            d_out.zero_()
        if method == "sorted":
            lib = N.require()
            s = N.stream_ptr(rows_in.device)
            k1 = int(k) + 1
            gbuf = torch.zeros(P * k1, dtype=torch.float32, device=rows_in.device)
            N.check(lib.fps_sgns_standard_coef(_c(rows_in).data_ptr(), _c(rows_out).data_ptr(), _c(pos_c).data_ptr(),
                                               _c(pos_o).data_ptr(), _c(pos_neg).data_ptr(), P, D, int(k), lr,
                                               _c(d_in).data_ptr(), N.ptr(wmap_in), N.ptr(loss), gbuf.data_ptr(), s,
                                               int(bf)),
                    "sgns_coef")
            keys = torch.cat([pos_o.reshape(P, 1), pos_neg.reshape(P, int(k))], dim=1).reshape(-1)
            srow, perm = torch.sort(keys.to(torch.int32))
            N.check(lib.fps_sgns_rows(_c(srow).data_ptr(), _c(perm).data_ptr(), gbuf.data_ptr(), _c(pos_c).data_ptr(),
                                      k1, P * k1, _c(rows_in).data_ptr(), D, _c(d_out).data_ptr(), N.ptr(wmap_out), s,
                                      int(bf), _c(d_out_bf16).data_ptr() if direct_ob else None),
                    "sgns_rows")
            if ob and not direct_ob:
                d_out_bf16.copy_(d_out)
            return loss
        N.check(N.require().fps_sgns_standard(_c(rows_in).data_ptr(), _c(rows_out).data_ptr(), _c(pos_c).data_ptr(),
                                              _c(pos_o).data_ptr(), _c(pos_neg).data_ptr(), P, D, int(k), lr,
                                              _c(d_in).data_ptr(), _c(d_out).data_ptr(), N.ptr(wmap_in),
                                              N.ptr(wmap_out), N.ptr(loss), N.stream_ptr(rows_in.device), int(bf)),
                "sgns_standard")
        if ob:
            d_out_bf16.copy_(d_out)
        return loss
    # CPU: the mini-batch form (every pair reads the rows as of the call); the
    # kernel's exact per-wave order is ``reference.sgns_standard`` (numerics tests)
    if rows_in.dtype != d_in.dtype or rows_out.dtype != d_out.dtype:  # bf16 wire rows: widened here
        rows_in, rows_out = rows_in.to(d_in.dtype), rows_out.to(d_out.dtype)
    if d_out_bf16 is not None:  # d_out is scratch: accumulate from zero, return narrowed
        d_out.zero_()
        loss = sgns_standard(rows_in, rows_out, pos_c, pos_o, pos_neg, k, lr, d_in, d_out, with_loss, method,
                             wmap_in, wmap_out)
        d_out_bf16.copy_(d_out)
        return loss
    if wmap_in is not None or wmap_out is not None:
        tmp_in = torch.zeros((rows_in.shape[0], D), dtype=d_in.dtype)
        tmp_out = torch.zeros((rows_out.shape[0], D), dtype=d_out.dtype)
        total = R.sgns_standard_batched(rows_in, rows_out, pos_c, pos_o, pos_neg, int(k), lr, tmp_in, tmp_out)
        for d, tmp, wm in ((d_in, tmp_in, wmap_in), (d_out, tmp_out, wmap_out)):
            if wm is None:
                d += tmp
            else:
                d.index_add_(0, wm.long(), tmp)
        return torch.tensor([total]) if with_loss else None
    total = R.sgns_standard_batched(rows_in, rows_out, pos_c, pos_o, pos_neg, int(k), lr, d_in, d_out)
    return torch.tensor([total]) if with_loss else None


TOPK_MAX_K = 256


def topk_merge(S: torch.Tensor, ids: torch.Tensor, best_s: torch.Tensor, best_i: torch.Tensor,
               fresh: bool = False) -> None:
    """Merge each row of ``S[B, n]`` (item ids ``ids[n]``) into the running top-k
    ``best_s``/``best_i`` ``[B, k]`` (sorted descending; start -inf / -1) in place (K13).
    ``fresh``: the running lists are still empty (-inf / -1) -- a plain selection, one
    wave per row on the GPU for ``n <= 4096`` (``fps_topk_select``, same result)."""
    B, n = S.shape
    k = best_s.shape[1]
    if _on_gpu(S):
        if k > TOPK_MAX_K:
            raise ValueError(f"topk_merge: k <= {TOPK_MAX_K}")
        if S.stride(1) != 1:
            raise ValueError("topk_merge: S needs unit column stride")
        if fresh and k <= 128 and k <= n <= 4096:
            redo = torch.zeros(B, dtype=torch.uint8, device=S.device)
            N.check(N.require().fps_topk_select(S.data_ptr(), S.stride(0), B, n, _c(ids.long()).data_ptr(),
                                                _c(best_s).data_ptr(), _c(best_i).data_ptr(), k, redo.data_ptr(),
                                                N.stream_ptr(S.device)), "topk_select")
            return
        N.check(N.require().fps_topk_merge(S.data_ptr(), S.stride(0), B, n, _c(ids.long()).data_ptr(),
                                           _c(best_s).data_ptr(), _c(best_i).data_ptr(), k, N.stream_ptr(S.device)),
                "topk_merge")
        return
    cand_s = torch.cat([best_s, S], 1)
    cand_i = torch.cat([best_i, ids.long().expand(B, n)], 1)
    top_s, j = torch.topk(cand_s, k, dim=1)
    best_s.copy_(top_s)
    best_i.copy_(torch.gather(cand_i, 1, j))


#: candidates kept per query and segment by ``score_filter`` (<= the merge's LDS capacity)
TOPK_CAND_CAP = 2048


def score_filter(Q: torch.Tensor, X: torch.Tensor, ids: torch.Tensor, best_s: torch.Tensor, cand_key: torch.Tensor,
                 cand_id: torch.Tensor, cnt: torch.Tensor) -> None:
    """Fused K8 scoring + threshold filter (GPU only): every ``<Q[b], X[i]>`` strictly above
    ``best_s[b, -1]`` is appended to row ``b`` of ``cand_key``/``cand_id`` ``[B, cap]``
    (order-preserving uint32 keys as int32 storage); ``cnt[b]`` (zeroed by the caller)
    counts all of them, so ``cnt > cap`` means the row overflowed."""
    B, D = Q.shape
    cap = cand_key.shape[1]
    N.check(N.require().fps_score_filter(_c(Q).data_ptr(), _c(X).data_ptr(), _c(ids).data_ptr(), B, X.shape[0], D,
                                         _c(best_s).data_ptr(), best_s.shape[1], _c(cand_key).data_ptr(),
                                         _c(cand_id).data_ptr(), _c(cnt).data_ptr(), cap, N.stream_ptr(Q.device)),
            "score_filter")


def score_filter_lemp(Q: torch.Tensor, X: torch.Tensor, ids: torch.Tensor, best_s: torch.Tensor,
                      cand_key: torch.Tensor, cand_id: torch.Tensor, cnt: torch.Tensor,
                      qlen: Optional[torch.Tensor] = None, xlen: Optional[torch.Tensor] = None) -> None:
    """``score_filter`` with the LEMP length bound applied per 64 x 64 tile on the device:
    with ``qlen`` [B] / ``xlen`` [n] (vector norms), a tile none of whose
    queries can be beaten by its longest item (``|q| max|x| <= best_s[q, -1]``, with an
    fp32 rounding slack) is skipped -- exact, and no host sync."""
    B, D = Q.shape
    n = X.shape[0]
    cap = cand_key.shape[1]
    if X.shape[1] != D or ids.numel() != n or best_s.shape[0] != B or cnt.numel() != B or cand_id.shape != (B, cap):
        raise ValueError("score_filter_lemp: shape mismatch")
    if (qlen is None) != (xlen is None):
        raise ValueError("score_filter_lemp: qlen and xlen go together")
    if qlen is not None and (qlen.numel() != B or xlen.numel() != n):
        raise ValueError("score_filter_lemp: qlen [B] / xlen [n]")
    slack = 1.0 + 1e-4 + D * 2.4e-7  # > the relative fp32 error of a D-term dot product and of |q| |x|
    N.check(N.require().fps_score_filter_lemp(
        _c(Q).data_ptr(), _c(X).data_ptr(), _c(ids).data_ptr(), B, n, D, _c(best_s).data_ptr(), best_s.shape[1],
        None if qlen is None else _c(qlen.float()).data_ptr(), None if xlen is None else _c(xlen.float()).data_ptr(),
        slack, _c(cand_key).data_ptr(), _c(cand_id).data_ptr(), _c(cnt).data_ptr(), cap, N.stream_ptr(Q.device)),
        "score_filter_lemp")


#: embedding dims the bf16 scorer is built for (``csrc/kernels/score_bf16.hip``)
BF16_SCORE_DIMS = (32, 64, 128)


def bf16_score_margin(D: int) -> float:
    """``c`` with ``|S_bf16 - S_fp32| <= c |q| |x|`` for RNE-rounded bf16 operands and fp32
    accumulation (``score_bf16.hip`` header: 2u + u^2 + 2 D 2^-24, u = 2^-8), widened by
    0.1 % for the fp32 norms."""
    u = 2.0 ** -8
    return (2 * u + u * u + 2 * D * 2.0 ** -24) * 1.001


def coord_block_bounds(X: torch.Tensor, xlen: torch.Tensor) -> torch.Tensor:
    """``[ceil(n / 32), D, 2]`` min / max of the normalised coordinates ``x_c / |x|``
    over every block of 32 consecutive items (the last block over its own items):
    the per-block table of the LEMP COORD bound in ``score_filter_bf16``."""
    n, D = X.shape
    xn = X.float() / xlen.float().clamp_min(1e-30).view(-1, 1)
    nb = -(-n // 32)
    pad = nb * 32 - n
    if pad:
        xn = torch.cat([xn, xn[-1:].expand(pad, D)], 0)
    xn = xn.view(nb, 32, D)
    return torch.stack([xn.amin(1), xn.amax(1)], 2).contiguous()


def topk_scan_prep(Q: torch.Tensor, k: int, bf16: bool = True):
    """The set-up of a fresh fused top-K scan in ONE launch (``topk.hip``
    ``topk_scan_prep_kernel``): ``(qlen [B] fp32 row norms, Qb [B, D] bf16 (RNE) or None,
    best_s [B, k] = -inf, best_i [B, k] = -1, cnt [B] int32 = 0, ovf [1] int32 = 0)``."""
    Q = _c(Q.float())
    B, D = Q.shape
    dev = Q.device
    if not Q.is_cuda or k <= 0 or k > TOPK_MAX_K:
        raise ValueError("topk_scan_prep: a cuda [B, D] query batch and 0 < k <= TOPK_MAX_K")
    qlen = torch.empty(B, dtype=torch.float32, device=dev)
    Qb = torch.empty((B, D), dtype=torch.bfloat16, device=dev) if bf16 else None
    best_s = torch.empty((B, k), dtype=torch.float32, device=dev)
    best_i = torch.empty((B, k), dtype=torch.int64, device=dev)
    cnt = torch.empty(B, dtype=torch.int32, device=dev)
    ovf = torch.empty(1, dtype=torch.int32, device=dev)
    N.check(N.require().fps_topk_scan_prep(Q.data_ptr(), B, D, k, qlen.data_ptr(),
                                           Qb.data_ptr() if Qb is not None else None, best_s.data_ptr(),
                                           best_i.data_ptr(), cnt.data_ptr(), ovf.data_ptr(),
                                           N.stream_ptr(dev)), "topk_scan_prep")
    return qlen, Qb, best_s, best_i, cnt, ovf


def block_max32(xlen: torch.Tensor) -> torch.Tensor:
    """``[ceil(n / 32)]`` max of every 32 consecutive entries (the last block over its own)."""
    n = xlen.numel()
    nb = -(-n // 32)
    x = xlen.float()
    if nb * 32 != n:
        x = torch.cat([x, x.new_zeros(nb * 32 - n)])
    return x.view(nb, 32).amax(1)


_SB_KNOBS = False


def score_filter_bf16(Qb: torch.Tensor, Xb: torch.Tensor, best_s: torch.Tensor, cand_pos: torch.Tensor,
                      cnt: torch.Tensor, qlen: torch.Tensor, xlen: Optional[torch.Tensor], coord=None,
                      stats: Optional[torch.Tensor] = None, gate: Optional[torch.Tensor] = None,
                      xbm: Optional[torch.Tensor] = None) -> None:
    """Candidate filter on bf16 MFMA (GPU only, K8 fast path): every item ``i`` whose bf16
    score can exceed ``best_s[b, -1]`` (margin ``bf16_score_margin(D) |q_b| max|x|``) gets
    its position appended to row ``b`` of ``cand_pos`` ``[B, cap]`` (int64); ``cnt[b]``
    (zeroed by the caller) counts them all.  ``cand_rescore`` turns the list into exact
    (key, id) candidates for ``topk_merge_cand``.  ``coord = (qf int32[B], qbf[B], cb)``
    turns on the LEMP COORD + length bounds per (32 queries, 32 items) block pair
    (``cb`` = ``coord_block_bounds`` of these items); ``stats`` (int32[2]) counts the
    block pairs scored / skipped; ``gate`` (int32[1], optional): the COORD bound is
    evaluated only while ``gate[0] != 0`` (``coord_gate``)."""
    B, D = Qb.shape
    n = Xb.shape[0]
    cap = cand_pos.shape[1]
    if Qb.dtype != torch.bfloat16 or Xb.dtype != torch.bfloat16 or Xb.shape[1] != D or D not in BF16_SCORE_DIMS:
        raise ValueError(f"score_filter_bf16: bf16 [B, D] / [n, D] with D in {BF16_SCORE_DIMS}")
    if xbm is None:  # the kernel reads the longest item of every 32-item block
        if xlen is None or xlen.numel() != n:
            raise ValueError("score_filter_bf16: xlen [n] or xbm [ceil(n / 32)]")
        xbm = block_max32(xlen)
    if best_s.shape[0] != B or cnt.numel() != B or cand_pos.dtype != torch.int64 or qlen.numel() != B \
            or xbm.numel() != -(-n // 32):
        raise ValueError("score_filter_bf16: shape mismatch")
    qf = qbf = cb = None
    if coord is not None:
        qf, qbf, cb = coord
        if qf.dtype != torch.int32 or qf.numel() != B or qbf.numel() != B or tuple(cb.shape) != (-(-n // 32), D, 2):
            raise ValueError("score_filter_bf16: coord = (int32 qf[B], qbf[B], cb[ceil(n/32), D, 2])")
        if DEBUG:
            check_index(qf, D, "score_filter_bf16 qf")
        qf, qbf, cb = _c(qf), _c(qbf.float()), _c(cb.float())
    slack = 1.0 + 1e-4 + D * 2.4e-7
    global _SB_KNOBS
    if not _SB_KNOBS:  # A/B switches, read once: FPS_SB_MIN_WGS = fewest workgroups per scorer launch (0: 1024
        _SB_KNOBS = True  # items each); FPS_SB_ILV=1: interleaved MFMA chains of the query blocks;
        # FPS_SB_PD = 1 / 2: prefetch distance of the LDS item stages; FPS_SB_CUR2=1: a stage's LDS operand reads
        # all issued at its start
        mw, ilv, pd = os.environ.get("FPS_SB_MIN_WGS"), os.environ.get("FPS_SB_ILV"), os.environ.get("FPS_SB_PD")
        if os.environ.get("FPS_SB_CUR2") is not None:
            N.require().fps_score_set_cur2(int(os.environ["FPS_SB_CUR2"]))
        if mw is not None:
            N.require().fps_score_set_min_wgs(int(mw))
        if ilv is not None:
            N.require().fps_score_set_ilv(int(ilv))
        if pd is not None:
            N.require().fps_score_set_pd(int(pd))
    N.check(N.require().fps_score_filter_bf16(
        _c(Qb).data_ptr(), _c(Xb).data_ptr(), B, n, D, _c(best_s).data_ptr(), best_s.shape[1],
        _c(qlen.float()).data_ptr(), _c(xbm.float()).data_ptr(), bf16_score_margin(D), slack,
        _c(cand_pos).data_ptr(), _c(cnt).data_ptr(), cap, N.ptr(qf), N.ptr(qbf), N.ptr(cb), N.ptr(stats),
        N.ptr(gate), N.stream_ptr(Qb.device)), "score_filter_bf16")


def coord_gate(stats: torch.Tensor, prev: torch.Tensor, gate: torch.Tensor, num: int = 1, den: int = 4,
               rest: int = 3) -> None:
    """Device-side COORD switch of a LEMP scan (GPU only; the scorer evaluates the
    bound while ``gate[0] > 0``).  After a segment that evaluated it: on if it skipped
    at least ``num / den`` of the (query, item) block pairs (``stats`` = cumulative
    scored / skipped, ``prev`` = their values at the previous call), else off for the
    next ``rest`` segments, then probed again.  No host sync: the bound is exact
    either way, the gate only decides whether evaluating it pays."""
    N.check(N.require().fps_coord_gate(_c(stats).data_ptr(), _c(prev).data_ptr(), _c(gate).data_ptr(), int(num),
                                       int(den), int(rest), N.stream_ptr(stats.device)), "coord_gate")


def cand_rescore(Q: torch.Tensor, X: torch.Tensor, ids: torch.Tensor, best_s: torch.Tensor, cand_key: torch.Tensor,
                 cand_id: torch.Tensor, cnt: torch.Tensor) -> None:
    """Exact fp32 scores of ``score_filter_bf16``'s candidates (GPU only): ``cand_id`` holds
    item positions in ``X`` on entry and ``ids[pos]`` on exit; ``cand_key`` the
    order-preserving keys, bit-identical to ``score_filter``'s (same fp32 MFMA chain), or 0
    where the exact score is not strictly above ``best_s[b, -1]``."""
    B, D = Q.shape
    cap = cand_key.shape[1]
    if X.shape[1] != D or D not in BF16_SCORE_DIMS or cand_id.shape != (B, cap) or cnt.numel() != B:
        raise ValueError("cand_rescore: shape mismatch")
    N.check(N.require().fps_cand_rescore(_c(Q).data_ptr(), _c(X).data_ptr(), _c(ids.long()).data_ptr(), B, D,
                                         _c(best_s).data_ptr(), best_s.shape[1], _c(cnt).data_ptr(), cap,
                                         _c(cand_key).data_ptr(), _c(cand_id).data_ptr(), N.stream_ptr(Q.device)),
            "cand_rescore")


def topk_merge_cand(cand_key: torch.Tensor, cand_id: torch.Tensor, cnt: torch.Tensor, best_s: torch.Tensor,
                    best_i: torch.Tensor, overflow: Optional[torch.Tensor] = None, reset_cnt: bool = False) -> None:
    """Merge ``score_filter`` candidate lists into the running top-k in place (K13).
    ``overflow`` (int32 [1]): set to 1 on the device when a row had more than ``cap``
    candidates (its merge is incomplete; the caller rescans).  ``reset_cnt``: ``cnt``
    (contiguous int32) is zeroed on the device once merged -- ready for the next
    segment's filter without a fill launch."""
    B, cap = cand_key.shape
    if reset_cnt and not (cnt.is_contiguous() and cnt.dtype == torch.int32):
        raise ValueError("topk_merge_cand: reset_cnt needs a contiguous int32 cnt")
    N.check(N.require().fps_topk_merge_cand(_c(cand_key).data_ptr(), _c(cand_id).data_ptr(), _c(cnt).data_ptr(), cap,
                                            B, _c(best_s).data_ptr(), _c(best_i).data_ptr(), best_s.shape[1],
                                            None if overflow is None else overflow.data_ptr(), int(reset_cnt),
                                            N.stream_ptr(best_s.device)), "topk_merge_cand")


def mf_online_phase(U: torch.Tensor, urow: Optional[torch.Tensor], irow: torch.Tensor,
                    target: Optional[torch.Tensor], lr: float, W: torch.Tensor, du: torch.Tensor,
                    trained: Optional[torch.Tensor] = None) -> None:
    """One SGD phase of the online MF + top-K worker (``mf_online.hip``, GPU only): for
    every entry t with ``irow[t] >= 0``: ``e = target[t] - <U[urow[t]], W[irow[t]]>``
    (target 0 when None: a negative), ``du[urow[t]] += lr e W[irow[t]]`` (distinct rows),
    ``W[irow[t]] += lr e U[urow[t]]`` (atomics), every entry reading the item rows as the
    phase starts; ``urow`` None = identity.  ``trained`` (int64 scalar, optional) counts
    the applied entries."""
    n, D = irow.numel(), U.shape[1]
    if not (U.is_cuda and U.dtype == W.dtype == du.dtype == torch.float32 and W.shape[1] == D == du.shape[1]):
        raise ValueError("mf_online_phase: cuda fp32 U / W / du with one D")
    if irow.dtype != torch.int64 or (urow is not None and (urow.dtype != torch.int64 or urow.numel() != n)) \
            or (target is not None and target.numel() != n) or D > 256:
        raise ValueError("mf_online_phase: int64 irow / urow [n], target [n], D <= 256")
    if DEBUG:
        check_index(irow, W.shape[0], "mf_online_phase irow", allow_negative=True)
    gbuf = torch.empty(n, dtype=torch.float32, device=U.device)
    N.check(N.require().fps_mf_online_phase(_c(U).data_ptr(), N.ptr(None if urow is None else _c(urow)),
                                            _c(irow).data_ptr(),
                                            N.ptr(None if target is None else _c(target.float())), n, D, float(lr),
                                            W.data_ptr(), du.data_ptr(), gbuf.data_ptr(), N.ptr(trained),
                                            N.stream_ptr(U.device)),
            "mf_online_phase")


def index_refresh(rows: torch.Tensor, pos: torch.Tensor, W: torch.Tensor, vecs: torch.Tensor,
                  vecs_bf: Optional[torch.Tensor], lengths: torch.Tensor) -> None:
    """Copy the local item rows ``W[rows]`` into a LEMP index at positions ``pos[row]``
    (``< 0``: not indexed): fp32 vectors, the bf16 shadow (RNE, as ``.bfloat16()``) and
    the lengths (``mf_online.hip``, GPU only)."""
    D = W.shape[1]
    if not (W.is_cuda and rows.dtype == pos.dtype == torch.int64 and vecs.shape[1] == D and D <= 256):
        raise ValueError("index_refresh: cuda, int64 rows / pos, D <= 256")
    if vecs_bf is not None and (vecs_bf.dtype != torch.bfloat16 or vecs_bf.shape != vecs.shape):
        raise ValueError("index_refresh: bf16 shadow of vecs' shape")
    N.check(N.require().fps_index_refresh(_c(rows).data_ptr(), rows.numel(), _c(pos).data_ptr(), _c(W).data_ptr(), D,
                                          vecs.data_ptr(), N.ptr(vecs_bf), lengths.data_ptr(),
                                          N.stream_ptr(W.device)), "index_refresh")


def round_plan(users: torch.Tensor):
    """``(by_user, rnd, first, nu)`` of a batch of users (GPU, one launch after the sort,
    ``topk.hip`` ``round_plan_kernel``): ``by_user`` = entries stably sorted by user,
    ``rnd[e]`` = e's occurrence round, ``first[e]`` = position in ``by_user`` of the
    first entry of e's user, ``nu[e]`` = that user's entry count (int32)."""
    B = users.numel()
    if not users.is_cuda or B > (1 << 20):
        raise ValueError("round_plan: a cuda tensor of at most 2^20 users")
    rnd = torch.empty(B, dtype=torch.int32, device=users.device)
    first = torch.empty_like(rnd)
    nu = torch.empty_like(rnd)
    su, by_user = torch.sort(users.long(), stable=True)
    N.check(N.require().fps_round_plan(su.data_ptr(), by_user.data_ptr(), B, rnd.data_ptr(), first.data_ptr(),
                                       nu.data_ptr(), N.stream_ptr(users.device)), "round_plan")
    return by_user, rnd, first, nu


def topk_seen_merge(ss: torch.Tensor, ii: torch.Tensor, K: int, users: torch.Tensor, items: torch.Tensor,
                    rnd: torch.Tensor, first: torch.Tensor, nu: torch.Tensor, by_user: torch.Tensor,
                    ring: torch.Tensor, ring_cur: torch.Tensor):
    """Seen-aware merge of gathered partial top-K lists for a whole micro-batch, all
    occurrence rounds at once (GPU only, K13; ``topk.hip`` ``seen_merge_kernel``), then
    the batch's rated items into the ring store.  ``ss`` / ``ii`` ``[B, m]`` partial
    scores / item ids; entry ``e`` of user ``users[e]`` is its user's ``rnd[e]``-th in the
    batch, the user's entries are ``by_user[first[e] : first[e] + nu[e]]`` (stable);
    ``ring`` ``[U, M]`` int32 / ``ring_cur`` ``[U]`` int64 the dense seen store (updated).
    Returns ``best_s`` / ``best_i`` ``[B, K]`` (key desc, ties by smaller id; -inf / -1 past
    the kept candidates)."""
    B, m = ss.shape
    M = ring.shape[1]
    if not (ss.is_cuda and ss.dtype == torch.float32 and ii.dtype == torch.int64 and ii.shape == ss.shape):
        raise ValueError("topk_seen_merge: cuda fp32 ss / int64 ii [B, m]")
    if m > TOPK_CAND_CAP or K > TOPK_MAX_K or M > TOPK_MAX_K or ring.dtype != torch.int32 \
            or ring_cur.dtype != torch.int64:
        raise ValueError("topk_seen_merge: m <= TOPK_CAND_CAP, K / M <= TOPK_MAX_K, int32 ring, int64 cursors")
    for t, dt in ((users, torch.int64), (items, torch.int64), (rnd, torch.int32), (first, torch.int32),
                  (nu, torch.int32), (by_user, torch.int64)):
        if t.dtype != dt or t.numel() != B:
            raise ValueError("topk_seen_merge: users / items / by_user int64 [B], rnd / first / nu int32 [B]")
    if DEBUG:
        check_index(users, ring.shape[0], "topk_seen_merge users")
    best_s = torch.empty((B, K), dtype=torch.float32, device=ss.device)
    best_i = torch.empty((B, K), dtype=torch.int64, device=ss.device)
    cpre = torch.empty(B, dtype=torch.int64, device=ss.device)
    N.check(N.require().fps_topk_seen_merge(
        _c(ss).data_ptr(), _c(ii).data_ptr(), B, m, int(K), _c(users).data_ptr(), _c(items).data_ptr(),
        _c(rnd).data_ptr(), _c(first).data_ptr(), _c(nu).data_ptr(), _c(by_user).data_ptr(), ring.data_ptr(),
        ring_cur.data_ptr(), M, cpre.data_ptr(), best_s.data_ptr(), best_i.data_ptr(), N.stream_ptr(ss.device)),
        "topk_seen_merge")
    return best_s, best_i


def score_gemm(Q: torch.Tensor, X: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
    """``out[b, i] = <Q[b], X[i]>`` on MFMA (fp32 in/accumulate, K8 scoring).  ``out`` may be
    a column slice of a wider buffer (row stride taken from it)."""
    B, D = Q.shape
    N = X.shape[0]
    if out is None:
        out = torch.empty((B, N), dtype=torch.float32, device=Q.device)
    if Q.is_cuda:
        if out.stride(1) != 1:
            raise ValueError("score_gemm output must have unit column stride")
        lib = N_.require()
        N_.check(lib.fps_score_gemm(_c(Q).data_ptr(), _c(X).data_ptr(), out.data_ptr(), B, N, D, out.stride(0),
                                    N_.stream_ptr(Q.device)), "score_gemm")
        return out
    out.copy_(Q.float() @ X.float().T)
    return out


N_ = N
PA_VARIANTS = {"PA": 0, "PA-I": 1, "PA-II": 2}
PA_MODES = {"ova": 0, "pb": 1, "ml": 2}


def flip_sentinel(table: torch.Tensor, rows: torch.Tensor) -> None:
    """Torch twin of the kernels' untouched-row sentinel flip: entries of ``table[rows]``
    holding -0.0 become +0.0 (``ShardedTable(touch_sentinel=True)``)."""
    r = rows.long()
    r = r[r >= 0]  # padding slots
    x = table[r]
    table[r] = torch.where((x == 0) & torch.signbit(x), torch.zeros_like(x), x)


def flip_masked(table: torch.Tensor, mask: torch.Tensor) -> None:
    """Sentinel flip of the rows whose ``mask`` entry is set (bool / uint8 ``[rows]``):
    their -0.0 entries become +0.0.  Rows outside the mask are not read."""
    if _on_gpu(table) and table.dtype == torch.float32:
        m = mask.view(torch.uint8) if mask.dtype == torch.bool else mask
        N.check(N.require().fps_flip_masked(_c(table).data_ptr(), _c(m).data_ptr(), table.shape[0],
                                            table[0].numel() if table.shape[0] else 0, N.stream_ptr(table.device)),
                "flip_masked")
        return
    w = table.view(table.shape[0], -1)
    w.masked_fill_((w == 0) & torch.signbit(w) & mask.bool().view(-1, 1), 0.0)


def _wmap_cpu(delta, rows: int):
    """CPU twin of the kernels' write map: a zero buffer over the pulled rows, added
    into ``delta`` at the map afterwards."""
    return torch.zeros((rows,) + tuple(delta.shape[1:]), dtype=delta.dtype)


def pa_binary(indptr, xval, pos, w, y, variant: str, C: float, delta, with_loss: bool = False,
              flip: Optional[torch.Tensor] = None, wmap: Optional[torch.Tensor] = None):
    """Binary PA on a CSR micro-batch (K10); returns ``(pred int8[B], loss or None)``.
    ``flip`` (the in-place path: the table itself): the first pull of a feature turns
    its untouched sentinel -0.0 into +0.0.  ``wmap`` (int32, optional): the delta of
    pulled row ``r`` is added to ``delta[wmap[r]]`` (a push the worker applies to the
    owner's table itself)."""
    B = indptr.numel() - 1
    if flip is not None and not xval.is_cuda:
        flip_sentinel(flip.view(-1, 1), pos)
    if xval.is_cuda:
        pred = torch.empty(B, dtype=torch.int8, device=xval.device)
        loss = torch.zeros(1, device=xval.device) if with_loss else None
        lib = N.require()
        wm = None if wmap is None else _c(wmap.to(torch.int32))
        N.check(lib.fps_pa_binary(_c(indptr).data_ptr(), _c(xval).data_ptr(), _c(pos).data_ptr(), _c(w).data_ptr(),
                                  _c(y).data_ptr(), B, PA_VARIANTS[variant], C, _c(delta).data_ptr(),
                                  pred.data_ptr(), N.ptr(loss), N.ptr(flip), N.ptr(wm), N.stream_ptr(xval.device)),
                "pa_binary")
        return pred, loss
    if wmap is not None:
        tmp = _wmap_cpu(delta.view(-1, 1), w.numel())
        pred, loss = R.pa_binary(indptr, xval, pos, w, y, PA_VARIANTS[variant], C, tmp.view(-1))
        delta.view(-1).index_add_(0, wmap.long(), tmp.view(-1))
        return pred, torch.tensor([loss])
    pred, loss = R.pa_binary(indptr, xval, pos, w, y, PA_VARIANTS[variant], C, delta)
    return pred, torch.tensor([loss])


def pa_multi(indptr, xval, pos, W, y, mode: str, variant: str, C: float, cost, delta, with_loss: bool = False,
             flip: Optional[torch.Tensor] = None, wmap: Optional[torch.Tensor] = None):
    """Multiclass PA (OVA / cost PB / cost ML) on a CSR micro-batch (K11/K12); L <= 64.
    ``flip`` / ``wmap``: as ``pa_binary``."""
    B = indptr.numel() - 1
    L = W.shape[1]
    if flip is not None and not xval.is_cuda:
        flip_sentinel(flip, pos)
    if xval.is_cuda:
        pred = torch.empty(B, dtype=torch.int32, device=xval.device)
        loss = torch.zeros(1, device=xval.device) if with_loss else None
        lib = N.require()
        wm = None if wmap is None else _c(wmap.to(torch.int32))
        N.check(lib.fps_pa_multi(_c(indptr).data_ptr(), _c(xval).data_ptr(), _c(pos).data_ptr(), _c(W).data_ptr(), L,
                                 _c(y).data_ptr(), B, PA_MODES[mode], PA_VARIANTS[variant], C, N.ptr(cost),
                                 _c(delta).data_ptr(), pred.data_ptr(), N.ptr(loss), N.ptr(flip), N.ptr(wm),
                                 N.stream_ptr(xval.device)), "pa_multi")
        return pred, loss
    if wmap is not None:
        tmp = _wmap_cpu(delta, W.shape[0])
        pred, loss = R.pa_multi(indptr, xval, pos, W, y, PA_MODES[mode], PA_VARIANTS[variant], C, cost, tmp)
        delta.index_add_(0, wmap.long(), tmp)
        return pred, torch.tensor([loss])
    pred, loss = R.pa_multi(indptr, xval, pos, W, y, PA_MODES[mode], PA_VARIANTS[variant], C, cost, delta)
    return pred, torch.tensor([loss])


def mf_sq_err(U, I, uid, iid, r) -> torch.Tensor:
    """Sum of squared rating errors (device scalar on GPU) (K14)."""
    if _on_gpu(U):
        out = torch.zeros(1, dtype=torch.float64, device=U.device)
        lib = N.require()
        N.check(lib.fps_mf_sq_err(_c(U).data_ptr(), _c(I).data_ptr(), _c(uid).data_ptr(), _c(iid).data_ptr(),
                                  _c(r).data_ptr(), uid.numel(), U.shape[1], out.data_ptr(), N.stream_ptr(U.device)),
                "mf_sq_err")
        return out
    return torch.tensor([R.mf_sq_err(U, I, uid, iid, r)], dtype=torch.float64)

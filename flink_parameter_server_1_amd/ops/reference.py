"""Plain-PyTorch reference implementations of every kernel in ``csrc/kernels``.

They define the semantics the HIP kernels are tested against (numerics tests
compare the gfx950 kernel with these on the same inputs) and are the CPU
execution path of the tensor engine (gloo multi-process tests, CPU boxes).
"""
from __future__ import annotations

import torch

M32 = 0xFFFFFFFF


def fmix32(x: torch.Tensor) -> torch.Tensor:
    """murmur3 finalizer on int64 tensors holding uint32 values."""
    x = x ^ (x >> 16)
    x = (x * 0x85EBCA6B) & M32
    x = x ^ (x >> 13)
    x = (x * 0xC2B2AE35) & M32
    x = x ^ (x >> 16)
    return x


def hash_uniform(seed: int, ids: torch.Tensor, j: torch.Tensor) -> torch.Tensor:
    """U[0,1) for every (id, j) pair; ids [N,1] int64, j [1,D] int64 -> [N, D] fp32."""
    h0 = fmix32(torch.tensor((seed ^ 0x9E3779B9) & M32, dtype=torch.int64))
    h = fmix32(h0 ^ (ids & M32))
    h = fmix32(h ^ ((ids >> 32) & M32) ^ 0x27D4EB2F)
    h = fmix32((h + j * 0x9E3779B9) & M32)
    return (h >> 8).to(torch.float32) * (1.0 / 16777216.0)


def init_rows(table: torch.Tensor, id_base: int, id_stride: int, lo: float, hi: float, seed: int):
    n, d = table.shape
    ids = (id_base + torch.arange(n, dtype=torch.int64) * id_stride).view(-1, 1)
    j = torch.arange(d, dtype=torch.int64).view(1, -1)
    u = hash_uniform(seed, ids, j).to(table.dtype)  # k / 2^24: exact in any float dtype
    table.copy_((lo + (hi - lo) * u).to(table.device))
    return table


def init_values(ids: torch.Tensor, dim: int, lo: float, hi: float, seed: int) -> torch.Tensor:
    j = torch.arange(dim, dtype=torch.int64).view(1, -1)
    return lo + (hi - lo) * hash_uniform(seed, ids.to(torch.int64).view(-1, 1).cpu(), j)


def gather_rows(table, idx, out_dtype=torch.float32, touched=None):
    """``table[idx]``; idx < 0 (a padding slot) serves a zero row and marks nothing."""
    idx = idx.long()
    keep = idx >= 0
    if touched is not None:
        touched[idx[keep]] = 1
    if table.shape[0] == 0:  # a rank without a shard serves only padding slots
        return torch.zeros((idx.numel(),) + tuple(table.shape[1:]), dtype=out_dtype, device=table.device)
    out = table[idx.clamp_min(0)].to(out_dtype)
    return torch.where(keep.view(-1, *([1] * (out.dim() - 1))), out, torch.zeros_like(out))


OPS = {"add": 0, "set": 1, "sgd": 2, "adagrad": 3}


def apply_rows(table, idx, delta, op="add", lr=0.0, eps=1e-10, state=None, touched=None):
    idx = idx.long()
    keep = idx >= 0
    idx, delta = idx[keep], delta[keep].to(table.dtype)
    # -0.0 deltas add as +0.0 (the kernels' pos0): an untouched row's -0.0 sentinel flips
    delta = torch.where(delta == 0, torch.zeros_like(delta), delta)
    if touched is not None:
        touched[idx] = 1
    if op == "add_unique" and idx.numel() and torch.unique(idx).numel() != idx.numel():
        # the GPU kernel is a plain read-modify-write per row: repeated rows lose updates
        raise ValueError("add_unique with repeated rows")
    if op in ("add", "add_unique"):
        table.index_add_(0, idx, delta)
    elif op == "set":
        table[idx] = delta
    elif op == "sgd":
        table.index_add_(0, idx, -lr * delta)
    elif op == "adagrad":
        state[idx] += delta * delta
        table[idx] -= lr * delta * torch.rsqrt(state[idx] + eps)
    elif op == "add_renorm":  # unique idx: w += g, state[row] = |w|
        table.index_add_(0, idx, delta.to(table.dtype))
        state[idx] = table[idx].norm(dim=1).to(state.dtype)
    else:
        raise ValueError(op)
    return table


def shard_of(keys: torch.Tensor, W: int, part_kind: int, block: int):
    k = keys.long().abs()
    if part_kind == 0:
        return k % W, k // W
    if part_kind == 2:  # sparse ids: the id itself is the owner's hash-table key
        return k % W, keys.long()
    d = torch.clamp(k // block, max=W - 1)
    return d, k - d * block


def dedup(keys: torch.Tensor, W: int, part_kind: int, block: int):
    """Unique keys grouped by destination shard (compact layout).

    Returns ``counts[W] int32, prefix[W+1] int32, uniq[U] int32 (local keys,
    shard-major), pos[B] int32`` with ``uniq[pos[b]] == local(keys[b])``.
    Inside a shard group unique keys keep first-occurrence order (the GPU
    kernel's order there is arbitrary).
    """
    keys = keys.long()
    uniq_g, first_idx = _unique_first(keys)
    dest, local = shard_of(uniq_g, W, part_kind, block)
    counts = torch.bincount(dest, minlength=W)
    order = torch.argsort(dest * (keys.numel() + 1) + first_idx, stable=True)
    slot_of = torch.empty_like(order)
    slot_of[order] = torch.arange(order.numel())
    uniq = local[order].to(torch.int32)
    inv = torch.searchsorted(uniq_g, keys)
    pos = slot_of[inv].to(torch.int32)
    prefix = torch.zeros(W + 1, dtype=torch.int32)
    prefix[1:] = torch.cumsum(counts, 0).to(torch.int32)
    return counts.to(torch.int32), prefix, uniq, pos


def route(keys: torch.Tensor, W: int, part_kind: int, block: int):
    """``dedup``'s layout without de-duplication: every request is an entry of
    ``uniq`` (shard-major, request order inside a shard), ``pos`` a permutation."""
    keys = keys.long()
    dest, local = shard_of(keys, W, part_kind, block)
    counts = torch.bincount(dest, minlength=W)
    order = torch.argsort(dest, stable=True)
    pos = torch.empty_like(order)
    pos[order] = torch.arange(order.numel(), device=keys.device)
    prefix = torch.zeros(W + 1, dtype=torch.int32, device=keys.device)
    prefix[1:] = torch.cumsum(counts, 0).to(torch.int32)
    return counts.to(torch.int32), prefix, local[order].to(torch.int32), pos.to(torch.int32)


def _unique_first(keys):
    uniq, inv = torch.unique(keys, sorted=True, return_inverse=True)
    first = torch.full((uniq.numel(),), keys.numel(), dtype=torch.long)
    first.scatter_reduce_(0, inv, torch.arange(keys.numel()), reduce="amin")
    return uniq, first


def bucketize(keys, W, part_kind, block):
    d, _ = shard_of(keys, W, part_kind, block)
    return d.to(torch.int32), torch.bincount(d, minlength=W).to(torch.int32)


def mf_sgd_local(U, I, uid, iid, r, lr, lam=0.0, user_atomic=False):
    uid, iid = uid.long(), iid.long()
    u, i = U[uid], I[iid]
    e = r - (u * i).sum(1)
    du = lr * (e[:, None] * i - lam * u)
    di = lr * (e[:, None] * u - lam * i)
    if user_atomic:
        U.index_add_(0, uid, du)
    else:
        U[uid] = u + du
    I.index_add_(0, iid, di)


def mf_sgd_pulled(U, uid, r, rows, pos, delta, lr, lam=0.0, user_atomic=False):
    uid, pos = uid.long(), pos.long()
    u, i = U[uid], rows[pos].to(U.dtype)
    e = r - (u * i).sum(1)
    du = lr * (e[:, None] * i - lam * u)
    di = lr * (e[:, None] * u - lam * i)
    if user_atomic:
        U.index_add_(0, uid, du)
    else:
        U[uid] = u + du
    delta.index_add_(0, pos, di)


def lock_acquire(lock, rows, src: int):
    """Sequential semantics of ``lock_acquire_kernel``: take free locks, keep own."""
    rows = rows.long()
    granted = torch.zeros(rows.numel(), dtype=torch.uint8)
    for b, r in enumerate(rows.tolist()):
        if int(lock[r]) in (-1, src):
            lock[r] = src
            granted[b] = 1
    return granted


def lock_release(lock, rows, granted):
    rows = rows.long()
    lock[rows[granted.bool()]] = -1


def rot_block_of(iid, W, half):
    """Item -> (block 2q+h, row inside the block) of the rotation layout (``rotate.hip``)."""
    i = iid.long()
    q = i % W
    loc = i // W
    hq = half.long()[q]
    h = (loc >= hq).long()
    return 2 * q + h, loc - h * hq


def rot_partition(uid, iid, rating, W, half):
    """Ratings grouped by item block: ``(counts[K], ptr[K+1], uid, row, rating)`` (stable order)."""
    K = 2 * W
    b, row = rot_block_of(iid, W, half)
    order = torch.argsort(b, stable=True)
    counts = torch.bincount(b, minlength=K).to(torch.int32)
    ptr = torch.zeros(K + 1, dtype=torch.int32)
    ptr[1:] = torch.cumsum(counts, 0)
    return counts, ptr, uid[order].to(torch.int32), row[order].to(torch.int32), rating[order]


def tile_partition(uid, iid, rating, W, half, R, T, P=1, upp=None):
    """Ratings grouped by (user phase ``uid // upp``, item block, tile of R rows):
    ``(ptr[P*2W*T+1], uid, row_in_block, rating)``."""
    b, row = rot_block_of(iid, W, half)
    phase = uid.long() // upp if (P > 1 and upp) else torch.zeros_like(b)
    bucket = (phase * 2 * W + b) * T + row // R
    KT = P * 2 * W * T
    order = torch.argsort(bucket, stable=True)
    counts = torch.bincount(bucket, minlength=KT)
    ptr = torch.zeros(KT + 1, dtype=torch.int32)
    ptr[1:] = torch.cumsum(counts, 0)
    return ptr, uid[order].to(torch.int32), row[order].to(torch.int32), rating[order]


def pair_sgd_pulled(rows, pa, pb, label, delta, lr, loss_kind=0):
    """Pairwise embedding SGD on pulled rows; returns the loss sum (see ``pair.hip``)."""
    pa, pb = pa.long(), pb.long()
    a, b = rows[pa].to(torch.float32), rows[pb].to(torch.float32)
    s = (a * b).sum(1)
    if loss_kind == 0:
        g = label - torch.sigmoid(s)
        z = torch.where(label > 0.5, s, -s)
        loss = torch.nn.functional.softplus(-z).sum()
    else:
        g = label - s
        loss = 0.5 * (g * g).sum()
    c = (lr * g)[:, None]
    delta.index_add_(0, pa, c * b)
    delta.index_add_(0, pb, c * a)
    return float(loss)


def csr_group(keys: torch.Tensor, n_groups: int):
    """Counting sort: ``ptr[G+1]`` offsets and ``order`` = request indices grouped by key."""
    k = keys.long()
    order = torch.argsort(k, stable=True).to(torch.int32)
    cnt = torch.bincount(k, minlength=n_groups)
    ptr = torch.zeros(n_groups + 1, dtype=torch.int32)
    ptr[1:] = torch.cumsum(cnt, 0).to(torch.int32)
    return ptr, order


def mf_sgd_grouped(U, I, uid, r, ptr, order, lr, lam=0.0, delta=None):
    """Per group (item / unique slot) sequential SGD in ``order``; ``delta`` given =
    pulled mode (``I`` read only, ``delta[g] = final - initial``), else ``I`` updated in place."""
    uid, ptr, order = uid.long(), ptr.long(), order.long()
    G = ptr.numel() - 1
    for g in range(G):
        a, b = int(ptr[g]), int(ptr[g + 1])
        if a == b:
            continue
        i0 = I[g].to(torch.float32).clone()
        i = i0.clone()
        for s in range(a, b):
            rb = int(order[s])
            u = U[uid[rb]].clone()
            e = float(r[rb]) - float(torch.dot(u, i))
            U[uid[rb]] = u + lr * (e * i - lam * u)
            i = i + lr * (e * u - lam * i)
        if delta is not None:
            delta[g] = i - i0
        else:
            I[g] = i


def _u32(x):
    return torch.as_tensor(x, dtype=torch.int64) & M32


def rnd(seed: int, counter: int, i: torch.Tensor, salt) -> torch.Tensor:
    """Counter-based RNG of ``csrc/kernels/sampling.hip`` (uint32 per index)."""
    i = i.to(torch.int64)
    h = fmix32(_u32(seed ^ 0x68BC21EB))
    h = fmix32(h ^ _u32(counter & M32))
    h = fmix32(h ^ _u32((counter >> 32) & M32) ^ (i & M32))
    salt = torch.as_tensor(salt, dtype=torch.int64)
    h = fmix32(h ^ ((i >> 32) & M32) ^ ((salt * 0x9E3779B9) & M32))
    return h


def sample_uniform_reject(n, k, n_items, positive=None, user=None, ring=None, mem=0, seed=0, counter=0,
                          known=None, known_count=None):
    t = torch.arange(n * k, dtype=torch.int64)
    b = t // k
    pos = positive.long()[b] if positive is not None else torch.full_like(t, -1)
    out = torch.zeros(n * k, dtype=torch.int64)
    done = torch.zeros(n * k, dtype=torch.bool)
    rows = ring.long().view(-1, mem)[user.long()[b]] if (ring is not None and user is not None and mem) else None
    span = max(int(known_count), 1) if known is not None else n_items
    for tries in range(32):
        cand = (rnd(seed, counter, t, tries) * span) >> 32
        if known is not None:
            cand = known.long()[cand]
        bad = cand == pos
        if rows is not None:
            bad |= (rows == cand[:, None]).any(1)
        take = ~done
        out[take] = cand[take]
        done |= ~bad
    return out.to(torch.int32)


def ring_push(ring, cursor, uid, iid, mem):
    """Sequential ring push (the GPU takes slots in atomic arrival order)."""
    for u, i in zip(uid.tolist(), iid.tolist()):
        ring[u * mem + int(cursor[u]) % mem] = i
        cursor[u] += 1


def known_append(flag, lst, count, iid):
    for i in iid.tolist():
        if int(flag[i]) == 0:
            flag[i] = 1
            lst[int(count[0])] = i
            count[0] += 1


def sample_alias(prob, alias, n, seed=0, counter=0):
    t = torch.arange(n, dtype=torch.int64)
    V = prob.numel()
    col = (rnd(seed, counter, t, 1) * V) >> 32
    u = (rnd(seed, counter, t, 2) >> 8).to(torch.float32) * (1.0 / 16777216.0)
    return torch.where(u < prob[col], col, alias.long()[col]).to(torch.int32)


def sgns_step(rows_in, rows_out, pos_c, pos_o, pos_neg, lr, neg_weight, d_in, d_out, neg_k=32, neg_group=1):
    """Block-shared-negative SGNS (32 pairs x ``neg_k`` negatives per block; ``neg_group``
    consecutive blocks share one set of negatives); returns the loss."""
    P = pos_c.numel()
    loss = 0.0
    Hall = rows_in.float()[pos_c.long()]
    Oall = rows_out.float()[pos_o.long()]
    for blk in range((P + 31) // 32):
        sl = slice(32 * blk, min(P, 32 * blk + 32))
        H, O = Hall[sl], Oall[sl]
        g = blk // neg_group
        negs = pos_neg.long()[neg_k * g: neg_k * g + neg_k]
        Nn = rows_out.float()[negs]
        sp = (H * O).sum(1)
        S = H @ Nn.T
        gpos = lr * (1 - torch.sigmoid(sp))
        G = -lr * neg_weight * torch.sigmoid(S)
        d_in.index_add_(0, pos_c.long()[sl], G @ Nn + gpos[:, None] * O)
        d_out.index_add_(0, negs, G.T @ H)
        d_out.index_add_(0, pos_o.long()[sl], gpos[:, None] * H)
        loss += float(-torch.log(torch.sigmoid(sp) + 1e-12).sum()
                      - neg_weight * torch.log(1 - torch.sigmoid(S) + 1e-12).sum())
    return loss


def _pa_tau(variant, loss, n2, C):
    if variant == 0:
        return torch.where(n2 > 0, loss / n2.clamp(min=1e-30), torch.zeros_like(loss))
    if variant == 1:
        return torch.where(n2 > 0, torch.clamp(loss / n2.clamp(min=1e-30), max=C), torch.zeros_like(loss))
    return loss / (n2 + 1.0 / (2.0 * C))


def pa_binary(indptr, xval, pos, w, y, variant, C, delta):
    """Returns (pred int8 [B], summed hinge loss); accumulates into ``delta[U]``."""
    B = indptr.numel() - 1
    seg = torch.repeat_interleave(torch.arange(B), (indptr[1:] - indptr[:-1]).long())
    m = torch.zeros(B).index_add_(0, seg, xval * w[pos.long()])
    n2 = torch.zeros(B).index_add_(0, seg, xval * xval)
    pred = torch.where(m > 0, 1, -1).to(torch.int8)
    yf = y.float()
    loss = torch.clamp(1 - yf * m, min=0) * (y != 0)
    mult = _pa_tau(variant, loss, n2, C) * yf
    delta.index_add_(0, pos.long(), mult[seg] * xval)
    return pred, float(loss.sum())


def pa_multi(indptr, xval, pos, W, y, mode, variant, C, cost, delta):
    B = indptr.numel() - 1
    L = W.shape[1]
    seg = torch.repeat_interleave(torch.arange(B), (indptr[1:] - indptr[:-1]).long())
    d = torch.zeros(B, L).index_add_(0, seg, xval[:, None] * W[pos.long()])
    n2 = torch.zeros(B).index_add_(0, seg, xval * xval)
    pred = torch.argmax(d, 1).to(torch.int32)
    total = 0.0
    lab = y.long()
    has = lab >= 0
    if mode == 0:
        yc = -torch.ones(B, L)
        yc[has, lab[has]] = 1.0
        loss = torch.clamp(1 - d * yc, min=0) * has[:, None]
        mult = _pa_tau(variant, loss, n2[:, None].expand_as(loss), C) * yc
        delta.index_add_(0, pos.long(), xval[:, None] * mult[seg])
        total = float(loss.sum())
    else:
        labc = lab.clamp(min=0)
        dy = d[torch.arange(B), labc]
        score = d if mode == 1 else d - dy[:, None] + torch.sqrt(cost[labc])
        q = torch.argmax(score, 1)
        act = has & (q != labc)
        loss = d[torch.arange(B), q] - dy + torch.sqrt(cost[labc, q])
        tau = torch.where(n2 > 0, loss / (2 * n2.clamp(min=1e-30)), torch.zeros_like(loss)) * act
        v = tau[seg] * xval
        rows = pos.long()
        dl = torch.zeros(xval.numel(), L)
        dl[torch.arange(xval.numel()), labc[seg]] += v
        dl[torch.arange(xval.numel()), q[seg]] -= v
        delta.index_add_(0, rows, dl)
        total = float((loss * act).sum())
    return pred, total


def mf_sq_err(U, I, uid, iid, r) -> float:
    e = r - (U[uid.long()] * I[iid.long()]).sum(1)
    return float((e.double() ** 2).sum())


HT_SALT = 0x2545F491


def ht_lookup(keys, tab, rowmap, rowkey, count, insert, rows=None, init_kind=-1, lo=0.0, hi=0.0, seed=0):  # noqa: C901
    """CPU twin of ``kernels/hash_table.hip`` ``fps_ht_lookup``: persistent
    open-addressing table (``tab`` int64: 0 empty, ``1<<32 | uint32(key)``
    occupied; linear probing from ``fmix32(key ^ SALT)``), compact rows handed
    out in first-insert order.  Returns ``(row int32[n], fresh uint8[n],
    overflow int)``."""
    cap = tab.numel()
    mask = cap - 1
    tb, rm, rk = tab.numpy(), rowmap.numpy(), rowkey.numpy()
    ks = keys.to(torch.int64).tolist()
    h0 = (fmix32((keys.to(torch.int64) & M32) ^ HT_SALT) & mask).tolist() if ks else []
    out = torch.full((len(ks),), -1, dtype=torch.int32)
    fresh = torch.zeros(len(ks), dtype=torch.uint8)
    overflow = 0
    cnt = int(count[0])
    for b, k in enumerate(ks):
        want = (1 << 32) | (k & M32)
        h = h0[b]
        for _ in range(cap):
            cur = int(tb[h])
            if cur == want:
                out[b] = int(rm[h])
                break
            if cur == 0:
                if not insert:
                    break
                if cnt >= rk.shape[0]:
                    overflow = 2
                    break
                tb[h] = want
                rm[h] = cnt
                rk[cnt] = k
                out[b] = cnt
                fresh[b] = 1
                cnt += 1
                break
            h = (h + 1) & mask
        else:
            overflow = 1
    count[0] = cnt
    if insert and rows is not None and init_kind >= 0 and fresh.any():
        sel = fresh.bool()
        r = out[sel].long()
        if init_kind == 0:
            rows[r] = 0
        elif init_kind == 1:
            rows[r] = lo
        else:
            rows[r] = init_values(keys[sel], rows.shape[1], lo, hi, seed).to(rows.dtype)
    return out, fresh, overflow


def ht_rehash(rowkey, count, tab, rowmap):
    cap = tab.numel()
    mask = cap - 1
    tb, rm = tab.numpy(), rowmap.numpy()
    ks = rowkey[:count].to(torch.int64)
    h0 = (fmix32((ks & M32) ^ HT_SALT) & mask).tolist()
    for r, k in enumerate(ks.tolist()):
        h = h0[r]
        while tb[h] != 0:
            h = (h + 1) & mask
        tb[h] = (1 << 32) | (k & M32)
        rm[h] = r


SGNS_STD_CHUNK = 16  # pairs per wave in kernels/sgns_std.hip


def sgns_standard(rows_in, rows_out, pos_c, pos_o, pos_neg, k, lr, d_in, d_out, method="atomic"):
    """CPU twin of ``fps_sgns_standard`` (sequential; center runs restart at every
    chunk of ``SGNS_STD_CHUNK`` pairs like the kernel's waves).  Returns the loss.
    ``method="sorted"``: the output-row deltas are ``g * rows_in[center]`` added
    after the pass (``rows_in`` after the center updates when ``d_in`` is
    ``rows_in``), the sorted form of ``ops.sgns_standard``."""
    import math

    deferred = []

    P = pos_c.numel()
    D = rows_in.shape[1]
    pc, po = pos_c.tolist(), pos_o.tolist()
    pn = pos_neg.reshape(P, k).tolist() if k else [[] for _ in range(P)]
    total = 0.0
    for s0 in range(0, P, SGNS_STD_CHUNK):
        cur, h, h0 = -1, None, None
        for p in range(s0, min(P, s0 + SGNS_STD_CHUNK)):
            c = pc[p]
            if c != cur:
                if cur >= 0:
                    d_in[cur] += (h - h0).to(d_in.dtype)
                cur = c
                h = rows_in[c].double().clone()
                h0 = h.clone()
            o = po[p]
            dh = torch.zeros(D, dtype=torch.float64)
            for x, lab in [(o, 1.0)] + [(n, 0.0) for n in pn[p] if n != o]:
                xv = rows_out[x].double()
                s = float(h @ xv)
                g = lr * (lab - 1.0 / (1.0 + math.exp(-s)))
                total += math.log1p(math.exp(-s)) if lab > 0 else math.log1p(math.exp(s))
                if method == "sorted":
                    deferred.append((x, g, c))
                else:
                    d_out[x] += (g * h).to(d_out.dtype)
                dh += g * xv
            h = h + dh
        if cur >= 0:
            d_in[cur] += (h - h0).to(d_in.dtype)
    for x, g, c in deferred:
        d_out[x] += (g * rows_in[c].double()).to(d_out.dtype)
    return total


def sgns_standard_batched(rows_in, rows_out, pos_c, pos_o, pos_neg, k, lr, d_in, d_out):
    """Mini-batch form of standard SGNS for CPU runs: every pair of the call reads
    the rows as they were before the call (the PS path's snapshot semantics),
    deltas are summed per row.  Returns the loss."""
    P = pos_c.numel()
    c, o = pos_c.long(), pos_o.long()
    x = torch.cat([o.view(P, 1), pos_neg.long().view(P, k)], 1) if k else o.view(P, 1)
    h = rows_in[c].double()
    X = rows_out[x].double()                                   # [P, 1+k, D]
    s = torch.einsum("pd,pjd->pj", h, X)
    lab = torch.zeros_like(s)
    lab[:, 0] = 1.0
    keep = torch.ones_like(s, dtype=torch.bool)
    keep[:, 1:] = x[:, 1:] != o.view(P, 1)                     # word2vec skips a negative equal to the target
    g = lr * (lab - torch.sigmoid(s)) * keep
    loss = torch.where(lab > 0, torch.nn.functional.softplus(-s), torch.nn.functional.softplus(s))[keep].sum()
    d_out.index_add_(0, x.reshape(-1), (g.unsqueeze(2) * h.unsqueeze(1)).reshape(-1, h.shape[1]).to(d_out.dtype))
    d_in.index_add_(0, c, torch.einsum("pj,pjd->pd", g, X).to(d_in.dtype))
    return float(loss)

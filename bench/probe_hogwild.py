#!/usr/bin/env python3
"""Lost user-row updates of the tiled MF step (the duplicate-user Hogwild race), measured.

    python bench/probe_hogwild.py [--users 1000000] [--items 100000] [--per-user 6.4] [--phases 4]

The tile-grouped SGD (``csrc/kernels/mf_tiled.hip``) gives every item row to one lane
group and updates user rows with plain stores: two ratings of one user that run in
two workgroups at the same time race on the user row (read, update, store), and one
of the two updates is lost.  This probe makes every update observable: user rows
start at 0 and the learning rate is tiny, so to first order each rating adds
``lr * r * item`` to its user row and leaves the item rows alone.  A user's row after
one step must then equal ``lr * sum_k r_k item_k`` (to ~1e-5 relative); a user whose
row misses by more than a fraction of one rating's share lost an update.  Reports
the fraction of users affected and the fraction of rating updates lost (least squares
per user: ``lost_update_count``) at the given density (the headline: 64M ratings over
10M users = 6.4 ratings per user per step, 4 user phases).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def lost_update_count(U, uid, v, users: int, nmax: int = 24, chunk: int = 200_000):
    """Updates missing from each user's row: the row must be ``sum_k c_k v_k`` with
    every ``c_k = 1`` (``v_k`` = rating k's contribution); ``c`` by least squares per
    user (<= ``nmax`` ratings, 64 dims), a lost update shows as ``c_k ~ 0``.  Returns
    ``(lost updates, ratings checked)``."""
    import torch

    dev = U.device
    order = torch.argsort(uid.long(), stable=True)
    su = uid.long()[order]
    cnt = torch.bincount(su, minlength=users)
    start = torch.cumsum(cnt, 0) - cnt
    rank = torch.arange(su.numel(), device=dev) - start[su]
    lost, checked = 0.0, 0
    for a in range(0, users, chunk):
        b = min(users, a + chunk)
        lo, hi = int(start[a]), int(start[b - 1] + cnt[b - 1])
        u_ = su[lo:hi] - a
        k_ = rank[lo:hi]
        ok = (k_ < nmax) & (cnt[su[lo:hi]] <= nmax)
        V = torch.zeros((b - a, nmax, v.shape[1]), dtype=torch.float64, device=dev)
        V[u_[ok], k_[ok]] = v[order[lo:hi][ok]].double()
        pad = torch.arange(nmax, device=dev).view(1, -1) >= cnt[a:b].view(-1, 1)
        G = V @ V.transpose(1, 2)
        # scale of this user's contributions; padded slots get it on the diagonal, and a
        # ridge of 1e-9 of it keeps a user who rated one item twice (parallel
        # contributions) solvable
        real_n = (~pad).sum(1, keepdim=True).clamp_min(1)
        scale = (G.diagonal(dim1=1, dim2=2) * (~pad)).sum(1, keepdim=True) / real_n
        scale = torch.where(scale > 0, scale, torch.ones_like(scale))
        G = G + torch.diag_embed(pad.double() * scale + 1e-9 * scale)
        rhs = (V @ U[a:b].double().unsqueeze(-1)).squeeze(-1)
        c = torch.linalg.solve(G, rhs)
        real = ~pad & (cnt[a:b] <= nmax).view(-1, 1)
        lost += float(((1.0 - c.clamp(0.0, 1.0)) * real).sum())
        checked += int(real.sum())
    return lost, checked


def lost_updates(users: int, items: int, per_user: float, phases: int, seed: int = 0, lr: float = 1e-4,
                 count_updates: bool = True, user_update: str = "store", world: int = 1,
                 overlap_substeps="auto") -> dict:
    """``users`` rows of ONE worker; ``world > 1``: that worker is rank 0 of a
    ``world``-GPU rotation job (``MFConfig(emulate_world=world)``: the same blocks,
    sub-steps and partition as one GPU of the real job, so the race is measured on
    the geometry the N-GPU bench runs)."""
    import torch

    from flink_parameter_server_1_amd.models.mf.fast import DistributedMF, MFConfig
    from flink_parameter_server_1_amd.parallel.comm import Comm

    dev = torch.device("cuda", 0)
    if world > 1:
        cfg = MFConfig(num_users=users * world, num_items=items, dim=64, learning_rate=lr, user_phases=phases,
                       prefetch_partition=False, user_update=user_update, exchange="rotate", emulate_world=world,
                       overlap_substeps=overlap_substeps)
    else:
        cfg = MFConfig(num_users=users, num_items=items, dim=64, learning_rate=lr, user_phases=phases,
                       prefetch_partition=False, user_update=user_update)
    m = DistributedMF(cfg, Comm(device=dev, local=True))
    assert m.users.n_local == users
    assert m.sgd_mode == "tiled"  # "atomic": the tiled kernel with float-atomic user deltas (exact)
    g = torch.Generator(device=dev).manual_seed(seed)
    with torch.no_grad():
        m.U.zero_()
        m.I.copy_(torch.rand(m.I.shape, generator=g, device=dev) * 0.2 - 0.1)
    n = int(users * per_user)
    uid = torch.randint(0, users, (n,), generator=g, device=dev, dtype=torch.int32)
    iid = torch.randint(0, items, (n,), generator=g, device=dev, dtype=torch.int32)
    r = torch.rand(n, generator=g, device=dev)
    I0 = m.I.clone()
    m.step(uid, iid, r)
    m.flush()
    torch.cuda.synchronize()
    v = lr * r.view(-1, 1) * I0[iid.long()]  # rating k's contribution to its user's row
    want = torch.zeros_like(m.U).index_add_(0, uid.long(), v)
    cnt = torch.bincount(uid.long(), minlength=users)
    err = (m.U - want).norm(dim=1)
    share = want.norm(dim=1) / cnt.clamp_min(1)  # ~ one rating's contribution
    lost = (err > 0.2 * share) & (cnt > 1)
    rated = cnt > 0
    if world > 1 and hasattr(m.rot, "close"):
        m.rot.close()
    out = {"users": users, "items": items, "ratings": n, "ratings_per_user": per_user, "world": world,
           "overlap_substeps": bool(getattr(m, "_overlap", False)) if world > 1 else None,
           "phases": getattr(m, "user_phases", None), "tile_rows": getattr(m, "tile_R", None), "user_update": cfg.user_update, "users_with_lost_update": int(lost.sum()),
           "rated_users": int(rated.sum()), "lost_user_fraction": float(lost.sum()) / max(int(rated.sum()), 1),
           "max_rel_err_clean": float((err / want.norm(dim=1).clamp_min(1e-30))[rated & ~lost].max())
           if bool((rated & ~lost).any()) else None}
    if count_updates:
        # users with more ratings than the solver's width are not counted (reported in updates_checked)
        nmax = max(24, min(64, int(cnt.max())))
        nl, nc = lost_update_count(m.U, uid, v, users, nmax=nmax, chunk=max(20_000, 200_000 * 24 // nmax))
        out.update({"lost_updates": nl, "updates_checked": nc, "lost_update_fraction": nl / max(nc, 1)})
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=1_000_000)
    ap.add_argument("--items", type=int, default=100_000)
    ap.add_argument("--per-user", type=float, default=6.4)
    ap.add_argument("--phases", default="1,4")
    ap.add_argument("--user-update", default="store", choices=["store", "sc1", "atomic"])
    ap.add_argument("--no-count", action="store_true", help="skip the per-update least-squares count")
    ap.add_argument("--world", type=int, default=1, help="rank 0 of an N-GPU rotation job (emulated schedule)")
    ap.add_argument("--overlap", default="auto", choices=["auto", "on", "off"],
                    help="world > 1: sub-steps on alternating streams (auto: from 4 ranks)")
    a = ap.parse_args(argv)
    for p in [int(x) for x in a.phases.split(",")]:
        print(json.dumps(lost_updates(a.users, a.items, a.per_user, p, count_updates=not a.no_count,
                                      user_update=a.user_update, world=a.world,
                                      overlap_substeps={"auto": "auto", "on": True,
                                                        "off": False}[a.overlap])), flush=True)


if __name__ == "__main__":
    main()

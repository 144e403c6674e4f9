"""Self-check of the multi-GPU MF step on the REAL process group (``bench.py --verify``).

The rotation (``parallel/rotation.py``) moves item blocks between the GPUs with
RCCL point-to-point transfers on the compute streams; its result must equal a
sequential replay of the same sub-step schedule (stratified SGD is serializable:
every item block is held by one rank per sub-step and every user row by its
worker -- ``FlinkParameterServer.scala:265-317``'s worker/PS feedback loop with
exact ownership).  This module runs a small instance of the job's own step
(same world, same schedule, same sub-step overlap, same kernels) on the job's
own communicator, gathers the tables to rank 0, replays the schedule in plain
fp32 PyTorch on the CPU and compares.  Batches hold distinct users and distinct
items, so the GPU kernels are deterministic and the comparison is to fp32
rounding (fused multiply-adds vs separate ones), not to a statistical bound.

A wrong peer, a missing stream wait, a buffer reused before its send completed
or a block never sent home changes item rows by O(lr * rating) -- far above the
tolerance -- so a mismatch means the exchange is broken and the bench must not
print a number.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import torch

from .comm import Comm
from .rotation import layout_world, shard_halves

#: the check's geometry: small enough for a CPU replay in seconds, large enough for
#: several tiles per block and every sub-step to carry ratings at 8 ranks
VERIFY_USERS, VERIFY_ITEMS, VERIFY_DIM, VERIFY_BATCH, VERIFY_STEPS = 40_000, 6_000, 64, 3_000, 2
RTOL, ATOL = 1e-5, 1e-6


def unique_batches(rank: int, steps: int, n_users_local: int, n_items: int, batch: int, seed: int = 7,
                   device="cpu") -> List[tuple]:
    """Per step ``batch`` distinct local users and ``batch`` distinct items (one rating per
    user row and per item row: the tiled kernel is then deterministic)."""
    g = torch.Generator(device="cpu").manual_seed(seed * 7919 + rank)
    out = []
    for _ in range(steps):
        u = torch.randperm(n_users_local, generator=g)[:batch].to(torch.int32)
        i = torch.randperm(n_items, generator=g)[:batch].to(torch.int32)
        r = torch.rand(batch, generator=g)
        out.append((u.to(device), i.to(device), r.to(device)))
    return out


def repeated_user_batches(rank: int, steps: int, n_users_local: int, n_items: int, batch: int, repeat: int = 8,
                          seed: int = 11, device="cpu") -> List[tuple]:
    """The collision regime: per step ``batch // repeat`` distinct local users, each rating
    ``repeat`` distinct items (``batch`` distinct items per step), shuffled -- every user row
    gets ``repeat`` deltas inside one launch, as the headline's ~6.4 ratings per user do."""
    g = torch.Generator(device="cpu").manual_seed(seed * 7919 + rank)
    out = []
    for _ in range(steps):
        nu = max(1, batch // repeat)
        u = torch.randperm(n_users_local, generator=g)[:nu].repeat(repeat)
        i = torch.randperm(n_items, generator=g)[: u.numel()]
        p = torch.randperm(u.numel(), generator=g)
        r = torch.rand(u.numel(), generator=g)
        out.append((u[p].to(torch.int32).to(device), i[p].to(torch.int32).to(device), r.to(device)))
    return out


def _occurrence_rounds(uid: torch.Tensor) -> torch.Tensor:
    """k for the k-th occurrence of each user in ``uid`` (0-based, in input order)."""
    order = torch.argsort(uid.long(), stable=True)
    su = uid.long()[order]
    start = torch.ones_like(su, dtype=torch.bool)
    start[1:] = su[1:] != su[:-1]
    idx = torch.arange(su.numel())
    first = torch.cummax(torch.where(start, idx, torch.zeros_like(idx)), 0).values
    k = torch.empty_like(idx)
    k[order] = idx - first
    return k


def active_blocks(rank: int, substep: int, world: int, schedule: str) -> List[int]:
    """Partition-layout blocks rank ``rank`` updates in sub-step ``substep``
    (``_Ring.order``: ring 0 direction +1; bidir ring 1 direction -1, base 2W)."""
    K = 2 * world
    out = [(2 * rank + substep) % K]
    if schedule == "bidir":
        out.append(K + (2 * rank + 1 - substep) % K)
    return out


def replay_rotation(world: int, schedule: str, cfg, batches: List[List[tuple]], users_mode: str = "jacobi"):
    """Sequential fp32 CPU replay of ``len(batches[0])`` rotation steps of ``world``
    ranks: returns ``(items [num_items, D], [user shard of rank r])``.

    ``users_mode`` -- how a user rated several times in one (rank, sub-step) is updated:
    "jacobi" sums the deltas all computed from the row at the sub-step's start (what the
    exact ``user_update="atomic"`` kernel does when every read lands before any add);
    "sequential" applies them one after another, in input order (the reference worker's
    order: ``PSOnlineMatrixFactorizationWorker.scala:41-55``); "store" keeps only one of
    them (last writer: what a lost-update race leaves).  With distinct users per sub-step
    all three equal the kernel exactly."""
    from ..ops import reference as R
    from .table import ShardedTable

    init = ("uniform", cfg.range_min, cfg.range_max)
    users = [ShardedTable(cfg.num_users, cfg.dim, r, world, "hash", init, cfg.user_seed(), "cpu",
                          track_touched=False).weight.clone() for r in range(world)]
    items = ShardedTable(cfg.num_items, cfg.dim, 0, 1, "hash", init, cfg.item_seed(), "cpu",
                         track_touched=False).weight.clone()
    Wv = layout_world(world, schedule)
    half = torch.tensor(shard_halves(cfg.num_items, Wv))
    steps = len(batches[0])
    for s in range(steps):
        for t in range(2 * world):
            for r in range(world):
                u, i, rt = (x.cpu() for x in batches[r][s])
                blk, _ = R.rot_block_of(i, Wv, half)
                sel = torch.isin(blk, torch.tensor(active_blocks(r, t, world, schedule)))
                u, i, rt = u[sel], i[sel], rt[sel]
                if users_mode == "sequential":
                    # k-th occurrence of each user in round k: users distinct inside a round,
                    # so the rounds in order are a sequential schedule (items are distinct)
                    k = _occurrence_rounds(u)
                    for q in range(int(k.max()) + 1 if k.numel() else 0):
                        m = k == q
                        R.mf_sgd_local(users[r], items, u[m], i[m], rt[m], cfg.learning_rate, cfg.lam)
                else:  # "jacobi" sums the deltas; "store" keeps the last writer's (a lost-update model)
                    R.mf_sgd_local(users[r], items, u, i, rt, cfg.learning_rate, cfg.lam,
                                   user_atomic=users_mode != "store")
    return items, users


def replay_ps(world: int, cfg, batches: List[List[tuple]], staleness: int):
    """Sequential fp32 CPU replay of the pull / push protocol with ``staleness`` (the
    bounded-staleness pipeline): step ``s`` of every rank reads the item rows as they
    were after the pushes of steps ``<= s - 1 - staleness`` were applied, updates its
    own users sequentially and pushes per-item delta sums (``SimplePSLogic``'s add)."""
    from ..ops import reference as R
    from .table import ShardedTable

    init = ("uniform", cfg.range_min, cfg.range_max)
    users = [ShardedTable(cfg.num_users, cfg.dim, r, world, "hash", init, cfg.user_seed(), "cpu",
                          track_touched=False).weight.clone() for r in range(world)]
    items = ShardedTable(cfg.num_items, cfg.dim, 0, 1, "hash", init, cfg.item_seed(), "cpu",
                         track_touched=False).weight.clone()
    steps = len(batches[0])
    pushes = []
    snaps = {}
    for s in range(steps + staleness + 1):
        if s - 1 - staleness >= 0:  # the push of step s - 1 - staleness lands
            items += pushes[s - 1 - staleness]
        snaps[s] = items.clone()
        if s < steps:
            delta = torch.zeros_like(items)
            for r in range(world):
                u, i, rt = (x.cpu() for x in batches[r][s])
                R.mf_sgd_pulled(users[r], u, rt, snaps[s], i, delta, cfg.learning_rate, cfg.lam)
            pushes.append(delta)
    return items, users


def _gather_rows(comm: Comm, t: torch.Tensor) -> List[torch.Tensor]:
    """All-gather of ``[n_r, ...]`` tensors of different lengths (padded on the wire)."""
    ns = [int(x) for x in comm.gather_floats(float(t.shape[0]))]
    cap = max(ns)
    pad = torch.zeros((cap,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    pad[: t.shape[0]] = t
    return [x[:n] for x, n in zip(comm.all_gather(pad), ns)]


def device_identity(comm: Comm) -> Dict[str, object]:
    """This rank's device: index, name and UUID (CUDA/HIP), for the per-rank report."""
    dev = comm.device
    if dev.type != "cuda":
        return {"device": str(dev)}
    p = torch.cuda.get_device_properties(dev)
    return {"device": str(dev), "name": p.name, "uuid": str(getattr(p, "uuid", "")),
            "pci_bus_id": getattr(p, "pci_bus_id", None)}


def rccl_version() -> Optional[str]:
    try:
        v = torch.cuda.nccl.version()
        return ".".join(map(str, v)) if isinstance(v, tuple) else str(v)
    except Exception:  # noqa: BLE001 -- no RCCL in this build (CPU)
        return None


def mutant_rotation(name: str):
    """Fault injection for the check's own tests (``FPS_VERIFY_MUTANT`` in ``bench.py``):
    a ``RingRotation`` with one realistic exchange bug.

    * ``wrong_buffer``: each sub-step sends the block the rank is ABOUT to update
      instead of the one it finished (the neighbour works on a stale copy);
    * ``no_home``: ``home()`` never returns the blocks (the PS shards keep old rows).
    """
    from . import rotation

    if name == "wrong_buffer":
        class WrongBuffer(rotation._Ring):
            def transfers(self):
                t = super().transfers()
                if t is None:
                    return None
                return (self.buf[self.A][: self.rows[self.order(self.s - 1)]], t[0][1]), t[1]

        class Rot(rotation.RingRotation):
            def __init__(self, *a, **k):
                super().__init__(*a, **k)
                for ring in self.rings:
                    ring.__class__ = WrongBuffer
        return Rot
    if name == "no_home":
        class Rot(rotation.RingRotation):
            def home(self):
                self.at_rest = True
                self.s = 0
        return Rot
    raise ValueError(f"unknown rotation mutant {name!r}")


def rotation_check(comm: Comm, schedule: str = "bidir", overlap="auto", steps: int = VERIFY_STEPS,
                   rotation_cls=None, sgd_mode: str = "auto", exchange: str = "rotate",
                   pipeline: bool = True, wire: str = "fp32", user_update: str = "auto",
                   repeated_users: bool = False, dim: int = VERIFY_DIM) -> Dict[str, object]:
    """Run ``steps`` steps of a small MF job on ``comm`` (the real world) and compare every
    rank's user rows and the whole item table with the sequential replay: the rotation
    schedule (``exchange="rotate"``) or the pull / push protocol with the pipeline's
    staleness (``"ps"``; bf16 on the wire is compared at bf16 tolerance).  Returns the
    same report on every rank (``verify_ok`` agreed by all ranks).  ``rotation_cls``
    replaces ``RingRotation`` (mutation tests).

    ``repeated_users`` (rotation only): the collision regime -- every user rated 8 times
    per step (``repeated_user_batches``), so user rows get several deltas inside one
    launch and across the overlapped sub-steps.  A lost user delta is first order in the
    learning rate; which reads see which adds is not deterministic, a second-order effect,
    so the tolerance is measured: 4x the gap between the two exact orders of the replay
    (summed deltas from one read vs one user delta after another) -- and the check asserts
    that the replay with lost updates (one writer per user and sub-step) lies beyond 2x it.  ``user_update="atomic"`` must pass; "store" (Hogwild)
    loses deltas and fails."""
    from ..models.mf.fast import DistributedMF, MFConfig

    if exchange not in ("rotate", "ps"):
        raise ValueError(f"verify: exchange must be 'rotate' or 'ps', not {exchange!r}")
    if repeated_users and exchange != "rotate":
        raise ValueError("verify: the collision regime checks the rotation exchange")
    lr = 0.01 if repeated_users else 0.05
    cfg = MFConfig(num_users=VERIFY_USERS, num_items=VERIFY_ITEMS, dim=dim, learning_rate=lr,
                   range_min=0.0, range_max=0.2, exchange=exchange, rotation=schedule, overlap_substeps=overlap,
                   sgd_mode=sgd_mode, pipeline=pipeline, wire_dtype=wire, user_update=user_update)
    m = DistributedMF(cfg, comm)
    if rotation_cls is not None:
        m.rot = rotation_cls(comm, m.items.weight, cfg.num_items, schedule)
    rtol, atol = (RTOL, ATOL) if wire == "fp32" else (2e-2, 2e-3)
    W, r = comm.world, comm.rank
    make = repeated_user_batches if repeated_users else unique_batches
    for u, i, rt in make(r, steps, m.users.n_local, cfg.num_items, VERIFY_BATCH, device=comm.device):
        m.step(u, i, rt)
    m.flush()
    ids, vals = m.item_vectors(only_touched=False)
    all_ids = _gather_rows(comm, ids.to(torch.int64).contiguous())
    all_vals = _gather_rows(comm, vals.contiguous())
    all_users = _gather_rows(comm, m.U.contiguous())
    bad = 0.0
    report = {"verify_world": W, "verify_exchange": exchange, "verify_schedule": schedule, "verify_steps": steps,
              "verify_sgd_mode": m.sgd_mode, "verify_overlap_substeps": bool(getattr(m, "_overlap", False)),
              "verify_user_update": m.user_update, "verify_dim": dim, "verify_wire": wire,
              "verify_repeated_users": repeated_users}
    if r == 0:
        batches = [make(q, steps, (cfg.num_users - q + W - 1) // W, cfg.num_items, VERIFY_BATCH)
                   for q in range(W)]
        if exchange == "rotate":
            ref_items, ref_users = replay_rotation(W, schedule, cfg, batches)
        else:
            ref_items, ref_users = replay_ps(W, cfg, batches, 1 if m.pipeline else 0)
        got_items = torch.empty_like(ref_items)
        got_items[torch.cat(all_ids).cpu().long()] = torch.cat(all_vals).cpu()
        err_i = float((got_items - ref_items).abs().max())
        err_u = max(float((all_users[q].cpu() - ref_users[q]).abs().max()) for q in range(W))
        moved = float((ref_items - ShardedInit.items(cfg)).abs().max())
        if repeated_users:
            # measured tolerance: the gap between the two exact orders, x 4; a lost delta
            # (the smallest user delta of the replay's first sub-step) must exceed it
            seq_items, seq_users = replay_rotation(W, schedule, cfg, batches, users_mode="sequential")
            gap_u = max(float((seq_users[q] - ref_users[q]).abs().max()) for q in range(W))
            gap_i = float((seq_items - ref_items).abs().max())
            tol_u, tol_i = 4 * gap_u + atol, 4 * gap_i + atol
            # what lost updates look like: the replay keeping one writer per user and sub-step
            _, lost_users = replay_rotation(W, schedule, cfg, batches, users_mode="store")
            lost_u = max(float((lost_users[q] - ref_users[q]).abs().max()) for q in range(W))
            ok = (err_u <= tol_u and err_i <= tol_i and lost_u > 2 * tol_u)
            report.update(verify_tol_users=tol_u, verify_tol_items=tol_i, verify_lost_update_err=lost_u)
        else:
            ok = (torch.allclose(got_items, ref_items, rtol=rtol, atol=atol)
                  and all(torch.allclose(all_users[q].cpu(), ref_users[q], rtol=rtol, atol=atol) for q in range(W)))
        ok = ok and moved > 100 * atol
        bad = 0.0 if ok else 1.0
        report.update(verify_max_abs_err_items=err_i, verify_max_abs_err_users=err_u, verify_ref_moved=moved)
    bad = comm.max_over_ranks(bad)  # every rank learns rank 0's verdict
    report["verify_ok"] = bad == 0.0
    return report


class ShardedInit:
    """The initial item table of a config (for the replay's 'did anything move' check)."""

    @staticmethod
    def items(cfg) -> torch.Tensor:
        from .table import ShardedTable

        return ShardedTable(cfg.num_items, cfg.dim, 0, 1, "hash", ("uniform", cfg.range_min, cfg.range_max),
                            cfg.item_seed(), "cpu", track_touched=False).weight

    @staticmethod
    def users(cfg, rank: int, world: int) -> torch.Tensor:
        from .table import ShardedTable

        return ShardedTable(cfg.num_users, cfg.dim, rank, world, "hash", ("uniform", cfg.range_min, cfg.range_max),
                            cfg.user_seed(), "cpu", track_touched=False).weight

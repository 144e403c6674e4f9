"""Model formats, data readers and checkpoint / resume.

* ``id;value`` text — one coordinate per line in coordinate order per id,
  users and items in separate files: the reference's dump format
  (``T/matrix/factorization/PSOnlineMatrixFactorizationImplicitTest.scala:76-91``),
  read by its notebooks.  ``write_factors_text`` / ``read_factors_text``.
* model streams — ``(id, value)`` iterables for ``transform_with_model_load``
  (``model_stream_from_text``) and the last-writer-wins fold of an output
  stream (``fold_model``).
* binary shard snapshots — ``ids int64[n] + values fp32[n, d]`` with a header
  (partitioner kind, num ids, dim, world, rank, step).  ``restore_table``
  re-shards: it reads every shard file and keeps the ids this rank owns, so a
  checkpoint written at P shards restores at any P'.
* ``Checkpointer`` — periodic snapshots of named tables + a JSON manifest,
  atomic publish (tmp + rename), ``restore_latest``.  The reference has no
  runtime checkpointing at all (``README.md:67-69``).
* rating logs — ``ts user item [rating]`` lines (space/comma/tab), the input
  format of the reference's experiment drivers (``read_ratings``).
* PA prediction log lines ``###PS###t;<label>;[k -> v,...]``
  (``M/passive/aggressive/classification/binary/PABinaryClassificationOffline.scala:356``).

Heavy lifting is in C++ (``csrc/host/fps_host.cpp``) with Python fallbacks.
"""
from __future__ import annotations

import glob
import json
import os
import time
from typing import Dict, Iterable, Iterator, List, Optional, Tuple

import numpy as np
import torch

from . import native_host as NH


# ------------------------------------------------------------------ id;value text
def write_factors_text(path: str, ids, values, append: bool = False) -> None:
    ids = np.ascontiguousarray(np.asarray(ids, dtype=np.int64))
    vals = np.ascontiguousarray(np.asarray(values, dtype=np.float32)).reshape(ids.size, -1)
    L = NH.lib()
    if L is not None:
        rc = L.fps_write_factors_text(path.encode(), NH._p(ids), NH._p(vals), ids.size, vals.shape[1], int(append))
        if rc != 0:
            raise OSError(f"cannot write {path}")
        return
    with open(path, "a" if append else "w") as f:
        for i, row in zip(ids.tolist(), vals):
            for v in row:
                f.write(f"{i};{float(v):.9g}\n")


def read_factors_text(path: str) -> Dict[int, np.ndarray]:
    """``{id: vector}``; consecutive lines with the same id form the vector."""
    L = NH.lib()
    if L is not None:
        n = L.fps_read_id_value_text(path.encode(), 0, None, None)
        if n < 0:
            raise FileNotFoundError(path)
        ids = np.empty(n, dtype=np.int64)
        vals = np.empty(n, dtype=np.float64)
        n = L.fps_read_id_value_text(path.encode(), n, NH._p(ids), NH._p(vals))
        ids, vals = ids[:n], vals[:n]
    else:
        rows = [ln.strip().split(";") for ln in open(path) if ln.strip()]
        ids = np.array([int(r[0]) for r in rows], dtype=np.int64)
        vals = np.array([float(r[1]) for r in rows], dtype=np.float64)
    out: Dict[int, list] = {}
    if ids.size:
        cut = np.flatnonzero(np.diff(ids)) + 1
        for seg_i, seg_v in zip(np.split(ids, cut), np.split(vals, cut)):
            out.setdefault(int(seg_i[0]), []).extend(seg_v.tolist())
    return {k: np.asarray(v) for k, v in out.items()}


def model_stream_from_text(path: str) -> Iterator[Tuple[int, np.ndarray]]:
    """``(id, vector)`` records for ``transform_with_model_load``."""
    yield from read_factors_text(path).items()


def fold_model(stream, side: str = "right") -> Dict[int, object]:
    """Last-writer-wins fold of an output stream (the model the stream describes)."""
    out = {}
    for e in stream:
        if (side == "right" and e.is_right) or (side == "left" and e.is_left):
            k, v = e.value
            out[k] = v
    return out


def write_prediction_log(lines: Iterable[Tuple[dict, object]], path: Optional[str] = None) -> List[str]:
    res = [f"###PS###t;{label};[{','.join(f'{k} -> {v}' for k, v in sorted(vec.items()))}]"
           for vec, label in lines]
    if path:
        with open(path, "w") as f:
            f.write("\n".join(res) + "\n")
    return res


# ------------------------------------------------------------------ rating logs
def read_ratings(path: str, default_rating: float = 1.0):
    """``ts user item [rating]`` lines -> numpy arrays (ts, user, item, rating)."""
    L = NH.lib()
    if L is not None:
        n = L.fps_count_lines(path.encode())
        if n < 0:
            raise FileNotFoundError(path)
        ts = np.empty(n, dtype=np.int64)
        u = np.empty(n, dtype=np.int32)
        i = np.empty(n, dtype=np.int32)
        r = np.empty(n, dtype=np.float32)
        m = L.fps_parse_ratings(path.encode(), n, NH._p(ts), NH._p(u), NH._p(i), NH._p(r), default_rating)
        return ts[:m], u[:m], i[:m], r[:m]
    rows = []
    for ln in open(path):
        parts = ln.replace(",", " ").replace("\t", " ").split()
        if len(parts) >= 3:
            rows.append((int(parts[0]), int(parts[1]), int(parts[2]),
                         float(parts[3]) if len(parts) > 3 else default_rating))
    a = np.array(rows, dtype=np.float64).reshape(-1, 4)
    return a[:, 0].astype(np.int64), a[:, 1].astype(np.int32), a[:, 2].astype(np.int32), a[:, 3].astype(np.float32)


def synthetic_ratings_host(n: int, n_local_users: int, n_items: int, seed: int = 0, offset: int = 0):
    """Multithreaded C++ synthetic rating generator (host-side data loader)."""
    u = np.empty(n, dtype=np.int32)
    i = np.empty(n, dtype=np.int32)
    r = np.empty(n, dtype=np.float32)
    L = NH.lib()
    if L is None:
        rng = np.random.default_rng(seed + offset)
        return (rng.integers(0, n_local_users, n, dtype=np.int32), rng.integers(0, n_items, n, dtype=np.int32),
                rng.random(n, dtype=np.float32))
    L.fps_gen_ratings(n, n_local_users, n_items, seed & 0xFFFFFFFF, offset, NH._p(u), NH._p(i), NH._p(r))
    return u, i, r


# ------------------------------------------------------------------ snapshots
def save_snapshot(path: str, ids: torch.Tensor, values: torch.Tensor, *, part_kind: int, num_ids: int, world: int,
                  rank: int, step: int = 0) -> None:
    ids_np = np.ascontiguousarray(ids.detach().to("cpu", torch.int64).numpy())
    v = values.detach().to("cpu", torch.float32)
    width = v.shape[-1] if v.dim() > 1 else (v.numel() // max(ids_np.size, 1) if ids_np.size else 1)
    vals_np = np.ascontiguousarray(v.reshape(ids_np.size, width).numpy())
    L = NH.lib()
    if L is not None:
        rc = L.fps_write_snapshot(path.encode(), part_kind, num_ids, vals_np.shape[1], world, rank, step,
                                  NH._p(ids_np), NH._p(vals_np), ids_np.size)
        if rc != 0:
            raise OSError(f"snapshot write failed ({rc}): {path}")
        return
    meta = dict(part_kind=part_kind, num_ids=num_ids, dim=vals_np.shape[1], world=world, rank=rank, step=step)
    np.savez(path + ".npz", ids=ids_np, values=vals_np, meta=json.dumps(meta))
    os.replace(path + ".npz", path)


def load_snapshot(path: str):
    """-> (meta dict, ids int64[n], values fp32[n, d])."""
    L = NH.lib()
    if L is not None:
        meta = np.zeros(7, dtype=np.int64)
        if L.fps_read_snapshot_header(path.encode(), NH._p(meta)) == 0:
            keys = ["part_kind", "num_ids", "dim", "world", "rank", "n_rows", "step"]
            m = dict(zip(keys, meta.tolist()))
            ids = np.empty(m["n_rows"], dtype=np.int64)
            vals = np.empty((m["n_rows"], m["dim"]), dtype=np.float32)
            if L.fps_read_snapshot(path.encode(), NH._p(ids), NH._p(vals), m["n_rows"]) != 0:
                raise OSError(f"corrupt snapshot {path}")
            return m, ids, vals
    z = np.load(path, allow_pickle=False)
    m = json.loads(str(z["meta"]))
    return m, z["ids"], z["values"]


def save_table(table, path: str, step: int = 0, only_touched: bool = False) -> None:
    """Shard snapshot of a ``ShardedTable``: the rows, plus -- next to it -- the
    optimizer state (Adagrad accumulators / add_renorm lengths: ``<path>.state``)
    and the touched flags (``<path>.touched``), so a resumed run applies the same
    update rule to the same state and dumps the same touched rows."""
    ids, vals = table.dump(only_touched, raw=True)
    save_snapshot(path, ids, vals, part_kind=table.part_kind, num_ids=table.num_ids, world=table.world,
                  rank=table.rank, step=step)
    loc = table.local_of(ids.to(table.device)) if ids.numel() else ids.long()
    if table.state is not None:
        st = table.state[loc.long()].reshape(ids.numel(), -1)
        save_snapshot(path + ".state", ids, st, part_kind=table.part_kind, num_ids=table.num_ids, world=table.world,
                      rank=table.rank, step=step)
    if table.touched is not None:
        t = torch.nonzero(table.touched, as_tuple=False).flatten()
        tid = table.global_ids(t)
        save_snapshot(path + ".touched", tid, torch.ones(tid.numel(), 1), part_kind=table.part_kind,
                      num_ids=table.num_ids, world=table.world, rank=table.rank, step=step)


def _shard_file_coords(path: str):
    """(rank, world) of a ``<name>.shard<r>-of-<w>.bin`` file, or None."""
    import re

    m = re.search(r"\.shard(\d+)-of-(\d+)\.bin$", path)
    return (int(m.group(1)), int(m.group(2))) if m else None


def snapshot_meta(path: str) -> dict:
    """A snapshot's header (partitioner kind, num ids, dim, world, rank, rows, step)
    without reading its rows."""
    L = NH.lib()
    if L is not None:
        meta = np.zeros(7, dtype=np.int64)
        if L.fps_read_snapshot_header(path.encode(), NH._p(meta)) == 0:
            return dict(zip(["part_kind", "num_ids", "dim", "world", "rank", "n_rows", "step"], meta.tolist()))
    return load_snapshot(path)[0]


def shard_files_for(table, files: List[str]) -> List[str]:
    """The shard files that can hold ids this rank owns, when the files were written
    with the same partitioning as ``table`` (header ``part_kind``): with hash
    partitioning a file of shard ``r`` of ``W`` (ids ``= r mod W``) overlaps shard
    ``r'`` of ``W'`` iff ``r = r' (mod gcd(W, W'))`` -- only its own file when the
    world size is unchanged; with range partitioning the id ranges are
    intersected.  A different partitioning (e.g. hash shards restored into a
    range-partitioned table), lookup partitioning and unnamed files: every file."""
    from math import gcd

    out = []
    for f in files:
        c = _shard_file_coords(f)
        if c is None or table.partition == "lookup" or snapshot_meta(f)["part_kind"] != table.part_kind:
            out.append(f)
            continue
        r, w = c
        if table.partition == "hash":
            if (r - table.rank) % gcd(w, table.world) == 0:
                out.append(f)
        else:
            blk = -(-table.num_ids // w)
            lo, hi = r * blk, min(table.num_ids, (r + 1) * blk) if r < w - 1 else table.num_ids
            mlo = table.rank * table.block
            mhi = table.num_ids if table.rank == table.world - 1 else min(table.num_ids, mlo + table.block)
            if lo < mhi and mlo < hi:
                out.append(f)
    return out


#: bytes of snapshot files read by ``restore_table`` in this process (restore-IO tests)
RESTORE_BYTES = {"bytes": 0}


def restore_table(table, pattern: str) -> int:
    """Restore this rank's rows (and optimizer state / touched flags) from the
    shard files matching ``pattern``; re-shards to the current world size, and
    reads only the files that can hold ids of this rank (``shard_files_for``)."""
    n = 0
    files = [f for f in sorted(glob.glob(pattern)) if not f.endswith((".state", ".touched"))]
    for f in shard_files_for(table, files):
        RESTORE_BYTES["bytes"] += os.path.getsize(f)
        _, ids, vals = load_snapshot(f)
        if not ids.size:
            continue
        ids_t = torch.from_numpy(ids)
        mine = table.part.shard_tensor(ids_t) == table.rank
        table.load(ids_t, torch.from_numpy(vals))
        n += int(mine.sum())
        if table.touched is not None and os.path.exists(f + ".touched"):
            loc = table.local_of(ids_t[mine].to(table.device))  # load() marked them: the saved flags decide
            table.touched[loc] = 0
        if table.state is not None and os.path.exists(f + ".state"):
            RESTORE_BYTES["bytes"] += os.path.getsize(f + ".state")
            _, sid, sv = load_snapshot(f + ".state")
            sid_t = torch.from_numpy(sid)
            m2 = table.part.shard_tensor(sid_t) == table.rank
            loc = table.local_of(sid_t[m2].to(table.device)).long()
            table.state[loc] = torch.from_numpy(sv)[m2].to(table.state.device).reshape(
                (loc.numel(),) + tuple(table.state.shape[1:]))
        if table.touched is not None and os.path.exists(f + ".touched"):
            RESTORE_BYTES["bytes"] += os.path.getsize(f + ".touched")
            _, tid, _ = load_snapshot(f + ".touched")
            tid_t = torch.from_numpy(tid)
            m3 = table.part.shard_tensor(tid_t) == table.rank
            table.touched[table.local_of(tid_t[m3].to(table.device)).long()] = 1
    return n


class Checkpointer:
    """Periodic snapshots of named ``ShardedTable``s (+ optimizer state + touched
    flags) and of per-rank auxiliary state (RNG counters, negative-sampling rings,
    the data cursor: ``aux_state() -> {name: tensor or number}`` /
    ``load_aux_state(dict)``).

    Layout: ``<dir>/step_<k>/<name>.shard<rank>-of-<world>.bin`` (+ ``.state``,
    ``.touched``), ``aux.rank<r>-of-<w>.pt`` and ``manifest.json`` written by rank
    0 after a barrier (the snapshot is complete when the manifest exists).
    ``restore_latest`` re-shards to the current world size, reading only the
    shard files that can hold this rank's ids; aux state is restored when the
    world size is unchanged.  ``before_save`` (e.g. ``DistributedMF.flush``) runs
    first, so in-flight pushes land and rotating item blocks are back home.
    """

    def __init__(self, directory: str, tables: Dict[str, object], comm=None, every_steps: int = 0, keep: int = 2,
                 before_save=None, aux=None):
        self.before_save = before_save
        self.dir = directory
        self.tables = tables
        self.comm = comm
        self.every = every_steps
        self.keep = keep
        self.aux = aux  # object with aux_state() / load_aux_state(d)
        os.makedirs(directory, exist_ok=True)

    def _rank_world(self):
        if self.comm is None:
            return 0, 1
        return self.comm.rank, self.comm.world

    def maybe_save(self, step: int, extra: Optional[dict] = None) -> bool:
        if self.every and step % self.every == 0 and step > 0:
            self.save(step, extra)
            return True
        return False

    def save(self, step: int, extra: Optional[dict] = None) -> str:
        if self.before_save is not None:
            self.before_save()
        rank, world = self._rank_world()
        d = os.path.join(self.dir, f"step_{step:09d}")
        os.makedirs(d, exist_ok=True)
        for name, t in self.tables.items():
            save_table(t, os.path.join(d, f"{name}.shard{rank}-of-{world}.bin"), step)
        if self.aux is not None:
            st = {k: (v.detach().cpu() if torch.is_tensor(v) else v) for k, v in self.aux.aux_state().items()}
            tmp = os.path.join(d, f"aux.rank{rank}-of-{world}.pt.tmp")
            torch.save(st, tmp)
            os.replace(tmp, tmp[:-4])
        if self.comm is not None:
            self.comm.barrier()
        if rank == 0:
            manifest = {"step": step, "world": world, "tables": sorted(self.tables), "time": time.time(),
                        "extra": extra or {}}
            with open(os.path.join(d, "manifest.json.tmp"), "w") as f:
                json.dump(manifest, f)
            os.replace(os.path.join(d, "manifest.json.tmp"), os.path.join(d, "manifest.json"))
            self._gc()
        if self.comm is not None:
            self.comm.barrier()
        return d

    def _gc(self):
        done = sorted(p for p in glob.glob(os.path.join(self.dir, "step_*"))
                      if os.path.exists(os.path.join(p, "manifest.json")))
        for p in done[:-self.keep] if self.keep else []:
            for f in glob.glob(os.path.join(p, "*")):
                os.remove(f)
            os.rmdir(p)

    def latest(self) -> Optional[str]:
        done = sorted(p for p in glob.glob(os.path.join(self.dir, "step_*"))
                      if os.path.exists(os.path.join(p, "manifest.json")))
        return done[-1] if done else None

    def restore_latest(self) -> Optional[dict]:
        d = self.latest()
        if d is None:
            return None
        with open(os.path.join(d, "manifest.json")) as f:
            manifest = json.load(f)
        for name, t in self.tables.items():
            restore_table(t, os.path.join(d, f"{name}.shard*-of-*.bin"))
        rank, world = self._rank_world()
        aux_path = os.path.join(d, f"aux.rank{rank}-of-{world}.pt")
        if self.aux is not None and os.path.exists(aux_path) and manifest.get("world") == world:
            self.aux.load_aux_state(torch.load(aux_path, weights_only=True))
        return manifest

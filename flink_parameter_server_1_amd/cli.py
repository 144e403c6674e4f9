"""Command line front-end: ``python -m flink_parameter_server_1_amd <command> ...``.

The reference has no CLI (only two ``main()`` test drivers,
``T/matrix/factorization/PSOnlineMatrixFactorizationImplicitTest.scala:31-97``);
every knob is a method parameter.  Here the same knobs are dataclass
configs (``MFConfig``, ``SGNSConfig``, ``PAConfig``) that can come from flags
or a YAML file (``--config``, safe-loaded).

Commands
  mf-online   per-record online MF on a rating log (``ts user item [rating]``),
              writes user / item factors as ``id;value`` files (the driver's output)
  mf-offline  per-record multi-epoch MF, same IO
  mf-gpu      MF on the tensor engine (GPU / CPU), synthetic or from a log; optional
              checkpoints; one process per GPU under torch.distributed.run
  topk        top-K recommendation from factor files + nDCG / hit-rate per period
  pa-train    PA classifier on a libsvm-style file (``label idx:val ...``)
  w2v         word2vec SGNS on a token file (whitespace separated ints) or synthetic
  bench       the headline benchmark (bench.py)
"""
from __future__ import annotations

import argparse
import dataclasses
import json
import os
import sys
import time


def _load_yaml(path):
    import yaml

    with open(path) as f:
        return yaml.safe_load(f) or {}


def _apply_config(cfg_cls, args, extra=None):
    vals = {}
    if getattr(args, "config", None):
        vals.update(_load_yaml(args.config))
    for f in dataclasses.fields(cfg_cls):
        v = getattr(args, f.name, None)
        if v is not None:
            vals[f.name] = v
    if extra:
        vals.update(extra)
    return cfg_cls(**{k: v for k, v in vals.items() if k in {f.name for f in dataclasses.fields(cfg_cls)}})


def _ratings_from_log(path):
    from .models.mf.core import Rating
    from .utils.io import read_ratings

    ts, u, i, r = read_ratings(path)
    return [Rating(int(a), int(b), float(c), int(t)) for t, a, b, c in zip(ts, u, i, r)]


def _write_factors(stream, users_out, items_out):
    import numpy as np

    from .utils.io import fold_model, write_factors_text

    for side, path in (("left", users_out), ("right", items_out)):
        if path:
            m = fold_model(stream, side)
            ids = np.array(sorted(m), dtype=np.int64)
            vals = np.stack([np.asarray(m[i], dtype=np.float32) for i in ids]) if len(ids) else np.zeros((0, 1))
            write_factors_text(path, ids, vals)


def cmd_mf(args, offline: bool):
    from .models.mf import apps

    if not offline and getattr(args, "engine", "python") == "native":
        return cmd_mf_native(args)
    ratings = _ratings_from_log(args.input)
    kw = dict(num_factors=args.num_factors, range_min=args.range_min, range_max=args.range_max,
              learning_rate=args.learning_rate, negative_sample_rate=args.negative_sample_rate,
              user_memory=args.user_memory, pull_limit=args.pull_limit, worker_parallelism=args.workers,
              ps_parallelism=args.ps, seed=args.seed)
    t0 = time.time()
    out = apps.ps_offline_mf(ratings, iterations=args.iterations, **kw) if offline else apps.ps_online_mf(ratings, **kw)
    _write_factors(out, args.users_out, args.items_out)
    print(json.dumps({"ratings": len(ratings), "seconds": time.time() - t0, "outputs": len(out)}))


def cmd_mf_native(args):
    """Online MF through the C++ record engine (same job, same output files)."""
    import numpy as np

    from .models.mf.native import ps_online_mf_native
    from .utils.io import write_factors_text

    ratings = _ratings_from_log(args.input)
    u = np.array([r.user for r in ratings], dtype=np.int64)
    it = np.array([r.item for r in ratings], dtype=np.int64)
    rt = np.array([r.rating for r in ratings], dtype=np.float64)
    t0 = time.time()
    res = ps_online_mf_native(u, it, rt, num_factors=args.num_factors, range_min=args.range_min,
                              range_max=args.range_max, learning_rate=args.learning_rate,
                              negative_sample_rate=args.negative_sample_rate, user_memory=args.user_memory,
                              pull_limit=args.pull_limit, worker_parallelism=args.workers, ps_parallelism=args.ps,
                              seed=args.seed or 0)
    dt = time.time() - t0
    for path, ids, vals in ((args.users_out, res.user_ids, res.user_vectors),
                            (args.items_out, res.item_ids, res.item_vectors)):
        if path:
            o = np.argsort(ids)
            write_factors_text(path, ids[o], vals[o].astype(np.float32))
    print(json.dumps({"ratings": len(ratings), "seconds": dt, "engine": "native", **res.stats}))


def cmd_mf_gpu(args):
    import torch

    from .models.mf.fast import DistributedMF, MFConfig, SyntheticRatings
    from .parallel.comm import Comm
    from .utils.io import Checkpointer, read_ratings

    comm = Comm.init_from_env()
    cfg = _apply_config(MFConfig, args)
    m = DistributedMF(cfg, comm)
    if args.input:
        ts, u, i, r = read_ratings(args.input)
        mine = (u % comm.world) == comm.rank
        dev = comm.device
        uid = torch.from_numpy(u[mine] // comm.world).to(dev)
        iid = torch.from_numpy(i[mine]).to(dev)
        rat = torch.from_numpy(r[mine]).to(dev)
        n = uid.numel()

        def batch(s):
            a = (s * args.batch) % max(n, 1)
            return uid[a:a + args.batch], iid[a:a + args.batch], rat[a:a + args.batch]
    else:
        data = SyntheticRatings(cfg.num_users, cfg.num_items, args.batch * 4, comm.rank, comm.world,
                                device=comm.device, truth_dim=args.truth_dim)
        batch = lambda s: data.batch(s, args.batch)  # noqa: E731
    ck = Checkpointer(args.checkpoint_dir, {"users": m.users, "items": m.items}, comm,
                      every_steps=args.checkpoint_every, before_save=m.flush, aux=m) if args.checkpoint_dir else None
    start, man = 0, None
    if ck and args.resume:
        man = ck.restore_latest()
        start = man["step"] if man else 0
    if man is None and (args.model_in_users or args.model_in_items):
        # warm start from id;value dumps -- only when no checkpoint was restored
        # (a restored checkpoint is newer than the initial model and wins)
        from .utils.io import read_factors_text

        m.load_model(read_factors_text(args.model_in_users) if args.model_in_users else None,
                     read_factors_text(args.model_in_items) if args.model_in_items else None)
    t0 = time.time()
    for s in range(start, start + args.steps):
        m.step(*batch(s))
        if ck:
            ck.maybe_save(s + 1)
    m.flush()
    rmse = m.rmse(*batch(0))
    if comm.rank == 0:
        print(json.dumps({"steps": args.steps, "seconds": time.time() - t0, "updates": m.updates * comm.world,
                          "rmse_first_batch": rmse}))
    from .utils.io import write_factors_text

    def out_path(p):  # one file per rank at N > 1 (each holds its shard's rows)
        return p if comm.world == 1 else f"{p}.{comm.rank}"

    if args.items_out:
        ids, vals = m.item_vectors(only_touched=False)
        o = torch.argsort(ids)
        write_factors_text(out_path(args.items_out), ids[o].cpu().numpy(), vals[o].cpu().numpy())
    if args.users_out:
        ids, vals = m.user_vectors()
        write_factors_text(out_path(args.users_out), ids.cpu().numpy(), vals.detach().cpu().numpy())


def cmd_topk(args):
    import numpy as np
    import torch

    from .models.mf.topk_fast import LempTopK
    from .utils.io import read_factors_text, read_ratings
    from .utils.metrics import NDCGAggregator

    users = read_factors_text(args.users)
    items = read_factors_text(args.items)
    iid = torch.tensor(sorted(items))
    X = torch.tensor(np.stack([items[int(i)] for i in iid]), dtype=torch.float32)
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    lemp = LempTopK(iid.to(dev), X.to(dev))
    ts, u, i, r = read_ratings(args.test)
    agg = NDCGAggregator(args.period)
    known = [k for k in range(len(u)) if int(u[k]) in users]
    for a in range(0, len(known), 4096):
        idx = known[a:a + 4096]
        Q = torch.tensor(np.stack([users[int(u[k])] for k in idx]), dtype=torch.float32, device=dev)
        _, top = lemp.query(Q, args.k)
        for row, k in zip(top.cpu().tolist(), idx):
            agg.add(int(ts[k]), row, int(i[k]))
    if args.csv:
        agg.to_csv(args.csv)
    print(json.dumps({"periods": agg.periods()[:10], "n": len(known)}))


def cmd_mf_topk(args):
    """psOnlineLearnerAndGenerator on a ``ts,user,item[,rating]`` log
    (``T/matrix/factorization/PSOnlineMatrixFactorizationAndTopKGeneratorTest.scala``): every rating
    is a top-K query answered before it is learned; nDCG@K per ``--period`` seconds
    (``nDCGSink.nDCGPeriodsToCsv``).  ``--engine tensor``: the tensor engine (GPU when present, one
    process; under torchrun the items are sharded over the ranks), ``record``: the per-record engine."""
    import numpy as np
    import torch

    from .models.mf.topk_tensor import as_reference_records, ps_online_learner_and_generator_tensor
    from .utils.io import read_ratings
    from .utils.metrics import NDCGAggregator

    ts, u, i, r = read_ratings(args.input)
    if args.limit:
        ts, u, i, r = ts[:args.limit], u[:args.limit], i[:args.limit], r[:args.limit]
    order = np.argsort(ts, kind="stable")
    ts, u, i, r = ts[order], u[order], i[order], r[order]
    n_users, n_items = int(u.max()) + 1, int(i.max()) + 1
    kw = dict(num_factors=args.num_factors, range_min=args.range_min, range_max=args.range_max,
              learning_rate=args.learning_rate, negative_sample_rate=args.negative_sample_rate,
              user_memory=args.user_memory, K=args.k, worker_k=args.worker_k, bucket_size=args.bucket,
              seed=args.seed)
    agg = NDCGAggregator(args.period)
    if args.engine == "record":
        from .models.mf.apps import ps_online_learner_and_generator
        from .models.mf.core import Rating

        recs = [Rating(int(a), int(b), float(c), int(t)) for a, b, c, t in zip(u, i, r, ts)]
        out = ps_online_learner_and_generator(recs, init="hash", worker_parallelism=1, ps_parallelism=1, **kw)
        for uu, ii, tt, top in out:
            agg.add(tt, [it for _, it in top], ii)
    else:
        from .parallel.comm import Comm

        comm = Comm.init_from_env()
        dev = comm.device
        B = args.batch
        batches = [(torch.from_numpy(u[s:s + B].astype(np.int64)).to(dev),
                    torch.from_numpy(i[s:s + B].astype(np.int64)).to(dev),
                    torch.from_numpy(ts[s:s + B].astype(np.int64)).to(dev),
                    torch.from_numpy(r[s:s + B].astype(np.float32)).to(dev)) for s in range(0, len(u), B)]
        out = ps_online_learner_and_generator_tensor(batches, n_users, n_items, comm=comm, **kw)
        if comm.rank != 0:
            return 0
        for uu, ii, tt, top in as_reference_records(out):
            agg.add(tt, [it for _, it in top], ii)
    if args.csv:
        agg.to_csv(args.csv)
    print(json.dumps({"ratings": int(len(u)), "periods": agg.periods()[:10]}))
    return 0


def _read_libsvm(path):
    labels, rows = [], []
    for ln in open(path):
        p = ln.split()
        if not p:
            continue
        labels.append(float(p[0]))
        rows.append([(int(t.split(":")[0]), float(t.split(":")[1])) for t in p[1:]])
    return labels, rows


def cmd_pa(args):
    import torch

    from .models.pa.fast import DistributedPA, PAConfig
    from .parallel.comm import Comm

    comm = Comm.init_from_env()
    cfg = _apply_config(PAConfig, args)
    m = DistributedPA(cfg, comm)
    labels, rows = _read_libsvm(args.input)
    dev = comm.device
    correct = total = 0
    for e in range(args.epochs):
        for a in range(comm.rank * args.batch, len(rows), args.batch * comm.world):
            chunk = rows[a:a + args.batch]
            lab = labels[a:a + args.batch]
            indptr = torch.tensor([0] + [len(r) for r in chunk]).cumsum(0).to(dev)
            idx = torch.tensor([k for r in chunk for k, _ in r], dtype=torch.int32, device=dev)
            val = torch.tensor([v for r in chunk for _, v in r], dtype=torch.float32, device=dev)
            if cfg.kind == "binary":
                y = torch.tensor([1 if x > 0 else -1 for x in lab], dtype=torch.int8, device=dev)
            else:
                y = torch.tensor([int(x) for x in lab], dtype=torch.int32, device=dev)
            pred, _ = m.train_step(indptr, idx, val, y)
            if e == args.epochs - 1:
                correct += int((pred.to(y.dtype) == y).sum())
                total += len(chunk)
    print(json.dumps({"examples": total, "online_accuracy_last_epoch": correct / max(total, 1)}))


def cmd_w2v(args):
    import torch

    from .models.w2v.sgns import DistributedSGNS, SGNSConfig, skipgram_pairs, synthetic_corpus
    from .parallel.comm import Comm

    comm = Comm.init_from_env()
    cfg = _apply_config(SGNSConfig, args)
    m = DistributedSGNS(cfg, comm=comm)
    if args.input:
        toks = torch.tensor([int(t) for t in open(args.input).read().split()], dtype=torch.int32)
    else:
        toks = synthetic_corpus(args.tokens, cfg.vocab_size, seed=comm.rank)
    toks = toks.to(comm.device)
    c, o = skipgram_pairs(toks, cfg.window)
    losses = []
    for a in range(0, c.numel(), args.batch):
        loss = m.step(c[a:a + args.batch], o[a:a + args.batch], with_loss=(a // args.batch) % 50 == 0)
        if loss is not None:
            losses.append(loss)
    print(json.dumps({"pairs": int(c.numel()), "loss_trace": losses[:20]}))


def build_parser():
    ap = argparse.ArgumentParser(prog="flink_parameter_server_1_amd")
    sub = ap.add_subparsers(dest="cmd", required=True)

    def mf_common(p):
        p.add_argument("--input", required=True)
        p.add_argument("--users-out")
        p.add_argument("--items-out")
        p.add_argument("--num-factors", type=int, default=10)
        p.add_argument("--range-min", type=float, default=-0.01)
        p.add_argument("--range-max", type=float, default=0.01)
        p.add_argument("--learning-rate", type=float, default=0.01)
        p.add_argument("--negative-sample-rate", type=int, default=0)
        p.add_argument("--user-memory", type=int, default=128)
        p.add_argument("--pull-limit", type=int, default=1600)
        p.add_argument("--workers", type=int, default=4)
        p.add_argument("--ps", type=int, default=4)
        p.add_argument("--seed", type=int, default=None)

    p = sub.add_parser("mf-online")
    mf_common(p)
    p.add_argument("--engine", choices=["python", "native"], default="python",
                   help="native: the C++ record engine (csrc/host/record_engine.cpp)")
    p = sub.add_parser("mf-offline")
    mf_common(p)
    p.add_argument("--iterations", type=int, default=10)

    p = sub.add_parser("mf-gpu")
    p.add_argument("--config")
    p.add_argument("--input")
    p.add_argument("--num-users", type=int)
    p.add_argument("--num-items", type=int)
    p.add_argument("--dim", type=int)
    p.add_argument("--learning-rate", type=float)
    p.add_argument("--wire-dtype")
    p.add_argument("--exchange", choices=["auto", "rotate", "ps", "local"])
    p.add_argument("--sgd-mode", choices=["auto", "tiled", "flat", "grouped"])
    p.add_argument("--negative-sample-rate", type=int)
    p.add_argument("--user-memory", type=int)
    p.add_argument("--batch", type=int, default=1 << 20)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--truth-dim", type=int, default=8)
    p.add_argument("--checkpoint-dir")
    p.add_argument("--checkpoint-every", type=int, default=0)
    p.add_argument("--resume", action="store_true")
    p.add_argument("--items-out", help="id;value dump of the item factors (per-rank suffix at N > 1)")
    p.add_argument("--users-out", help="id;value dump of the user factors (per-rank suffix at N > 1)")
    p.add_argument("--model-in-users", help="warm start: id;value user factors")
    p.add_argument("--model-in-items", help="warm start: id;value item factors")

    p = sub.add_parser("topk")
    p.add_argument("--users", required=True)
    p.add_argument("--items", required=True)
    p.add_argument("--test", required=True)
    p.add_argument("--k", type=int, default=100)
    p.add_argument("--period", type=int, default=86400)
    p.add_argument("--csv")

    p = sub.add_parser("mf-topk", help="online MF + top-K generation with nDCG per period "
                                        "(psOnlineLearnerAndGenerator)")
    p.add_argument("--input", required=True, help="ts,user,item[,rating] lines")
    p.add_argument("--engine", choices=["tensor", "record"], default="tensor")
    p.add_argument("--num-factors", type=int, default=10)
    p.add_argument("--range-min", type=float, default=-0.01)
    p.add_argument("--range-max", type=float, default=0.01)
    p.add_argument("--learning-rate", type=float, default=0.2)
    p.add_argument("--negative-sample-rate", type=int, default=9)
    p.add_argument("--user-memory", type=int, default=4)
    p.add_argument("--k", type=int, default=100)
    p.add_argument("--worker-k", type=int, default=100)
    p.add_argument("--bucket", type=int, default=100)
    p.add_argument("--batch", type=int, default=1024, help="tensor engine: ratings per micro-batch")
    p.add_argument("--period", type=int, default=86400)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--limit", type=int, default=0, help="first N ratings only (0: all)")
    p.add_argument("--csv", help="nDCG per period (nDCGPeriodsToCsv)")

    p = sub.add_parser("pa-train")
    p.add_argument("--config")
    p.add_argument("--input", required=True)
    p.add_argument("--feature-count", type=int, required=False)
    p.add_argument("--kind")
    p.add_argument("--label-count", type=int)
    p.add_argument("--variant")
    p.add_argument("--aggressiveness", type=float)
    p.add_argument("--batch", type=int, default=4096)
    p.add_argument("--epochs", type=int, default=1)

    p = sub.add_parser("w2v")
    p.add_argument("--config")
    p.add_argument("--input")
    p.add_argument("--vocab-size", type=int)
    p.add_argument("--dim", type=int)
    p.add_argument("--window", type=int)
    p.add_argument("--learning-rate", type=float)
    p.add_argument("--tokens", type=int, default=1 << 20)
    p.add_argument("--batch", type=int, default=1 << 16)

    p = sub.add_parser("split-log", help="31-day train / 14-day test split (Data_Manipulation notebook)")
    p.add_argument("--input", required=True)
    p.add_argument("--train-out", required=True)
    p.add_argument("--test-out", required=True)
    p.add_argument("--train-days", type=float, default=31)
    p.add_argument("--test-days", type=float, default=14)

    p = sub.add_parser("eval-factors", help="top-k recall/precision of dumped factors (Tester notebook)")
    p.add_argument("--users", required=True)
    p.add_argument("--items", required=True)
    p.add_argument("--test", required=True)
    p.add_argument("--train")
    p.add_argument("--k", type=int, default=5)

    p = sub.add_parser("bench")
    p.add_argument("rest", nargs=argparse.REMAINDER)
    ap.add_argument("--log-level", default=None, help="package log level (default FPS_LOG_LEVEL or WARNING)")
    ap.add_argument("--log-messages", action="store_true",
                    help="DEBUG line per record / pull answer / PS message (the reference main-jar logging)")
    return ap


def cmd_split_log(args):
    from .utils.eval_tools import split_log_file

    n_tr, n_te = split_log_file(args.input, args.train_out, args.test_out, args.train_days, args.test_days)
    print(json.dumps({"train": n_tr, "test": n_te}))
    return 0


def cmd_eval_factors(args):
    from .utils.eval_tools import evaluate_factor_files

    print(json.dumps(evaluate_factor_files(args.users, args.items, args.test, args.k, args.train)))
    return 0


def main(argv=None):
    args = build_parser().parse_args(argv)
    from .utils import logs

    logs.configure(args.log_level, True if args.log_messages else None)
    if args.cmd == "split-log":
        return cmd_split_log(args)
    if args.cmd == "eval-factors":
        return cmd_eval_factors(args)
    if args.cmd in ("mf-online", "mf-offline"):
        return cmd_mf(args, offline=args.cmd == "mf-offline")
    if args.cmd == "mf-gpu":
        return cmd_mf_gpu(args)
    if args.cmd == "topk":
        return cmd_topk(args)
    if args.cmd == "mf-topk":
        return cmd_mf_topk(args)
    if args.cmd == "pa-train":
        return cmd_pa(args)
    if args.cmd == "w2v":
        return cmd_w2v(args)
    if args.cmd == "bench":
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        import bench

        return bench.main(args.rest)
    return 1


if __name__ == "__main__":
    sys.exit(main())

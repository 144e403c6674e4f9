"""Spawn a gloo process group on CPU (the Flink mini-cluster analogue)."""
import os
import socket
import tempfile
import traceback

import torch.multiprocessing as mp


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _entry(rank, world, port, fn, args, out_dir):
    import pickle

    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = fn(rank, world, *args)
        err = None
    except Exception:  # pragma: no cover - reported by the parent
        res, err = None, traceback.format_exc()
    with open(os.path.join(out_dir, f"r{rank}.pkl"), "wb") as f:
        pickle.dump((res, err), f)
    if dist.is_initialized():  # fn may have left the group itself (Comm.shutdown)
        dist.destroy_process_group()


def run_ranks(fn, world, *args):
    """Run ``fn(rank, world, *args)`` on ``world`` gloo ranks; returns the list of results."""
    import pickle

    out_dir = tempfile.mkdtemp(prefix="fps_dist_")
    for attempt in range(2):
        try:
            mp.spawn(_entry, args=(world, free_port(), fn, args, out_dir), nprocs=world, join=True)
            break
        except Exception as e:  # a rendezvous port taken by a parallel test worker: once more
            if attempt or not any(m in str(e) for m in ("Address already in use", "EADDRINUSE")):
                raise
    return _collect(out_dir, world)


def _collect(out_dir, world):
    """Per-rank results; on failure every failed rank's traceback, the root cause (an
    error that is not a peer's closed connection) first."""
    import pickle

    results, errs = [], []
    for r in range(world):
        with open(os.path.join(out_dir, f"r{r}.pkl"), "rb") as f:
            res, err = pickle.load(f)
        if err:
            errs.append((r, err))
        results.append(res)
    if errs:
        errs.sort(key=lambda e: "Connection closed" in e[1] or "Connection reset" in e[1])
        raise AssertionError("\n".join(f"rank {r} failed:\n{e}" for r, e in errs))
    return results


def _nccl_entry(rank, world, port, fn, args, out_dir):
    """One rank of a real multi-GPU world: GPU ``rank``, RCCL (``nccl``) process group."""
    import pickle

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch
    import torch.distributed as dist

    try:
        torch.cuda.set_device(rank)
        dev = torch.device("cuda", rank)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        from flink_parameter_server_1_amd.parallel.comm import Comm

        res, err = fn(Comm(device=dev), *args), None
        torch.cuda.synchronize(dev)
    except Exception:  # pragma: no cover - reported by the parent
        res, err = None, traceback.format_exc()
    with open(os.path.join(out_dir, f"r{rank}.pkl"), "wb") as f:
        pickle.dump((res, err), f)
    if dist.is_initialized():
        dist.destroy_process_group()


def run_nccl(fn, world, *args):
    """Run ``fn(comm, *args)`` on ``world`` processes, one GPU each, over RCCL.  Every
    child is a fresh interpreter (spawn), so nothing of the parent's GPU state is
    inherited.  Returns the list of results (CPU objects)."""
    import pickle

    out_dir = tempfile.mkdtemp(prefix="fps_nccl_")
    mp.spawn(_nccl_entry, args=(world, free_port(), fn, args, out_dir), nprocs=world, join=True)
    return _collect(out_dir, world)

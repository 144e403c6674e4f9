"""Diagnostic: the aten ops of one PA PS-path step (bench/bench_pa.py --ps-path geometry) by
call site -- which Python lines launch the small per-step kernels."""
import collections
import sys
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

sys.path.insert(0, ".")
from flink_parameter_server_1_amd.models.pa.fast import DistributedPA, PAConfig, synthetic_sparse_batch  # noqa: E402
from flink_parameter_server_1_amd.parallel.comm import Comm  # noqa: E402


def main():
    comm = Comm.init_from_env()
    dev = comm.device
    m = DistributedPA(PAConfig(feature_count=1_000_000_000, kind="binary", local_direct=False), comm)
    batches = [synthetic_sparse_batch(65536, 64, 1_000_000_000, seed=1, step=s, device=dev) for s in range(4)]
    for s in range(4):
        m.train_step(*batches[s])
    torch.cuda.synchronize()
    seen = collections.Counter()

    class _Log(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            fr = [f for f in traceback.extract_stack()[:-1] if "flink_parameter_server_1_amd" in f.filename]
            where = " < ".join(f"{f.filename.split('flink_parameter_server_1_amd/')[-1]}:{f.lineno}" for f in fr[-3:][::-1])
            seen[(str(func.overloadpacket.__name__), where)] += 1
            return func(*args, **(kwargs or {}))

    with _Log():
        m.train_step(*batches[0])
    torch.cuda.synchronize()
    print("aten ops of one step by call site:", sum(seen.values()))
    for (op, where), n in sorted(seen.items(), key=lambda x: -x[1]):
        print(f"{n:4d} {op:24s} {where}")


if __name__ == "__main__":
    main()

"""Diagnostic: which Python lines launch the small per-batch torch kernels of the online
MF + top-K step (bench/bench_mf_topk.py geometry).  Prints the profiler's op table
grouped by the calling stack (fills, copies, elementwise ops)."""
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, ".")
from flink_parameter_server_1_amd.core.tensor_engine import TensorRuntime  # noqa: E402
from flink_parameter_server_1_amd.models.mf.topk_tensor import OnlineMFTopKWorker  # noqa: E402
from flink_parameter_server_1_amd.parallel.comm import Comm  # noqa: E402
from flink_parameter_server_1_amd.ps.device_logics import DeviceSimplePSLogic  # noqa: E402


def main():
    users, items, dim, batch = 1_000_000, 1_000_000, 64, 4096
    comm = Comm.init_from_env()
    dev = comm.device
    worker = OnlineMFTopKWorker(items, dim, 0.01, K=100, worker_k=75, memory=16, negative_sample_rate=2,
                                bucket_size=65536, range_min=-0.1, range_max=0.1, prefill_items=True,
                                num_users=users)
    logic = DeviceSimplePSLogic(users, dim, op="add_renorm", init=("uniform", -0.1, 0.1))
    logic.emit = "none"
    rt = TensorRuntime(comm, staleness=0, output_sink=lambda e: None).start(worker, logic)
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    data = [(torch.randint(0, users, (batch,), generator=g, device=dev),
             torch.randint(0, items, (batch,), generator=g, device=dev),
             torch.arange(s * batch, (s + 1) * batch, device=dev),
             torch.rand(batch, generator=g, device=dev)) for s in range(4)]
    for s in range(4):
        rt.submit(data[s])
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        for s in range(4):
            rt.submit(data[s])
        torch.cuda.synchronize()
    # which package lines issue the aten ops of one batch (a dispatch-mode log)
    import collections
    import traceback

    from torch.utils._python_dispatch import TorchDispatchMode

    seen = collections.Counter()

    class _Log(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            fr = [f for f in traceback.extract_stack()[:-1] if "flink_parameter_server_1_amd" in f.filename]
            where = " < ".join(f"{f.filename.split('flink_parameter_server_1_amd/')[-1]}:{f.lineno}" for f in fr[-3:][::-1])
            seen[(str(func.overloadpacket.__name__), where)] += 1
            return func(*args, **(kwargs or {}))

    with _Log():
        rt.submit(data[0])
    torch.cuda.synchronize()
    print("aten ops of one batch by call site:", sum(seen.values()))
    for (op, where), n in sorted(seen.items(), key=lambda x: -x[1]):
        print(f"{n:4d} {op:24s} {where}")
    ka = prof.key_averages(group_by_stack_n=6)
    rows = [e for e in ka if e.device_time_total > 0 and not e.key.startswith("fps") and e.count >= 4
            and any(t in e.key for t in ("fill", "copy", "zero", "full", "add", "mul", "where", "remainder",
                                           "arange", "cat", "index", "sum", "max", "sqrt", "lt", "ge", "eq",
                                           "to", "clone", "sub", "div", "ne", "gather", "scatter", "sort"))]
    rows.sort(key=lambda e: -e.count)
    for e in rows[:45]:
        print(f"{e.key:28s} n={e.count:4d} dev_us={e.device_time_total:8.1f}")
        for fr in e.stack[:6]:
            print("      ", fr)


if __name__ == "__main__":
    main()

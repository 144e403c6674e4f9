"""Probe: does a one-rank RCCL group take point-to-point sends / receives to itself through
``Comm.p2p`` (batch_isend_irecv), with the works waited on from two streams?"""
import os
import socket
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.distributed as dist

from flink_parameter_server_1_amd.parallel.comm import Comm

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
s = socket.socket()
s.bind(("127.0.0.1", 0))
port = s.getsockname()[1]
s.close()
dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
comm = Comm(device=dev)
a = torch.randn(1 << 20, device=dev)
b = torch.empty_like(a)
side = torch.cuda.Stream(dev)
side.wait_stream(torch.cuda.current_stream(dev))
try:
    with torch.cuda.stream(side):
        works = comm.p2p([(a, 0)], [(b, 0)])
    for w in works:
        w.wait()
    with torch.cuda.stream(side):
        for w in works:
            w.wait()
    torch.cuda.synchronize()
    print("self p2p ok", bool(torch.equal(a, b)), len(works))
except Exception as e:  # report, do not hide
    print("self p2p failed:", type(e).__name__, str(e)[:300])
dist.destroy_process_group()

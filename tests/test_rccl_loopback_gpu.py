"""GPU: ``parallel.comm.Comm`` through a one-rank RCCL group -- the rotation's
point-to-point contract (posted from one stream, waited on from others, three
rotating buffers reused) and the PS all-to-alls run as RCCL kernels on a one-GPU box.
The multi-rank data flow itself is covered by the virtual world (``test_vworld_gpu.py``)."""
import pytest
import torch

from flink_parameter_server_1_amd.parallel.comm import Comm

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def test_rccl_p2p_rotation_pattern_to_self(rccl_loopback):
    """Sub-steps alternate two compute streams; each posts a send + receive (here: to
    its own rank) from the previous sub-step's stream, the next sub-step's stream and
    the posting stream both wait on the works, and the three buffers rotate roles --
    the data every receive delivers is the block its send read, every time."""
    comm = Comm(device=DEV)
    assert comm.backend == "nccl" and comm.world == 1
    main = torch.cuda.current_stream(DEV)
    aux = torch.cuda.Stream(DEV)
    aux.wait_stream(main)
    bufs = [torch.full((1 << 18, 64), float(i), device=DEV) for i in range(3)]
    A, P, F = 0, 1, 2
    streams = (main, aux)
    for s in range(12):
        cur, prev = streams[s % 2], streams[(s - 1) % 2]
        with torch.cuda.stream(prev):
            works = comm.p2p([(bufs[P], 0)], [(bufs[F], 0)])
        with torch.cuda.stream(cur):
            bufs[A].add_(1.0)  # this sub-step's compute on the active block
        nxt = streams[(s + 1) % 2]
        for st in (nxt, cur):
            with torch.cuda.stream(st):
                for w in works:
                    w.wait()
        with torch.cuda.stream(nxt):
            assert_eq = (bufs[F] == bufs[P]).all()
        A, P, F = F, A, P
        torch.cuda.synchronize()
        assert bool(assert_eq), s
    main.wait_stream(aux)
    torch.cuda.synchronize()


def test_rccl_all_to_all_loopback_matches_local_copy(rccl_loopback):
    """``Comm.all_to_all`` / ``all_to_all_async`` through RCCL (loopback) == the
    world-1 local copy, for the fixed-shape plans' equal splits and uneven ones."""
    comm = Comm(device=DEV)
    comm.loopback = True
    x = torch.randn(1000, 16, device=DEV)
    out = comm.all_to_all(x, [1000], [1000])
    assert torch.equal(out, x) and out.data_ptr() != x.data_ptr()
    y, w = comm.all_to_all_async(x[:700], [700], [700])
    w.wait()
    torch.cuda.synchronize()
    assert torch.equal(y, x[:700])

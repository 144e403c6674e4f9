"""Probe: per-user integer atomics at the headline geometry (64M ratings, 10M users).
Design input for exact user rows (docs/ROUND5.md): what a per-rating ordinal
(returning atomicAdd) or a per-rating lock (CAS + exchange) costs on gfx950."""
import ctypes
import json
import os

import torch

LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libprobe_atomics.so")


def main():
    lib = ctypes.CDLL(LIB)
    lib.probe_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                              ctypes.c_void_p]
    n, users = 1 << 26, 10_000_000
    dev = torch.device("cuda")
    uid = torch.randint(0, users, (n,), dtype=torch.int32, device=dev)
    cnt = torch.zeros(users, dtype=torch.int32, device=dev)
    ord_ = torch.empty(n, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    names = {0: "plain gather (baseline)", 1: "returning atomicAdd", 2: "no-return atomicAdd",
             3: "lock CAS + exchange", 4: "returning atomicAdd, 1 lane per 16"}
    if os.environ.get("FPS_PROBE_ROWS"):  # only the row-update probes
        return rows(lib, dev, st)
    for which in (0, 1, 2, 3, 4):
        ts = []
        for rep in range(4):
            cnt.zero_()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rc = lib.probe_run(which, uid.data_ptr(), cnt.data_ptr(), ord_.data_ptr(), n, st)
            e1.record()
            torch.cuda.synchronize()
            assert rc == 0, rc
            if rep:
                ts.append(e0.elapsed_time(e1))
        ok = None
        if which in (1, 4):  # ordinals of each user are 0..c-1
            c = torch.bincount(uid.long(), minlength=users)
            ok = bool(torch.equal(cnt.long(), c)) and int(ord_.max()) == int(c.max()) - 1
        if which == 3:
            ok = int(cnt.abs().sum()) == 0
        print(json.dumps({"probe": names[which], "ms": min(ts), "per_s": n / (min(ts) / 1e3), "ok": ok}), flush=True)

    rows(lib, dev, st)


def rows(lib, dev, st):
    """256-B row updates (one wave per update): plain read-modify-write (Hogwild) vs
    float atomics, rows random over the table or owned by one XCD each
    (``s_getreg HW_REG_XCC_ID``).  Design input for exact user rows."""
    lib.probe_rows.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                               ctypes.c_void_p]
    names = {0: "row RMW plain (Hogwild)", 1: "row float atomics, agent scope", 2: "row float atomics, workgroup scope",
             3: "row float atomics, agent scope, XCD-owned rows", 4: "row float atomics, workgroup scope, XCD-owned rows"}
    n = 1 << 24  # one user phase of the headline step
    # working sets (rows of 256 B): 4 MB (one XCD's L2), 16 / 64 MB (the rotation's active
    # item block at N = 8 / 2), 200 MB (inside the 256 MiB Infinity Cache), then the round-5
    # sets 640 MB / 2.5 GB; FPS_PROBE_ROW_SETS="16384,65536" picks others
    sets = [int(x) for x in os.environ.get("FPS_PROBE_ROW_SETS", "16384,65536,262144,819200,2500000,10000000")
            .split(",")]
    for nrows, layout in [(r, lay) for r in sets for lay in ("random", "tile")]:
        if layout == "random":
            uid = torch.randint(0, nrows, (n,), dtype=torch.int32, device=dev)
        else:  # tile-clustered: each run of 4096 updates stays inside one 256-row tile (a tile SGD chunk)
            tiles = max(1, nrows // 256)
            t = torch.randint(0, tiles, (n // 4096 + 1,), dtype=torch.int32, device=dev).repeat_interleave(4096)[:n]
            uid = (t * 256 + torch.randint(0, min(256, nrows), (n,), dtype=torch.int32, device=dev)).clamp_(max=nrows - 1)
        tab = torch.zeros(nrows, 64, device=dev)
        for mode in (0, 1, 2, 3, 4):
            ts = []
            for rep in range(4):
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                rc = lib.probe_rows(mode, uid.data_ptr(), tab.data_ptr(), n, nrows, st)
                e1.record()
                torch.cuda.synchronize()
                assert rc == 0, rc
                if rep:
                    ts.append(e0.elapsed_time(e1))
            ms = min(ts)
            print(json.dumps({"probe": names[mode], "rows": nrows, "MB": nrows * 256 / 2**20, "layout": layout,
                              "updates": n, "ms": ms,
                              "GB_per_s_256B": n * 256 / (ms / 1e3) / 1e9}), flush=True)
        del tab


if __name__ == "__main__":
    main()

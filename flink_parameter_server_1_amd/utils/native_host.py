"""ctypes binding of ``_lib/libfps_host.so`` (csrc/host/fps_host.cpp).

Host-native data loading / model IO / sparse store.  Every entry point has a
pure-Python fallback in its caller (``utils.io``), used only when the library
is not built.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_SO = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_lib", "libfps_host.so")
_lib = None
_err = None

c_int, c_i64, c_f32, c_u32, c_vp, c_cp = (ctypes.c_int, ctypes.c_int64, ctypes.c_float, ctypes.c_uint32,
                                          ctypes.c_void_p, ctypes.c_char_p)
_SIG = {
    "fps_parse_ratings": ([c_cp, c_i64, c_vp, c_vp, c_vp, c_vp, c_f32], c_i64),
    "fps_count_lines": ([c_cp], c_i64),
    "fps_write_factors_text": ([c_cp, c_vp, c_vp, c_i64, c_int, c_int], c_int),
    "fps_read_id_value_text": ([c_cp, c_i64, c_vp, c_vp], c_i64),
    "fps_write_snapshot": ([c_cp, c_int, c_i64, c_int, c_int, c_int, c_i64, c_vp, c_vp, c_i64], c_int),
    "fps_read_snapshot_header": ([c_cp, c_vp], c_int),
    "fps_read_snapshot": ([c_cp, c_vp, c_vp, c_i64], c_int),
    "fps_gen_ratings": ([c_i64, c_i64, c_i64, c_u32, c_i64, c_vp, c_vp, c_vp], None),
    "fps_hs_create": ([c_int, c_f32, c_f32, c_u32, c_i64], c_vp),
    "fps_hs_destroy": ([c_vp], None),
    "fps_hs_size": ([c_vp], c_i64),
    "fps_hs_pull": ([c_vp, c_vp, c_i64, c_vp], None),
    "fps_hs_push": ([c_vp, c_vp, c_i64, c_vp, c_int], None),
    "fps_hs_dump": ([c_vp, c_vp, c_vp, c_i64], c_i64),
    "fps_mf_online_record": ([c_vp, c_vp, c_vp, c_i64, c_int, c_int, c_int, ctypes.c_double, ctypes.c_double,
                              ctypes.c_double, ctypes.c_double, c_u32, c_i64, c_int, c_int, c_vp, c_vp, c_i64, c_vp,
                              c_vp, c_i64, c_vp, c_vp], c_int),
}


def lib():
    global _lib, _err
    if _lib is None and _err is None:
        try:
            h = ctypes.CDLL(_SO)
            for name, (args, res) in _SIG.items():
                fn = getattr(h, name)
                fn.argtypes, fn.restype = args, res
            _lib = h
        except OSError as e:
            _err = e
    return _lib


def available() -> bool:
    return lib() is not None


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


class HashStore:
    """Open-addressing ``int64 id -> fp32[dim]`` store with lazy hash-RNG init
    (the generic sparse-id PS store; same init values as the device tables)."""

    def __init__(self, dim: int, lo: float = -0.01, hi: float = 0.01, seed: int = 0, capacity: int = 1024):
        L = lib()
        if L is None:
            raise RuntimeError(f"host library unavailable: {_err}")
        self.dim = dim
        self._h = L.fps_hs_create(dim, lo, hi, seed & 0xFFFFFFFF, capacity)

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.fps_hs_destroy(self._h)
            self._h = None

    def __len__(self):
        return int(lib().fps_hs_size(self._h))

    def pull(self, keys) -> np.ndarray:
        k = np.ascontiguousarray(keys, dtype=np.int64)
        out = np.empty((k.size, self.dim), dtype=np.float32)
        lib().fps_hs_pull(self._h, _p(k), k.size, _p(out))
        return out

    def push(self, keys, deltas, op: str = "add"):
        k = np.ascontiguousarray(keys, dtype=np.int64)
        d = np.ascontiguousarray(deltas, dtype=np.float32).reshape(k.size, self.dim)
        lib().fps_hs_push(self._h, _p(k), k.size, _p(d), 0 if op == "add" else 1)

    def dump(self):
        n = len(self)
        k = np.empty(n, dtype=np.int64)
        v = np.empty((n, self.dim), dtype=np.float32)
        m = lib().fps_hs_dump(self._h, _p(k), _p(v), n)
        return k[:m], v[:m]

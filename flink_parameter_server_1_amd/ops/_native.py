"""ctypes binding of the in-tree gfx950 kernel library ``_lib/libfps_kernels.so``.

The library exposes a plain C ABI (``fps_*`` launchers: device pointers, sizes
and a ``hipStream_t``) so it does not depend on torch's C++ ABI and builds in
seconds with hipcc.  It must be loaded *after* ``import torch``: torch ships
the HIP runtime (``libamdhip64.so.7``) and the library binds to that loaded
copy, so kernels run on torch's device/context and streams.

On a GPU box a missing / unloadable library is an error (``require()``),
never a silent fallback to eager PyTorch.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must precede the library load, see docstring)

_LIB_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_lib")
KERNELS_SO = os.environ.get("FPS_KERNELS_SO") or os.path.join(_LIB_DIR, "libfps_kernels.so")  # override: A/B of builds

_lock = threading.Lock()
_lib = None
_err = None

c_int, c_i64, c_f32, c_u32, c_vp = ctypes.c_int, ctypes.c_int64, ctypes.c_float, ctypes.c_uint32, ctypes.c_void_p
c_u64 = ctypes.c_uint64
c_double = ctypes.c_double

_SIGNATURES = {
    "fps_abi_version": [],
    "fps_init_rows": [c_vp, c_i64, c_int, c_i64, c_i64, c_f32, c_f32, c_u32, c_vp],
    "fps_mark_rows": [c_vp, c_vp, c_i64, c_vp],
    "fps_pack_counts": [c_vp, c_int, c_int, c_int, c_vp, c_vp],
    "fps_segment_fill_set_link_wgs": [c_int],
    "fps_static_plan": [c_vp, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp],
    "fps_flip_masked": [c_vp, c_vp, c_i64, c_int, c_vp],
    "fps_dedup_flags": [c_vp, c_i64, c_vp, c_vp, c_u32, c_i64, c_int, c_int, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp,
                        c_vp],
    "fps_dedup_flags_ws_ints": [c_i64, c_int],
    "fps_gather_rows": [c_vp, c_vp, c_int, c_i64, c_int, c_vp, c_int, c_vp, c_int, c_vp],
    "fps_apply_rows": [c_vp, c_vp, c_vp, c_i64, c_int, c_vp, c_int, c_int, c_f32, c_f32, c_vp, c_vp],
    "fps_dedup": [c_vp, c_i64, c_vp, c_u32, c_int, c_int, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp],
    "fps_route_requests": [c_vp, c_i64, c_int, c_int, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp],
    "fps_dedup_hashed": [c_vp, c_i64, c_vp, c_i64, c_u32, c_int, c_int, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                         c_vp],
    "fps_pair_sgd_pulled": [c_vp, c_int, c_vp, c_vp, c_vp, c_vp, c_i64, c_int, c_f32, c_int, c_vp, c_vp],
    "fps_mf_sgd_local_seg": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_int, c_f32, c_f32, c_int, c_vp],
    "fps_rot_partition": [c_vp, c_vp, c_vp, c_i64, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp],
    "fps_tile_partition_ws_ints": [c_int, c_int, c_int],
    "fps_tile_partition_set_h16": [c_int],
    "fps_tile_partition_set_grid": [c_int],
    "fps_tile_partition_set_slim": [c_int],
    "fps_segment_fill": [c_vp, c_i64, c_i64, c_vp, c_vp, c_int, c_vp, c_double],
    "fps_tile_partition_get_slim": [],
    "fps_tile_partition": [c_vp, c_vp, c_vp, c_i64, c_int, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp, c_vp,
                           c_vp, c_vp, c_int, c_vp, c_vp],
    "fps_mf_sgd_tiled": [c_vp, c_vp, c_vp, c_int, c_vp, c_int, c_int, c_i64, c_vp, c_vp, c_i64, c_int, c_int, c_f32,
                         c_f32, c_vp, c_int, c_i64, c_int, c_vp],
    "fps_score_filter": [c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp, c_int, c_vp, c_vp, c_vp, c_int, c_vp],
    "fps_topk_merge_cand": [c_vp, c_vp, c_vp, c_int, c_int, c_vp, c_vp, c_int, c_vp, c_int, c_vp],
    "fps_mf_online_phase": [c_vp, c_vp, c_vp, c_vp, c_i64, c_int, c_f32, c_vp, c_vp, c_vp, c_vp, c_vp],
    "fps_index_refresh": [c_vp, c_i64, c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_vp],
    "fps_round_plan": [c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_vp],
    "fps_topk_scan_prep": [c_vp, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp],
    "fps_topk_seen_merge": [c_vp, c_vp, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int,
                            c_vp, c_vp, c_vp, c_vp],
    "fps_score_filter_lemp": [c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp, c_int, c_vp, c_vp, c_f32, c_vp, c_vp, c_vp,
                              c_int, c_vp],
    "fps_score_filter_bf16": [c_vp, c_vp, c_int, c_int, c_int, c_vp, c_int, c_vp, c_vp, c_f32, c_f32, c_vp, c_vp, c_int,
                              c_vp, c_vp, c_vp, c_vp, c_vp, c_vp],
    "fps_score_set_min_wgs": [c_int],
    "fps_score_set_ilv": [c_int],
    "fps_score_set_pd": [c_int],
    "fps_score_set_cur2": [c_int],
    "fps_coord_gate": [c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp],
    "fps_cand_rescore": [c_vp, c_vp, c_vp, c_int, c_int, c_vp, c_int, c_vp, c_int, c_vp, c_vp, c_vp],
    "fps_lock_acquire": [c_vp, c_vp, c_i64, ctypes.c_int32, c_vp, c_vp],
    "fps_lock_release": [c_vp, c_vp, c_i64, c_vp, c_vp],
    "fps_topk_merge": [c_vp, c_i64, c_int, c_int, c_vp, c_vp, c_vp, c_int, c_vp],
    "fps_topk_select": [c_vp, c_i64, c_int, c_int, c_vp, c_vp, c_vp, c_int, c_vp, c_vp],
    "fps_bucketize": [c_vp, c_i64, c_int, c_int, c_i64, c_vp, c_vp, c_vp],
    "fps_mf_sgd_local": [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_int, c_f32, c_f32, c_int, c_vp],
    "fps_mf_sgd_pulled": [c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_i64, c_int, c_f32, c_f32, c_int, c_vp],
    "fps_mf_sq_err": [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_int, c_vp, c_vp],
    "fps_csr_count": [c_vp, c_i64, c_vp, c_vp],
    "fps_csr_scatter": [c_vp, c_i64, c_vp, c_vp, c_vp, c_vp],
    "fps_mf_sgd_grouped": [c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_vp, c_i64, c_int, c_f32, c_f32, c_vp, c_vp],
    "fps_sample_uniform_reject": [c_i64, c_int, ctypes.c_int32, c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_u32,
                                  ctypes.c_uint64, c_vp, c_vp],
    "fps_ring_push": [c_vp, c_vp, c_vp, c_vp, c_i64, c_int, c_vp],
    "fps_known_append": [c_vp, c_vp, c_vp, c_vp, c_i64, c_vp],
    "fps_sample_alias": [c_vp, c_vp, ctypes.c_int32, c_i64, c_u32, ctypes.c_uint64, c_vp, c_vp],
    "fps_sgns_step": [c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_i64, c_int, c_f32, c_f32, c_vp, c_vp, c_vp, c_vp],
    "fps_sgns_step_v4g": [c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_i64, c_int, c_f32, c_f32, c_vp, c_vp, c_vp, c_int, c_vp],
    "fps_pa_binary": [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_int, c_f32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp],
    "fps_score_gemm": [c_vp, c_vp, c_vp, c_int, c_int, c_int, c_i64, c_vp],
    "fps_pa_multi": [c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_i64, c_int, c_int, c_f32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp],
    "fps_ht_lookup": [c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_int,
                      c_int, c_f32, c_f32, c_u32, c_vp],
    "fps_ht_rehash": [c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp],
    "fps_sgns_standard": [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_int, c_int, c_f32, c_vp, c_vp, c_vp, c_vp, c_vp,
                          c_vp, c_int],
    "fps_sgns_standard_coef": [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_int, c_int, c_f32, c_vp, c_vp, c_vp, c_vp,
                               c_vp, c_int],
    "fps_sgns_rows": [c_vp, c_vp, c_vp, c_vp, c_int, c_i64, c_vp, c_int, c_vp, c_vp, c_vp, c_int, c_vp],
}
#: optional symbols (added by later kernel files); bound when present
OPTIONAL = {}
#: launchers / sizers returning int64 (the rest return an int status)
RESTYPE_I64 = {"fps_tile_partition_ws_ints", "fps_dedup_flags_ws_ints"}


def register(name, argtypes):
    OPTIONAL[name] = argtypes


def load():
    """Load the kernel library once; returns the ctypes handle or None."""
    global _lib, _err
    if _lib is not None or _err is not None:
        return _lib
    with _lock:
        if _lib is not None or _err is not None:
            return _lib
        if not os.path.exists(KERNELS_SO):
            _err = FileNotFoundError(f"{KERNELS_SO} missing: run `python csrc/build.py`")
            return None
        try:
            lib = ctypes.CDLL(KERNELS_SO)
            for name, args in list(_SIGNATURES.items()) + list(OPTIONAL.items()):
                fn = getattr(lib, name, None)
                if fn is None:
                    if name in _SIGNATURES:
                        raise AttributeError(f"{name} missing from {KERNELS_SO}")
                    continue
                fn.argtypes = args
                fn.restype = c_i64 if name in RESTYPE_I64 else c_int
            _lib = lib
        except OSError as e:  # pragma: no cover
            _err = e
    return _lib


def require():
    lib = load()
    if lib is None:
        raise RuntimeError(f"gfx950 kernel library unavailable: {_err}")
    return lib


def available() -> bool:
    return load() is not None


def check(rc: int, what: str):
    if rc != 0:
        raise RuntimeError(f"{what} failed with hipError {rc}")


#: the current stream's raw handle without building a Stream object (the launch path's
#: ``torch.cuda.current_stream(device)`` resolved the device index and wrapped the stream
#: in Python on every kernel launch: ~1/10 of a PS micro-batch's host time)
_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_ptr(device=None) -> int:
    if _RAW_STREAM is not None:
        if isinstance(device, torch.device) and device.type == "cuda":
            return _RAW_STREAM(device.index if device.index is not None else torch.cuda.current_device())
        if device is None:
            return _RAW_STREAM(torch.cuda.current_device())
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t):
    """Optional kernel operand (None -> nullptr); must be a GPU tensor."""
    if t is None:
        return None
    if not t.is_cuda:
        raise ValueError(f"kernel operand on {t.device}: expected a GPU tensor")
    return t.data_ptr()

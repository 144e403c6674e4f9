"""Tracing hooks: roctx ranges around pipeline stages + torch.profiler export.

The reference only logs every message at DEBUG (``M/FlinkParameterServer.scala:237,247,284``).
Here ``trace_range("pull-a2a")`` etc. emit roctx ranges (``torch.cuda.nvtx``
maps to roctx on ROCm builds) that show up in ``rocprofv3 --marker-trace``
timelines; ``FPS_TRACE=0`` turns them into no-ops.  ``profile_to`` wraps a
block in ``torch.profiler`` and writes a Chrome trace.
"""
from __future__ import annotations

import os
from contextlib import contextmanager, nullcontext

_ENABLED = os.environ.get("FPS_TRACE", "1") != "0"
_NV = False  # False: not looked up yet; None: no roctx (no GPU, or FPS_TRACE=0)


def _nvtx():
    """``torch.cuda.nvtx`` (roctx on ROCm) if a GPU is present, looked up once: every
    pipeline stage opens a range, and a per-call ``torch.cuda.is_available()`` was
    ~1/10 of a PS-path micro-batch's host time (profiles/r6_pa_host_profile.txt)."""
    global _NV
    if _NV is False:
        _NV = None
        if _ENABLED:
            try:
                import torch

                if torch.cuda.is_available():
                    _NV = torch.cuda.nvtx
            except Exception:  # pragma: no cover
                pass
    return _NV


class _Range:
    """roctx range + optional ``utils.metrics.StageTimer`` stage as a plain context
    manager (a generator-based one cost two frames per stage on the host)."""

    __slots__ = ("name", "timer", "_nv", "_t")

    def __init__(self, name: str, timer=None):
        self.name, self.timer, self._t = name, timer, None
        self._nv = _nvtx()

    def __enter__(self):
        if self._nv is not None:
            self._nv.range_push(self.name)
        if self.timer is not None:
            self._t = self.timer.stage(self.name)
            self._t.__enter__()
        return self

    def __exit__(self, *exc):
        if self._t is not None:
            self._t.__exit__(*exc)
        if self._nv is not None:
            self._nv.range_pop()
        return False


def trace_range(name: str) -> _Range:
    return _Range(name)


def stage(name: str, timer=None) -> _Range:
    """A pipeline stage: roctx range (``rocprofv3 --marker-trace``) plus, when a
    ``utils.metrics.StageTimer`` is attached, HIP-event timing of the stage."""
    return _Range(name, timer)


@contextmanager
def profile_to(path: str, enabled: bool = True):
    if not enabled:
        with nullcontext():
            yield None
        return
    import torch

    acts = [torch.profiler.ProfilerActivity.CPU]
    if torch.cuda.is_available():
        acts.append(torch.profiler.ProfilerActivity.CUDA)
    with torch.profiler.profile(activities=acts, record_shapes=False) as prof:
        yield prof
    prof.export_chrome_trace(path)

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


def _nvtx():
    try:
        import torch

        if torch.cuda.is_available():
            return torch.cuda.nvtx
    except Exception:  # pragma: no cover
        pass
    return None


@contextmanager
def trace_range(name: str):
    nv = _nvtx() if _ENABLED else None
    if nv is None:
        yield
        return
    nv.range_push(name)
    try:
        yield
    finally:
        nv.range_pop()


@contextmanager
def stage(name: str, timer=None):
    """A pipeline stage: roctx range (``rocprofv3 --marker-trace``) plus, when a
    ``utils.metrics.StageTimer`` is attached, HIP-event timing of the stage."""
    if timer is None:
        with trace_range(name):
            yield
        return
    with trace_range(name), timer.stage(name):
        yield


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

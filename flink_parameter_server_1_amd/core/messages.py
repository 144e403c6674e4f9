"""L1 message vocabulary of the parameter server.

Mirrors the reference wire vocabulary (``M/entities/Messages.scala:3-8``):
``WorkerToPS(workerPartitionIndex, Either[Pull, Push])``,
``PSToWorker(workerPartitionIndex, PullAnswer)``, ``Pull(paramId)``,
``Push(paramId, delta)``, ``PullAnswer(paramId, param)``.

These record types are used by the per-record *compat* path (CPU, event
driven).  The GPU fast path never materialises them: it moves the same
information as structure-of-arrays tensors (``keys int32[N]``,
``values [N, D]``) through RCCL all-to-all (see ``parallel/``).

``Left`` / ``Right`` model Scala's ``Either``: the engines return a stream
of ``Left(worker_output)`` / ``Right(ps_output)`` exactly like
``transform`` does in ``M/FlinkParameterServer.scala:325-328``.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Generic, TypeVar

A = TypeVar("A")
B = TypeVar("B")


class Either(Generic[A, B]):
    """Scala-style ``Either``.  ``Left`` = worker side, ``Right`` = PS side."""

    __slots__ = ("value",)
    is_left: bool = False
    is_right: bool = False

    def __init__(self, value):
        self.value = value

    def __eq__(self, other):
        return type(self) is type(other) and self.value == other.value

    def __hash__(self):
        return hash((type(self).__name__, _hashable(self.value)))

    def __repr__(self):
        return f"{type(self).__name__}({self.value!r})"

    # pickling support for __slots__ classes
    def __getstate__(self):
        return self.value

    def __setstate__(self, state):
        self.value = state


class Left(Either):
    __slots__ = ()
    __match_args__ = ("value",)
    is_left = True


class Right(Either):
    __slots__ = ()
    __match_args__ = ("value",)
    is_right = True


def _hashable(v):
    try:
        hash(v)
        return v
    except TypeError:
        return repr(v)


@dataclass(frozen=True, slots=True)
class Pull:
    param_id: int


@dataclass(frozen=True, slots=True)
class Push:
    param_id: int
    delta: Any


@dataclass(frozen=True, slots=True)
class PullAnswer:
    param_id: int
    param: Any


@dataclass(frozen=True, slots=True)
class WorkerToPS:
    """Worker -> PS message; ``msg`` is ``Left(Pull)`` or ``Right(Push)``."""

    worker_partition_index: int
    msg: Either

    @property
    def param_id(self) -> int:
        return self.msg.value.param_id


@dataclass(frozen=True, slots=True)
class PSToWorker:
    """PS -> worker message carrying a pull answer for ``worker_partition_index``."""

    worker_partition_index: int
    msg: PullAnswer


def left_values(stream):
    """Worker outputs of an output stream (``Left`` side)."""
    return [e.value for e in stream if e.is_left]


def right_values(stream):
    """PS outputs of an output stream (``Right`` side)."""
    return [e.value for e in stream if e.is_right]

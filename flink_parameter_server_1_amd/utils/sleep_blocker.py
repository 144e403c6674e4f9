"""Manual back-pressure: delay a stream once before its first record.

``block(stream, ms)`` mirrors ``FlinkSleepBlocker.block`` (``M/utils/FlinkSleepBlocker.scala:23-36``):
a lazy sleeper runs before the first element of each (sub)stream, e.g. to
hold training data back until a model has been loaded into the PS.  Works on
any iterable; ``block_partitions`` applies it to every partition of a
``PartitionedInput``.
"""
from __future__ import annotations

import time
from typing import Iterable, Iterator

from ..core.engine import PartitionedInput


class _Blocked:
    def __init__(self, stream: Iterable, milliseconds: float):
        self.stream = stream
        self.ms = milliseconds

    def __iter__(self) -> Iterator:
        first = True
        for x in self.stream:
            if first:
                time.sleep(self.ms / 1000.0)
                first = False
            yield x


def block(stream: Iterable, milliseconds: float) -> Iterable:
    return _Blocked(stream, milliseconds)


def block_partitions(inp: PartitionedInput, milliseconds: float) -> PartitionedInput:
    return PartitionedInput([block(p, milliseconds) for p in inp.parts])

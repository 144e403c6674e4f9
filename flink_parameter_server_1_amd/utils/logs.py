"""Logging configuration (C57).

The reference ships two log4j files: the main jar logs ``hu.sztaki.ilab`` at
DEBUG -- every incoming record, pull answer and PS message
(``M/FlinkParameterServer.scala:237,247,284``, ``src/main/resources/log4j.properties:5``)
-- and the tests at ERROR (``src/test/resources/log4j.properties``).

Here the package logger is ``flink_parameter_server_1_amd``; ``configure``
installs one console handler.  Per-message tracing of the per-record engine
uses the child logger ``flink_parameter_server_1_amd.messages`` and is only
formatted when that logger is enabled for DEBUG (``message_tracing()``), so
the default costs one attribute test per message, not a string format.

Environment: ``FPS_LOG_LEVEL`` (default WARNING), ``FPS_LOG_MESSAGES=1``
(enable per-message DEBUG lines, the reference main-jar behaviour).
"""
from __future__ import annotations

import logging
import os
import sys
from typing import Optional

ROOT = "flink_parameter_server_1_amd"
MESSAGES = ROOT + ".messages"
_FORMAT = "%(asctime)s %(levelname)s %(name)s [rank %(rank)s] %(message)s"


class _RankFilter(logging.Filter):
    def filter(self, record):
        if not hasattr(record, "rank"):
            record.rank = os.environ.get("RANK", "0")
        return True


def configure(level: Optional[str] = None, messages: Optional[bool] = None, stream=None) -> logging.Logger:
    """Configure the package loggers (idempotent)."""
    level = level or os.environ.get("FPS_LOG_LEVEL", "WARNING")
    if messages is None:
        messages = os.environ.get("FPS_LOG_MESSAGES", "0") == "1"
    root = logging.getLogger(ROOT)
    root.setLevel(getattr(logging, str(level).upper(), logging.WARNING))
    if not any(getattr(h, "_fps", False) for h in root.handlers):
        h = logging.StreamHandler(stream or sys.stderr)
        h.setFormatter(logging.Formatter(_FORMAT))
        h.addFilter(_RankFilter())
        h._fps = True
        root.addHandler(h)
        root.propagate = False
    logging.getLogger(MESSAGES).setLevel(logging.DEBUG if messages else logging.WARNING)
    return root


def get(name: str) -> logging.Logger:
    return logging.getLogger(f"{ROOT}.{name}")


_msg_log = logging.getLogger(MESSAGES)


def message_tracing() -> bool:
    """True when per-message DEBUG lines are on (checked once per message)."""
    return _msg_log.isEnabledFor(logging.DEBUG)


def trace_message(kind: str, subtask: int, payload) -> None:
    _msg_log.debug("%s @%d: %r", kind, subtask, payload)

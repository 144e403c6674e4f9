"""LEMP candidate pruning for exact top-K inner-product retrieval.

Strategies (``M/matrix/factorization/pruning/LEMPPruningStrategy.scala:6-75``):
``LENGTH``, ``COORD``, ``INCR(n)``, ``LC(t)``, ``LI(n, t)`` with the same
``from_string`` syntax (``length``, ``coord``, ``incr:N``, ``lc:T``, ``li:N:T``).

Predicates (``M/matrix/factorization/pruning/LEMPPruningFunctions.scala:20-89``).
SURVEY B6: the reference compares the *squared* item length with the
*unsquared* bound ``theta/|u|``; ``length_pruning`` here squares the bound
(the LEMP paper's test) unless ``reference_quirks=True``.  B7: the reference's
INCR focus set ranges over ``0 until len-1`` (skips the last coordinate);
``focus_set`` includes every coordinate unless ``reference_quirks=True``.
"""
from __future__ import annotations

import math
import re
from dataclasses import dataclass
from typing import Sequence

import numpy as np


class LEMPPruningStrategy:
    @staticmethod
    def from_string(s: str) -> "LEMPPruningStrategy":
        m = None
        if re.fullmatch(r"length", s):
            return LENGTH()
        if re.fullmatch(r"coord", s):
            return COORD()
        m = re.fullmatch(r"incr:(\d*)", s)
        if m:
            return INCR(int(m.group(1)))
        m = re.fullmatch(r"lc:([0-9.]*)", s)
        if m:
            return LC(float(m.group(1)))
        m = re.fullmatch(r"li:(\d*):([0-9.]*)", s)
        if m:
            return LI(int(m.group(1)), float(m.group(2)))
        raise ValueError(f"Invalid LEMP Pruning strategy string {s}")

    fromString = from_string

    @property
    def num_focus(self) -> int:
        return 0


@dataclass(frozen=True)
class LENGTH(LEMPPruningStrategy):
    pass


@dataclass(frozen=True)
class COORD(LEMPPruningStrategy):
    pass


@dataclass(frozen=True)
class INCR(LEMPPruningStrategy):
    num_focus_coordinates: int

    @property
    def num_focus(self):
        return self.num_focus_coordinates


@dataclass(frozen=True)
class LC(LEMPPruningStrategy):
    algorithm_switch_threshold: float


@dataclass(frozen=True)
class LI(LEMPPruningStrategy):
    num_focus_coordinates: int
    algorithm_switch_threshold: float

    @property
    def num_focus(self):
        return self.num_focus_coordinates


def length_pruning(min_length: float, reference_quirks: bool = False):
    """Keep items with ``|p| >= theta/|u|`` (pass ``theta/|u|``)."""
    if reference_quirks:
        return lambda item: item[1][0] * item[1][0] >= min_length
    bound = min_length * min_length if min_length > 0 else -math.inf
    return lambda item: item[1][0] * item[1][0] >= bound


def coord_pruning(f: int, user, theta_b_q: float):
    """COORD bound on the normalised focus coordinate ``f``."""
    ulen, uvec = user
    q_bar_f = uvec[f] / ulen if ulen > 0 else 0.0
    a = q_bar_f * theta_b_q
    b = math.sqrt(max(0.0, (1 - theta_b_q * theta_b_q) * (1 - q_bar_f * q_bar_f)))
    lf_p, uf_p = a - b, a + b
    with np.errstate(divide="ignore", invalid="ignore"):
        ratio = theta_b_q / q_bar_f if q_bar_f != 0 else math.inf
    l_f = lf_p if (q_bar_f >= 0 or lf_p > ratio) else -1.0
    u_f = uf_p if (q_bar_f <= 0 or uf_p < ratio) else 1.0

    def pred(item):
        plen, pvec = item[1]
        p_bar_f = pvec[f] / plen if plen > 0 else 0.0
        return l_f <= p_bar_f <= u_f

    return pred


def incr_pruning(F: Sequence[int], user, theta: float):
    """INCR bound using the ``F`` focus coordinates (Cauchy-Schwarz on the rest)."""
    ulen, uvec = user
    F = np.asarray(F, dtype=np.int64)
    qF = uvec[F]
    q_mF_sqr = ulen * ulen - float(np.dot(qF, qF))

    def pred(item):
        plen, pvec = item[1]
        pF = pvec[F]
        q_F_p_F = float(np.dot(qF, pF))
        p_F_sqr = float(np.dot(pF, pF))
        ub = theta - q_F_p_F
        return ub < 0.0 or q_mF_sqr * (plen * plen - p_F_sqr) >= ub * ub

    return pred


def focus_coordinate(uvec) -> int:
    """Coordinate with the largest magnitude (COORD focus)."""
    return int(np.argmax(np.asarray(uvec) ** 2))


def focus_set(uvec, n: int, reference_quirks: bool = False) -> np.ndarray:
    d = len(uvec) - 1 if reference_quirks else len(uvec)
    sq = np.asarray(uvec[:d]) ** 2
    return np.argsort(-sq, kind="stable")[:n]


# Scala-spelled aliases
lengthPruning, coordPruning, incrPruning = length_pruning, coord_pruning, incr_pruning

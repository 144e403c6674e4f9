"""Offline evaluation tools: the reference's notebooks as library functions (C55).

``Notebooks/Data_Manipulation.ipynb`` splits a Last.fm-style session log into
a 31-day training and a 14-day test window; ``Notebooks/Tester.ipynb`` loads
the dumped ``UserVector.map`` / ``ItemVector.map`` factor files (``id;value``
one coordinate per line, the C54 output format), recommends the top 5 items
per user and reports recall / precision.  Same steps here, usable from Python
or the CLI (``python -m flink_parameter_server_1_amd split-log|eval-factors``).
"""
from __future__ import annotations

from collections import defaultdict
from typing import Dict, Optional, Sequence, Tuple

import numpy as np

from .io import read_factors_text, read_ratings
from .metrics import recall_precision_at_k, top_k_from_factors

DAY = 86400


def split_by_time(ts: np.ndarray, train_days: float = 31, test_days: float = 14,
                  start: Optional[int] = None) -> Tuple[np.ndarray, np.ndarray]:
    """Boolean masks (train, test): ``[start, start+train)`` and ``[start+train, start+train+test)``."""
    ts = np.asarray(ts)
    t0 = int(ts.min()) if start is None else int(start)
    t1 = t0 + int(train_days * DAY)
    t2 = t1 + int(test_days * DAY)
    return (ts >= t0) & (ts < t1), (ts >= t1) & (ts < t2)


def split_log_file(path: str, train_out: str, test_out: str, train_days: float = 31, test_days: float = 14):
    """Split a ``ts user item [rating]`` log into two files; returns (n_train, n_test)."""
    ts, u, i, r = read_ratings(path)
    tr, te = split_by_time(ts, train_days, test_days)
    for mask, out in ((tr, train_out), (te, test_out)):
        with open(out, "w") as f:
            for a, b, c, d in zip(ts[mask].tolist(), u[mask].tolist(), i[mask].tolist(), r[mask].tolist()):
                f.write(f"{a} {b} {c} {d:g}\n")
    return int(tr.sum()), int(te.sum())


def relevant_items(users: Sequence[int], items: Sequence[int]) -> Dict[int, set]:
    rel: Dict[int, set] = defaultdict(set)
    for a, b in zip(users, items):
        rel[int(a)].add(int(b))
    return dict(rel)


def evaluate_factor_files(user_file: str, item_file: str, test_log: str, k: int = 5,
                          train_log: Optional[str] = None) -> Dict[str, float]:
    """Tester.ipynb: top-``k`` recommendation from dumped factors, recall/precision@k on the
    test window (items already seen in ``train_log`` excluded when given)."""
    users = read_factors_text(user_file)
    items = read_factors_text(item_file)
    _, tu, ti, _ = read_ratings(test_log)
    relevant = {u: s for u, s in relevant_items(tu, ti).items() if u in users}
    exclude = None
    if train_log is not None:
        _, ru, ri, _ = read_ratings(train_log)
        exclude = relevant_items(ru, ri)
    rec = top_k_from_factors({u: users[u] for u in relevant}, items, k, exclude)
    recall, precision = recall_precision_at_k(rec, relevant, k)
    return {"recall": recall, "precision": precision, "users": float(len(relevant)), "k": float(k)}

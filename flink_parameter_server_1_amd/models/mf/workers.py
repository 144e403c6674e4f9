"""Per-record MF worker logics (compat engine; exact reference semantics).

* ``PSOnlineMatrixFactorizationWorker`` — ``M/matrix/factorization/workers/PSOnlineMatrixFactorizationWorker.scala:22-90``
* ``PSOfflineMatrixFactorizationWorker`` — ``.../PSOfflineMatrixFactorizationWorker.scala:27-150``.
  The reference spawns a thread on EOF that issues the epochs' pulls while
  the operator thread handles answers (a race) and its per-epoch
  ``Random.shuffle`` result is discarded (B2).  Here EOF issues every epoch's
  pulls through the (buffering) pull limiter, which releases them as answers
  arrive -- the same pull order and flow control, no foreign thread -- and
  each epoch is really shuffled.
* ``PSTopKGeneratorWorker`` — LEMP top-K over the worker-resident item shard
  (``.../PSTopKGeneratorWorker.scala:13-120``).
* ``PSOnlineMatrixFactorizationAndTopKGeneratorWorker`` — top-K + owner-side
  SGD with negatives (``.../PSOnlineMatrixFactorizationAndTopKGeneratorWorker.scala:28-195``).
* ``CollectTopKFromEachWorker`` — merge of the partial top-Ks
  (``M/matrix/factorization/utils/CollectTopKFromEachWorker.scala:23-74``).
"""
from __future__ import annotations

import random
from collections import defaultdict, deque
from typing import Dict, List, Optional

import numpy as np
from sortedcontainers import SortedList

from ...api.futures import BaseMFWorkerLogic
from ...api.logic import WorkerLogic
from ...core.messages import Left
from .core import (RangedRandomFactorInitializerDescriptor, Rating, SGDUpdater, TopKQueue, attach_length,
                   dot_product, vector_sum)
from .pruning import (COORD, INCR, LC, LENGTH, LI, coord_pruning, focus_coordinate, focus_set, incr_pruning,
                      length_pruning)


class _SeenMemory:
    """Per-user bounded memory of seen items (set + FIFO)."""

    def __init__(self, user_memory: int):
        self.user_memory = user_memory
        self.sets: Dict[int, set] = defaultdict(set)
        self.queues: Dict[int, deque] = defaultdict(deque)

    def add_evict_first(self, user, item):
        """Online/offline MF order: evict when full, then add (``:61-68``)."""
        s, q = self.sets[user], self.queues[user]
        if len(q) >= self.user_memory and q:
            s.discard(q.popleft())
        s.add(item)
        q.append(item)
        return s

    def add_evict_after(self, user, item):
        """Top-K worker order: add if new, then evict past memory (``:128-138``)."""
        s, q = self.sets[user], self.queues[user]
        if item not in s:
            s.add(item)
            q.append(item)
            if len(q) > self.user_memory:
                s.discard(q.popleft())
        return s


class PSOnlineMatrixFactorizationWorker(WorkerLogic):
    def __init__(self, num_factors: int, range_min: float, range_max: float, learning_rate: float,
                 user_memory: int = 128, negative_sample_rate: int = 0, seed: Optional[int] = None,
                 lam: float = 0.0, factor_init=None):
        self.factor_init = (factor_init.open() if factor_init is not None else
                            RangedRandomFactorInitializerDescriptor(num_factors, range_min, range_max, seed).open())
        self.factor_update = SGDUpdater(learning_rate, lam)
        self.negative_sample_rate = negative_sample_rate
        self.user_vectors: Dict[int, np.ndarray] = {}
        self.rating_buffer: Dict[int, deque] = {}
        self.item_ids: List[int] = []
        self.seen = _SeenMemory(user_memory)
        self.rng = random.Random(seed)

    def on_recv(self, data: Rating, ps):
        seen = self.seen.add_evict_first(data.user, data.item)
        ids = self.item_ids
        for _ in range(min(len(ids) - len(seen), self.negative_sample_rate)):
            neg = ids[self.rng.randrange(len(ids))]
            while neg in seen:
                neg = ids[self.rng.randrange(len(ids))]
            self.rating_buffer[neg].append(Rating(data.user, neg, 0.0, data.timestamp))
            ps.pull(neg)
        q = self.rating_buffer.get(data.item)
        if q is None:
            q = self.rating_buffer[data.item] = deque()
            ids.append(data.item)
        q.append(data)
        ps.pull(data.item)

    def on_pull_recv(self, item_id, item_vec, ps):
        rating = self.rating_buffer[item_id].popleft()
        user = self.user_vectors.get(rating.user)
        if user is None:
            user = self.factor_init.next_factor(rating.user)
        du, di = self.factor_update.delta(rating.rating, user, item_vec)
        new_user = vector_sum(user, du)
        self.user_vectors[rating.user] = new_user
        ps.output((rating.user, new_user))
        ps.push(item_id, di)


class PSOfflineMatrixFactorizationWorker(WorkerLogic):
    """Input: ``Left(EOF)`` / ``Right(Rating)`` (the ``flatMapWithEOF`` stream)."""

    def __init__(self, num_factors: int, range_min: float, range_max: float, learning_rate: float,
                 negative_sample_rate: int = 0, user_memory: int = 128, iterations: int = 1,
                 seed: Optional[int] = None, lam: float = 0.0, shuffle: bool = True):
        self.factor_init = RangedRandomFactorInitializerDescriptor(num_factors, range_min, range_max, seed).open()
        self.factor_update = SGDUpdater(learning_rate, lam)
        self.negative_sample_rate = negative_sample_rate
        self.iterations = iterations
        self.shuffle = shuffle
        self.rbs: List[List[Rating]] = []
        self.user_vectors: Dict[int, np.ndarray] = {}
        self.rating_buffer: Dict[int, deque] = defaultdict(deque)
        self.seen = _SeenMemory(user_memory)
        self.all_items_set = set()
        self.all_items: List[int] = []
        self.started = False
        self.rng = random.Random(seed)

    def on_recv(self, value, ps):
        if value.is_right:
            rating = value.value
            if self.started:
                raise RuntimeError("Should not have started training while waiting for further elements.")
            if rating.item not in self.all_items_set:
                self.all_items_set.add(rating.item)
                self.all_items.append(rating.item)
            seen = self.seen.add_evict_first(rating.user, rating.item)
            rs = []
            for _ in range(min(len(self.all_items_set) - len(seen), self.negative_sample_rate)):
                neg = self.all_items[self.rng.randrange(len(self.all_items))]
                while neg in seen:
                    neg = self.all_items[self.rng.randrange(len(self.all_items))]
                rs.append(Rating.from_tuple((rating.user, neg, 0.0)))
            rs.append(rating)
            self.rbs.append(rs)
        else:  # EOF: run every epoch's pulls (released by the pull limiter)
            self.started = True
            for _ in range(self.iterations):
                order = list(self.rbs)
                if self.shuffle:
                    self.rng.shuffle(order)
                for rs in order:
                    for r in rs:
                        self.rating_buffer[r.item].append((r.user, r.rating))
                        ps.pull(r.item)

    def on_pull_recv(self, item, item_vec, ps):
        user, rating = self.rating_buffer[item].popleft()
        uvec = self.user_vectors.get(user)
        if uvec is None:
            uvec = self.factor_init.next_factor(user)
        du, di = self.factor_update.delta(rating, uvec, item_vec)
        new_user = vector_sum(uvec, du)
        self.user_vectors[user] = new_user
        ps.output((user, new_user))
        ps.push(item, di)


# ---------------------------------------------------------------------- LEMP
def lemp_top_k(user, items_desc: SortedList, model: Dict[int, tuple], worker_k: int, bucket_size: int,
               pruning, reference_quirks: bool = False) -> TopKQueue:
    """Length-bucketed exact top-K with LEMP candidate pruning (``PSTopKGeneratorWorker.scala:46-110``).

    ``items_desc`` holds ``(-length, item)`` so it iterates by descending length.
    """
    ulen, uvec = user
    top = TopKQueue()
    if ulen == 0 or len(items_desc) == 0:
        return top
    f = focus_coordinate(uvec)
    fs = focus_set(uvec, pruning.num_focus, reference_quirks)
    entries = list(items_desc)
    for start in range(0, len(entries), bucket_size):
        bucket = entries[start:start + bucket_size]
        head_len = -bucket[0][0]
        if not (len(top) < worker_k or head_len * ulen > top.head[0]):
            break
        theta = 0.0 if len(top) < worker_k else top.head[0]
        denom = head_len * ulen
        theta_b_q = theta / denom if denom > 0 else 0.0
        last_len = -bucket[-1][0]
        if isinstance(pruning, LENGTH):
            pred = length_pruning(theta / ulen, reference_quirks)
        elif isinstance(pruning, COORD):
            pred = coord_pruning(f, user, theta_b_q)
        elif isinstance(pruning, INCR):
            pred = incr_pruning(fs, user, theta)
        elif isinstance(pruning, LC):
            pred = length_pruning(theta / ulen, reference_quirks) if head_len > last_len * \
                pruning.algorithm_switch_threshold else coord_pruning(f, user, theta_b_q)
        elif isinstance(pruning, LI):
            pred = length_pruning(theta / ulen, reference_quirks) if head_len > last_len * \
                pruning.algorithm_switch_threshold else incr_pruning(fs, user, theta)
        else:
            pred = None
        for neg_len, item in bucket:
            lv = model[item]
            if pred is not None and not pred((item, lv)):
                continue
            top.offer(dot_product(uvec, lv[1]), item, worker_k)
    return top


class PSTopKGeneratorWorker(BaseMFWorkerLogic):
    """Items are worker-resident ``(len, vec)``; users are pulled from the PS."""

    def __init__(self, worker_k: int, bucket_size: int, worker_parallelism: int, pruning,
                 reference_quirks: bool = False):
        super().__init__()
        self.worker_k, self.bucket_size = worker_k, bucket_size
        self.worker_parallelism = worker_parallelism
        self.pruning = pruning
        self.quirks = reference_quirks
        self.items_desc = SortedList()
        self.rating_buffer: Dict[int, deque] = defaultdict(deque)
        self.worker_id = -1

    def on_recv(self, data, ps):
        if self.worker_id == -1:
            self.worker_id = data.target_worker
        self.rating_buffer[data.user].append(data)
        ps.pull(data.user)

    def on_pull_recv(self, user_id, user_and_len, ps):
        rate = self.rating_buffer[user_id].popleft()
        if user_and_len[0] == -1:  # invalid user
            ps.output((rate, TopKQueue()))
            return
        top = lemp_top_k(user_and_len, self.items_desc, self.model, self.worker_k, self.bucket_size,
                         self.pruning, self.quirks)
        ps.output((rate, top))

    def update_model(self, item_id, param):
        old = self.model.get(item_id)
        if old is not None:
            self.items_desc.discard((-old[0], item_id))
        param = (float(param[0]), np.asarray(param[1], dtype=np.float64))
        self.model[item_id] = param
        self.items_desc.add((-param[0], item_id))


class PSOnlineMatrixFactorizationAndTopKGeneratorWorker(WorkerLogic):
    def __init__(self, negative_sample_rate: int, user_memory: int, worker_k: int, bucket_size: int, pruning,
                 worker_parallelism: int, factor_init_desc, factor_update, seed: Optional[int] = None,
                 reference_quirks: bool = False):
        self.negative_sample_rate = negative_sample_rate
        self.worker_k, self.bucket_size = worker_k, bucket_size
        self.pruning = pruning
        self.worker_parallelism = worker_parallelism
        self.factor_init_desc = factor_init_desc
        self.factor_update = factor_update
        self.model: Dict[int, tuple] = {}
        self.items_desc = SortedList()
        self.item_ids: List[int] = []
        self.rating_buffer: Dict[int, deque] = defaultdict(deque)
        self.seen = _SeenMemory(user_memory)
        self.worker_id = -1
        self.rng = random.Random(seed)
        self.quirks = reference_quirks
        self._init = None

    def on_recv(self, data, ps):
        if self.worker_id == -1:
            self.worker_id = data.target_worker
        self.rating_buffer[data.user].append(data)
        ps.pull(data.user)

    def on_pull_recv(self, user_id, user_and_len, ps):
        rate = self.rating_buffer[user_id].popleft()
        ulen, uvec = user_and_len
        top = lemp_top_k(user_and_len, self.items_desc, self.model, self.worker_k, self.bucket_size,
                         self.pruning, self.quirks)
        ps.output((rate, top))
        if hash(rate.item) % self.worker_parallelism == self.worker_id:
            seen = self.seen.add_evict_after(rate.user, rate.item)
            u_delta = np.zeros(len(uvec))
            for _ in range(min(len(self.model) - len(seen), self.negative_sample_rate)):
                neg = self.item_ids[self.rng.randrange(len(self.item_ids))]
                counter = 32
                while counter > 0 and neg in seen:
                    neg = self.item_ids[self.rng.randrange(len(self.item_ids))]
                    counter -= 1
                if counter > 0:
                    neg_vec = self.model[neg][1]
                    uu, idelta = self.factor_update.delta(0.0, uvec, neg_vec)
                    u_delta = vector_sum(u_delta, uu)
                    self._update_no_init(neg, attach_length(vector_sum(neg_vec, idelta)))
            item_vec = self.model[rate.item][1] if rate.item in self.model else self._initialize(rate.item)[1]
            ud, idelta = self.factor_update.delta(rate.rating, uvec, item_vec)
            self._update_no_init(rate.item, attach_length(vector_sum(item_vec, idelta)))
            ps.push(user_id, (float("nan"), vector_sum(u_delta, ud)))

    def _update_no_init(self, item_id, param):
        old = self.model[item_id]
        self.items_desc.discard((-old[0], item_id))
        self.model[item_id] = param
        self.items_desc.add((-param[0], item_id))

    def update_model(self, item_id, param):
        if item_id in self.model:
            self.items_desc.discard((-self.model[item_id][0], item_id))
        else:
            self.item_ids.append(item_id)
        self.model[item_id] = param
        self.items_desc.add((-param[0], item_id))

    def _initialize(self, item_id):
        if self._init is None:
            self._init = self.factor_init_desc.open()
        lv = attach_length(self._init.next_factor(item_id))
        self.update_model(item_id, lv)
        return lv


class CollectTopKFromEachWorker:
    """Merge ``worker_parallelism`` partial top-Ks per rating id; drop items the user
    has seen (bounded memory), sort descending, keep ``K``.  Emits
    ``(user, item, timestamp, [(score, item), ...])``."""

    def __init__(self, K: int, memory: int, worker_parallelism: int):
        self.K, self.memory, self.wp = K, memory, worker_parallelism
        self.outputs: Dict[float, list] = {}
        self.seen_set: Dict[int, set] = defaultdict(set)
        self.seen_list: Dict[int, deque] = defaultdict(deque)

    def flat_map(self, value, out):
        if not value.is_left:
            return
        rate, top = value.value
        parts = self.outputs.setdefault(rate.rating_id, [None] * self.wp)
        parts[rate.target_worker] = top
        if all(p is not None for p in parts):
            seen = self.seen_set[rate.user]
            merged = [x for p in parts for x in p]
            lst = sorted((x for x in merged if x[1] not in seen), key=lambda x: -x[0])[: self.K]
            out((rate.user, rate.item, rate.timestamp, lst))
            del self.outputs[rate.rating_id]
            seen.add(rate.item)
            self.seen_list[rate.user].append(rate.item)
            if self.memory > -1 and len(self.seen_list[rate.user]) > self.memory:
                seen.discard(self.seen_list[rate.user].popleft())

    def run(self, stream) -> list:
        res = []
        for e in stream:
            self.flat_map(e, res.append)
        return res

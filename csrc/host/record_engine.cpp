// Native per-record engine for the online MF job (BASELINE config #1 on CPU).
//
// The reference runs psOnlineMF as Flink subtasks exchanging one message per
// pull, pull answer and push (M/FlinkParameterServer.scala:195-336, worker
// M/matrix/factorization/workers/PSOnlineMatrixFactorizationWorker.scala:22-90,
// PS = SimplePSLogic with vector add M/server/SimplePSLogic.scala:7-26, pull
// limiter M/WorkerLogic.scala:176-225).  This engine runs the same protocol with
// the same per-record semantics in one C++ thread:
//
// * W worker and P PS subtasks; input partitioned by |user| % W, params by
//   |id| % P (core/partitioners.py);
// * FIFO mailboxes per subtask (pull answers of one (worker, PS) pair arrive
//   in request order, which the per-item rating FIFO of the worker relies on);
// * the scheduling turn of core/engine.py LocalRuntime: per worker up to 64
//   pull answers then up to 64 input records, then per PS up to 64 messages;
// * worker: optional negatives (rejection-sampled among the worker's known items,
//   excluding the user's last user_memory items), rating FIFO per item, pull
//   limiter (at most pull_limit outstanding, excess queued FIFO); on an answer:
//   lazy user init, e = r - u.i, u += lr (e i - lam u), push lr (e u - lam i);
// * PS: lazy init on first pull, add on push (a push to an unknown id stores
//   the delta), NaN check (FactorIsNotANumberException, Vector.scala:72-84);
// * init U[lo, hi) by a hash of (seed, id, coordinate) -- deterministic per id
//   like PseudoRandomFactorInitializer, same function as the GPU tables.
//
// Outputs: the reference emits (user, vec) per answer and (item, vec) per push;
// their last-writer-wins fold is the final model, which is what this returns
// (plus counts of every message kind).  Doubles throughout (the reference's
// Array[Double] factors).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <deque>
#include <vector>

#define FPS_HOST_API extern "C" __attribute__((visibility("default")))

namespace {

inline uint32_t fmix32(uint32_t x) {
  x ^= x >> 16; x *= 0x85ebca6bu;
  x ^= x >> 13; x *= 0xc2b2ae35u;
  x ^= x >> 16;
  return x;
}

inline float hash_uniform(uint32_t seed, int64_t id, uint32_t j) {  // = csrc/kernels/common.h
  uint32_t h = fmix32(seed ^ 0x9e3779b9u);
  h = fmix32(h ^ (uint32_t)(id & 0xffffffff));
  h = fmix32(h ^ (uint32_t)((uint64_t)id >> 32) ^ 0x27d4eb2fu);
  h = fmix32(h + j * 0x9e3779b9u);
  return (float)(h >> 8) * (1.0f / 16777216.0f);
}

// |a| % m, the reference's Math.abs(id.hashCode) % P without its negative result
// for the most negative id: |a| taken as unsigned
inline int64_t abs_mod(int64_t a, int64_t m) {
  const uint64_t x = a < 0 ? (uint64_t)0 - (uint64_t)a : (uint64_t)a;
  return (int64_t)(x % (uint64_t)m);
}

// open-addressing int64 -> dense index
struct IndexMap {
  static constexpr int64_t kEmpty = INT64_MIN;
  std::vector<int64_t> keys;
  std::vector<int32_t> idx;
  int64_t size = 0;
  IndexMap() : keys(64, kEmpty), idx(64, -1) {}
  static uint32_t h(int64_t k) { return fmix32((uint32_t)k ^ fmix32((uint32_t)((uint64_t)k >> 32))); }
  int32_t find(int64_t k) const {
    const int64_t m = (int64_t)keys.size() - 1;
    for (int64_t i = h(k) & m;; i = (i + 1) & m) {
      if (keys[i] == k) return idx[i];
      if (keys[i] == kEmpty) return -1;
    }
  }
  void insert(int64_t k, int32_t v) {  // k must be absent
    if ((size + 1) * 2 > (int64_t)keys.size()) grow();
    const int64_t m = (int64_t)keys.size() - 1;
    int64_t i = h(k) & m;
    while (keys[i] != kEmpty) i = (i + 1) & m;
    keys[i] = k;
    idx[i] = v;
    ++size;
  }
  void grow() {
    std::vector<int64_t> ok;
    std::vector<int32_t> oi;
    ok.swap(keys);
    oi.swap(idx);
    keys.assign(ok.size() * 2, kEmpty);
    idx.assign(ok.size() * 2, -1);
    size = 0;
    for (size_t i = 0; i < ok.size(); ++i)
      if (ok[i] != kEmpty) insert(ok[i], oi[i]);
  }
};

// dense rows of D doubles addressed through an IndexMap
struct RowStore {
  int D;
  IndexMap map;
  std::vector<int64_t> ids;
  std::vector<double> vals;
  explicit RowStore(int d) : D(d) {}
  double* row(int32_t i) { return &vals[(size_t)i * D]; }
  int32_t add(int64_t id) {
    const int32_t i = (int32_t)ids.size();
    ids.push_back(id);
    vals.resize(vals.size() + D);
    map.insert(id, i);
    return i;
  }
  void init_row(int32_t i, double lo, double hi, uint32_t seed) {
    double* v = row(i);
    for (int j = 0; j < D; ++j) v[j] = lo + (hi - lo) * (double)hash_uniform(seed, ids[i], (uint32_t)j);
  }
};

// FIFO ring of messages (id, worker, kind, D doubles of payload) grown by doubling:
// one contiguous payload slot per message instead of per-double deque operations
struct MsgRing {
  int D;
  std::vector<int64_t> id;
  std::vector<int32_t> worker, kind;
  std::vector<double> val;
  size_t head = 0, count = 0;
  explicit MsgRing(int d) : D(d) { grow(256); }
  bool empty() const { return count == 0; }
  size_t cap() const { return id.size(); }
  void grow(size_t c) {
    std::vector<int64_t> i2(c);
    std::vector<int32_t> w2(c), k2(c);
    std::vector<double> v2(c * (size_t)D);
    for (size_t q = 0; q < count; ++q) {
      const size_t s = (head + q) % cap();
      i2[q] = id[s];
      w2[q] = worker[s];
      k2[q] = kind[s];
      std::memcpy(&v2[q * D], &val[s * D], sizeof(double) * D);
    }
    id.swap(i2);
    worker.swap(w2);
    kind.swap(k2);
    val.swap(v2);
    head = 0;
  }
  void push(int64_t i, int32_t w, int32_t k, const double* v) {
    if (count == cap()) grow(cap() * 2);
    const size_t s = (head + count) % cap();
    id[s] = i;
    worker[s] = w;
    kind[s] = k;
    if (v != nullptr) std::memcpy(&val[s * D], v, sizeof(double) * D);
    ++count;
  }
  size_t front() const { return head; }  // slot of the oldest message
  const double* payload(size_t slot) const { return &val[slot * D]; }
  void pop() {
    head = (head + 1) % cap();
    --count;
  }
};

struct Worker {
  int D;
  RowStore users;
  // per-item FIFO of buffered ratings: index by item slot, nodes in a pool
  IndexMap item_slot;
  std::vector<int64_t> item_ids;       // worker's known items (negative sampling domain)
  std::vector<int32_t> head, tail;     // per item slot, -1 = empty
  std::vector<int32_t> nxt;            // node pool
  std::vector<int64_t> nuser;
  std::vector<double> nrating;
  std::vector<int32_t> free_nodes;
  // pull limiter
  int64_t outstanding = 0;
  std::deque<int64_t> pending_pulls;
  // input
  std::vector<int64_t> input;  // rating indices of this partition, in order
  size_t cursor = 0;
  // pull answers: (item, value[D])
  MsgRing answers;
  // per-user memory of seen items (negative sampling)
  IndexMap user_slot;
  std::vector<std::deque<int64_t>> seen_fifo;  // may hold repeats (FIFO of every rated item)
  std::vector<std::vector<int64_t>> seen_set;   // distinct items (a repeat evicted from the FIFO
                                                // leaves the set, as in the reference)
  uint64_t rng;
  explicit Worker(int d, uint64_t seed) : D(d), users(d), answers(d), rng(seed * 0x9e3779b97f4a7c15ull + 1) {}

  uint64_t next_rand() {  // splitmix64
    uint64_t z = (rng += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
  }
  int32_t slot_of_item(int64_t item) {
    int32_t s = item_slot.find(item);
    if (s < 0) {
      s = (int32_t)item_ids.size();
      item_slot.insert(item, s);
      item_ids.push_back(item);
      head.push_back(-1);
      tail.push_back(-1);
    }
    return s;
  }
  void enqueue(int32_t slot, int64_t user, double rating) {
    int32_t n;
    if (!free_nodes.empty()) {
      n = free_nodes.back();
      free_nodes.pop_back();
    } else {
      n = (int32_t)nxt.size();
      nxt.push_back(-1);
      nuser.push_back(0);
      nrating.push_back(0.0);
    }
    nxt[n] = -1;
    nuser[n] = user;
    nrating[n] = rating;
    if (tail[slot] < 0) head[slot] = n;
    else nxt[tail[slot]] = n;
    tail[slot] = n;
  }
  bool dequeue(int32_t slot, int64_t& user, double& rating) {
    const int32_t n = head[slot];
    if (n < 0) return false;
    user = nuser[n];
    rating = nrating[n];
    head[slot] = nxt[n];
    if (head[slot] < 0) tail[slot] = -1;
    free_nodes.push_back(n);
    return true;
  }
};

}  // namespace

// Runs the online MF job over n ratings.  users_out / items_out receive the
// final (folded) model: ids and D doubles per row, up to the caps; counts[0..1]
// = rows written, stats[0..6] = pulls, pushes, answers, worker outputs, PS
// outputs, scheduling turns, negatives drawn.  Returns 0, or -1 on a NaN factor
// (FactorIsNotANumberException), -2 on a pull answer without a buffered rating,
// -3 on bad arguments (D in 1..256, W, P, pull_limit >= 1).
FPS_HOST_API int fps_mf_online_record(const int64_t* user, const int64_t* item, const double* rating, int64_t n,
                                      int W, int P, int D, double lr, double lam, double lo, double hi,
                                      uint32_t seed, int64_t pull_limit, int neg_rate, int user_memory,
                                      int64_t* users_out_ids, double* users_out_vals, int64_t users_cap,
                                      int64_t* items_out_ids, double* items_out_vals, int64_t items_cap,
                                      int64_t* counts, int64_t* stats) {
  constexpr int kBatch = 64;  // LocalRuntime.batch
  if (D <= 0 || D > 256 || W <= 0 || P <= 0 || pull_limit <= 0) return -3;
  const uint32_t user_seed = seed ^ 0x5bd1e995u;
  std::vector<Worker> workers;
  workers.reserve(W);
  for (int w = 0; w < W; ++w) workers.emplace_back(D, (uint64_t)seed * 1000003ull + (uint64_t)w);
  for (int64_t k = 0; k < n; ++k) workers[abs_mod(user[k], W)].input.push_back(k);
  std::vector<RowStore> ps;
  ps.reserve(P);
  for (int p = 0; p < P; ++p) ps.emplace_back(D);
  std::vector<MsgRing> ps_inbox;  // pulls (kind 0) and pushes with their delta (kind 1)
  ps_inbox.reserve(P);
  for (int p = 0; p < P; ++p) ps_inbox.emplace_back(D);
  int64_t n_pull = 0, n_push = 0, n_ans = 0, n_wout = 0, n_psout = 0, turns = 0, n_neg = 0;
  std::vector<double> du(D), di(D);

  auto send_pull = [&](int w, int64_t id) {
    const int p = (int)abs_mod(id, P);
    ps_inbox[p].push(id, w, 0, nullptr);
    ++n_pull;
  };
  auto limited_pull = [&](Worker& wk, int w, int64_t id) {  // M/WorkerLogic.scala:176-225
    if (wk.outstanding < pull_limit) {
      ++wk.outstanding;
      send_pull(w, id);
    } else {
      wk.pending_pulls.push_back(id);
    }
  };

  bool progressed = true;
  while (progressed) {
    progressed = false;
    ++turns;
    for (int w = 0; w < W; ++w) {
      Worker& wk = workers[w];
      // ---- pull answers (limiter first: release one queued pull per answer)
      for (int a = 0; a < kBatch && !wk.answers.empty(); ++a) {
        const size_t slot_a = wk.answers.front();
        const int64_t iid = wk.answers.id[slot_a];
        double iv[256];
        std::memcpy(iv, wk.answers.payload(slot_a), sizeof(double) * D);
        wk.answers.pop();
        int64_t u;
        double r;
        const int32_t slot = wk.item_slot.find(iid);
        if (slot < 0 || !wk.dequeue(slot, u, r)) return -2;
        int32_t ui = wk.users.map.find(u);
        if (ui < 0) {
          ui = wk.users.add(u);
          wk.users.init_row(ui, lo, hi, user_seed);
        }
        double* uv = wk.users.row(ui);
        double dot = 0.0;
        for (int j = 0; j < D; ++j) dot += uv[j] * iv[j];
        const double e = r - dot;
        if (lam != 0.0) {  // the reference's operation order (SGDUpdater)
          for (int j = 0; j < D; ++j) {
            du[j] = lr * (e * iv[j] - lam * uv[j]);
            di[j] = lr * (e * uv[j] - lam * iv[j]);
          }
        } else {
          const double g = lr * e;
          for (int j = 0; j < D; ++j) {
            du[j] = g * iv[j];
            di[j] = g * uv[j];
          }
        }
        for (int j = 0; j < D; ++j) {
          uv[j] += du[j];
          if (std::isnan(uv[j])) return -1;
        }
        ++n_wout;  // output((user, vec))
        const int p = (int)abs_mod(iid, P);
        ps_inbox[p].push(iid, w, 1, di.data());
        ++n_push;
        ++n_ans;
        // limiter after the logic (its push goes first): release one queued pull
        --wk.outstanding;
        if (!wk.pending_pulls.empty()) {
          const int64_t q = wk.pending_pulls.front();
          wk.pending_pulls.pop_front();
          ++wk.outstanding;
          send_pull(w, q);
        }
        progressed = true;
      }
      // ---- input records
      for (int a = 0; a < kBatch && wk.cursor < wk.input.size(); ++a) {
        const int64_t k = wk.input[wk.cursor++];
        const int64_t u = user[k], it = item[k];
        if (neg_rate > 0) {  // PSOnlineMatrixFactorizationWorker.scala:61-79
          int32_t us = wk.user_slot.find(u);
          if (us < 0) {
            us = (int32_t)wk.seen_fifo.size();
            wk.user_slot.insert(u, us);
            wk.seen_fifo.emplace_back();
            wk.seen_set.emplace_back();
          }
          std::deque<int64_t>& fifo = wk.seen_fifo[us];
          std::vector<int64_t>& set = wk.seen_set[us];
          auto in_set = [&set](int64_t x) {
            for (int64_t y : set)
              if (y == x) return true;
            return false;
          };
          if ((int64_t)fifo.size() >= user_memory && !fifo.empty()) {  // evict first, then add
            const int64_t x = fifo.front();
            fifo.pop_front();
            for (size_t q = 0; q < set.size(); ++q)
              if (set[q] == x) { set[q] = set.back(); set.pop_back(); break; }
          }
          if (!in_set(it)) set.push_back(it);
          fifo.push_back(it);
          const int64_t known = (int64_t)wk.item_ids.size();
          const int64_t draws = std::min<int64_t>(known - (int64_t)set.size(), neg_rate);
          for (int64_t d = 0; d < draws; ++d) {
            int64_t neg;
            do {
              neg = wk.item_ids[(size_t)(wk.next_rand() % (uint64_t)known)];
            } while (in_set(neg));
            wk.enqueue(wk.slot_of_item(neg), u, 0.0);
            limited_pull(wk, w, neg);
            ++n_neg;
          }
        }
        wk.enqueue(wk.slot_of_item(it), u, rating[k]);
        limited_pull(wk, w, it);
        progressed = true;
      }
    }
    for (int p = 0; p < P; ++p) {
      RowStore& st = ps[p];
      for (int a = 0; a < kBatch && !ps_inbox[p].empty(); ++a) {
        MsgRing& box = ps_inbox[p];
        const size_t slot_m = box.front();
        const int64_t mid = box.id[slot_m];
        const int32_t mworker = box.worker[slot_m], mkind = box.kind[slot_m];
        int32_t i = st.map.find(mid);
        if (mkind == 0) {  // pull: lazy init, answer to the asking worker
          if (i < 0) {
            i = st.add(mid);
            st.init_row(i, lo, hi, seed);
          }
          workers[mworker].answers.push(mid, 0, 0, st.row(i));
        } else {  // push: add (or store the delta for an unknown id), output (id, value)
          const double* d = box.payload(slot_m);
          double* v;
          if (i < 0) {
            i = st.add(mid);
            v = st.row(i);
            for (int j = 0; j < D; ++j) v[j] = d[j];
          } else {
            v = st.row(i);
            for (int j = 0; j < D; ++j) v[j] += d[j];
          }
          for (int j = 0; j < D; ++j)
            if (std::isnan(v[j])) return -1;
          ++n_psout;
        }
        box.pop();
        progressed = true;
      }
    }
  }
  // ---- folded model
  int64_t nu = 0, ni = 0;
  for (Worker& wk : workers)
    for (size_t r = 0; r < wk.users.ids.size() && nu < users_cap; ++r, ++nu) {
      users_out_ids[nu] = wk.users.ids[r];
      std::memcpy(users_out_vals + nu * D, wk.users.row((int32_t)r), sizeof(double) * D);
    }
  for (RowStore& st : ps)
    for (size_t r = 0; r < st.ids.size() && ni < items_cap; ++r, ++ni) {
      items_out_ids[ni] = st.ids[r];
      std::memcpy(items_out_vals + ni * D, st.row((int32_t)r), sizeof(double) * D);
    }
  counts[0] = nu;
  counts[1] = ni;
  stats[0] = n_pull;
  stats[1] = n_push;
  stats[2] = n_ans;
  stats[3] = n_wout;
  stats[4] = n_psout;
  stats[5] = turns;
  stats[6] = n_neg;
  return 0;
}

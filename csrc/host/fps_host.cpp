// Host-side native runtime pieces (C++17, no GPU): data loading, model IO,
// synthetic data generation, and a sparse-id parameter store.
//
//  * rating-log parser  -- "ts user item [rating]" lines (space / comma / tab),
//    the format the reference's experiment drivers read
//    (T/matrix/factorization/PSOnlineMatrixFactorizationImplicitTest.scala:31-97).
//  * id;value factor files -- one coordinate per line "<id>;<value>" in
//    coordinate order per id: the reference's model dump format, consumed by
//    its notebooks (Notebooks/Tester.ipynb).  Writer formats in parallel.
//  * binary shard snapshots -- header + ids int64[n] + values fp32[n, d].
//  * synthetic rating generator -- counter-based hash RNG, multithreaded,
//    deterministic per (seed, rank, index) regardless of thread count.
//  * HashStore -- open-addressing int64 -> fp32[dim] table with lazy
//    deterministic init (the "generic sparse id" PS store).
//
// C ABI, loaded with ctypes (flink_parameter_server_1_amd/utils/native_host.py).
#include <algorithm>
#include <atomic>
#include <cerrno>
#include <charconv>
#include <cmath>
#include <climits>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#define FPS_HOST_API extern "C" __attribute__((visibility("default")))

namespace {

inline uint32_t fmix32(uint32_t x) {
  x ^= x >> 16; x *= 0x85ebca6bu;
  x ^= x >> 13; x *= 0xc2b2ae35u;
  x ^= x >> 16;
  return x;
}

// identical to hash_uniform in csrc/kernels/common.h
inline float hash_uniform(uint32_t seed, int64_t id, uint32_t j) {
  uint32_t h = fmix32(seed ^ 0x9e3779b9u);
  h = fmix32(h ^ (uint32_t)(id & 0xffffffff));
  h = fmix32(h ^ (uint32_t)((uint64_t)id >> 32) ^ 0x27d4eb2fu);
  h = fmix32(h + j * 0x9e3779b9u);
  return (float)(h >> 8) * (1.0f / 16777216.0f);
}

int n_threads(int64_t work) {
  unsigned hc = std::thread::hardware_concurrency();
  const char* e = std::getenv("OMP_NUM_THREADS");
  if (e) hc = (unsigned)std::max(1, std::atoi(e));
  int64_t t = std::min<int64_t>(hc ? hc : 4, std::max<int64_t>(1, work / 65536));
  return (int)std::max<int64_t>(1, t);
}

bool read_file(const char* path, std::string& buf) {
  FILE* f = std::fopen(path, "rb");
  if (!f) return false;
  std::fseek(f, 0, SEEK_END);
  long sz = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  buf.resize(sz > 0 ? (size_t)sz : 0);
  size_t got = sz > 0 ? std::fread(&buf[0], 1, (size_t)sz, f) : 0;
  std::fclose(f);
  buf.resize(got);
  return true;
}

inline bool is_sep(char c) { return c == ' ' || c == ',' || c == '\t' || c == ';'; }

const char* parse_i64(const char* p, const char* end, int64_t& v, bool& ok) {
  while (p < end && is_sep(*p)) ++p;
  auto r = std::from_chars(p, end, v);
  ok = r.ec == std::errc();
  return r.ptr;
}

const char* parse_f64(const char* p, const char* end, double& v, bool& ok) {
  while (p < end && is_sep(*p)) ++p;
  if (p >= end || *p == '\r') { ok = false; return p; }  // field absent on this line
  char* q = nullptr;
  v = std::strtod(p, &q);  // stops at the line's '\n' (not a numeric char)
  ok = q != p && q <= end;
  return ok ? q : p;
}

}  // namespace

// ------------------------------------------------------------------ rating logs
// Lines: "<ts> <user> <item> [<rating>]".  Missing rating -> default_rating
// (implicit feedback).  Returns the number of parsed records (<= cap), or -1.
FPS_HOST_API int64_t fps_parse_ratings(const char* path, int64_t cap, int64_t* ts, int32_t* users, int32_t* items,
                                       float* ratings, float default_rating) {
  std::string buf;
  if (!read_file(path, buf)) return -1;
  const char* p = buf.data();
  const char* end = p + buf.size();
  int64_t n = 0;
  while (p < end && n < cap) {
    const char* eol = (const char*)std::memchr(p, '\n', (size_t)(end - p));
    if (!eol) eol = end;
    bool ok1, ok2, ok3, ok4;
    int64_t t, u, i;
    const char* q = parse_i64(p, eol, t, ok1);
    q = parse_i64(q, eol, u, ok2);
    q = parse_i64(q, eol, i, ok3);
    double r = default_rating;
    if (ok1 && ok2 && ok3) {
      double rr;
      parse_f64(q, eol, rr, ok4);
      if (ok4) r = rr;
      ts[n] = t; users[n] = (int32_t)u; items[n] = (int32_t)i; ratings[n] = (float)r;
      ++n;
    }
    p = eol + 1;
  }
  return n;
}

FPS_HOST_API int64_t fps_count_lines(const char* path) {
  std::string buf;
  if (!read_file(path, buf)) return -1;
  int64_t n = std::count(buf.begin(), buf.end(), '\n');
  if (!buf.empty() && buf.back() != '\n') ++n;
  return n;
}

// ------------------------------------------------------------------ id;value
FPS_HOST_API int fps_write_factors_text(const char* path, const int64_t* ids, const float* vals, int64_t n, int d,
                                        int append) {
  const int T = n_threads(n * d);
  std::vector<std::string> parts(T);
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t) {
    th.emplace_back([&, t] {
      const int64_t lo = n * t / T, hi = n * (t + 1) / T;
      std::string& s = parts[t];
      s.reserve((size_t)(hi - lo) * d * 24);
      char tmp[64];
      for (int64_t r = lo; r < hi; ++r) {
        for (int j = 0; j < d; ++j) {
          int len = std::snprintf(tmp, sizeof(tmp), "%lld;%.9g\n", (long long)ids[r], (double)vals[r * d + j]);
          s.append(tmp, (size_t)len);
        }
      }
    });
  }
  for (auto& x : th) x.join();
  FILE* f = std::fopen(path, append ? "ab" : "wb");
  if (!f) return -1;
  for (auto& s : parts) std::fwrite(s.data(), 1, s.size(), f);
  std::fclose(f);
  return 0;
}

// Reads "<id>;<value>" lines; consecutive lines of one id form its vector.
// First call with ids == nullptr returns the number of lines (upper bound of
// values); second call fills ids_per_line / values and returns the count.
FPS_HOST_API int64_t fps_read_id_value_text(const char* path, int64_t cap, int64_t* ids, double* vals) {
  std::string buf;
  if (!read_file(path, buf)) return -1;
  const char* p = buf.data();
  const char* end = p + buf.size();
  int64_t n = 0;
  while (p < end) {
    const char* eol = (const char*)std::memchr(p, '\n', (size_t)(end - p));
    if (!eol) eol = end;
    if (eol > p) {
      if (ids == nullptr) {
        ++n;
      } else if (n < cap) {
        bool ok1, ok2;
        int64_t id;
        double v;
        const char* q = parse_i64(p, eol, id, ok1);
        parse_f64(q, eol, v, ok2);
        if (ok1 && ok2) { ids[n] = id; vals[n] = v; ++n; }
      }
    }
    p = eol + 1;
  }
  return n;
}

// ------------------------------------------------------------------ snapshots
struct SnapHeader {
  char magic[8];      // "FPSSNAP1"
  int32_t version;
  int32_t part_kind;  // 0 hash, 1 range
  int64_t num_ids;
  int32_t dim;
  int32_t world;
  int32_t rank;
  int32_t dtype;      // 0 fp32
  int64_t n_rows;
  int64_t step;
  int64_t reserved[4];
};

FPS_HOST_API int fps_write_snapshot(const char* path, int part_kind, int64_t num_ids, int dim, int world, int rank,
                                    int64_t step, const int64_t* ids, const float* vals, int64_t n) {
  SnapHeader h{};
  std::memcpy(h.magic, "FPSSNAP1", 8);
  h.version = 1; h.part_kind = part_kind; h.num_ids = num_ids; h.dim = dim; h.world = world; h.rank = rank;
  h.dtype = 0; h.n_rows = n; h.step = step;
  std::string tmp = std::string(path) + ".tmp";
  FILE* f = std::fopen(tmp.c_str(), "wb");
  if (!f) return -1;
  bool ok = std::fwrite(&h, sizeof(h), 1, f) == 1;
  ok = ok && (n == 0 || std::fwrite(ids, sizeof(int64_t), (size_t)n, f) == (size_t)n);
  ok = ok && (n == 0 || std::fwrite(vals, sizeof(float), (size_t)(n * dim), f) == (size_t)(n * dim));
  ok = (std::fflush(f) == 0) && ok;
  std::fclose(f);
  if (!ok) return -2;
  return std::rename(tmp.c_str(), path) == 0 ? 0 : -3;  // atomic publish
}

// meta: [part_kind, num_ids, dim, world, rank, n_rows, step]
FPS_HOST_API int fps_read_snapshot_header(const char* path, int64_t* meta) {
  FILE* f = std::fopen(path, "rb");
  if (!f) return -1;
  SnapHeader h{};
  bool ok = std::fread(&h, sizeof(h), 1, f) == 1 && std::memcmp(h.magic, "FPSSNAP1", 8) == 0;
  std::fclose(f);
  if (!ok) return -2;
  meta[0] = h.part_kind; meta[1] = h.num_ids; meta[2] = h.dim; meta[3] = h.world; meta[4] = h.rank;
  meta[5] = h.n_rows; meta[6] = h.step;
  return 0;
}

FPS_HOST_API int fps_read_snapshot(const char* path, int64_t* ids, float* vals, int64_t cap_rows) {
  FILE* f = std::fopen(path, "rb");
  if (!f) return -1;
  SnapHeader h{};
  if (std::fread(&h, sizeof(h), 1, f) != 1 || h.n_rows > cap_rows) { std::fclose(f); return -2; }
  const int64_t n = h.n_rows;
  bool ok = (n == 0 || std::fread(ids, sizeof(int64_t), (size_t)n, f) == (size_t)n);
  ok = ok && (n == 0 || std::fread(vals, sizeof(float), (size_t)(n * h.dim), f) == (size_t)(n * h.dim));
  std::fclose(f);
  return ok ? 0 : -3;
}

// ------------------------------------------------------------------ synthetic ratings
// users in [0, n_local_users) (rank-local rows), items in [0, n_items), ratings U[0,1)
FPS_HOST_API void fps_gen_ratings(int64_t n, int64_t n_local_users, int64_t n_items, uint32_t seed, int64_t offset,
                                  int32_t* users, int32_t* items, float* ratings) {
  const int T = n_threads(n);
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t) {
    th.emplace_back([&, t] {
      for (int64_t k = n * t / T; k < n * (t + 1) / T; ++k) {
        const int64_t gk = offset + k;
        users[k] = (int32_t)(((uint64_t)fmix32((uint32_t)gk ^ fmix32(seed)) * (uint64_t)n_local_users) >> 32);
        items[k] = (int32_t)(((uint64_t)fmix32((uint32_t)(gk >> 32) ^ fmix32((uint32_t)gk + 0x9e3779b9u ^ seed)) *
                              (uint64_t)n_items) >> 32);
        ratings[k] = hash_uniform(seed + 1, gk, 7);
      }
    });
  }
  for (auto& x : th) x.join();
}

// ------------------------------------------------------------------ HashStore
namespace {
struct HashStore {
  int dim;
  float lo, hi;
  uint32_t seed;
  int64_t size = 0;
  // empty slot marker: INT64_MIN (ids are any other int64, negative ones
  // included -- the reference's Int ids may be negative, only the
  // partitioner takes |id|, M/FlinkParameterServer.scala:355-366)
  static constexpr int64_t kEmpty = INT64_MIN;
  std::vector<int64_t> keys;
  std::vector<float> vals;
  std::mutex mu;

  HashStore(int d, float l, float h, uint32_t s, int64_t cap) : dim(d), lo(l), hi(h), seed(s) { rehash(cap); }

  void rehash(int64_t cap) {
    int64_t c = 16;
    while (c < cap * 2) c <<= 1;
    std::vector<int64_t> ok = std::move(keys);
    std::vector<float> ov = std::move(vals);
    keys.assign((size_t)c, kEmpty);
    vals.assign((size_t)c * dim, 0.f);
    size = 0;
    for (size_t i = 0; i < ok.size(); ++i)
      if (ok[i] != kEmpty) std::memcpy(&vals[(size_t)slot_insert(ok[i]) * dim], &ov[i * dim], sizeof(float) * dim);
  }

  int64_t mask() const { return (int64_t)keys.size() - 1; }

  int64_t find(int64_t k) const {
    int64_t i = (int64_t)(fmix32((uint32_t)k ^ fmix32((uint32_t)((uint64_t)k >> 32))) & mask());
    while (true) {
      if (keys[i] == k) return i;
      if (keys[i] == kEmpty) return -1;
      i = (i + 1) & mask();
    }
  }

  int64_t slot_insert(int64_t k) {
    if ((size + 1) * 2 > (int64_t)keys.size()) rehash(size + 1);
    int64_t i = (int64_t)(fmix32((uint32_t)k ^ fmix32((uint32_t)((uint64_t)k >> 32))) & mask());
    while (keys[i] != kEmpty && keys[i] != k) i = (i + 1) & mask();
    if (keys[i] == kEmpty) { keys[i] = k; ++size; }
    return i;
  }

  float* get_or_init(int64_t k) {
    int64_t i = find(k);
    if (i < 0) {
      i = slot_insert(k);
      float* v = &vals[(size_t)i * dim];
      for (int j = 0; j < dim; ++j) v[j] = lo + (hi - lo) * hash_uniform(seed, k, (uint32_t)j);
      return v;
    }
    return &vals[(size_t)i * dim];
  }
};
}  // namespace

FPS_HOST_API void* fps_hs_create(int dim, float lo, float hi, uint32_t seed, int64_t cap) {
  return new HashStore(dim, lo, hi, seed, cap);
}
FPS_HOST_API void fps_hs_destroy(void* h) { delete (HashStore*)h; }
FPS_HOST_API int64_t fps_hs_size(void* h) { return ((HashStore*)h)->size; }

// pull: values for keys (lazy init of unseen ids)
FPS_HOST_API void fps_hs_pull(void* h, const int64_t* keys, int64_t n, float* out) {
  HashStore* s = (HashStore*)h;
  std::lock_guard<std::mutex> g(s->mu);
  for (int64_t r = 0; r < n; ++r) std::memcpy(out + r * s->dim, s->get_or_init(keys[r]), sizeof(float) * s->dim);
}

// push: add (op 0) or set (op 1); an unseen key takes the delta itself (SimplePSLogic semantics)
FPS_HOST_API void fps_hs_push(void* h, const int64_t* keys, int64_t n, const float* delta, int op) {
  HashStore* s = (HashStore*)h;
  std::lock_guard<std::mutex> g(s->mu);
  for (int64_t r = 0; r < n; ++r) {
    int64_t i = s->find(keys[r]);
    const float* d = delta + r * s->dim;
    if (i < 0 || op == 1) {
      if (i < 0) i = s->slot_insert(keys[r]);
      std::memcpy(&s->vals[(size_t)i * s->dim], d, sizeof(float) * s->dim);
    } else {
      float* v = &s->vals[(size_t)i * s->dim];
      for (int j = 0; j < s->dim; ++j) v[j] += d[j];
    }
  }
}

// dump: keys / values of every stored id (cap rows); returns the count
FPS_HOST_API int64_t fps_hs_dump(void* h, int64_t* keys, float* vals, int64_t cap) {
  HashStore* s = (HashStore*)h;
  std::lock_guard<std::mutex> g(s->mu);
  int64_t n = 0;
  for (size_t i = 0; i < s->keys.size() && n < cap; ++i) {
    if (s->keys[i] == HashStore::kEmpty) continue;
    keys[n] = s->keys[i];
    std::memcpy(vals + n * s->dim, &s->vals[i * s->dim], sizeof(float) * s->dim);
    ++n;
  }
  return n;
}

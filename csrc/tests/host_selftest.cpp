// Self-test of the host runtime (csrc/host/fps_host.cpp), built with
// AddressSanitizer + UBSan by `python csrc/build.py --asan-selftest`
// (sanitizers on host code; GPU ASan is not available).
// Exercises every exported entry point on small inputs, including the edge
// cases (missing trailing newline, malformed lines, table growth).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

extern "C" {
int64_t fps_parse_ratings(const char*, int64_t, int64_t*, int32_t*, int32_t*, float*, float);
int64_t fps_count_lines(const char*);
int fps_write_factors_text(const char*, const int64_t*, const float*, int64_t, int, int);
int64_t fps_read_id_value_text(const char*, int64_t, int64_t*, double*);
int fps_write_snapshot(const char*, int, int64_t, int, int, int, int64_t, const int64_t*, const float*, int64_t);
int fps_read_snapshot_header(const char*, int64_t*);
int fps_read_snapshot(const char*, int64_t*, float*, int64_t);
void fps_gen_ratings(int64_t, int64_t, int64_t, uint32_t, int64_t, int32_t*, int32_t*, float*);
void* fps_hs_create(int, float, float, uint32_t, int64_t);
void fps_hs_destroy(void*);
int64_t fps_hs_size(void*);
void fps_hs_pull(void*, const int64_t*, int64_t, float*);
void fps_hs_push(void*, const int64_t*, int64_t, const float*, int);
int64_t fps_hs_dump(void*, int64_t*, float*, int64_t);
int fps_mf_online_record(const int64_t*, const int64_t*, const double*, int64_t, int, int, int, double, double,
                         double, double, uint32_t, int64_t, int, int, int64_t*, double*, int64_t, int64_t*, double*,
                         int64_t, int64_t*, int64_t*);
}

static int failures = 0;
#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) { std::fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c); ++failures; } \
  } while (0)

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  // ratings: last line without newline, a malformed line, an optional rating column
  const std::string rp = dir + "/fps_selftest_ratings.txt";
  {
    FILE* f = std::fopen(rp.c_str(), "w");
    std::fputs("10 1 2 0.5\n11 3 4\nbad line\n12 5 6 1.5", f);
    std::fclose(f);
  }
  CHECK(fps_count_lines(rp.c_str()) == 4);
  std::vector<int64_t> ts(4);
  std::vector<int32_t> u(4), it(4);
  std::vector<float> r(4);
  const int64_t n = fps_parse_ratings(rp.c_str(), 4, ts.data(), u.data(), it.data(), r.data(), 1.0f);
  CHECK(n == 3);
  CHECK(ts[0] == 10 && u[0] == 1 && it[0] == 2 && std::fabs(r[0] - 0.5f) < 1e-6f);
  CHECK(ts[1] == 11 && std::fabs(r[1] - 1.0f) < 1e-6f);
  CHECK(ts[2] == 12 && u[2] == 5 && std::fabs(r[2] - 1.5f) < 1e-6f);
  CHECK(fps_parse_ratings(rp.c_str(), 1, ts.data(), u.data(), it.data(), r.data(), 1.0f) == 1);  // cap respected

  // id;value text round trip
  const std::string fp = dir + "/fps_selftest_factors.txt";
  const int64_t ids[3] = {7, 3, 9};
  const float vals[6] = {0.25f, -1.f, 2.f, 3.5f, 1e-7f, -4.f};
  CHECK(fps_write_factors_text(fp.c_str(), ids, vals, 3, 2, 0) == 0);
  const int64_t m = fps_read_id_value_text(fp.c_str(), 0, nullptr, nullptr);
  CHECK(m == 6);
  std::vector<int64_t> rid(6);
  std::vector<double> rv(6);
  CHECK(fps_read_id_value_text(fp.c_str(), 6, rid.data(), rv.data()) == 6);
  for (int k = 0; k < 6; ++k) {
    CHECK(rid[k] == ids[k / 2]);
    CHECK(std::fabs(rv[k] - vals[k]) <= 1e-6 * std::fmax(1.0, std::fabs(vals[k])));
  }

  // snapshot round trip
  const std::string sp = dir + "/fps_selftest.snap";
  CHECK(fps_write_snapshot(sp.c_str(), 1, 100, 2, 4, 3, 77, ids, vals, 3) == 0);
  int64_t meta[7];
  CHECK(fps_read_snapshot_header(sp.c_str(), meta) == 0);
  CHECK(meta[0] == 1 && meta[1] == 100 && meta[2] == 2 && meta[3] == 4 && meta[4] == 3 && meta[5] == 3 && meta[6] == 77);
  std::vector<int64_t> sid(3);
  std::vector<float> sv(6);
  CHECK(fps_read_snapshot(sp.c_str(), sid.data(), sv.data(), 2) == -2);  // capacity check
  CHECK(fps_read_snapshot(sp.c_str(), sid.data(), sv.data(), 3) == 0);
  CHECK(std::memcmp(sv.data(), vals, sizeof(vals)) == 0 && sid[2] == 9);

  // synthetic generator: ranges
  std::vector<int32_t> gu(100000), gi(100000);
  std::vector<float> gr(100000);
  fps_gen_ratings(100000, 1000, 77, 5, 123, gu.data(), gi.data(), gr.data());
  for (int k = 0; k < 100000; ++k) CHECK(gu[k] >= 0 && gu[k] < 1000 && gi[k] >= 0 && gi[k] < 77 && gr[k] >= 0 && gr[k] < 1);

  // hash store: lazy init, add/set, growth past the initial capacity, dump
  void* h = fps_hs_create(3, -1.f, 1.f, 9, 4);
  std::vector<int64_t> keys(5000);
  for (int k = 0; k < 5000; ++k) keys[k] = (int64_t)k * 7919 - 100000;  // negative ids too
  std::vector<float> out(5000 * 3), out2(5000 * 3);
  fps_hs_pull(h, keys.data(), 5000, out.data());
  CHECK(fps_hs_size(h) == 5000);
  fps_hs_pull(h, keys.data(), 5000, out2.data());
  CHECK(std::memcmp(out.data(), out2.data(), out.size() * sizeof(float)) == 0);  // deterministic init
  std::vector<float> ones(5000 * 3, 1.f);
  fps_hs_push(h, keys.data(), 5000, ones.data(), 0);
  fps_hs_pull(h, keys.data(), 1, out2.data());
  CHECK(std::fabs(out2[0] - (out[0] + 1.f)) < 1e-6f);
  const int64_t newk = 123456789;
  const float setv[3] = {5.f, 6.f, 7.f};
  fps_hs_push(h, &newk, 1, setv, 0);  // unseen key takes the delta
  fps_hs_pull(h, &newk, 1, out2.data());
  CHECK(out2[0] == 5.f && out2[2] == 7.f);
  std::vector<int64_t> dk(6000);
  std::vector<float> dv(6000 * 3);
  CHECK(fps_hs_dump(h, dk.data(), dv.data(), 6000) == 5001);
  CHECK(fps_hs_dump(h, dk.data(), dv.data(), 10) == 10);  // cap respected
  fps_hs_destroy(h);

  // native record engine: negatives + limiter + negative ids, exact message counts
  {
    const int64_t n = 4000;
    std::vector<int64_t> u(n), it(n);
    std::vector<double> r(n);
    for (int64_t k = 0; k < n; ++k) { u[k] = (k * 7) % 97; it[k] = (k * 13) % 61 - 30; r[k] = (k % 5) * 0.2; }
    std::vector<int64_t> uid(97), iid(61), counts(2), stats(7);
    std::vector<double> uv(97 * 6), iv(61 * 6);
    CHECK(fps_mf_online_record(u.data(), it.data(), r.data(), n, 3, 2, 6, 0.05, 0.01, -0.1, 0.1, 5, 4, 2, 16,
                               uid.data(), uv.data(), 97, iid.data(), iv.data(), 61, counts.data(),
                               stats.data()) == 0);
    CHECK(counts[0] == 97);
    CHECK(stats[0] == stats[1] && stats[0] == n + stats[6]);
    CHECK(fps_mf_online_record(u.data(), it.data(), r.data(), n, 3, 2, 300, 0.05, 0.0, -0.1, 0.1, 5, 4, 0, 16,
                               uid.data(), uv.data(), 97, iid.data(), iv.data(), 61, counts.data(),
                               stats.data()) == -3);  // D > 256 rejected
  }

  std::remove(rp.c_str());
  std::remove(fp.c_str());
  std::remove(sp.c_str());
  if (failures) { std::fprintf(stderr, "%d failure(s)\n", failures); return 1; }
  std::printf("host selftest OK\n");
  return 0;
}

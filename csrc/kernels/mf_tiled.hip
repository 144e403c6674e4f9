// Tile-grouped MF SGD (gfx950): no global item atomics, no LDS float atomics.
//
// Why: the flat kernel (mf.hip) pushes every rating's item delta with a
// 256-B global float-atomic wave-instruction; those execute at the memory
// side at ~1.3 TB/s chip-wide (MI355X_MICROARCH.md "Global float atomics"),
// so the measured 3.9e9 ratings/s sits on that ceiling (profiles/README.md).
// Staging the item rows in LDS and adding with ds_add_f32 instead was slower
// still: SQ_LDS_IDX_ACTIVE showed the LDS busy for the whole kernel, ~3 LDS
// cycles per float atomic lane (profiles/r1_tiled_lds_atomics.md).
//
// This kernel: the ratings of a micro-batch are bucketed by tile of R item rows
// (tile_partition below, no global atomics); one workgroup takes one tile,
// stages up to CAP of its rating records in LDS, counting-sorts them by row
// (one LDS int atomic per rating), and gives every row to ONE lane group.  The
// lane group reads the item row once into registers, streams the row's ratings
// with PF user rows in flight, updates each user row (plain store) against the
// row's value at the start of the chunk, sums the item deltas in registers and
// writes the row back once with a plain store.  Global traffic per rating:
// user row read + write (512 B) + 16 B record; per item row and chunk: 512 B.
//
// Semantics: inside one chunk (<= CAP ratings of a tile) an item's ratings see
// the item as of the chunk start and their deltas are summed -- the per-item
// mini-batch the PS path has (rows pulled once per micro-batch, deltas summed
// and pushed: M/matrix/factorization/workers/PSOnlineMatrixFactorizationWorker.scala:41-55,
// PS add M/matrix/factorization/PSOnlineMatrixFactorization.scala:58-60).
// User rows are Hogwild across workgroups, as in the flat kernel.
//
// Lane layout: TPR lanes per rating / row, each holding V float4 (D = 4*TPR*V;
// D = 64 -> 16 lanes x 1 float4: every row access is one 256-B coalesced
// wave-quarter).
#include "common.h"

#include <cstdlib>
#include <type_traits>

using namespace fps;

namespace {

// ---------------------------------------------------------------- partition
// bucket of a rating = (phase * 2W + block) * T + row_in_block / R (block layout of
// rotate.hip: b = 2q + h, q = i % W, h = (i / W >= half[q])); W = 1 with half[0] =
// num_items gives a single block (the whole local table).  phase = uid / upp: the
// SGD runs the phases one after another, so the user rows one launch touches
// (upp of them) mostly stay in the 256 MiB Infinity Cache (P = 1: upp > users).
//
// The divisions by W, R and upp use multiply-shift reciprocals: with four
// hardware integer divisions per rating the count kernel was VALU-bound.
struct FastDiv {  // n / d for 0 <= n < 2^31: (n * M) >> k, k = 31 + ceil(log2 d), M = ceil(2^k / d)
  uint64_t M;
  int k;
  __device__ __forceinline__ int32_t div(int32_t n) const { return (int32_t)(((uint64_t)(uint32_t)n * M) >> k); }
};

static FastDiv make_fastdiv(int d) {
  int l = 0;
  while ((1ll << l) < d) ++l;
  const int k = 31 + l;
  return FastDiv{((1ull << k) + (uint64_t)d - 1) / (uint64_t)d, k};
}

struct TileGeo {
  int W, R, T;
  FastDiv dW, dR, dU;
  const int32_t* half;
};

static TileGeo make_geo(int W, const int32_t* half, int R, int T, int upp) {
  return TileGeo{W, R, T, make_fastdiv(W), make_fastdiv(R), make_fastdiv(upp), half};
}

__device__ __forceinline__ void tile_bucket(int32_t i, int32_t u, const TileGeo& g, int& bucket, int32_t& row) {
  const int32_t loc = g.dW.div(i);
  const int q = i - loc * g.W;
  const int32_t hq = g.half[q];
  const int h = loc >= hq;
  row = loc - (h ? hq : 0);
  bucket = (g.dU.div(u) * 2 * g.W + 2 * q + h) * g.T + g.dR.div(row);  // user phase, item block, tile
}

constexpr int TP_MAX_BUCKETS = 16384;  // 64 KiB of LDS counters

typedef int tp_i2 __attribute__((ext_vector_type(2)));
typedef int tp_i3 __attribute__((ext_vector_type(3)));
typedef int tp_i4 __attribute__((ext_vector_type(4)));

// streaming access (NT: non-temporal -- the partition's inputs are read once and
// its outputs are read by the next step's SGD, long after any cache kept them;
// marking them streaming keeps the L2 / Infinity Cache for the SGD's user rows)
template <bool NT, typename T>
__device__ __forceinline__ T tp_ld(const T* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT, typename T>
__device__ __forceinline__ void tp_st(T* p, T v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

typedef float tp_f4 __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ float4 f4_ld(const float4* p) {
  if constexpr (NT) {
    const tp_f4 v = __builtin_nontemporal_load(reinterpret_cast<const tp_f4*>(p));
    return make_float4(v.x, v.y, v.z, v.w);
  } else {
    return *p;
  }
}
template <bool NT>
__device__ __forceinline__ void f4_st(float4* p, float4 v) {
  if constexpr (NT) __builtin_nontemporal_store(tp_f4{v.x, v.y, v.z, v.w}, reinterpret_cast<tp_f4*>(p));
  else *p = v;
}

// Non-temporal scatter accesses are the default (same box, bench.py, 3 alternating runs
// each: plain 9.85e9, non-temporal 10.05e9 updates/s = +2 %; 12-B level-1 records as
// three dword accesses beat 16-B slots, 9.93e9; non-temporal count-kernel loads or
// tile-SGD record reads on top: no further gain; profiles/r2_partition.md).
static int tp_nt() {  // FPS_TP_NT: 0 plain, 1 non-temporal (12-B records, default), 2 non-temporal (16-B slots)
  static const int m = [] { const char* e = getenv("FPS_TP_NT"); return e ? atoi(e) : 1; }();
  return m;
}


// K1: per-workgroup histogram H[w][KT] (plain stores, no global atomics)
__global__ void __launch_bounds__(1024) tile_hist_kernel(const int32_t* __restrict__ uid,
                                                         const int32_t* __restrict__ iid, int64_t n, int64_t chunk,
                                                         TileGeo g,
                                                         int KT, int32_t* __restrict__ H, uint8_t* __restrict__ seen) {
  __shared__ int32_t cnt[TP_MAX_BUCKETS];
  for (int k = threadIdx.x; k < KT; k += blockDim.x) cnt[k] = 0;
  __syncthreads();
  const int64_t lo = (int64_t)blockIdx.x * chunk, hi = min(n, lo + chunk);
  for (int64_t x = lo + threadIdx.x; x < hi; x += blockDim.x) {
    const int32_t i = iid[x];
    int bk; int32_t row;
    tile_bucket(i, uid[x], g, bk, row);
    atomicAdd(cnt + bk, 1);
    if (seen != nullptr) seen[i] = 1;
  }
  __syncthreads();
  int32_t* Hw = H + (int64_t)blockIdx.x * KT;
  for (int k = threadIdx.x; k < KT; k += blockDim.x) Hw[k] = cnt[k];
}

// K2: per bucket, exclusive scan over the G workgroups (coalesced across buckets)
__global__ void tile_colscan_kernel(int32_t* __restrict__ H, int G, int KT, int32_t* __restrict__ totals) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= KT) return;
  int32_t run = 0;
  for (int w = 0; w < G; ++w) {
    const int32_t v = H[(int64_t)w * KT + k];
    H[(int64_t)w * KT + k] = run;
    run += v;
  }
  totals[k] = run;
}

// K3: exclusive scan of KT totals into ptr[KT+1] (one 1024-thread workgroup)
__global__ void __launch_bounds__(1024) tile_scan_kernel(const int32_t* __restrict__ totals_g, int KT,
                                                         int32_t* __restrict__ ptr) {
  __shared__ int32_t part[1024];
  __shared__ int32_t totals[16384];  // KT <= TP_MAX_BUCKETS: staged by coalesced loads
  for (int k = threadIdx.x; k < KT; k += 1024) totals[k] = totals_g[k];
  __syncthreads();
  const int per = (KT + 1023) / 1024;
  const int k0 = threadIdx.x * per;
  int32_t s = 0;
  for (int k = k0; k < min(KT, k0 + per); ++k) s += totals[k];
  part[threadIdx.x] = s;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {  // Hillis-Steele inclusive scan
    const int32_t v = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  int32_t run = threadIdx.x ? part[threadIdx.x - 1] : 0;
  for (int k = k0; k < min(KT, k0 + per); ++k) { ptr[k] = run; run += totals[k]; }
  if (threadIdx.x == 1023) ptr[KT] = part[1023];
}

// Packed rating records.  REC8 (users < 2^24, R <= 256): 8 B {uid | row_in_tile << 24,
// rating bits}; else 16 B {uid, row-in-block, rating bits, bucket}.
template <bool REC8>
__device__ __forceinline__ void put_rec(void* rec, int64_t o, int32_t uid, int32_t row, float rating, int bucket,
                                        int R) {
  if (REC8) reinterpret_cast<int2*>(rec)[o] = make_int2(uid | ((row & (R - 1)) << 24), __float_as_int(rating));
  else reinterpret_cast<int4*>(rec)[o] = make_int4(uid, row, __float_as_int(rating), bucket);
}

// K4: scatter packed records to ptr[bucket] + H[w][bucket] + LDS slot (one
// store per rating instead of three scattered 4-B stores)
template <bool REC8>
__global__ void __launch_bounds__(1024) tile_scatter_kernel(const int32_t* __restrict__ uid,
                                                            const int32_t* __restrict__ iid,
                                                            const float* __restrict__ rating, int64_t n,
                                                            int64_t chunk, TileGeo g, int KT,
                                                            const int32_t* __restrict__ H,
                                                            const int32_t* __restrict__ ptr,
                                                            void* __restrict__ rec) {
  __shared__ int32_t cur[TP_MAX_BUCKETS];
  const int32_t* Hw = H + (int64_t)blockIdx.x * KT;
  for (int k = threadIdx.x; k < KT; k += blockDim.x) cur[k] = ptr[k] + Hw[k];
  __syncthreads();
  const int64_t lo = (int64_t)blockIdx.x * chunk, hi = min(n, lo + chunk);
  for (int64_t x = lo + threadIdx.x; x < hi; x += blockDim.x) {
    int bk; int32_t row;
    tile_bucket(iid[x], uid[x], g, bk, row);
    const int32_t o = atomicAdd(cur + bk, 1);
    put_rec<REC8>(rec, o, uid[x], row, rating[x], bk, g.R);
  }
}

// ---- two-level partition (default): coarse key (bucket >> cshift, ~128
// keys) then the full bucket, each level with few open output runs per
// workgroup so the scattered 16-B stores combine in L2 (the single-level
// scatter above keeps ~16k runs open per workgroup: ~4 records each).
// Reservations use one global atomic per (workgroup, key); no histograms
// matrix, no column scan.  Order inside a bucket is arbitrary.
constexpr int TP2_MAX_COARSE = 1024;

// both histograms in one pass over iid: coarse counts and per-bucket counts
__global__ void __launch_bounds__(1024) tp2_count_kernel(const int32_t* __restrict__ uid,
                                                         const int32_t* __restrict__ iid, int64_t n, int64_t chunk,
                                                         TileGeo g,
                                                         int cshift, int NC, int KT, int32_t* __restrict__ ccount,
                                                         int32_t* __restrict__ bcount, uint8_t* __restrict__ seen,
                                                         int32_t* __restrict__ H1 = nullptr) {
  __shared__ int32_t hb[TP_MAX_BUCKETS];
  __shared__ int32_t hc[TP2_MAX_COARSE];
  for (int k = threadIdx.x; k < KT; k += blockDim.x) hb[k] = 0;
  for (int k = threadIdx.x; k < NC; k += blockDim.x) hc[k] = 0;
  __syncthreads();
  const int64_t lo = (int64_t)blockIdx.x * chunk, hi = min(n, lo + chunk);
  for (int64_t x = lo + threadIdx.x; x < hi; x += blockDim.x) {
    const int32_t i = iid[x];
    int bk; int32_t row;
    tile_bucket(i, uid[x], g, bk, row);
    atomicAdd(hb + bk, 1);
    atomicAdd(hc + (bk >> cshift), 1);
    if (seen != nullptr) seen[i] = 1;
  }
  __syncthreads();
  for (int k = threadIdx.x; k < KT; k += blockDim.x)
    if (hb[k]) atomicAdd(bcount + k, hb[k]);
  for (int k = threadIdx.x; k < NC; k += blockDim.x) {
    if (hc[k]) atomicAdd(ccount + k, hc[k]);
    if (H1 != nullptr) H1[(int64_t)blockIdx.x * NC + k] = hc[k];  // tp3: per-workgroup coarse counts
  }
}

// LEVEL 1: records from (uid, iid, rating), key = coarse; out = {uid, row, rating, bucket}
// LEVEL 2: records from tmp, key = bucket (tmp.w); out = the same record
template <int LEVEL, bool REC8>
__global__ void __launch_bounds__(1024) tp2_scatter_kernel(const int32_t* __restrict__ uid,
                                                           const int32_t* __restrict__ iid,
                                                           const float* __restrict__ rating,
                                                           const int4* __restrict__ tmp, int64_t n, int64_t chunk,
                                                           TileGeo g,
                                                           int cshift, int nkeys, const int32_t* __restrict__ ptr,
                                                           int32_t* __restrict__ cursor, void* __restrict__ out) {
  __shared__ int32_t h[TP_MAX_BUCKETS];
  for (int k = threadIdx.x; k < nkeys; k += blockDim.x) h[k] = 0;
  __syncthreads();
  const int64_t lo = (int64_t)blockIdx.x * chunk, hi = min(n, lo + chunk);
  for (int64_t x = lo + threadIdx.x; x < hi; x += blockDim.x) {
    int key;
    if (LEVEL == 1) {
      int bk; int32_t row;
      tile_bucket(iid[x], uid[x], g, bk, row);
      key = bk >> cshift;
    } else {
      key = tmp[x].w;
    }
    atomicAdd(h + key, 1);
  }
  __syncthreads();
  for (int k = threadIdx.x; k < nkeys; k += blockDim.x)
    if (h[k]) h[k] = ptr[k] + atomicAdd(cursor + k, h[k]);  // this workgroup's range of key k
  __syncthreads();
  for (int64_t x = lo + threadIdx.x; x < hi; x += blockDim.x) {
    int4 r;
    int key;
    if (LEVEL == 1) {
      int bk; int32_t row;
      tile_bucket(iid[x], uid[x], g, bk, row);
      r = make_int4(uid[x], row, __float_as_int(rating[x]), bk);
      key = bk >> cshift;
    } else {
      r = tmp[x];
      key = r.w;
    }
    const int32_t o = atomicAdd(h + key, 1);
    if (LEVEL == 1) reinterpret_cast<int4*>(out)[o] = r;  // level 1 keeps the bucket for level 2
    else put_rec<REC8>(out, o, r.x, r.y, __int_as_float(r.z), r.w, g.R);
  }
}

// ---- two-level partition with LDS-sorted batches (default).  Both scatters
// above leave each lane's store on its own output run, so a wave's 64 stores
// hit ~64 different lines and the L2 writes lines back half-filled (1.2-2.5
// TB/s, profiles/r1_mf_partition_levels.md).  Here every workgroup stages a
// batch of TP3_B records in LDS, counting-sorts it by key (<= TP3_MAXK keys:
// ~128 coarse keys at level 1, the <= 2^cshift buckets of one coarse key at
// level 2), reserves one output range per (batch, key) with a global atomic,
// and writes the sorted batch out so consecutive lanes store consecutive
// records of one run (32-128 records per run at uniform keys).  Level 2 walks
// work items (coarse key, sub-range of CH records) so its key span is bounded
// whatever the key skew.
constexpr int TP3_B = 4096;      // records per LDS batch (64 KiB of int4)
constexpr int TP3_MAXK = 256;    // keys per batch sort
constexpr int TP3_CH = 32768;    // level-2 records per work item

// exclusive scan of cnt[0..nk) (nk <= 256) into off[] by wave 0; 4 keys per lane
__device__ __forceinline__ void tp3_scan(const int32_t* cnt, int32_t* off, int nk) {
  if (threadIdx.x >= 64) return;
  const int l = threadIdx.x;
  int32_t v[4], s = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) { const int k = 4 * l + q; v[q] = k < nk ? cnt[k] : 0; s += v[q]; }
  int32_t inc = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int32_t y = __shfl_up(inc, o, 64);
    if (l >= o) inc += y;
  }
  int32_t run = inc - s;
#pragma unroll
  for (int q = 0; q < 4; ++q) { const int k = 4 * l + q; if (k < nk) off[k] = run; run += v[q]; }
}

// tp3 counts: fine-bucket histogram per count workgroup (row 1 + g of bcount,
// plain stores, summed by tp3_colsum_kernel) and coarse counts per level-1 chunk
// (H1[chunk][NC]).  Each workgroup covers `sub` consecutive level-1 chunks, so
// <= 512 fine histograms are written however many level-1 chunks there are.
// (Flushing the fine histogram with global atomics cost 16M atomics per step
// at KT = 15.6k buckets and 65k-rating chunks, 4M with 256 workgroups.)
__global__ void __launch_bounds__(1024) tp3_count_kernel(const int32_t* __restrict__ uid,
                                                         const int32_t* __restrict__ iid, int64_t n, int64_t chunk,
                                                         int G, int sub, TileGeo g, int cshift, int NC, int KT,
                                                         int32_t* __restrict__ ccount, int32_t* __restrict__ bcount,
                                                         uint8_t* __restrict__ seen, int32_t* __restrict__ H1) {
  // One LDS atomic per rating (LDS atomics run at ~1 lane per CU cycle and
  // bound this kernel); the coarse counts of a chunk are read off the fine
  // histogram afterwards: 8 lanes per coarse key sum its 2^cshift buckets.
  __shared__ int32_t hb[TP_MAX_BUCKETS];
  __shared__ int32_t hc_prev[TP3_MAXK];
  for (int k = threadIdx.x; k < KT; k += blockDim.x) hb[k] = 0;
  if (threadIdx.x < NC) hc_prev[threadIdx.x] = 0;
  __syncthreads();
  const int span = 1 << cshift;
  const int per = (span + 7) / 8;
  const int ck = threadIdx.x >> 3, cl = threadIdx.x & 7;  // coarse key, lane in its group of 8
  const int c0 = blockIdx.x * sub, c1 = min(G, c0 + sub);
  for (int c = c0; c < c1; ++c) {
    const int64_t lo = (int64_t)c * chunk, hi = min(n, lo + chunk);
    constexpr int U4 = 8;  // loads in flight per thread (a lone dependent load pair per
                           // iteration left the kernel latency-bound at ~1.7 TB/s)
    for (int64_t x0 = lo + threadIdx.x; x0 < hi; x0 += U4 * blockDim.x) {
      int32_t iv[U4], uv[U4];
#pragma unroll
      for (int j = 0; j < U4; ++j) {
        const int64_t x = x0 + (int64_t)j * blockDim.x;
        iv[j] = x < hi ? iid[x] : -1;
        uv[j] = x < hi ? uid[x] : 0;
      }
#pragma unroll
      for (int j = 0; j < U4; ++j) {
        if (iv[j] < 0) continue;
        int bk; int32_t row;
        tile_bucket(iv[j], uv[j], g, bk, row);
        atomicAdd(hb + bk, 1);
        if (seen != nullptr) seen[iv[j]] = 1;
      }
    }
    __syncthreads();
    int32_t tot = 0;
    if (ck < NC)
      for (int q = 0; q < per; ++q) {
        const int b = (ck << cshift) + cl * per + q;
        if (cl * per + q < span && b < KT) tot += hb[b];
      }
    tot += __shfl_xor(tot, 1, 64);
    tot += __shfl_xor(tot, 2, 64);
    tot += __shfl_xor(tot, 4, 64);
    if (ck < NC && cl == 0) {
      const int32_t v = tot - hc_prev[ck];
      hc_prev[ck] = tot;
      if (v) atomicAdd(ccount + ck, v);
      H1[(int64_t)c * NC + ck] = v;
    }
    __syncthreads();  // hb is read above before the next chunk adds to it
  }
  int32_t* Hf = bcount + (int64_t)(blockIdx.x + 1) * KT;  // row 0 = the totals (tp3_colsum_kernel)
  for (int k = threadIdx.x; k < KT; k += blockDim.x) Hf[k] = hb[k];
}

// bcount[k] = sum of the count workgroups' rows bcount[1 + g][k]: 64 columns x 16
// row groups per workgroup, independent loads, LDS reduction
__global__ void __launch_bounds__(1024) tp3_colsum_kernel(int32_t* __restrict__ bcount, int G, int KT) {
  __shared__ int32_t part[16][64];
  const int col = blockIdx.x * 64 + (threadIdx.x & 63), rg = threadIdx.x >> 6;
  int32_t s = 0;
  if (col < KT)
    for (int g = rg; g < G; g += 16) s += bcount[(int64_t)(g + 1) * KT + col];
  part[rg][threadIdx.x & 63] = s;
  __syncthreads();
  if (rg == 0 && col < KT) {
    int32_t t = 0;
#pragma unroll
    for (int q = 0; q < 16; ++q) t += part[q][threadIdx.x];
    bcount[col] = t;
  }
}

// tp3 level-1 bases: H1[w][k] = cptr[k] + sum over w' < w of H1[w'][k]; one
// workgroup per coarse key, one thread per partition workgroup (G <= 1024)
__global__ void __launch_bounds__(1024) tp3_colscan_kernel(int32_t* __restrict__ H1, int G, int NC,
                                                           const int32_t* __restrict__ cptr) {
  __shared__ int32_t wsum[16];
  const int k = blockIdx.x, w = threadIdx.x, l = w & 63, wv = w >> 6;
  const int32_t v = w < G ? H1[(int64_t)w * NC + k] : 0;
  int32_t inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int32_t y = __shfl_up(inc, o, 64);
    if (l >= o) inc += y;
  }
  if (l == 63) wsum[wv] = inc;
  __syncthreads();
  int32_t before = cptr[k];
  for (int q = 0; q < wv; ++q) before += wsum[q];
  if (w < G) H1[(int64_t)w * NC + k] = before + inc - v;
}

// work items of level 2: wptr[c] = sum over c' < c of ceil(ccount[c'] / CH)
__global__ void tp3_workptr_kernel(const int32_t* __restrict__ ccount, int NC, int32_t* __restrict__ wptr) {
  if (threadIdx.x != 0) return;
  int32_t run = 0;
  for (int c = 0; c < NC; ++c) { wptr[c] = run; run += (ccount[c] + TP3_CH - 1) / TP3_CH; }
  wptr[NC] = run;
}

// LEVEL 1: (uid, iid, rating)[chunk of this workgroup] -> tmp grouped by coarse key
//          (bucket >> cshift); kptr = cptr, cursor = ccursor.  tmp records: REC8
//          12 B {uid | row_in_tile << 24, rating bits, bucket}, else 16 B {uid, row,
//          rating bits, bucket}
// LEVEL 2: tmp[work item] -> out (8- or 16-B records) grouped by bucket; kptr = ptr,
//          cursor = bcursor; work items from wptr / cptr
// NTM: 0 = plain accesses; 1 = non-temporal, 12-B level-1 records as three dwords;
// 2 = non-temporal, 12-B records in 16-B slots (one 3-dword vector access each)
template <int LEVEL, bool REC8, bool PIPE = true, int NTM = 0>
__global__ void __launch_bounds__(1024) tp3_scatter_kernel(const int32_t* __restrict__ uid,
                                                           const int32_t* __restrict__ iid,
                                                           const float* __restrict__ rating,
                                                           const int4* __restrict__ tmp, int64_t n, int64_t chunk,
                                                           TileGeo g,
                                                           int cshift, int NC, int KT,
                                                           const int32_t* __restrict__ kptr,
                                                           int32_t* __restrict__ cursor,
                                                           const int32_t* __restrict__ cptr,
                                                           const int32_t* __restrict__ wptr,
                                                           const int32_t* __restrict__ H1,
                                                           void* __restrict__ out) {
  constexpr int E = TP3_B / 1024;
  __shared__ int4 srt[TP3_B];
  __shared__ int32_t cnt[TP3_MAXK], off[TP3_MAXK], base[TP3_MAXK];
  __shared__ int32_t s_item[3];  // level 2: lo, hi, key base of the current work item
  const int tid = threadIdx.x;
  const int nwork = LEVEL == 1 ? 1 : wptr[NC];
  for (int w = LEVEL == 1 ? 0 : blockIdx.x; w < nwork; w += (LEVEL == 1 ? 1 : gridDim.x)) {
    int64_t lo, hi;
    int kb, nk;
    if (LEVEL == 1) {
      lo = (int64_t)blockIdx.x * chunk;
      hi = min(n, lo + chunk);
      kb = 0;
      nk = NC;
      if (tid < nk) base[tid] = H1[(int64_t)blockIdx.x * NC + tid];  // this workgroup's run starts
    } else {
      if (tid == 0) {
        int c = 0;
        while (wptr[c + 1] <= w) ++c;  // NC <= 256: linear search
        const int32_t a = cptr[c] + (w - wptr[c]) * TP3_CH;
        s_item[0] = a;
        s_item[1] = min(cptr[c + 1], a + TP3_CH);
        s_item[2] = c << cshift;
      }
      __syncthreads();
      lo = s_item[0];
      hi = s_item[1];
      kb = s_item[2];
      nk = min(1 << cshift, KT - kb);
      __syncthreads();  // s_item is rewritten for the next work item
    }
    // software pipeline: the raw inputs of batch b+1 are loaded into registers
    // while batch b is sorted and written (its loads were issued one batch earlier)
    int32_t ru[E], ri[E], rr[E];
    int4 rt[E];
    auto load_batch = [&](int64_t bs) {
      const int nbs = (int)min((int64_t)TP3_B, hi - bs);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int p = e * 1024 + tid;
        if (p < nbs) {
          const int64_t x = bs + p;
          constexpr bool NT = NTM > 0;
          if (LEVEL == 1) {
            ru[e] = tp_ld<NT>(uid + x);
            ri[e] = tp_ld<NT>(iid + x);
            rr[e] = __float_as_int(tp_ld<NT>(rating + x));
          } else if (REC8 && NTM == 2) {
            const tp_i3 t = tp_ld<true>(reinterpret_cast<const tp_i3*>(tmp) + x);  // 16-B slots
            rt[e] = make_int4(t.x, t.y, t.z, 0);
          } else if (REC8) {
            const int* q = reinterpret_cast<const int*>(tmp) + 3 * x;
            rt[e] = make_int4(tp_ld<NT>(q), tp_ld<NT>(q + 1), tp_ld<NT>(q + 2), 0);
          } else {
            const tp_i4 t = tp_ld<NT>(reinterpret_cast<const tp_i4*>(tmp) + x);
            rt[e] = make_int4(t.x, t.y, t.z, t.w);
          }
        }
      }
    };
    if (PIPE && lo < hi) load_batch(lo);
    for (int64_t b0 = lo; b0 < hi; b0 += TP3_B) {
      const int nb = (int)min((int64_t)TP3_B, hi - b0);
      if (!PIPE) load_batch(b0);  // A/B: loads of a batch right before its use
      if (tid < nk) cnt[tid] = 0;
      int4 r[E];
      int k[E], slot[E];
#pragma unroll
      for (int e = 0; e < E; ++e) {  // this batch's records (registers loaded last iteration)
        k[e] = 0;
        if (e * 1024 + tid >= nb) continue;  // no record: registers hold stale values
        if (LEVEL == 1) {
          int bk; int32_t row;
          tile_bucket(ri[e], ru[e], g, bk, row);
          if (REC8) r[e] = make_int4(ru[e] | ((row & (g.R - 1)) << 24), rr[e], bk, 0);
          else r[e] = make_int4(ru[e], row, rr[e], bk);
          k[e] = bk >> cshift;
        } else {
          r[e] = rt[e];
          k[e] = (REC8 ? rt[e].z : rt[e].w) - kb;
        }
      }
      if (PIPE && b0 + TP3_B < hi) load_batch(b0 + TP3_B);  // in flight during the sort below
      __syncthreads();  // cnt zeroed
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int p = e * 1024 + tid;
        slot[e] = -1;
        if (p < nb) {
          slot[e] = atomicAdd(cnt + k[e], 1);
        }
      }
      __syncthreads();
      tp3_scan(cnt, off, nk);
      if (LEVEL == 2 && tid < nk && cnt[tid]) base[tid] = kptr[kb + tid] + atomicAdd(cursor + kb + tid, cnt[tid]);
      __syncthreads();
#pragma unroll
      for (int e = 0; e < E; ++e)
        if (slot[e] >= 0) srt[off[k[e]] + slot[e]] = r[e];
      __syncthreads();
      for (int p = tid; p < nb; p += 1024) {
        const int4 x = srt[p];
        const int bk = REC8 ? x.z : x.w;
        const int kk = LEVEL == 1 ? (bk >> cshift) : bk - kb;
        const int64_t o = (int64_t)base[kk] + (p - off[kk]);
        constexpr bool NT = NTM > 0;
        if (LEVEL == 1 && REC8 && NTM == 2) tp_st<true>(reinterpret_cast<tp_i3*>(out) + o, tp_i3{x.x, x.y, x.z});
        else if (LEVEL == 1 && REC8) {
          int* q = reinterpret_cast<int*>(out) + 3 * o;
          tp_st<NT>(q, x.x);
          tp_st<NT>(q + 1, x.y);
          tp_st<NT>(q + 2, x.z);
        } else if (LEVEL == 1) tp_st<NT>(reinterpret_cast<tp_i4*>(out) + o, tp_i4{x.x, x.y, x.z, x.w});
        else if (REC8) tp_st<NT>(reinterpret_cast<tp_i2*>(out) + o, tp_i2{x.x, x.y});
        else put_rec<false>(out, o, x.x, x.y, __int_as_float(x.z), x.w, g.R);
      }
      __syncthreads();  // LDS reused by the next batch
      if (LEVEL == 1 && tid < nk) base[tid] += cnt[tid];  // same thread zeroes cnt[tid] next
    }
  }
}

// ---- tp4: capacity-slot partition (default).  No counting pass.  tp3's count
// kernel (one LDS atomic per rating into a 16k-bucket histogram, 79 % of its LDS
// cycles bank conflicts, profiles/r1_partition_pmc.md) ran ~200 us alone and
// ~2 ms beside the SGD, whose LDS it starved.  Here every coarse key and every
// bucket owns a slot of its own in the output, sized from the counts of the
// previous run of the same partitioner (a stationary stream's bucket sizes barely
// move between micro-batches): cap_k = floor(prev_k * n * slack / n_prev) + pad
// (the first run: uniform).  Each LDS-sorted batch reserves its runs with one
// global atomic per (batch, key) on the key's cursor; the cursors end as the exact
// counts, which size the next run.  Records past a slot's capacity go to an
// overflow list (one atomic per (batch, key) again) that a flat SGD kernel
// processes after the tiles of their block (tp4_ovf_sgd_kernel): nothing is
// dropped whatever the skew, only slower.  Traffic: level 1 reads the 12-B input
// and writes 12-B records, level 2 reads them and writes 8-B records (44 B per
// rating against tp3's 52 B).
constexpr float TP4_SLACK = 1.125f;
constexpr int TP4_PAD = 64;

// starts[0..K] = exclusive scan of the capacities (one 1024-thread workgroup, K <= 16384)
__global__ void __launch_bounds__(1024) tp4_plan_kernel(const int32_t* __restrict__ prev, int K, int64_t n_prev,
                                                        int64_t n, int32_t* __restrict__ starts) {
  __shared__ int32_t part[1024];
  const int per = (K + 1023) / 1024;
  const int k0 = threadIdx.x * per;
  const double scale = n_prev > 0 ? (double)n * TP4_SLACK / (double)n_prev : 0.0;
  const int32_t uni = (int32_t)((double)n * TP4_SLACK / K);
  auto cap = [&](int k) -> int32_t {
    return (n_prev > 0 ? (int32_t)((double)prev[k] * scale) : uni) + TP4_PAD;
  };
  int32_t s = 0;
  for (int k = k0; k < min(K, k0 + per); ++k) s += cap(k);
  part[threadIdx.x] = s;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const int32_t v = threadIdx.x >= o ? part[threadIdx.x - o] : 0;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  int32_t run = threadIdx.x ? part[threadIdx.x - 1] : 0;
  for (int k = k0; k < min(K, k0 + per); ++k) { starts[k] = run; run += cap(k); }
  if (threadIdx.x == 1023) starts[K] = part[1023];
}

// level-2 work items over the FILLED part of every coarse slot
__global__ void tp4_workptr_kernel(const int32_t* __restrict__ ccursor, const int32_t* __restrict__ cstart, int NC,
                                   int32_t* __restrict__ wptr) {
  if (threadIdx.x != 0) return;
  int32_t run = 0;
  for (int c = 0; c < NC; ++c) {
    wptr[c] = run;
    const int32_t filled = min(ccursor[c], cstart[c + 1] - cstart[c]);
    run += (filled + TP3_CH - 1) / TP3_CH;
  }
  wptr[NC] = run;
}

// overflow record {uid, row in block, rating bits, bucket} from a staged record
template <bool REC8, int LEVEL>
__device__ __forceinline__ int4 tp4_ovf_rec(const int4& x, int bk, const TileGeo& g) {
  if (REC8) {
    const int32_t u = x.x & 0xffffff;
    const int rit = (int)((uint32_t)x.x >> 24);
    return make_int4(u, (bk % g.T) * g.R + rit, x.y, bk);
  }
  return x;  // {uid, row, rating bits, bucket}
}

// LEVEL 1: (uid, iid, rating) of this workgroup's chunk -> coarse slots of tmp
//          (REC8: 12-B {uid | row_in_tile << 24, rating bits, bucket}; else 16-B
//          {uid, row, rating bits, bucket}); kstart = cstart, cursor = ccursor.
// LEVEL 2: the filled part of the coarse slots -> bucket slots of rec (8- or 16-B
//          records); kstart = bstart, cursor = bcursor; work items from wptr.
template <int LEVEL, bool REC8>
__global__ void __launch_bounds__(1024) tp4_scatter_kernel(const int32_t* __restrict__ uid,
                                                           const int32_t* __restrict__ iid,
                                                           const float* __restrict__ rating,
                                                           const void* __restrict__ tmp, int64_t n, int64_t chunk,
                                                           TileGeo g, int cshift, int NC, int KT,
                                                           const int32_t* __restrict__ kstart,
                                                           int32_t* __restrict__ cursor,
                                                           const int32_t* __restrict__ cstart,
                                                           const int32_t* __restrict__ ccursor,
                                                           const int32_t* __restrict__ wptr,
                                                           void* __restrict__ out, int4* __restrict__ ovf,
                                                           int32_t* __restrict__ ovf_cnt, uint8_t* __restrict__ seen) {
  constexpr int E = TP3_B / 1024;
  __shared__ int4 srt[TP3_B];
  __shared__ int32_t cnt[TP3_MAXK], off[TP3_MAXK], base[TP3_MAXK], obase[TP3_MAXK];
  __shared__ int32_t kst[TP3_MAXK], kcap[TP3_MAXK];
  __shared__ int32_t s_item[3];
  const int tid = threadIdx.x;
  const int nwork = LEVEL == 1 ? 1 : wptr[NC];
  for (int w = LEVEL == 1 ? 0 : blockIdx.x; w < nwork; w += (LEVEL == 1 ? 1 : gridDim.x)) {
    int64_t lo, hi;
    int kb, nk;
    if (LEVEL == 1) {
      lo = (int64_t)blockIdx.x * chunk;
      hi = min(n, lo + chunk);
      kb = 0;
      nk = NC;
    } else {
      if (tid == 0) {
        int c = 0;
        while (wptr[c + 1] <= w) ++c;  // NC <= 256: linear search
        const int32_t filled = min(ccursor[c], cstart[c + 1] - cstart[c]);
        const int32_t a = (w - wptr[c]) * TP3_CH;
        s_item[0] = cstart[c] + a;
        s_item[1] = cstart[c] + min(filled, a + TP3_CH);
        s_item[2] = c << cshift;
      }
      __syncthreads();
      lo = s_item[0];
      hi = s_item[1];
      kb = s_item[2];
      nk = min(1 << cshift, KT - kb);
    }
    if (tid < nk) {
      kst[tid] = kstart[kb + tid];
      kcap[tid] = kstart[kb + tid + 1] - kstart[kb + tid];
    }
    __syncthreads();  // s_item / kst / kcap visible; s_item rewritten only after the batches below
    for (int64_t b0 = lo; b0 < hi; b0 += TP3_B) {
      const int nb = (int)min((int64_t)TP3_B, hi - b0);
      if (tid < nk) cnt[tid] = 0;
      __syncthreads();
      int4 r[E];
      int k[E], slot[E];
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int p = e * 1024 + tid;
        slot[e] = -1;
        if (p < nb) {
          const int64_t x = b0 + p;
          int bk;
          if (LEVEL == 1) {
            const int32_t i = iid[x], u = uid[x];
            int32_t row;
            tile_bucket(i, u, g, bk, row);
            if (REC8) r[e] = make_int4(u | ((row & (g.R - 1)) << 24), __float_as_int(rating[x]), bk, 0);
            else r[e] = make_int4(u, row, __float_as_int(rating[x]), bk);
            if (seen != nullptr) seen[i] = 1;
            k[e] = bk >> cshift;
          } else if (REC8) {
            const int3 t = reinterpret_cast<const int3*>(tmp)[x];
            r[e] = make_int4(t.x, t.y, t.z, 0);
            k[e] = t.z - kb;
          } else {
            r[e] = reinterpret_cast<const int4*>(tmp)[x];
            k[e] = r[e].w - kb;
          }
          slot[e] = atomicAdd(cnt + k[e], 1);
        }
      }
      __syncthreads();
      tp3_scan(cnt, off, nk);
      if (tid < nk && cnt[tid]) {  // this batch's run of key tid: slot range, overflow beyond capacity
        const int32_t o = atomicAdd(cursor + kb + tid, cnt[tid]);
        base[tid] = o;
        const int32_t ex = o + cnt[tid] - kcap[tid];
        if (ex > 0) obase[tid] = atomicAdd(ovf_cnt, min(ex, cnt[tid]));
      }
      __syncthreads();
#pragma unroll
      for (int e = 0; e < E; ++e)
        if (slot[e] >= 0) srt[off[k[e]] + slot[e]] = r[e];
      __syncthreads();
      for (int p = tid; p < nb; p += 1024) {
        const int4 x = srt[p];
        const int bk = REC8 ? x.z : x.w;
        const int kk = LEVEL == 1 ? (bk >> cshift) : bk - kb;
        const int32_t idx = base[kk] + (p - off[kk]);
        if (idx < kcap[kk]) {
          const int64_t o = (int64_t)kst[kk] + idx;
          if (LEVEL == 1 && REC8) reinterpret_cast<int3*>(out)[o] = make_int3(x.x, x.y, x.z);
          else if (LEVEL == 1) reinterpret_cast<int4*>(out)[o] = x;
          else if (REC8) reinterpret_cast<int2*>(out)[o] = make_int2(x.x, x.y);
          else put_rec<false>(out, o, x.x, x.y, __int_as_float(x.z), x.w, g.R);
        } else {
          ovf[obase[kk] + (idx - max(kcap[kk], base[kk]))] = tp4_ovf_rec<REC8, LEVEL>(x, bk, g);
        }
      }
      __syncthreads();  // LDS reused by the next batch
    }
  }
}

// Flat SGD over the overflow records of buckets [b_lo, b_lo + nblk * T): one lane
// group per record, user row stored (Hogwild, as in the tiles), item delta by
// float atomics.  Runs after the tiled launch of the same blocks; a fixed grid
// reads the record count on the device (no host sync) and exits at once when the
// list is empty -- the common case.
template <int TPR, int V>
__global__ void __launch_bounds__(256) tp4_ovf_sgd_kernel(float* __restrict__ U, float* __restrict__ I0,
                                                          float* __restrict__ I1, const int4* __restrict__ ovf,
                                                          const int32_t* __restrict__ ovf_cnt, int b_lo, int T,
                                                          int nblk, float lr, float lambda) {
  constexpr int D4 = TPR * V;
  constexpr int GPW = 64 / TPR;
  const int n = *ovf_cnt;
  const int lane = threadIdx.x & 63;
  const int j = lane % TPR;
  const int64_t g0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / TPR;
  const int64_t gs = (int64_t)gridDim.x * blockDim.x / TPR;
  (void)GPW;
  for (int64_t x = g0; x < n; x += gs) {
    const int4 r = ovf[x];
    const int rel = r.w - b_lo;
    if (rel < 0 || rel >= nblk * T) continue;  // uniform in the lane group
    float4* Ig = reinterpret_cast<float4*>(rel < T ? I0 : I1) + (int64_t)r.y * D4;
    float4* Ug = reinterpret_cast<float4*>(U) + (int64_t)r.x * D4;
    const float rt = __int_as_float(r.z);
    float4 uv[V], iv[V];
    float p = 0.f;
#pragma unroll
    for (int v = 0; v < V; ++v) {
      uv[v] = Ug[j + v * TPR];
      iv[v] = Ig[j + v * TPR];
      p += uv[v].x * iv[v].x + uv[v].y * iv[v].y + uv[v].z * iv[v].z + uv[v].w * iv[v].w;
    }
    const float e = rt - group_sum<TPR>(p);
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const float4 u = uv[v], i = iv[v];
      Ug[j + v * TPR] = make_float4(u.x + lr * (e * i.x - lambda * u.x), u.y + lr * (e * i.y - lambda * u.y),
                                    u.z + lr * (e * i.z - lambda * u.z), u.w + lr * (e * i.w - lambda * u.w));
      float* ip = reinterpret_cast<float*>(Ig + j + v * TPR);
      atomic_add_noret(ip + 0, lr * (e * u.x - lambda * i.x));
      atomic_add_noret(ip + 1, lr * (e * u.y - lambda * i.y));
      atomic_add_noret(ip + 2, lr * (e * u.z - lambda * i.z));
      atomic_add_noret(ip + 3, lr * (e * u.w - lambda * i.w));
    }
  }
}

// ---------------------------------------------------------------- SGD
// records staged per chunk: 8-B records 4608 (38 KiB of LDS: 4 workgroups per CU; the bench's tiles hold Poisson(~4096) ratings, so a cap of 4096
// split half of them into a second, nearly empty chunk), 16-B records 4096
template <bool REC8>
constexpr int tg_cap() { return REC8 ? 4608 : 4096; }
constexpr int TG_MAX_R = 256;   // rows per tile

template <bool REC8>
struct RecT { using type = int4; };
template <>
struct RecT<true> { using type = int2; };

// (uid, row in tile, rating) of a staged record
template <bool REC8>
__device__ __forceinline__ void get_rec(const typename RecT<REC8>::type& x, int64_t r0, int32_t& uid, int& row,
                                        float& rating) {
  if constexpr (REC8) {
    uid = x.x & 0xffffff;
    row = (int)((uint32_t)x.x >> 24);
    rating = __int_as_float(x.y);
  } else {
    uid = x.x;
    row = (int)(x.y - r0);
    rating = __int_as_float(x.z);
  }
}

// NTI: item rows loaded / stored non-temporal (each is read and written once per
// chunk; the cache is worth more to the random user rows).  Default on: +0.7 %
// same box (profiles/r2_partition.md); non-temporal user-row stores: no gain.
template <int TPR, int V, int PF, bool REC8, bool PIPE = false, bool NTI = false>
__global__ void __launch_bounds__(512) mf_sgd_tilegroup_kernel(float* __restrict__ U, float* __restrict__ I,
                                                               const void* __restrict__ rec_,
                                                               const int32_t* __restrict__ ptr, int R,
                                                               int64_t block_rows, float lr, float lambda,
                                                               float* __restrict__ I1, int64_t block_rows1, int T0,
                                                               const int32_t* __restrict__ tcnt) {
  using Rec = typename RecT<REC8>::type;
  constexpr int TG_CAP = tg_cap<REC8>();
  const Rec* __restrict__ rec = reinterpret_cast<const Rec*>(rec_);
  __shared__ Rec srec[TG_CAP];       // the chunk, counting-sorted by row
  __shared__ int32_t cnt[TG_MAX_R + 1];
  __shared__ int32_t start[TG_MAX_R + 1];
  constexpr int D4 = TPR * V;
  constexpr int GPW = 64 / TPR;  // lane groups per wave
  // tiles [0, T0) cover item block I, tiles [T0, grid) the next block I1 (one launch
  // for two blocks with disjoint item rows: half the launch tails)
  const int t = blockIdx.x;
  const bool second = t >= T0;
  const int tl = second ? t - T0 : t;
  if (second) { I = I1; block_rows = block_rows1; }
  const int64_t r0 = (int64_t)tl * R;
  const int nr = (int)min((int64_t)R, block_rows - r0);
  // tp4 slots: the tile's records fill [ptr[t], ptr[t] + count) of its slot (the
  // cursor may exceed the slot: the excess went to the overflow list)
  const int32_t beg = ptr[t], end = tcnt != nullptr ? min(ptr[t + 1], beg + tcnt[t]) : ptr[t + 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ngroups = (blockDim.x >> 6) * GPW;
  const int grp = wave * GPW + lane / TPR, j = lane % TPR;
  float4* Ig = reinterpret_cast<float4*>(I) + r0 * D4;
  float4* Ug = reinterpret_cast<float4*>(U);
  for (int32_t c0 = beg; c0 < end; c0 += TG_CAP) {
    const int nc = min(TG_CAP, end - c0);
    for (int k = threadIdx.x; k <= nr; k += blockDim.x) cnt[k] = 0;
    __syncthreads();
    for (int k = threadIdx.x; k < nc; k += blockDim.x) {  // count rows (the chunk is re-read below: L2)
      int32_t u; int rw; float rt;
      get_rec<REC8>(rec[c0 + k], r0, u, rw, rt);
      atomicAdd(cnt + rw, 1);
    }
    __syncthreads();
    if (threadIdx.x < 64) {  // exclusive scan of <= 256 counters: 4 per lane + a wave scan
      int32_t c4[4], sum = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int k = 4 * lane + q;
        c4[q] = k < nr ? cnt[k] : 0;
        sum += c4[q];
      }
      int32_t inc = sum;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int32_t y = __shfl_up(inc, o, 64);
        if (lane >= o) inc += y;
      }
      int32_t run = inc - sum;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int k = 4 * lane + q;
        if (k < nr) { start[k] = run; cnt[k] = run; }
        run += c4[q];
      }
      if (lane == 63) start[nr] = inc;
    }
    __syncthreads();
    for (int k = threadIdx.x; k < nc; k += blockDim.x) {  // counting-sort placement
      const Rec x = rec[c0 + k];
      int32_t u; int rw; float rt;
      get_rec<REC8>(x, r0, u, rw, rt);
      srec[atomicAdd(cnt + rw, 1)] = x;
    }
    __syncthreads();
    for (int row = grp; row < nr; row += ngroups) {
      const int a = start[row], b = start[row + 1];
      if (a == b) continue;  // uniform in the lane group
      float4 iv[V], acc[V];
#pragma unroll
      for (int v = 0; v < V; ++v) {
        iv[v] = f4_ld<NTI>(Ig + (int64_t)row * D4 + j + v * TPR);
        acc[v] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
      // float4 offsets of the user rows: 32-bit for 8-B records (user < 2^24, D4 <= 64),
      // 14 fewer live VGPRs than 64-bit offsets
      using Off = typename std::conditional<REC8, uint32_t, int64_t>::type;
      float4 uvn[PF][V];  // PIPE: the next batch, loaded before this batch's user-row stores
      Off urn[PF];
      float rvn[PF];
      auto load_batch = [&](int k0, float4 (&uvx)[PF][V], Off (&urx)[PF], float (&rvx)[PF]) {
#pragma unroll
        for (int q = 0; q < PF; ++q) {  // all PF user rows in flight (index clamped, result masked)
          int32_t u; int rw;
          get_rec<REC8>(srec[min(k0 + q, b - 1)], r0, u, rw, rvx[q]);
          urx[q] = (Off)u * D4;
#pragma unroll
          for (int v = 0; v < V; ++v) uvx[q][v] = Ug[urx[q] + j + v * TPR];
        }
      };
      if (PIPE) load_batch(a, uvn, urn, rvn);
      for (int k0 = a; k0 < b; k0 += PF) {
        float4 uv[PF][V];
        Off ur[PF];
        float rv[PF];
        if (PIPE) {
          // vmcnt retires in issue order: loads issued after this batch's stores would
          // wait for them, so the next batch's rows are requested first
#pragma unroll
          for (int q = 0; q < PF; ++q) {
            ur[q] = urn[q];
            rv[q] = rvn[q];
#pragma unroll
            for (int v = 0; v < V; ++v) uv[q][v] = uvn[q][v];
          }
          if (k0 + PF < b) load_batch(k0 + PF, uvn, urn, rvn);
        } else {
          load_batch(k0, uv, ur, rv);
        }
#pragma unroll
        for (int q = 0; q < PF; ++q) {
          float p = 0.f;
#pragma unroll
          for (int v = 0; v < V; ++v)
            p += uv[q][v].x * iv[v].x + uv[q][v].y * iv[v].y + uv[q][v].z * iv[v].z + uv[q][v].w * iv[v].w;
          const float e = rv[q] - group_sum<TPR>(p);
          if (k0 + q >= b) continue;  // uniform in the lane group
#pragma unroll
          for (int v = 0; v < V; ++v) {
            const float4 u = uv[q][v], i = iv[v];
            float4 nu;
            nu.x = u.x + lr * (e * i.x - lambda * u.x);
            nu.y = u.y + lr * (e * i.y - lambda * u.y);
            nu.z = u.z + lr * (e * i.z - lambda * u.z);
            nu.w = u.w + lr * (e * i.w - lambda * u.w);
            Ug[ur[q] + j + v * TPR] = nu;
            acc[v].x += lr * (e * u.x - lambda * i.x);
            acc[v].y += lr * (e * u.y - lambda * i.y);
            acc[v].z += lr * (e * u.z - lambda * i.z);
            acc[v].w += lr * (e * u.w - lambda * i.w);
          }
        }
      }
#pragma unroll
      for (int v = 0; v < V; ++v) {
        float4 o = iv[v];
        o.x += acc[v].x; o.y += acc[v].y; o.z += acc[v].z; o.w += acc[v].w;
        f4_st<NTI>(Ig + (int64_t)row * D4 + j + v * TPR, o);
      }
    }
    __syncthreads();  // LDS reused by the next chunk
  }
}

}  // namespace

// Ratings per partition workgroup: longer chunks give longer runs per bucket in
// the scatter (chunk / KT records land contiguously), fewer give more parallelism.
// Level 3 (default) sizes the chunk from the bucket count unless set explicitly
// (FPS_TILE_PARTITION_CHUNK): ~16 records per bucket and workgroup, 65536 .. 262144
// (tp3_chunk).  Same box, alternating: at KT = 15.6k buckets (10M users, 4 phases)
// 65536 10.41 / 10.54e9, 262144 10.68 / 10.69e9 updates/s; at KT = 3.9k (2.5M users,
// 1 phase) 65536 9.89 / 9.88e9, 262144 9.69 / 9.73e9 (profiles/r2_partition.md).
static int64_t g_tp_chunk = 65536;
static bool g_tp_chunk_set = false;

FPS_API void fps_tile_partition_set_chunk(int64_t chunk) {
  g_tp_chunk = chunk > 1024 ? chunk : 1024;
  g_tp_chunk_set = true;
}

static int tp3_groups(int64_t n, int KT) {
  int64_t c = g_tp_chunk;
  if (!g_tp_chunk_set) {
    c = 65536;
    while (c < 16 * (int64_t)KT && c < 262144) c <<= 1;
  }
  int64_t g = (n + c - 1) / c;
  if (g < 1) g = 1;
  if (g > 1024) g = 1024;
  return (int)g;
}

// Workspace: H holds G * KT int32 (G = fps_tile_partition_groups(n)), totals KT.
FPS_API int fps_tile_partition_groups(int64_t n) {
  int64_t g = (n + g_tp_chunk - 1) / g_tp_chunk;
  if (g < 1) g = 1;
  if (g > 1024) g = 1024;
  return (int)g;
}

// rec: n packed records (8 B if rec8, else 16 B; see put_rec) grouped by bucket
FPS_API int fps_tile_partition(const int32_t* uid, const int32_t* iid, const float* rating, int64_t n, int W,
                               const int32_t* half, int R, int T, int P, int upp, int32_t* H, int32_t* totals, int32_t* ptr,
                               void* rec, int rec8, uint8_t* seen, void* stream) {
  const int KT = P * 2 * W * T;
  if (KT > TP_MAX_BUCKETS || R <= 0 || T <= 0) return (int)hipErrorInvalidValue;
  const TileGeo g = make_geo(W, half, R, T, upp);
  hipStream_t s = (hipStream_t)stream;
  const int G = fps_tile_partition_groups(n);
  const int64_t chunk = (n + G - 1) / G;
  hipLaunchKernelGGL(tile_hist_kernel, dim3(G), dim3(1024), 0, s, uid, iid, n, chunk, g,  KT, H, seen);
  hipLaunchKernelGGL(tile_colscan_kernel, dim3((KT + 255) / 256), dim3(256), 0, s, H, G, KT, totals);
  hipLaunchKernelGGL(tile_scan_kernel, dim3(1), dim3(1024), 0, s, (const int32_t*)totals, KT, ptr);
  if (n > 0) {
    if (rec8)
      hipLaunchKernelGGL(tile_scatter_kernel<true>, dim3(G), dim3(1024), 0, s, uid, iid, rating, n, chunk, g,
                          KT, (const int32_t*)H, (const int32_t*)ptr, rec);
    else
      hipLaunchKernelGGL(tile_scatter_kernel<false>, dim3(G), dim3(1024), 0, s, uid, iid, rating, n, chunk, g,
                          KT, (const int32_t*)H, (const int32_t*)ptr, rec);
  }
  FPS_CHECK_LAUNCH();
  return 0;
}

// Two-level partition.  Workspace (int32): ccount[NC], ccursor[NC], cptr[NC+1],
// bcount[KT], bcursor[KT] (all zeroed here), tmp: n int4.  ptr[KT+1] = tile
// offsets, rec: n records {uid, row-in-block, rating bits, bucket}.
FPS_API int fps_tile_partition2(const int32_t* uid, const int32_t* iid, const float* rating, int64_t n, int W,
                                const int32_t* half, int R, int T, int P, int upp, int32_t* ws, int4* tmp, int32_t* ptr, void* rec,
                                int rec8, uint8_t* seen, void* stream) {
  const int KT = P * 2 * W * T;
  if (KT > TP_MAX_BUCKETS || R <= 0 || T <= 0) return (int)hipErrorInvalidValue;
  int cshift = 0;
  while (((KT - 1) >> cshift) + 1 > 128) ++cshift;  // ~128 coarse keys
  const int NC = ((KT - 1) >> cshift) + 1;
  const TileGeo g = make_geo(W, half, R, T, upp);
  hipStream_t s = (hipStream_t)stream;
  int32_t* ccount = ws;
  int32_t* ccursor = ccount + NC;
  int32_t* cptr = ccursor + NC;
  int32_t* bcount = cptr + NC + 1;
  int32_t* bcursor = bcount + KT;
  hipError_t e = hipMemsetAsync(ws, 0, sizeof(int32_t) * (size_t)(3 * NC + 1 + 2 * KT), s);
  if (e != hipSuccess) return (int)e;
  const int G = fps_tile_partition_groups(n);
  const int64_t chunk = (n + G - 1) / G;
  hipLaunchKernelGGL(tp2_count_kernel, dim3(G), dim3(1024), 0, s, uid, iid, n, chunk, g,  cshift, NC, KT,
                     ccount, bcount, seen);
  hipLaunchKernelGGL(tile_scan_kernel, dim3(1), dim3(1024), 0, s, (const int32_t*)ccount, NC, cptr);
  hipLaunchKernelGGL(tile_scan_kernel, dim3(1), dim3(1024), 0, s, (const int32_t*)bcount, KT, ptr);
  if (n > 0) {
    hipLaunchKernelGGL((tp2_scatter_kernel<1, false>), dim3(G), dim3(1024), 0, s, uid, iid, rating,
                       (const int4*)nullptr, n, chunk, g,  cshift, NC, (const int32_t*)cptr, ccursor,
                       (void*)tmp);
    if (rec8)
      hipLaunchKernelGGL((tp2_scatter_kernel<2, true>), dim3(G), dim3(1024), 0, s, uid, iid, rating,
                         (const int4*)tmp, n, chunk, g,  cshift, KT, (const int32_t*)ptr, bcursor, rec);
    else
      hipLaunchKernelGGL((tp2_scatter_kernel<2, false>), dim3(G), dim3(1024), 0, s, uid, iid, rating,
                         (const int4*)tmp, n, chunk, g,  cshift, KT, (const int32_t*)ptr, bcursor, rec);
  }
  FPS_CHECK_LAUNCH();
  return 0;
}

FPS_API int64_t fps_tile_partition2_ws_ints(int W, int T, int P) {
  const int KT = P * 2 * W * T;
  int cshift = 0;
  while (((KT - 1) >> cshift) + 1 > 128) ++cshift;
  const int NC = ((KT - 1) >> cshift) + 1;
  return 3 * (int64_t)NC + 1 + 2 * (int64_t)KT;
}

// Two-level partition with LDS-sorted batches (tp3 above).  Workspace (int32,
// fps_tile_partition3_ws_ints): ccount[NC], ccursor[NC], cptr[NC+1], bcount[KT],
// bcursor[KT], wptr[NC+1] (zeroed here); tmp: n int4.
static int tp3_cshift(int KT) {
  int cshift = 0;
  while (((KT - 1) >> cshift) + 1 > 128) ++cshift;  // ~128 coarse keys of <= 128 buckets
  return cshift;
}

FPS_API int64_t fps_tile_partition3_ws_ints(int W, int T, int P) {
  const int KT = P * 2 * W * T;
  const int NC = ((KT - 1) >> tp3_cshift(KT)) + 1;
  // + H1[G <= 1024][NC] + fine histograms [1 + 512][KT]
  return 4 * (int64_t)NC + 2 + 2 * (int64_t)KT + 1024 * (int64_t)NC + 513 * (int64_t)KT;
}

FPS_API int fps_tile_partition3(const int32_t* uid, const int32_t* iid, const float* rating, int64_t n, int W,
                                const int32_t* half, int R, int T, int P, int upp, int32_t* ws, int4* tmp, int32_t* ptr, void* rec,
                                int rec8, uint8_t* seen, void* stream) {
  const int KT = P * 2 * W * T;
  if (KT > TP_MAX_BUCKETS || R <= 0 || T <= 0) return (int)hipErrorInvalidValue;
  const int cshift = tp3_cshift(KT);
  const int NC = ((KT - 1) >> cshift) + 1;
  if (NC > TP3_MAXK || (1 << cshift) > TP3_MAXK) return (int)hipErrorInvalidValue;
  const TileGeo g = make_geo(W, half, R, T, upp);
  hipStream_t s = (hipStream_t)stream;
  int32_t* ccount = ws;
  int32_t* ccursor = ccount + NC;
  int32_t* cptr = ccursor + NC;
  int32_t* bcount = cptr + NC + 1;
  int32_t* bcursor = bcount + KT;
  int32_t* wptr = bcursor + KT;
  int32_t* H1 = wptr + NC + 1;
  hipError_t e = hipMemsetAsync(ws, 0, sizeof(int32_t) * (size_t)(4 * NC + 2 + 2 * KT), s);
  if (e != hipSuccess) return (int)e;
  const int G = tp3_groups(n, KT);
  const int64_t chunk = (n + G - 1) / G;
  const int sub = (G + 511) / 512;  // <= 512 count workgroups (2 per CU)
  const int Gc = (G + sub - 1) / sub;
  int32_t* bhist = H1 + 1024 * (int64_t)NC;  // [1 + Gc][KT]: totals, then one row per count workgroup
  hipLaunchKernelGGL(tp3_count_kernel, dim3(Gc), dim3(1024), 0, s, uid, iid, n, chunk, G, sub, g, cshift, NC, KT, ccount, bhist, seen, H1);
  hipLaunchKernelGGL(tp3_colsum_kernel, dim3((KT + 63) / 64), dim3(1024), 0, s, bhist, Gc, KT);
  bcount = bhist;
  hipLaunchKernelGGL(tile_scan_kernel, dim3(1), dim3(1024), 0, s, (const int32_t*)ccount, NC, cptr);
  hipLaunchKernelGGL(tile_scan_kernel, dim3(1), dim3(1024), 0, s, (const int32_t*)bcount, KT, ptr);
  hipLaunchKernelGGL(tp3_colscan_kernel, dim3(NC), dim3(1024), 0, s, H1, G, NC, (const int32_t*)cptr);
  hipLaunchKernelGGL(tp3_workptr_kernel, dim3(1), dim3(64), 0, s, (const int32_t*)ccount, NC, wptr);
  if (n > 0) {
    int64_t g2 = n / TP3_CH + NC + 1;  // >= the number of work items
    // (capping the level-2 workgroups at 512 / 256 instead: no gain, profiles/r2_partition.md)
    if (g2 > 1024) g2 = 1024;
    // FPS_TP3_PIPE=1: the scatters with the register prefetch of the next batch --
    // measured slower (level 1: 530 vs 401 us per 64M ratings, bench 9.73-9.76e9 vs
    // 9.75-9.78e9, profiles/r2_partition.md), so off by default
    static const bool pipe = [] { const char* e = getenv("FPS_TP3_PIPE"); return e && e[0] == '1'; }();
    const int ntm = tp_nt();
#define FPS_TP3(L, R8, GRID, TMP, KPTR, CUR, H1P, OUT)                                                            \
    if (pipe) hipLaunchKernelGGL((tp3_scatter_kernel<L, R8, true>), dim3(GRID), dim3(1024), 0, s, uid, iid, rating, \
                                 TMP, n, chunk, g, cshift, NC, KT, KPTR, CUR, (const int32_t*)cptr,                \
                                 (const int32_t*)wptr, H1P, OUT);                                                  \
    else if (ntm == 1) hipLaunchKernelGGL((tp3_scatter_kernel<L, R8, false, 1>), dim3(GRID), dim3(1024), 0, s, uid, \
                                    iid, rating, TMP, n, chunk, g, cshift, NC, KT, KPTR, CUR, (const int32_t*)cptr, \
                                    (const int32_t*)wptr, H1P, OUT);                                               \
    else if (ntm == 2) hipLaunchKernelGGL((tp3_scatter_kernel<L, R8, false, 2>), dim3(GRID), dim3(1024), 0, s, uid, \
                                    iid, rating, TMP, n, chunk, g, cshift, NC, KT, KPTR, CUR, (const int32_t*)cptr, \
                                    (const int32_t*)wptr, H1P, OUT);                                               \
    else hipLaunchKernelGGL((tp3_scatter_kernel<L, R8, false>), dim3(GRID), dim3(1024), 0, s, uid, iid, rating,     \
                            TMP, n, chunk, g, cshift, NC, KT, KPTR, CUR, (const int32_t*)cptr, (const int32_t*)wptr, \
                            H1P, OUT)
    if (rec8) { FPS_TP3(1, true, G, (const int4*)nullptr, (const int32_t*)cptr, ccursor, (const int32_t*)H1, (void*)tmp); }
    else { FPS_TP3(1, false, G, (const int4*)nullptr, (const int32_t*)cptr, ccursor, (const int32_t*)H1, (void*)tmp); }
    if (rec8) { FPS_TP3(2, true, (int)g2, (const int4*)tmp, (const int32_t*)ptr, bcursor, (const int32_t*)nullptr, rec); }
    else { FPS_TP3(2, false, (int)g2, (const int4*)tmp, (const int32_t*)ptr, bcursor, (const int32_t*)nullptr, rec); }
#undef FPS_TP3
  }
  FPS_CHECK_LAUNCH();
  return 0;
}

// One launch per item block: T tiles of R (<= 256) rows of I[block_rows, D];
// ptr = the block's T+1 tile offsets (device).  D must be 16, 32, 64, 128 or 256.
FPS_API int fps_mf_sgd_tiled2(float* U, float* I, const void* rec, int rec8, const int32_t* ptr, int T, int R,
                              int64_t block_rows, float* I1, int64_t block_rows1, int nblk, int D, float lr,
                              float lambda, void* stream);

FPS_API int fps_mf_sgd_tiled(float* U, float* I, const void* rec, int rec8, const int32_t* ptr, int T, int R,
                             int64_t block_rows, int D, float lr, float lambda, void* stream) {
  return fps_mf_sgd_tiled2(U, I, rec, rec8, ptr, T, R, block_rows, I, block_rows, 1, D, lr, lambda, stream);
}

// nblk = 2: tiles ptr[0..2T] of two consecutive item blocks (I: block_rows, I1:
// block_rows1) in one launch of 2T workgroups.
FPS_API int fps_mf_sgd_tiled3(float* U, float* I, const void* rec, int rec8, const int32_t* ptr,
                              const int32_t* tcnt, int T, int R, int64_t block_rows, float* I1, int64_t block_rows1,
                              int nblk, int D, float lr, float lambda, void* stream);

FPS_API int fps_mf_sgd_tiled2(float* U, float* I, const void* rec, int rec8, const int32_t* ptr, int T, int R,
                              int64_t block_rows, float* I1, int64_t block_rows1, int nblk, int D, float lr,
                              float lambda, void* stream) {
  return fps_mf_sgd_tiled3(U, I, rec, rec8, ptr, nullptr, T, R, block_rows, I1, block_rows1, nblk, D, lr, lambda,
                           stream);
}

// tcnt (tp4 slots, may be null): per-tile record counts, ptr = the slot starts
FPS_API int fps_mf_sgd_tiled3(float* U, float* I, const void* rec, int rec8, const int32_t* ptr,
                              const int32_t* tcnt, int T, int R, int64_t block_rows, float* I1, int64_t block_rows1,
                              int nblk, int D, float lr, float lambda, void* stream) {
  if (T <= 0) return 0;
  if (nblk != 1 && nblk != 2) return (int)hipErrorInvalidValue;
  const int grid = nblk * T;
  if (R <= 0 || R > TG_MAX_R) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  constexpr int PF = 8;
  // FPS_MF_PIPE=1 (A/B): 4 user rows per batch, the next batch requested before this
  // batch's stores (same registers as 8 rows per batch without the pipeline)
  static const bool pipe = [] { const char* e = std::getenv("FPS_MF_PIPE"); return e && e[0] == '1'; }();
  // FPS_SGD_NT=0: item rows with plain accesses (A/B)
  static const bool nti = [] { const char* e = std::getenv("FPS_SGD_NT"); return !(e && e[0] == '0'); }();
#define FPS_TILED(TPR_, V_)                                                                                    \
  if (pipe && rec8) hipLaunchKernelGGL((mf_sgd_tilegroup_kernel<TPR_, V_, PF / 2, true, true>), dim3(grid),   \
                                       dim3(512), 0, s, U, I, rec, ptr, R, block_rows, lr, lambda, I1,         \
                                       block_rows1, T, tcnt);                                                  \
  else if (rec8 && nti) hipLaunchKernelGGL((mf_sgd_tilegroup_kernel<TPR_, V_, PF, true, false, true>), dim3(grid), \
                                           dim3(512), 0, s, U, I, rec, ptr, R, block_rows, lr, lambda, I1,     \
                                           block_rows1, T, tcnt);                                              \
  else if (rec8) hipLaunchKernelGGL((mf_sgd_tilegroup_kernel<TPR_, V_, PF, true>), dim3(grid), dim3(512), 0, s, \
                                    U, I, rec, ptr, R, block_rows, lr, lambda, I1, block_rows1, T, tcnt);      \
  else hipLaunchKernelGGL((mf_sgd_tilegroup_kernel<TPR_, V_, PF, false>), dim3(grid), dim3(512), 0, s, U, I,    \
                          rec, ptr, R, block_rows, lr, lambda, I1, block_rows1, T, tcnt)
  switch (D) {
    case 16: FPS_TILED(4, 1); break;
    case 32: FPS_TILED(8, 1); break;
    case 64: FPS_TILED(16, 1); break;
    case 128: FPS_TILED(16, 2); break;
    case 256: FPS_TILED(16, 4); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef FPS_TILED
  FPS_CHECK_LAUNCH();
  return 0;
}

// ---- tp4 host side.  Workspace (int32, fps_tile_partition4_ws_ints): cstart[NC+1],
// ccursor[NC], wptr[NC+1]; bstart[KT+1] / bcursor[KT] are the caller's (the SGD
// reads them: slot starts and counts); tmp holds fps_tile_partition4_cap(n, NC)
// 12- or 16-B records, rec fps_tile_partition4_cap(n, KT) 8- or 16-B records,
// ovf n 16-B records.  n_prev: the n of this partitioner's previous run (0: first),
// whose cursors (still in ccursor / bcursor) size this run's slots.
FPS_API int64_t fps_tile_partition4_ws_ints(int W, int T, int P) {
  const int KT = P * 2 * W * T;
  const int NC = ((KT - 1) >> tp3_cshift(KT)) + 1;
  return 3 * (int64_t)NC + 2;
}

FPS_API int64_t fps_tile_partition4_cap(int64_t n, int K) {
  return (int64_t)((double)n * TP4_SLACK) + (int64_t)K * (TP4_PAD + 1) + 16;
}

FPS_API int fps_tile_partition4(const int32_t* uid, const int32_t* iid, const float* rating, int64_t n,
                                int64_t n_prev, int W, const int32_t* half, int R, int T, int P, int upp,
                                int32_t* ws, void* tmp, int32_t* bstart, int32_t* bcursor, void* rec, int rec8,
                                int4* ovf, int32_t* ovf_cnt, uint8_t* seen, void* stream) {
  const int KT = P * 2 * W * T;
  if (KT > TP_MAX_BUCKETS || R <= 0 || T <= 0) return (int)hipErrorInvalidValue;
  const int cshift = tp3_cshift(KT);
  const int NC = ((KT - 1) >> cshift) + 1;
  if (NC > TP3_MAXK || (1 << cshift) > TP3_MAXK) return (int)hipErrorInvalidValue;
  const TileGeo g = make_geo(W, half, R, T, upp);
  hipStream_t s = (hipStream_t)stream;
  int32_t* cstart = ws;
  int32_t* ccursor = cstart + NC + 1;
  int32_t* wptr = ccursor + NC;
  // slots from the previous run's cursors, then zero the cursors
  hipLaunchKernelGGL(tp4_plan_kernel, dim3(1), dim3(1024), 0, s, (const int32_t*)ccursor, NC, n_prev, n, cstart);
  hipLaunchKernelGGL(tp4_plan_kernel, dim3(1), dim3(1024), 0, s, (const int32_t*)bcursor, KT, n_prev, n, bstart);
  hipError_t e = hipMemsetAsync(ccursor, 0, sizeof(int32_t) * (size_t)NC, s);
  if (e == hipSuccess) e = hipMemsetAsync(bcursor, 0, sizeof(int32_t) * (size_t)KT, s);
  if (e == hipSuccess) e = hipMemsetAsync(ovf_cnt, 0, sizeof(int32_t), s);
  if (e != hipSuccess) return (int)e;
  if (n > 0) {
    const int G = fps_tile_partition_groups(n);
    const int64_t chunk = (n + G - 1) / G;
#define FPS_TP4_L1(R8)                                                                                         \
    hipLaunchKernelGGL((tp4_scatter_kernel<1, R8>), dim3(G), dim3(1024), 0, s, uid, iid, rating,             \
                       (const void*)nullptr, n, chunk, g, cshift, NC, KT, (const int32_t*)cstart, ccursor,    \
                       (const int32_t*)cstart, (const int32_t*)ccursor, (const int32_t*)wptr, tmp, ovf, ovf_cnt, \
                       seen)
    if (rec8) FPS_TP4_L1(true); else FPS_TP4_L1(false);
#undef FPS_TP4_L1
    hipLaunchKernelGGL(tp4_workptr_kernel, dim3(1), dim3(64), 0, s, (const int32_t*)ccursor, (const int32_t*)cstart,
                       NC, wptr);
    int64_t g2 = n / TP3_CH + NC + 1;  // >= the number of work items
    // (capping the level-2 workgroups at 512 / 256 instead: no gain, profiles/r2_partition.md)
    if (g2 > 1024) g2 = 1024;
#define FPS_TP4_L2(R8)                                                                                         \
    hipLaunchKernelGGL((tp4_scatter_kernel<2, R8>), dim3((int)g2), dim3(1024), 0, s, uid, iid, rating,        \
                       (const void*)tmp, n, (int64_t)0, g, cshift, NC, KT, (const int32_t*)bstart, bcursor,     \
                       (const int32_t*)cstart, (const int32_t*)ccursor, (const int32_t*)wptr, rec, ovf, ovf_cnt,  \
                       (uint8_t*)nullptr)
    if (rec8) FPS_TP4_L2(true); else FPS_TP4_L2(false);
#undef FPS_TP4_L2
  }
  FPS_CHECK_LAUNCH();
  return 0;
}

// Overflow records of buckets [b_lo, b_lo + nblk*T) (item rows I0: first block, I1: second)
FPS_API int fps_mf_sgd_ovf(float* U, float* I0, float* I1, const int4* ovf, const int32_t* ovf_cnt, int b_lo, int T,
                           int nblk, int D, float lr, float lambda, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int grid = 512;  // fixed: the count lives on the device
#define FPS_OVF(TPR_, V_) hipLaunchKernelGGL((tp4_ovf_sgd_kernel<TPR_, V_>), dim3(grid), dim3(256), 0, s, U, I0, I1, \
                                             ovf, ovf_cnt, b_lo, T, nblk, lr, lambda)
  switch (D) {
    case 16: FPS_OVF(4, 1); break;
    case 32: FPS_OVF(8, 1); break;
    case 64: FPS_OVF(16, 1); break;
    case 128: FPS_OVF(16, 2); break;
    case 256: FPS_OVF(16, 4); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef FPS_OVF
  FPS_CHECK_LAUNCH();
  return 0;
}

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
  FastDiv dW, dR, dU, dT, d2W;
  const int32_t* half;
  int32_t nu, ni;  // valid local user / item ids: [0, nu) x [0, ni); a rating outside is dropped
};

static TileGeo make_geo(int W, const int32_t* half, int R, int T, int upp, int nu, int ni) {
  return TileGeo{W, R, T, make_fastdiv(W), make_fastdiv(R), make_fastdiv(upp), make_fastdiv(T), make_fastdiv(2 * W),
                 half, nu > 0 ? nu : INT32_MAX, ni > 0 ? ni : INT32_MAX};
}

// a rating the partition may bucket: an out-of-range id would index past the bucket
// counters here and past the tables in the SGD (a device fault), so it is dropped
__device__ __forceinline__ bool tile_valid(int32_t i, int32_t u, const TileGeo& g) {
  return (uint32_t)i < (uint32_t)g.ni && (uint32_t)u < (uint32_t)g.nu;
}

// the global item of a record from its bucket and row in block (tile_bucket's inverse)
__device__ __forceinline__ int32_t tile_item(int bucket, int32_t row_in_block, const TileGeo& g) {
  const int32_t a = g.dT.div(bucket);                // user phase * 2W + 2q + h
  const int32_t b = a - g.d2W.div(a) * (2 * g.W);    // 2q + h
  const int q = b >> 1;
  const int32_t loc = row_in_block + ((b & 1) ? g.half[q] : 0);
  return loc * g.W + q;
}

__device__ __forceinline__ void tile_bucket(int32_t i, int32_t u, const TileGeo& g, int& bucket, int32_t& row) {
  const int32_t loc = g.dW.div(i);
  const int q = i - loc * g.W;
  const int32_t hq = g.half[q];
  const int h = loc >= hq;
  row = loc - (h ? hq : 0);
  bucket = (g.dU.div(u) * 2 * g.W + 2 * q + h) * g.T + g.dR.div(row);  // user phase, item block, tile
}

// LDS counters of the count kernel: KT ints of dynamic LDS (64 KiB at KT = 16k: two
// 1024-thread workgroups per CU; up to 128 KiB -- a workgroup may declare 160 KiB)
constexpr int TP_MAX_BUCKETS = 32768;

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

// K3: exclusive scan of KT totals into ptr[KT+1] (one 1024-thread workgroup).  No
// staging of the totals in LDS: a 128 KiB static LDS array made this one-workgroup
// launch wait for a CU with that much free LDS while the SGD workgroups of the
// previous step held them (0.45 ms average, 1.2 ms max on the side stream,
// profiles/r4_final_bench_kernel_stats.csv); it now needs 64 B of LDS and runs
// beside them.  Each thread sums `per` consecutive totals from global memory, the
// 1024 partial sums are scanned by wave shuffles + 16 wave totals.
__global__ void __launch_bounds__(1024) tile_scan_kernel(const int32_t* __restrict__ totals, int KT,
                                                         int32_t* __restrict__ ptr) {
  __shared__ int32_t wsum[16];
  const int per = (KT + 1023) / 1024;
  const int k0 = threadIdx.x * per, k1 = min(KT, k0 + per);
  int32_t s = 0;
  for (int k = k0; k < k1; ++k) s += totals[k];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int32_t inc = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int32_t y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  if (lane == 63) wsum[wv] = inc;
  __syncthreads();
  int32_t run = inc - s;
  for (int q = 0; q < wv; ++q) run += wsum[q];
  for (int k = k0; k < k1; ++k) { const int32_t t = totals[k]; ptr[k] = run; run += t; }
  if (threadIdx.x == 1023) {
    int32_t tot = 0;
    for (int q = 0; q < 16; ++q) tot += wsum[q];
    ptr[KT] = tot;
  }
}

// Packed rating records.  REC8 (users < 2^24, R <= 256): 8 B {uid | row_in_tile << 24,
// rating bits}; else 16 B {uid, row-in-block, rating bits, bucket}.
template <bool REC8>
__device__ __forceinline__ void put_rec(void* rec, int64_t o, int32_t uid, int32_t row, float rating, int bucket,
                                        int R) {
  if (REC8) reinterpret_cast<int2*>(rec)[o] = make_int2(uid | ((row & (R - 1)) << 24), __float_as_int(rating));
  else reinterpret_cast<int4*>(rec)[o] = make_int4(uid, row, __float_as_int(rating), bucket);
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
//
// H16: two 16-bit counters per LDS word (KT / 2 words: 62.5 KiB instead of 125 KiB
// at the N = 8 layout's 31k buckets, so a count workgroup leaves room for two
// tile-SGD workgroups on its CU -- the partition of batch k+1 runs beside the SGD
// of batch k, profiles/r3_emulate8_timeline.md).  Overflow-safe: the ratings are
// counted in sub-batches of H16_SB per workgroup; a counter that reaches 2^15 sets a
// flag, and at the next sub-batch boundary the whole histogram is flushed into the
// workgroup's global row (which then accumulates) and zeroed.  A counter is below
// 2^15 at the start of every sub-batch and grows by at most H16_SB = 2^15 in it,
// so it never exceeds 2^16 - 1.  Uniform keys never flush (~8 counts per bucket).
constexpr int H16_SB = 32768;
// FPS_TP_NORET=1: the 16-bit counters are incremented with non-returning LDS atomics and
// the "a counter reached 2^15" test reads the histogram at each sub-batch end (KT / 2
// words, 128-bit reads) instead of every returned old value (A/B knob)
#ifndef FPS_TP_NORET
#define FPS_TP_NORET 0
#endif

template <bool H16>
__device__ __forceinline__ int32_t hb_get(const int32_t* hb, int b) {
  if constexpr (H16) return (int32_t)(((uint32_t)hb[b >> 1] >> ((b & 1) << 4)) & 0xffffu);
  else return hb[b];
}

// The partition kernels come in two shapes (``fps_tile_partition_set_slim``):
//  * fat: 1024-thread workgroups (the round-1..5 shape), fastest alone;
//  * slim: 256-thread workgroups of <= 32 VGPRs and <= ~35 KiB of LDS.  The tile SGD
//    beside which the partition of the next batch runs holds 3 workgroups per CU at
//    80 VGPRs (6 of 8 waves per SIMD, 480 of 512 registers, 114 KiB of LDS); a fat
//    partition workgroup fits only where one of them left, so every one displaced a
//    third of a CU's SGD.  A slim one fits in what the three leave free (one wave per
//    SIMD, 32 registers, 46 KiB): the partition then takes memory bandwidth from the SGD
//    but no occupancy.
template <bool H16, int BS, int U4>
__device__ __forceinline__ void tp3_count_body(const int32_t* __restrict__ uid, const int32_t* __restrict__ iid,
                                               int64_t n, int64_t chunk, int G, int sub, const TileGeo& g, int cshift,
                                               int NC, int KT, int32_t* __restrict__ ccount,
                                               int32_t* __restrict__ bcount, int32_t* __restrict__ H1) {
  // One LDS atomic per rating (LDS atomics run at ~1 lane per CU cycle and
  // bound this kernel); the coarse counts of a chunk are read off the fine
  // histogram afterwards: 8 lanes per coarse key sum its 2^cshift buckets.
  extern __shared__ __attribute__((aligned(16))) int32_t hb[];  // [KT] ints, or [ceil(KT / 2)] words of two 16-bit counters (dynamic LDS)
  __shared__ int32_t hc_prev[TP3_MAXK], hc_acc[TP3_MAXK];
  __shared__ int32_t s_ovf, s_flushed;
  const int KW = H16 ? (KT + 1) / 2 : KT;
  for (int k = threadIdx.x; k < KW; k += BS) hb[k] = 0;
  for (int k = threadIdx.x; k < NC; k += BS) { hc_prev[k] = 0; hc_acc[k] = 0; }
  if (threadIdx.x == 0) { s_ovf = 0; s_flushed = 0; }
  __syncthreads();
  int32_t* Hf = bcount + (int64_t)(blockIdx.x + 1) * KT;  // row 0 = the totals (tp3_colsum_kernel)
  const int span = 1 << cshift;
  const int per = (span + 7) / 8;
  const int cl = threadIdx.x & 7;  // lane in a coarse key's group of 8
  // coarse key ck's count now (summed by its 8 lanes; every lane of the group gets the total)
  auto coarse_now = [&](int ck) {
    int32_t tot = 0;
    if (ck < NC)
      for (int q = 0; q < per; ++q) {
        const int b = (ck << cshift) + cl * per + q;
        if (cl * per + q < span && b < KT) tot += hb_get<H16>(hb, b);
      }
    tot += __shfl_xor(tot, 1, 64);
    tot += __shfl_xor(tot, 2, 64);
    tot += __shfl_xor(tot, 4, 64);
    return tot;
  };
  // the coarse keys of this thread's group of 8 (NC <= 256: one pass at BS = 1024 and NC <= 128)
  constexpr int CKS = BS / 8;
  const int c0 = blockIdx.x * sub, c1 = min(G, c0 + sub);
  for (int c = c0; c < c1; ++c) {
    const int64_t lo = (int64_t)c * chunk, hi = min(n, lo + chunk);
    // U4: loads in flight per thread (a lone dependent load pair per iteration left the
    // kernel latency-bound at ~1.7 TB/s)
    const int64_t step = (int64_t)U4 * BS;
    for (int64_t s0 = lo; s0 < hi; s0 += (H16 ? H16_SB : hi - lo)) {
      const int64_t s1 = H16 ? min(hi, s0 + H16_SB) : hi;
      for (int64_t x0 = s0 + threadIdx.x; x0 < s1; x0 += step) {
        int32_t iv[U4], uv[U4];
#pragma unroll
        for (int j = 0; j < U4; ++j) {
          const int64_t x = x0 + (int64_t)j * BS;
          iv[j] = x < s1 ? iid[x] : -1;
          uv[j] = x < s1 ? uid[x] : 0;
        }
#pragma unroll
        for (int j = 0; j < U4; ++j) {
          if (iv[j] < 0 || !tile_valid(iv[j], uv[j], g)) continue;
          int bk; int32_t row;
          tile_bucket(iv[j], uv[j], g, bk, row);
          if constexpr (H16) {
            const int sh = (bk & 1) << 4;
#if FPS_TP_NORET
            atomicAdd(reinterpret_cast<uint32_t*>(hb) + (bk >> 1), 1u << sh);
#else
            const uint32_t old = atomicAdd(reinterpret_cast<uint32_t*>(hb) + (bk >> 1), 1u << sh);
            if (((old >> sh) & 0xffffu) >= 32767u) s_ovf = 1;  // this counter reached 2^15
#endif
          } else {
            atomicAdd(hb + bk, 1);
          }
        }
      }
      if constexpr (H16) {
        __syncthreads();
#if FPS_TP_NORET
        {  // any counter >= 2^15?  (KW words; 4 per 128-bit read where aligned)
          bool hit = false;
          const int KW4 = KW >> 2;
          const uint4* h4 = reinterpret_cast<const uint4*>(hb);
          for (int k = threadIdx.x; k < KW4; k += BS) {
            const uint4 w = h4[k];
            hit |= ((w.x | w.y | w.z | w.w) & 0x80008000u) != 0u;
          }
          for (int k = 4 * KW4 + threadIdx.x; k < KW; k += BS) hit |= (hb[k] & 0x80008000u) != 0u;
          if (hit) s_ovf = 1;
        }
        __syncthreads();
#endif
        const bool ovf = s_ovf;
        // every thread has read the flag before any can start the next sub-batch and set it again
        __syncthreads();
        if (ovf) {  // uniform: flush the histogram into the global row and restart it at zero
          for (int ck0 = 0; ck0 < NC; ck0 += CKS) {
            const int ck = ck0 + (threadIdx.x >> 3);
            const int32_t tot = coarse_now(ck);
            if (ck < NC && cl == 0) { hc_acc[ck] += tot - hc_prev[ck]; hc_prev[ck] = 0; }
          }
          const bool first = !s_flushed;
          for (int k = threadIdx.x; k < KT; k += BS) Hf[k] = (first ? 0 : Hf[k]) + hb_get<true>(hb, k);
          __syncthreads();
          for (int k = threadIdx.x; k < KW; k += BS) hb[k] = 0;
          if (threadIdx.x == 0) { s_ovf = 0; s_flushed = 1; }
          __syncthreads();
        }
      }
    }
    __syncthreads();
    for (int ck0 = 0; ck0 < NC; ck0 += CKS) {
      const int ck = ck0 + (threadIdx.x >> 3);
      const int32_t tot = coarse_now(ck);
      if (ck < NC && cl == 0) {
        const int32_t v = hc_acc[ck] + tot - hc_prev[ck];
        hc_prev[ck] = tot;
        hc_acc[ck] = 0;
        if (v) atomicAdd(ccount + ck, v);
        H1[(int64_t)c * NC + ck] = v;
      }
    }
    __syncthreads();  // hb is read above before the next chunk adds to it
  }
  const bool flushed = s_flushed;
  for (int k = threadIdx.x; k < KT; k += BS) Hf[k] = (flushed ? Hf[k] : 0) + hb_get<H16>(hb, k);
}

template <bool H16>
__global__ void __launch_bounds__(1024) tp3_count_kernel(const int32_t* __restrict__ uid,
                                                         const int32_t* __restrict__ iid, int64_t n, int64_t chunk,
                                                         int G, int sub, TileGeo g, int cshift, int NC, int KT,
                                                         int32_t* __restrict__ ccount, int32_t* __restrict__ bcount,
                                                         uint8_t* __restrict__ seen, int32_t* __restrict__ H1) {
  tp3_count_body<H16, 1024, 8>(uid, iid, n, chunk, G, sub, g, cshift, NC, KT, ccount, bcount, H1);
}

template <bool H16>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_num_vgpr(32)))
tp3_count_slim_kernel(const int32_t* __restrict__ uid, const int32_t* __restrict__ iid, int64_t n, int64_t chunk,
                      int G, int sub, TileGeo g, int cshift, int NC, int KT, int32_t* __restrict__ ccount,
                      int32_t* __restrict__ bcount, uint8_t* __restrict__ seen, int32_t* __restrict__ H1) {
  tp3_count_body<H16, 256, 4>(uid, iid, n, chunk, G, sub, g, cshift, NC, KT, ccount, bcount, H1);
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

// work items of level 2: wptr[c] = sum over c' < c of ceil(ccount[c'] / CH); one wave,
// 4 coarse keys per lane (NC <= 256) and a shuffle scan (was one thread walking NC
// dependent loads)
__global__ void tp3_workptr_kernel(const int32_t* __restrict__ ccount, int NC, int32_t* __restrict__ wptr) {
  if (threadIdx.x >= 64) return;
  const int l = threadIdx.x;
  int32_t v[4], s = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = 4 * l + q;
    v[q] = c < NC ? (ccount[c] + TP3_CH - 1) / TP3_CH : 0;
    s += v[q];
  }
  int32_t inc = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int32_t y = __shfl_up(inc, o, 64);
    if (l >= o) inc += y;
  }
  int32_t run = inc - s;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = 4 * l + q;
    if (c < NC) wptr[c] = run;
    run += v[q];
  }
  if (l == 63) wptr[NC] = inc;
}


// LEVEL 1: (uid, iid, rating)[chunk of this workgroup] -> tmp grouped by coarse key
//          (bucket >> cshift); kptr = cptr, cursor = ccursor.  tmp records: REC8
//          12 B {uid | row_in_tile << 24, rating bits, bucket} (three dwords), else
//          16 B {uid, row, rating bits, bucket}
// LEVEL 2: tmp[work item] -> out (8- or 16-B records) grouped by bucket; kptr = ptr,
//          cursor = bcursor; work items from wptr / cptr
// Every access is non-temporal: the inputs are read once and the outputs are read by
// the next step's SGD long after any cache kept them, so streaming them keeps the L2
// / Infinity Cache for the SGD's user rows (+2 % end to end, profiles/r2_partition.md;
// a register prefetch of the next batch and 16-B level-1 slots were measured slower
// and removed in round 3).
// BS threads, B records per LDS batch (fat: 1024 / TP3_B; slim: 256 / 1024)
template <int LEVEL, bool REC8, int BS, int B>
__device__ __forceinline__ void tp3_scatter_body(const int32_t* __restrict__ uid, const int32_t* __restrict__ iid,
                                                 const float* __restrict__ rating, const int4* __restrict__ tmp,
                                                 int64_t n, int64_t chunk, const TileGeo& g, int cshift, int NC,
                                                 int KT, const int32_t* __restrict__ kptr,
                                                 int32_t* __restrict__ cursor, const int32_t* __restrict__ cptr,
                                                 const int32_t* __restrict__ wptr, const int32_t* __restrict__ H1,
                                                 void* __restrict__ out, uint8_t* __restrict__ seen) {
  static_assert(BS >= TP3_MAXK, "one thread per key of a batch sort (nk <= TP3_MAXK)");
  constexpr int E = B / BS;
  __shared__ int4 srt[B];
  __shared__ int32_t cnt[TP3_MAXK], off[TP3_MAXK], base[TP3_MAXK];
  __shared__ int32_t s_item[3];  // level 2: lo, hi, key base of the current work item
  const int tid = threadIdx.x;
  // level 1: one work item per chunk (a grid smaller than the chunk count loops);
  // level 2: the work items of wptr
  const int nwork = LEVEL == 1 ? (int)((n + chunk - 1) / chunk) : wptr[NC];
  for (int w = blockIdx.x; w < nwork; w += gridDim.x) {
    int64_t lo, hi;
    int kb, nk;
    if (LEVEL == 1) {
      lo = (int64_t)w * chunk;
      hi = min(n, lo + chunk);
      kb = 0;
      nk = NC;
      if (tid < nk) base[tid] = H1[(int64_t)w * NC + tid];  // this chunk's run starts
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
    for (int64_t b0 = lo; b0 < hi; b0 += B) {
      const int nb = (int)min((int64_t)B, hi - b0);
      if (tid < nk) cnt[tid] = 0;
      int4 r[E];
      int k[E], slot[E];
      bool ok[E];
#pragma unroll
      for (int e = 0; e < E; ++e) {  // this batch's records
        k[e] = 0;
        const int p = e * BS + tid;
        ok[e] = p < nb;
        if (p >= nb) continue;
        const int64_t x = b0 + p;
        if (LEVEL == 1) {
          const int32_t u = tp_ld<true>(uid + x), i = tp_ld<true>(iid + x);
          const int32_t rb = __float_as_int(tp_ld<true>(rating + x));
          ok[e] = tile_valid(i, u, g);  // the count pass skipped it too
          if (!ok[e]) continue;
          int bk; int32_t row;
          tile_bucket(i, u, g, bk, row);
          if (REC8) r[e] = make_int4(u | ((row & (g.R - 1)) << 24), rb, bk, 0);
          else r[e] = make_int4(u, row, rb, bk);
          k[e] = bk >> cshift;
        } else if (REC8) {
          const int* q = reinterpret_cast<const int*>(tmp) + 3 * x;
          r[e] = make_int4(tp_ld<true>(q), tp_ld<true>(q + 1), tp_ld<true>(q + 2), 0);
          k[e] = r[e].z - kb;
        } else {
          const tp_i4 t = tp_ld<true>(reinterpret_cast<const tp_i4*>(tmp) + x);
          r[e] = make_int4(t.x, t.y, t.z, t.w);
          k[e] = r[e].w - kb;
        }
      }
      __syncthreads();  // cnt zeroed
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int p = e * BS + tid;
        slot[e] = ok[e] ? atomicAdd(cnt + k[e], 1) : -1;
      }
      __syncthreads();
      tp3_scan(cnt, off, nk);
      if (LEVEL == 2 && tid < nk && cnt[tid]) base[tid] = kptr[kb + tid] + atomicAdd(cursor + kb + tid, cnt[tid]);
      __syncthreads();
#pragma unroll
      for (int e = 0; e < E; ++e)
        if (slot[e] >= 0) srt[off[k[e]] + slot[e]] = r[e];
      __syncthreads();
      const int nv = off[nk - 1] + cnt[nk - 1];  // records kept (level 1 drops invalid ones)
      for (int p = tid; p < nv; p += BS) {
        const int4 x = srt[p];
        const int bk = REC8 ? x.z : x.w;
        const int kk = LEVEL == 1 ? (bk >> cshift) : bk - kb;
        const int64_t o = (int64_t)base[kk] + (p - off[kk]);
        if (LEVEL == 1 && REC8) {
          int* q = reinterpret_cast<int*>(out) + 3 * o;
          tp_st<true>(q, x.x);
          tp_st<true>(q + 1, x.y);
          tp_st<true>(q + 2, x.z);
        } else if (LEVEL == 1) tp_st<true>(reinterpret_cast<tp_i4*>(out) + o, tp_i4{x.x, x.y, x.z, x.w});
        else if (REC8) tp_st<true>(reinterpret_cast<tp_i2*>(out) + o, tp_i2{x.x, x.y});
        else put_rec<false>(out, o, x.x, x.y, __int_as_float(x.z), x.w, g.R);
        if (LEVEL == 2 && seen != nullptr) {
          // the batch's items (presence / touched flags), marked here rather than in the
          // count pass: the records leave the sort grouped by tile, so a wave's 64 byte
          // stores fall in a tile's few hundred bytes instead of 64 random lines (the count
          // pass's per-rating random byte stores slowed the SGD beside it:
          // profiles/r5_presence_ab.txt)
          const int32_t rib = REC8 ? (int32_t)(bk - g.dT.div(bk) * g.T) * g.R + (int32_t)((uint32_t)x.x >> 24) : x.y;
          seen[tile_item(bk, rib, g)] = 1;
        }
      }
      __syncthreads();  // LDS reused by the next batch
      if (LEVEL == 1 && tid < nk) base[tid] += cnt[tid];  // same thread zeroes cnt[tid] next
    }
  }
}


template <int LEVEL, bool REC8>
__global__ void __launch_bounds__(1024) tp3_scatter_kernel(const int32_t* __restrict__ uid,
                                                           const int32_t* __restrict__ iid,
                                                           const float* __restrict__ rating,
                                                           const int4* __restrict__ tmp, int64_t n, int64_t chunk,
                                                           TileGeo g, int cshift, int NC, int KT,
                                                           const int32_t* __restrict__ kptr,
                                                           int32_t* __restrict__ cursor,
                                                           const int32_t* __restrict__ cptr,
                                                           const int32_t* __restrict__ wptr,
                                                           const int32_t* __restrict__ H1,
                                                           void* __restrict__ out, uint8_t* __restrict__ seen) {
  tp3_scatter_body<LEVEL, REC8, 1024, TP3_B>(uid, iid, rating, tmp, n, chunk, g, cshift, NC, KT, kptr, cursor, cptr,
                                             wptr, H1, out, seen);
}

// slim shape (see tp3_count_body): 1024-record batches, 16 KiB of LDS
constexpr int TP3_SLIM_B = 1024;
template <int LEVEL, bool REC8>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_num_vgpr(32)))
tp3_scatter_slim_kernel(const int32_t* __restrict__ uid, const int32_t* __restrict__ iid,
                        const float* __restrict__ rating, const int4* __restrict__ tmp, int64_t n, int64_t chunk,
                        TileGeo g, int cshift, int NC, int KT, const int32_t* __restrict__ kptr,
                        int32_t* __restrict__ cursor, const int32_t* __restrict__ cptr,
                        const int32_t* __restrict__ wptr, const int32_t* __restrict__ H1, void* __restrict__ out,
                        uint8_t* __restrict__ seen) {
  tp3_scatter_body<LEVEL, REC8, 256, TP3_SLIM_B>(uid, iid, rating, tmp, n, chunk, g, cshift, NC, KT, kptr, cursor,
                                                 cptr, wptr, H1, out, seen);
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

// Item rows are loaded / stored non-temporal (each is read and written once per
// chunk; the cache is worth more to the random user rows): +0.7 % same box
// (profiles/r2_partition.md); non-temporal user-row stores: no gain.
//
// Two item blocks per launch: tiles [0, T0) cover block I (tile offsets ptr),
// tiles [T0, grid) block I1 (offsets ptr1) -- two blocks with disjoint item rows
// need no ordering, and one launch instead of two halves the tail of partly filled
// waves (the local layout's two halves; the bidirectional rotation's two rings).
//
// DELTA (the PS path, one block): the item rows I are READ-ONLY (the pulled rows)
// and the kernel writes the micro-batch's delta of every row of the block to Dl --
// what the PS then adds (SimplePSLogic's vector sum).  With dl_init every row of
// every tile is written in its tile's first chunk (zero when the chunk has none of
// its ratings, the whole tile when the tile has no ratings); a later chunk of the
// tile -- or a later launch without dl_init (the next user phase) -- starts from
// I + Dl (the row as the earlier work left it) and adds its sum to Dl.  Replaces a working copy of the pulled rows and a subtraction pass
// (round 3: clone + SGD + sub_, 1.3 GB of extra traffic at 1M x 64 rows).
// UM (user-row mode): 0 = plain loads / stores (Hogwild across workgroups);
// 1 = write-through (`sc1`: loads bypass the CU's L1, stores drop the line from the
// writing XCD's L2), so a user row updated on another CU or XCD is not re-read from a
// stale cached copy (about half the lost updates, profiles/r4_hogwild.md);
// 2 = exact: sc1 loads and the user delta ADDED with float atomics (executed at the
// memory side, never lost: a concurrent update of the same user is summed, as the
// item deltas of one tile are; the read it was computed from may be stale, as a
// Hogwild read).  Buffer addressing (UM >= 1): the table must be < 4 GiB.
typedef unsigned int tg_u4 __attribute__((ext_vector_type(4)));

template <bool REC8>
struct TgShared {
  typename RecT<REC8>::type srec[tg_cap<REC8>()];  // the chunk, counting-sorted by row
  int32_t cnt[TG_MAX_R + 1];
  int32_t start[TG_MAX_R + 1];
};

// one tile of the tile-grouped SGD (see mf_sgd_tilegroup_kernel)
template <int TPR, int V, int PF, bool REC8, bool DELTA, int UM>
__device__ __forceinline__ void tilegroup_tile(TgShared<REC8>& sh, const int t, float* __restrict__ U,
                                               float* __restrict__ I, const void* __restrict__ rec_,
                                               const int32_t* __restrict__ ptr, int R, int64_t block_rows,
                                               float lr, float lambda, float* __restrict__ I1,
                                               int64_t block_rows1, int T0, const int32_t* __restrict__ ptr1,
                                               float* __restrict__ Dl, int dl_init, uint32_t ubytes) {
  using Rec = typename RecT<REC8>::type;
  constexpr int TG_CAP = tg_cap<REC8>();
  const Rec* __restrict__ rec = reinterpret_cast<const Rec*>(rec_);
  Rec* srec = sh.srec;
  int32_t* cnt = sh.cnt;
  int32_t* start = sh.start;
  constexpr int D4 = TPR * V;
  constexpr int GPW = 64 / TPR;  // lane groups per wave
  const bool second = t >= T0;
  const int tl = second ? t - T0 : t;
  if (second) { I = I1; block_rows = block_rows1; ptr = ptr1; }
  const int64_t r0 = (int64_t)tl * R;
  const int nr = (int)min((int64_t)R, block_rows - r0);
  const int32_t beg = ptr[tl], end = ptr[tl + 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ngroups = (blockDim.x >> 6) * GPW;
  const int grp = wave * GPW + lane / TPR, j = lane % TPR;
  float4* Ig = reinterpret_cast<float4*>(I) + r0 * D4;
  float4* Ug = reinterpret_cast<float4*>(U);
  float4* Dg = DELTA ? reinterpret_cast<float4*>(Dl) + r0 * D4 : nullptr;
  __amdgpu_buffer_rsrc_t urs;
  if constexpr (UM >= 1) urs = __builtin_amdgcn_make_buffer_rsrc(U, (short)0, (int)ubytes, 0x00020000);
  if (DELTA && dl_init && beg == end) {  // no ratings in this tile: its rows' deltas are zero
    for (int k = threadIdx.x; k < nr * D4; k += blockDim.x) f4_st<true>(Dg + k, make_float4(0.f, 0.f, 0.f, 0.f));
    return;
  }
  for (int32_t c0 = beg; c0 < end; c0 += TG_CAP) {
    // first: Dl of this tile holds nothing yet (its first chunk of a launch that
    // initialises Dl); else every row continues from I + Dl (an earlier chunk, or an
    // earlier launch over the same rows -- the user phases)
    const bool first = DELTA && dl_init && c0 == beg;
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
      if (a == b) {  // uniform in the lane group
        if (DELTA && first)
#pragma unroll
          for (int v = 0; v < V; ++v) f4_st<true>(Dg + (int64_t)row * D4 + j + v * TPR, make_float4(0.f, 0.f, 0.f, 0.f));
        continue;
      }
      float4 iv[V], acc[V], dv[V];
#pragma unroll
      for (int v = 0; v < V; ++v) {
        iv[v] = f4_ld<true>(Ig + (int64_t)row * D4 + j + v * TPR);
        acc[v] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (DELTA && !first) {  // the earlier chunks' sum: the row continues from I + Dl
          dv[v] = f4_ld<true>(Dg + (int64_t)row * D4 + j + v * TPR);
          iv[v].x += dv[v].x; iv[v].y += dv[v].y; iv[v].z += dv[v].z; iv[v].w += dv[v].w;
        }
      }
      // float4 offsets of the user rows: 32-bit for 8-B records (user < 2^24, D4 <= 64),
      // 14 fewer live VGPRs than 64-bit offsets
      using Off = typename std::conditional<REC8, uint32_t, int64_t>::type;
      for (int k0 = a; k0 < b; k0 += PF) {
        float4 uv[PF][V];
        Off ur[PF];
        float rv[PF];
#pragma unroll
        for (int q = 0; q < PF; ++q) {  // all PF user rows in flight (index clamped, result masked)
          int32_t u; int rw;
          get_rec<REC8>(srec[min(k0 + q, b - 1)], r0, u, rw, rv[q]);
          ur[q] = (Off)u * D4;
#pragma unroll
          for (int v = 0; v < V; ++v) {
            if constexpr (UM >= 1)
              uv[q][v] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                                        urs, (int)((uint32_t)(ur[q] + j + v * TPR) * 16u), 0, 16));
            else
              uv[q][v] = Ug[ur[q] + j + v * TPR];
          }
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
            if constexpr (UM == 2) {
              // the delta added with contiguous float atomics: lane j of the group holds
              // elements 4j .. 4j+3 of this 4*TPR-float chunk; atomic instruction c adds
              // element TPR*c + j, fetched from lane (TPR*c + j) / 4 -- every instruction then
              // covers 4*TPR contiguous bytes of the row (one 64-B request per row at
              // TPR = 16) instead of 4-B lanes at a 16-B stride (4x the atomic requests)
              const float dx = nu.x - u.x, dy = nu.y - u.y, dz = nu.z - u.z, dw = nu.w - u.w;
              float* up = reinterpret_cast<float*>(Ug + ur[q] + v * TPR);
#pragma unroll
              for (int c = 0; c < 4; ++c) {
                const int src = (TPR * c + j) >> 2, comp = j & 3;
                const float a0 = __shfl(dx, src, TPR), a1 = __shfl(dy, src, TPR);
                const float a2 = __shfl(dz, src, TPR), a3 = __shfl(dw, src, TPR);
                atomic_add_noret(up + TPR * c + j, comp == 0 ? a0 : comp == 1 ? a1 : comp == 2 ? a2 : a3);
              }
            } else if constexpr (UM == 1)
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(tg_u4, nu), urs,
                                                     (int)((uint32_t)(ur[q] + j + v * TPR) * 16u), 0, 16);
            else
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
        if constexpr (DELTA) {
          float4 o = acc[v];
          if (!first) { o.x += dv[v].x; o.y += dv[v].y; o.z += dv[v].z; o.w += dv[v].w; }
          f4_st<true>(Dg + (int64_t)row * D4 + j + v * TPR, o);
        } else {
          float4 o = iv[v];
          o.x += acc[v].x; o.y += acc[v].y; o.z += acc[v].z; o.w += acc[v].w;
          f4_st<true>(Ig + (int64_t)row * D4 + j + v * TPR, o);
        }
      }
    }
    __syncthreads();  // LDS reused by the next chunk
  }
}

// Build-time knobs of the tile SGD (A/B variants: csrc/build.py --variant NAME -D ...):
// user rows in flight per lane group, and the minimum waves per SIMD the register
// allocation must leave room for (2 = two 512-thread workgroups per CU).  4 rows in
// flight: 79 VGPRs, three 512-thread workgroups per CU (8 rows: 109 VGPRs, two) --
// 0.5 % faster on the headline in two same-box A/Bs; 6 or 10 rows, or a forced 3rd /
// 4th workgroup with spills, were slower (profiles/r5_tile_sgd_variants_ab.txt)
#ifndef FPS_TG_PF
#define FPS_TG_PF 4
#endif
#ifndef FPS_TG_MINW
#define FPS_TG_MINW 2
#endif

// One workgroup per tile.  (A persistent grid taking tiles from a device counter, to
// drop the tail round of the 16 small launches per step at N = 8, was measured slower:
// 9.58e9 vs 9.87e9 updates/s at N = 1, 7.64 vs 7.45 ms emulated N = 8 --
// profiles/r4_persistent_sgd_ab.txt; removed.)
template <int TPR, int V, int PF, bool REC8, bool DELTA, int UM>
__global__ void __launch_bounds__(512, FPS_TG_MINW) mf_sgd_tilegroup_kernel(float* __restrict__ U, float* __restrict__ I,
                                                               const void* __restrict__ rec_,
                                                               const int32_t* __restrict__ ptr, int R,
                                                               int64_t block_rows, float lr, float lambda,
                                                               float* __restrict__ I1, int64_t block_rows1, int T0,
                                                               const int32_t* __restrict__ ptr1,
                                                               float* __restrict__ Dl, int dl_init, uint32_t ubytes) {
  __shared__ TgShared<REC8> sh;
  tilegroup_tile<TPR, V, PF, REC8, DELTA, UM>(sh, blockIdx.x, U, I, rec_, ptr, R, block_rows, lr, lambda, I1,
                                                block_rows1, T0, ptr1, Dl, dl_init, ubytes);
}

}  // namespace

// Level 3 partition's chunk: ~16 records per bucket and workgroup, 65536 .. 262144
// ratings (same box, alternating: at KT = 15.6k buckets 65536 gave 10.41 / 10.54e9,
// 262144 10.68 / 10.69e9 updates/s; at KT = 3.9k 65536 9.89 / 9.88e9, 262144 9.69 /
// 9.73e9, profiles/r2_partition.md)
static int tp3_groups(int64_t n, int KT) {
  int64_t c = 65536;
  while (c < 16 * (int64_t)KT && c < 262144) c <<= 1;
  int64_t g = (n + c - 1) / c;
  if (g < 1) g = 1;
  if (g > 1024) g = 1024;
  return (int)g;
}

static int tp3_cshift(int KT) {
  int cshift = 0;
  while (((KT - 1) >> cshift) + 1 > 128) ++cshift;  // ~128 coarse keys of <= 128 buckets
  return cshift;
}

// Workspace (int32): ccount[NC], ccursor[NC], cptr[NC+1], bcount[KT], bcursor[KT],
// wptr[NC+1] (zeroed here), H1[G <= 1024][NC], fine histograms [1 + 512][KT]
FPS_API int64_t fps_tile_partition_ws_ints(int W, int T, int P) {
  const int KT = P * 2 * W * T;
  const int NC = ((KT - 1) >> tp3_cshift(KT)) + 1;
  return 4 * (int64_t)NC + 2 + 2 * (int64_t)KT + 1024 * (int64_t)NC + 513 * (int64_t)KT;
}

// Two-level partition with LDS-sorted batches: a counting pass (fine and coarse
// histograms), level 1 scatters into ~128 coarse keys, level 2 into the KT buckets.
// ptr[KT+1] = bucket offsets; rec = n records (8 B if rec8, else 16 B) grouped by
// bucket; tmp = n 16-B slots (12-B records when rec8).  The counting-only
// single-level scatter, the atomic two-level scatter and a capacity-slot variant
// without counting pass were measured slower and removed in round 3
// (profiles/r1_mf_partition_levels.md, r2_tp4.md).
// count-kernel counter width: 16-bit packed unless set to 0 (A/B switch, FPS_TP_H16=0;
// above 16k buckets always 16-bit)
static int g_tp_h16 = 1;
FPS_API void fps_tile_partition_set_h16(int v) { g_tp_h16 = v; }
// most workgroups per partition launch (0 = as many as there is work): fewer, looping
// workgroups occupy fewer CUs beside the SGD of the previous batch (A/B knob, FPS_TP_GRID)
static int g_tp_grid = 0;
FPS_API void fps_tile_partition_set_grid(int v) { g_tp_grid = v; }
// partition kernel shape (tp3_count_body): 0 = fat (1024-thread workgroups), 1 = slim
// (256 threads, <= 32 VGPRs: co-resident with the tile SGD's three workgroups per CU)
static int g_tp_slim = 0;
FPS_API void fps_tile_partition_set_slim(int v) { g_tp_slim = v; }
FPS_API int fps_tile_partition_get_slim() { return g_tp_slim; }

FPS_API int fps_tile_partition(const int32_t* uid, const int32_t* iid, const float* rating, int64_t n, int W,
                               const int32_t* half, int R, int T, int P, int upp, int nu, int ni, int32_t* ws,
                               int4* tmp, int32_t* ptr, void* rec, int rec8, uint8_t* seen, void* stream) {
  const int KT = P * 2 * W * T;
  if (KT > TP_MAX_BUCKETS || R <= 0 || T <= 0) return (int)hipErrorInvalidValue;
  const int cshift = tp3_cshift(KT);
  const int NC = ((KT - 1) >> cshift) + 1;
  if (NC > TP3_MAXK || (1 << cshift) > TP3_MAXK) return (int)hipErrorInvalidValue;
  // user ids past the phases' range would land past the KT bucket counters
  if (nu <= 0 || (int64_t)nu > (int64_t)P * upp) nu = (int)min((int64_t)P * upp, (int64_t)INT32_MAX);
  const TileGeo g = make_geo(W, half, R, T, upp, nu, ni);
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
  const int cmax = g_tp_grid > 0 ? min(512, g_tp_grid) : 512;
  const int sub = (G + cmax - 1) / cmax;  // <= 512 count workgroups (2 per CU)
  const int Gc = (G + sub - 1) / sub;
  int32_t* bhist = H1 + 1024 * (int64_t)NC;  // [1 + Gc][KT]: totals, then one row per count workgroup
  // 16-bit LDS counters (<= 64 KiB at 31k buckets, the default dynamic-LDS ceiling,
  // and room on the CU for two SGD workgroups beside the count workgroup).  Also below
  // 16k buckets, where 32-bit ones would fit: half the LDS per count workgroup, and the
  // SGD beside it ran +0.4 % (local headline) / +0.8 % (PS path), same box
  // (profiles/r4_count_width_ab.txt)
  const bool h16 = g_tp_h16 != 0 || KT > 16384;  // 32-bit counters only fit 16k buckets
  const size_t hb_bytes = sizeof(int32_t) * (size_t)(h16 ? (KT + 1) / 2 : KT);
  // slim: the 16-bit histogram within what three SGD workgroups leave of a CU's LDS
  const bool slim = g_tp_slim != 0 && h16 && hb_bytes <= 40 * 1024;
  if (slim) {
    hipLaunchKernelGGL(tp3_count_slim_kernel<true>, dim3(Gc), dim3(256), hb_bytes, s, uid, iid, n, chunk, G, sub, g,
                       cshift, NC, KT, ccount, bhist, (uint8_t*)nullptr, H1);
  } else if (h16) {
    hipLaunchKernelGGL(tp3_count_kernel<true>, dim3(Gc), dim3(1024), hb_bytes, s, uid, iid, n, chunk, G, sub, g,
                       cshift, NC, KT, ccount, bhist, (uint8_t*)nullptr, H1);
  } else {
    hipLaunchKernelGGL(tp3_count_kernel<false>, dim3(Gc), dim3(1024), hb_bytes, s, uid, iid, n, chunk, G, sub, g,
                       cshift, NC, KT, ccount, bhist, (uint8_t*)nullptr, H1);
  }
  hipLaunchKernelGGL(tp3_colsum_kernel, dim3((KT + 63) / 64), dim3(1024), 0, s, bhist, Gc, KT);
  hipLaunchKernelGGL(tile_scan_kernel, dim3(1), dim3(1024), 0, s, (const int32_t*)ccount, NC, cptr);
  hipLaunchKernelGGL(tile_scan_kernel, dim3(1), dim3(1024), 0, s, (const int32_t*)bhist, KT, ptr);
  hipLaunchKernelGGL(tp3_colscan_kernel, dim3(NC), dim3(1024), 0, s, H1, G, NC, (const int32_t*)cptr);
  hipLaunchKernelGGL(tp3_workptr_kernel, dim3(1), dim3(64), 0, s, (const int32_t*)ccount, NC, wptr);
  if (n > 0) {
    int64_t g2 = n / TP3_CH + NC + 1;  // >= the number of work items
    if (g2 > 1024) g2 = 1024;
    if (g_tp_grid > 0 && g2 > g_tp_grid) g2 = g_tp_grid;
    const int g1 = g_tp_grid > 0 ? min(G, g_tp_grid) : G;
#define FPS_TP3(L, R8, GRID, TMP, KPTR, CUR, H1P, OUT)                                                            \
    if (slim)                                                                                                        \
      hipLaunchKernelGGL((tp3_scatter_slim_kernel<L, R8>), dim3(GRID), dim3(256), 0, s, uid, iid, rating, TMP, n,   \
                         chunk, g, cshift, NC, KT, KPTR, CUR, (const int32_t*)cptr, (const int32_t*)wptr, H1P, OUT, \
                         L == 2 ? seen : (uint8_t*)nullptr);                                                         \
    else                                                                                                             \
      hipLaunchKernelGGL((tp3_scatter_kernel<L, R8>), dim3(GRID), dim3(1024), 0, s, uid, iid, rating, TMP, n, chunk, \
                         g, cshift, NC, KT, KPTR, CUR, (const int32_t*)cptr, (const int32_t*)wptr, H1P, OUT,       \
                         L == 2 ? seen : (uint8_t*)nullptr)
    if (rec8) { FPS_TP3(1, true, g1, (const int4*)nullptr, (const int32_t*)cptr, ccursor, (const int32_t*)H1, (void*)tmp); }
    else { FPS_TP3(1, false, g1, (const int4*)nullptr, (const int32_t*)cptr, ccursor, (const int32_t*)H1, (void*)tmp); }
    if (rec8) { FPS_TP3(2, true, (int)g2, (const int4*)tmp, (const int32_t*)ptr, bcursor, (const int32_t*)nullptr, rec); }
    else { FPS_TP3(2, false, (int)g2, (const int4*)tmp, (const int32_t*)ptr, bcursor, (const int32_t*)nullptr, rec); }
#undef FPS_TP3
  }
  FPS_CHECK_LAUNCH();
  return 0;
}

// Tiled SGD over one or two item blocks: block 0 = rows I0[rows0, D] with tile
// offsets ptr0[T+1], block 1 (nblk = 2) = I1[rows1, D] with ptr1[T+1]; T tiles of
// R (<= 256) rows each.  D must be 16, 32, 64, 128 or 256.
// delta0 != nullptr (nblk = 1): DELTA mode -- I0 read-only, the block's deltas written
// to delta0 (delta_init) or added to it (a later user phase over the same rows).
FPS_API int fps_mf_sgd_tiled(float* U, float* I0, const void* rec, int rec8, const int32_t* ptr0, int T, int R,
                             int64_t rows0, float* I1, const int32_t* ptr1, int64_t rows1, int nblk, int D, float lr,
                             float lambda, float* delta0, int delta_init, int64_t users_bytes, int user_mode,
                             void* stream) {
  if (T <= 0) return 0;
  if (nblk != 1 && nblk != 2) return (int)hipErrorInvalidValue;
  if (delta0 != nullptr && nblk != 1) return (int)hipErrorInvalidValue;
  if (R <= 0 || R > TG_MAX_R) return (int)hipErrorInvalidValue;
  if (user_mode < 0 || user_mode > 2) return (int)hipErrorInvalidValue;
  if (nblk == 1) { I1 = I0; ptr1 = ptr0; rows1 = rows0; }
  const int grid = nblk * T;
  hipStream_t s = (hipStream_t)stream;
  constexpr int PF = FPS_TG_PF;
  // user-row mode (UM above: 0 plain, 1 write-through sc1, 2 exact atomic deltas); modes
  // 1 / 2 address users with 32-bit offsets of 8-B records and a buffer descriptor: the
  // table must be < 4 GiB
  if (user_mode && !(rec8 && users_bytes > 0 && users_bytes < (int64_t)0xFFFFFFFF)) return (int)hipErrorInvalidValue;
  const uint32_t ubytes = (uint32_t)(user_mode ? users_bytes : 0);
#define FPS_TILED_K(TPR_, V_, R8_, DL_, UM_)                                                                               \
  hipLaunchKernelGGL((mf_sgd_tilegroup_kernel<TPR_, V_, PF, R8_, DL_, UM_>), dim3(grid), dim3(512), 0, s, U, I0,   \
                     rec, ptr0, R, rows0, lr, lambda, I1, rows1, T, ptr1, delta0, delta_init, ubytes)
#define FPS_TILED_(TPR_, V_, DL_)                                 \
  if (rec8 && user_mode == 2) { FPS_TILED_K(TPR_, V_, true, DL_, 2); }       \
  else if (rec8 && user_mode == 1) { FPS_TILED_K(TPR_, V_, true, DL_, 1); }  \
  else if (rec8) { FPS_TILED_K(TPR_, V_, true, DL_, 0); }                    \
  else { FPS_TILED_K(TPR_, V_, false, DL_, 0); }
#define FPS_TILED(TPR_, V_)                      \
  if (delta0 != nullptr) { FPS_TILED_(TPR_, V_, true); } \
  else { FPS_TILED_(TPR_, V_, false); }
  switch (D) {
    case 16: FPS_TILED(4, 1); break;
    case 32: FPS_TILED(8, 1); break;
    case 64: FPS_TILED(16, 1); break;
    case 128: FPS_TILED(16, 2); break;
    case 256: FPS_TILED(16, 4); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef FPS_TILED
#undef FPS_TILED_
#undef FPS_TILED_K
  FPS_CHECK_LAUNCH();
  return 0;
}

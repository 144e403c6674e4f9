// Standard skip-gram negative sampling (gfx950), kernel K6 "standard": every
// (center, context) pair has k INDEPENDENT negatives (word2vec's own objective;
// the block-shared-negative kernels of sgns.hip are the labelled alternative).
//
// One wave per chunk of consecutive pairs.  Pairs arrive center-major (a
// center's whole window, then the next center: skipgram_pairs), so a wave
// walks runs of pairs that share a center: the center row h is loaded once per
// run into registers and updated there after every pair (sequential SGD inside
// the run), and only the run's total change is added to the center's row at the
// end (one 4*D-byte atomic wave-instruction per run instead of one per pair).
//
// Per pair: the context row and the k negative rows are loaded in groups of
// four (independent 256-B coalesced loads in flight), their dot products with h
// are reduced across the wave with xor-shuffles (four at a time), then
//   g_o = lr * (1 - sigma(h.o)),  g_n = lr * (0 - sigma(h.n))   (n != o)
//   W_out[x] += g_x * h                      (no-return float atomics)
//   h        += sum_x g_x * x               (registers)
// A negative equal to the context is skipped, as in word2vec.  Lane l owns the
// coordinates l, l + 64, ... (NPL = ceil(D / 64) floats per lane).
//
// Memory per pair at D = 300, k = 5: 6 rows read (7.2 KB) and 6 rows of float
// atomics (7.2 KB); the matrix cores have nothing GEMM-shaped to do here (every
// pair has its own rows: batched dot products), so this kernel is bound by the
// atomic rate (MI355X_MICROARCH.md "Global float atomics").
//
// rows_in / rows_out are the rows read (the tables themselves on the local path,
// the pulled rows on the PS path); d_in / d_out receive the deltas (the tables
// themselves -> Hogwild in place; or per-unique-row delta buffers to push).
// wmap_in / wmap_out (nullable) redirect the delta of row r to row wmap[r]: the
// PS path at world 1 adds its pushes straight into the owner's tables (pulled
// row r = table row wmap[r]) while reading the pulled snapshot.
#include "common.h"

using namespace fps;

namespace {

constexpr int SG = 4;  // rows per load group

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float sigmoidf(float s) { return 1.f / (1.f + __expf(-s)); }

// log(1 + exp(x)) without overflow
__device__ __forceinline__ float softplusf(float x) { return x > 0.f ? x + log1pf(__expf(-x)) : log1pf(__expf(x)); }

// float -> bf16, round to nearest even (torch's conversion; NaN stays a quiet NaN)
__device__ __forceinline__ uint16_t f32_to_bf16_rne(float f) {
  const uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40u);
  return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

// Row layout in a wave.  fp32 rows: lane l owns coordinates l + 64 m (NPL = ceil(D / 64)
// floats).  bf16 rows (BF, the PS path's wire rows read as pulled, even D): lane l owns
// the coordinate PAIRS 128 m' + 2 l, + 1 (NPL = 2 ceil(D / 128) floats), one 4-B load per
// pair widened in registers -- a 2-B load per coordinate (the fp32 map on bf16) ran the
// kernels 2.5x slower (round 6), and a separate widening pass cost a full read + write
// of every pulled row.  The fp32 delta buffers are addressed through the same map.
template <bool BF>
__device__ __forceinline__ int sg_coord(int lane, int m) {
  if constexpr (BF) return 128 * (m >> 1) + 2 * lane + (m & 1);
  else return lane + 64 * m;
}

template <int NPL, bool BF>
__device__ __forceinline__ void sg_load_row(const void* __restrict__ base, int64_t row, int D, int lane, bool valid,
                                            float (&v)[NPL]) {
  if constexpr (BF) {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint16_t*>(base) + row * D);
#pragma unroll
    for (int mp = 0; mp < NPL / 2; ++mp) {
      const int j = 128 * mp + 2 * lane;
      const uint32_t w = (valid && j < D) ? src[j >> 1] : 0u;
      v[2 * mp] = __uint_as_float(w << 16);             // coordinate j (the low half)
      v[2 * mp + 1] = __uint_as_float(w & 0xffff0000u);  // coordinate j + 1
    }
  } else {
    const float* src = reinterpret_cast<const float*>(base) + row * D;
#pragma unroll
    for (int m = 0; m < NPL; ++m) {
      const int j = lane + 64 * m;
      v[m] = (valid && j < D) ? src[j] : 0.f;
    }
  }
}

// GOUT = false: output-row deltas by float atomics (above).  GOUT = true: the
// output rows are not touched here; the pair's coefficient g_x goes to
// gbuf[p * (k + 1) + x] and sgns_rows_kernel below applies sum_x g_x * h per
// output row from the coefficients sorted by row (no atomics on the hot rows).
template <int NPL, bool GOUT, bool BF = false>
__global__ void __launch_bounds__(256) sgns_std_kernel(const void* __restrict__ rows_in,
                                                       const void* __restrict__ rows_out,
                                                       const int32_t* __restrict__ pos_c,
                                                       const int32_t* __restrict__ pos_o,
                                                       const int32_t* __restrict__ pos_neg, int64_t P, int D, int k,
                                                       float lr, float* __restrict__ d_in, float* __restrict__ d_out,
                                                       const int32_t* __restrict__ wmap_in,
                                                       const int32_t* __restrict__ wmap_out,
                                                       float* __restrict__ loss, int chunk,
                                                       float* __restrict__ gbuf) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t p0 = wave * chunk;
  if (p0 >= P) return;  // wave-uniform
  const int64_t p1 = min(P, p0 + chunk);
  float h[NPL], h0[NPL];
  int32_t cur = -1;
  float lsum = 0.f;
  auto flush = [&]() {
    if (cur < 0) return;
    float* dst = d_in + (int64_t)(wmap_in != nullptr ? wmap_in[cur] : cur) * D;
#pragma unroll
    for (int m = 0; m < NPL; ++m) {
      const int j = sg_coord<BF>(lane, m);
      if (j < D) atomic_add_noret(dst + j, h[m] - h0[m]);
    }
  };
  for (int64_t p = p0; p < p1; ++p) {
    const int32_t c = pos_c[p];
    if (c != cur) {  // a new center run: push the previous run's change, load this center
      flush();
      cur = c;
      sg_load_row<NPL, BF>(rows_in, c, D, lane, true, h);
#pragma unroll
      for (int m = 0; m < NPL; ++m) h0[m] = h[m];
    }
    const int32_t o = pos_o[p];
    float dh[NPL];
#pragma unroll
    for (int m = 0; m < NPL; ++m) dh[m] = 0.f;
    for (int x0 = 0; x0 <= k; x0 += SG) {  // x = 0: the context, x >= 1: negative x-1
      int32_t row[SG];
      float xv[SG][NPL], part[SG];
#pragma unroll
      for (int q = 0; q < SG; ++q) {
        const int x = x0 + q;
        row[q] = x == 0 ? o : (x <= k ? pos_neg[p * k + x - 1] : -1);
        if (x > 0 && row[q] == o) row[q] = -1;  // word2vec skips a negative equal to the target
      }
#pragma unroll
      for (int q = 0; q < SG; ++q)  // all loads of the group in flight
        sg_load_row<NPL, BF>(rows_out, row[q] < 0 ? 0 : row[q], D, lane, row[q] >= 0, xv[q]);
#pragma unroll
      for (int q = 0; q < SG; ++q) {
        float s = 0.f;
#pragma unroll
        for (int m = 0; m < NPL; ++m) s += h[m] * xv[q][m];
        part[q] = s;
      }
#pragma unroll
      for (int o2 = 32; o2 > 0; o2 >>= 1) {  // four wave reductions interleaved
#pragma unroll
        for (int q = 0; q < SG; ++q) part[q] += __shfl_xor(part[q], o2, 64);
      }
#pragma unroll
      for (int q = 0; q < SG; ++q) {
        if (row[q] < 0) continue;  // wave-uniform
        const float label = (x0 + q == 0) ? 1.f : 0.f;
        const float s = part[q];
        const float g = lr * (label - sigmoidf(s));
        if (loss != nullptr && lane == 0) lsum += label > 0.f ? softplusf(-s) : softplusf(s);
        if constexpr (GOUT) {
          if (lane == 0) gbuf[p * (k + 1) + x0 + q] = g;
#pragma unroll
          for (int m = 0; m < NPL; ++m) dh[m] += g * xv[q][m];
        } else {
          float* dst = d_out + (int64_t)(wmap_out != nullptr ? wmap_out[row[q]] : row[q]) * D;
#pragma unroll
          for (int m = 0; m < NPL; ++m) {
            const int j = sg_coord<BF>(lane, m);
            if (j < D) atomic_add_noret(dst + j, g * h[m]);
            dh[m] += g * xv[q][m];
          }
        }
      }
    }
#pragma unroll
    for (int m = 0; m < NPL; ++m) h[m] += dh[m];
  }
  flush();
  if (loss != nullptr && lane == 0) atomicAdd(loss, lsum);
}

// Output-row pass of the sorted form.  srow[n] = output rows sorted, perm[n] =
// their entry e = p * (k + 1) + x in gbuf; the delta of row r is
// sum over its entries of gbuf[e] * rows_h[pos_c[e / (k + 1)]].  One wave per
// C consecutive sorted entries: the wave stages its entries' (row, center, g)
// in LDS with parallel loads, then walks them with RG center rows in flight,
// summing each run of equal rows in registers.  A run that lies wholly inside
// the wave's range is the row's only writer: plain read-modify-write; the (at
// most two) runs cut by the range ends are shared with a neighbour wave: float
// atomics.  The hottest output rows (Zipf contexts) thus cost one atomic per
// wave range instead of one per pair.
constexpr int SR_C = 256;  // sorted entries per wave
constexpr int SR_G = 8;    // center rows in flight per lane

// OB (bf16 push output, BF rows only, no wmap): d_out is scratch -- a run wholly inside
// the range writes bf16(sum) straight into out_bf (the push's wire buffer: no zero-fill
// of d_out, no widening of d_out afterwards); a run cut by a range end adds its sum with
// float atomics into d_out, whose cut rows sgns_cut_rows_kernel zeroes before and
// converts into out_bf after.
template <int NPL, bool BF = false, bool OB = false>
__global__ void __launch_bounds__(256) sgns_rows_kernel(const int32_t* __restrict__ srow,
                                                        const int64_t* __restrict__ perm,
                                                        const float* __restrict__ gbuf,
                                                        const int32_t* __restrict__ pos_c, int k1, int64_t n,
                                                        const void* __restrict__ rows_h, int D,
                                                        float* __restrict__ d_out,
                                                        const int32_t* __restrict__ wmap_out,
                                                        uint16_t* __restrict__ out_bf) {
  static_assert(!OB || BF, "bf16 push output pairs with the bf16 row layout");
  __shared__ int32_t s_row[4][SR_C], s_cen[4][SR_C];
  __shared__ float s_g[4][SR_C];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t t0 = ((int64_t)blockIdx.x * 4 + wv) * SR_C;
  const int m_n = t0 < n ? (int)min((int64_t)SR_C, n - t0) : 0;
  for (int i = lane; i < m_n; i += 64) {
    const int64_t e = perm[t0 + i];
    s_row[wv][i] = srow[t0 + i];
    s_g[wv][i] = gbuf[e];
    s_cen[wv][i] = pos_c[e / k1];
  }
  __syncthreads();
  if (m_n == 0) return;  // after the only barrier
  // A run that starts inside the range loads its row when it starts (the load hides
  // behind the run's gathers) and stores row + sum when it ends; a run cut by a range
  // end adds its sum with atomics instead.
  float acc[NPL], base[NPL];
  int32_t cur = s_row[wv][0];
  bool whole = t0 == 0 || srow[t0 - 1] != cur;  // the current run starts inside this range
  auto start = [&]() {
    const float* dst = d_out + (int64_t)(wmap_out != nullptr ? wmap_out[cur] : cur) * D;
#pragma unroll
    for (int m = 0; m < NPL; ++m) {
      const int j = sg_coord<BF>(lane, m);
      acc[m] = 0.f;
      base[m] = (!OB && whole && j < D) ? dst[j] : 0.f;
    }
  };
  auto flush = [&](bool complete) {
    float* dst = d_out + (int64_t)(wmap_out != nullptr ? wmap_out[cur] : cur) * D;
    if (OB && complete) {  // one 4-B store per coordinate pair
      uint32_t* ob = reinterpret_cast<uint32_t*>(out_bf + (int64_t)cur * D);
#pragma unroll
      for (int mp = 0; mp < NPL / 2; ++mp) {
        const int j = 128 * mp + 2 * lane;
        if (j < D) ob[j >> 1] = (uint32_t)f32_to_bf16_rne(acc[2 * mp]) | ((uint32_t)f32_to_bf16_rne(acc[2 * mp + 1]) << 16);
      }
      return;
    }
#pragma unroll
    for (int m = 0; m < NPL; ++m) {
      const int j = sg_coord<BF>(lane, m);
      if (j < D) {
        if (complete) dst[j] = base[m] + acc[m];
        else atomic_add_noret(dst + j, acc[m]);
      }
    }
  };
  start();
  for (int i0 = 0; i0 < m_n; i0 += SR_G) {
    float hv[SR_G][NPL];
#pragma unroll
    for (int q = 0; q < SR_G; ++q) {  // all SR_G center rows in flight
      const int i = min(i0 + q, m_n - 1);
      sg_load_row<NPL, BF>(rows_h, s_cen[wv][i], D, lane, true, hv[q]);
    }
#pragma unroll
    for (int q = 0; q < SR_G; ++q) {
      const int i = i0 + q;
      if (i >= m_n) break;  // wave-uniform
      const int32_t r = s_row[wv][i];
      if (r != cur) {  // the run of `cur` ended inside the range
        flush(whole);
        cur = r;
        whole = true;
        start();
      }
      const float g = s_g[wv][i];
#pragma unroll
      for (int m = 0; m < NPL; ++m) acc[m] += g * hv[q][m];
    }
  }
  flush(whole && (t0 + m_n == n || srow[t0 + m_n] != cur));
}

// The rows cut by a range end of sgns_rows_kernel (its SR_C-entry ranges): the first row
// of a range that continues the previous range's last run, and the last row of a range
// that the next range continues.  ZERO: zero them in d_out (before the OB pass: their
// partial sums arrive by atomics); else write bf16(d_out) into out_bf (after).  A row cut
// several times is handled by several waves with the same values.
template <bool ZERO>
__global__ void __launch_bounds__(256) sgns_cut_rows_kernel(const int32_t* __restrict__ srow, int64_t n, int D,
                                                            float* __restrict__ d_out, uint16_t* __restrict__ out_bf) {
  const int lane = threadIdx.x & 63;
  const int64_t w = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t t0 = w * SR_C;
  if (t0 >= n) return;
  const int64_t t1 = min(n, t0 + SR_C) - 1;  // last entry of the range
  const int32_t first = srow[t0], last = srow[t1];
  const bool cut_first = t0 > 0 && srow[t0 - 1] == first;
  const bool cut_last = t1 + 1 < n && srow[t1 + 1] == last;
  for (int c = 0; c < 2; ++c) {
    const bool cut = c == 0 ? cut_first : cut_last;
    if (!cut) continue;  // wave-uniform
    const int64_t r = c == 0 ? first : last;
    float* dst = d_out + r * D;
    for (int j = lane; j < D; j += 64) {
      if (ZERO) dst[j] = 0.f;
      else out_bf[r * D + j] = f32_to_bf16_rne(dst[j]);
    }
  }
}

}  // namespace

// Sorted form, pass 1: centers as in fps_sgns_standard (d_in), output-row
// coefficients into gbuf[P * (k + 1)] (zeroed by the caller; skipped negatives
// stay 0).
FPS_API int fps_sgns_standard_coef(const void* rows_in, const void* rows_out, const int32_t* pos_c,
                                   const int32_t* pos_o, const int32_t* pos_neg, int64_t P, int D, int k, float lr,
                                   float* d_in, const int32_t* wmap_in, float* loss, float* gbuf, void* stream,
                                   int rows_bf16) {
  if (P <= 0) return 0;
  if (D <= 0 || D > 512 || k < 0 || (rows_bf16 && D % 2)) return (int)hipErrorInvalidValue;
  const int chunk = 16;
  const int64_t waves = (P + chunk - 1) / chunk;
  const int64_t blocks = (waves + 3) / 4;
  if (blocks > INT32_MAX) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
#define FPS_SGC(NPL_, BF_)                                                                                       \
  hipLaunchKernelGGL((sgns_std_kernel<NPL_, true, BF_>), dim3((unsigned)blocks), dim3(256), 0, s, rows_in,         \
                     rows_out, pos_c, pos_o, pos_neg, P, D, k, lr, d_in, (float*)nullptr, wmap_in,                 \
                     (const int32_t*)nullptr, loss, chunk, gbuf)
  if (rows_bf16) {
    if (D <= 128) FPS_SGC(2, true);
    else if (D <= 256) FPS_SGC(4, true);
    else if (D <= 384) FPS_SGC(6, true);
    else FPS_SGC(8, true);
  } else if (D <= 64) FPS_SGC(1, false);
  else if (D <= 128) FPS_SGC(2, false);
  else if (D <= 256) FPS_SGC(4, false);
  else if (D <= 320) FPS_SGC(5, false);
  else FPS_SGC(8, false);
#undef FPS_SGC
  FPS_CHECK_LAUNCH();
  return 0;
}

// Sorted form, pass 2: d_out[srow[t]] += gbuf[perm[t]] * rows_h[pos_c[perm[t] / k1]]
// over the n = P * k1 entries sorted by output row.
// out_bf16 (nullable; bf16 rows and no wmap only): the deltas leave as bf16 in out_bf16
// (rows of the n entries' row ids) and d_out is scratch (see sgns_rows_kernel OB)
FPS_API int fps_sgns_rows(const int32_t* srow, const int64_t* perm, const float* gbuf, const int32_t* pos_c, int k1,
                          int64_t n, const void* rows_h, int D, float* d_out, const int32_t* wmap_out,
                          void* stream, int rows_bf16, uint16_t* out_bf16) {
  if (n <= 0) return 0;
  if (D <= 0 || D > 512 || k1 <= 0 || (rows_bf16 && D % 2)) return (int)hipErrorInvalidValue;
  if (out_bf16 != nullptr && (!rows_bf16 || wmap_out != nullptr)) return (int)hipErrorInvalidValue;
  const int64_t blocks = (n + 4 * SR_C - 1) / (4 * SR_C);
  if (blocks > INT32_MAX) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
#define FPS_SGR(NPL_, BF_)                                                                                       \
  hipLaunchKernelGGL((sgns_rows_kernel<NPL_, BF_>), dim3((unsigned)blocks), dim3(256), 0, s, srow, perm, gbuf,     \
                     pos_c, k1, n, rows_h, D, d_out, wmap_out, (uint16_t*)nullptr)
#define FPS_SGRO(NPL_)                                                                                           \
  hipLaunchKernelGGL((sgns_rows_kernel<NPL_, true, true>), dim3((unsigned)blocks), dim3(256), 0, s, srow, perm,   \
                     gbuf, pos_c, k1, n, rows_h, D, d_out, wmap_out, out_bf16)
  if (out_bf16 != nullptr) {
    const int64_t cut_blocks = ((n + SR_C - 1) / SR_C + 3) / 4;  // one wave per range
    hipLaunchKernelGGL(sgns_cut_rows_kernel<true>, dim3((unsigned)cut_blocks), dim3(256), 0, s, srow, n, D, d_out,
                       out_bf16);
    if (D <= 128) FPS_SGRO(2);
    else if (D <= 256) FPS_SGRO(4);
    else if (D <= 384) FPS_SGRO(6);
    else FPS_SGRO(8);
    hipLaunchKernelGGL(sgns_cut_rows_kernel<false>, dim3((unsigned)cut_blocks), dim3(256), 0, s, srow, n, D, d_out,
                       out_bf16);
  } else if (rows_bf16) {
    if (D <= 128) FPS_SGR(2, true);
    else if (D <= 256) FPS_SGR(4, true);
    else if (D <= 384) FPS_SGR(6, true);
    else FPS_SGR(8, true);
  } else if (D <= 64) FPS_SGR(1, false);
  else if (D <= 128) FPS_SGR(2, false);
  else if (D <= 256) FPS_SGR(4, false);
  else if (D <= 320) FPS_SGR(5, false);
  else FPS_SGR(8, false);
#undef FPS_SGRO
#undef FPS_SGR
  FPS_CHECK_LAUNCH();
  return 0;
}

// P pairs: centers pos_c[P] (rows of rows_in / d_in), contexts pos_o[P] and
// k negatives per pair pos_neg[P * k] (rows of rows_out / d_out); fp32 rows,
// D <= 512.  loss (optional, zeroed by the caller) receives the summed loss.
FPS_API int fps_sgns_standard(const void* rows_in, const void* rows_out, const int32_t* pos_c,
                              const int32_t* pos_o, const int32_t* pos_neg, int64_t P, int D, int k, float lr,
                              float* d_in, float* d_out, const int32_t* wmap_in, const int32_t* wmap_out, float* loss,
                              void* stream, int rows_bf16) {
  if (P <= 0) return 0;
  if (D <= 0 || D > 512 || k < 0 || (rows_bf16 && D % 2)) return (int)hipErrorInvalidValue;
  // ~16 pairs per wave: long enough to reuse a center across its window, short
  // enough for >= 32k waves at 1M pairs (the GPU holds ~8k)
  const int chunk = 16;
  const int64_t waves = (P + chunk - 1) / chunk;
  const int64_t blocks = (waves + 3) / 4;
  if (blocks > INT32_MAX) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
#define FPS_SGS(NPL_, BF_)                                                                                       \
  hipLaunchKernelGGL((sgns_std_kernel<NPL_, false, BF_>), dim3((unsigned)blocks), dim3(256), 0, s, rows_in,        \
                     rows_out, pos_c, pos_o, pos_neg, P, D, k, lr, d_in, d_out, wmap_in, wmap_out, loss, chunk,    \
                     (float*)nullptr)
  if (rows_bf16) {
    if (D <= 128) FPS_SGS(2, true);
    else if (D <= 256) FPS_SGS(4, true);
    else if (D <= 384) FPS_SGS(6, true);
    else FPS_SGS(8, true);
  } else if (D <= 64) FPS_SGS(1, false);
  else if (D <= 128) FPS_SGS(2, false);
  else if (D <= 256) FPS_SGS(4, false);
  else if (D <= 320) FPS_SGS(5, false);
  else FPS_SGS(8, false);
#undef FPS_SGS
  FPS_CHECK_LAUNCH();
  return 0;
}

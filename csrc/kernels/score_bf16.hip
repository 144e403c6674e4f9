// Top-K scoring on bf16 MFMA with an exact fp32 re-score (gfx950).  Kernel K8, fast path.
//
// The fp32 scorer (score_gemm.hip) runs v_mfma_f32_32x32x2_f32: 32 MFMAs per 32 x 32
// score tile at D = 64, ~100 TF/s -- it was 70 % of an online MF + top-K batch
// (profiles/r2_mf_topk.md).  v_mfma_f32_32x32x16_bf16 does the same tile in 4
// MFMAs at 16x the rate, but bf16 operands change the scores, and the reference's
// top-K (M/matrix/factorization/workers/PSTopKGeneratorWorker.scala:46-110) is exact.
// Exactness is kept with a filter-then-rescore split:
//
//   1. score_filter_bf16_kernel: S~ = bf16(Q) . bf16(X) on MFMA, fp32 accumulate.  Per
//      product |bf16(q)bf16(x) - qx| <= (2u + u^2)|q||x| with u = 2^-8 (RNE), and by
//      Cauchy-Schwarz sum_k |q_k||x_k| <= |q| |x|, so |S~ - S| <= c |q| |x| with
//      c = 2u + u^2 + 2 * D * 2^-24 (the fp32 accumulations of both scorers).  An item
//      is a candidate iff S~ > theta_q - c |q| max|x| (theta_q = the query's current
//      k-th best, max over the 32 items of an MFMA block): a superset of the items
//      with S > theta_q.  Candidate positions go to the query's list (count
//      atomics, cap as in score_filter_kernel).
//   2. cand_rescore_kernel: each candidate's exact score with the SAME fp32 MFMA
//      chain as score_gemm / score_filter (v_mfma_f32_32x32x2_f32 over k pairs 0,1 |
//      2,3 | ... in order, the query broadcast over the A rows, 32 candidates on the
//      B columns), so keys are bit-identical to the fp32 path; a candidate whose
//      exact score is not strictly above theta_q (the fp32 path's test) gets key 0,
//      below every real key, and never enters the merge.
//
// Operand layout (v_mfma_f32_32x32x16_bf16, MI355X guide "A/B operand lane maps"):
// lane l (r = l & 31, h = l >> 5) holds A[row r][k = 8h + j] and B[k = 8h + j][col r],
// j = 0..7.  The dot product sums over k, so any k order shared by A and B is
// valid: k-step s of lane half h takes elements 8s .. 8s+7 of the row's half h
// (dims h*D/2 + 8s + j) -- each lane reads its D/2 contiguous bf16 (64 B at D = 64)
// with 16-B loads, no LDS.  A = 32 items, B = 32 queries, so the accumulator
// column (lane & 31) is one query: its threshold and norm sit in two registers,
// rows (reg & 3) + 8 (reg >> 2) + 4h are items.
#include "common.h"

// 32-query blocks per wave at D = 64: 2 (118 VGPRs, 4 waves / SIMD) scores the online
// MF + top-K batches 4 % faster than 4 (164 VGPRs, 3 waves / SIMD) and LEMP the same
// (profiles/r5_scorer_qb_ab.txt)
#ifndef FPS_SB_QB64
#define FPS_SB_QB64 2
#endif
// items per LDS stage (a multiple of 64; one barrier per stage)
#ifndef FPS_SB_ST
#define FPS_SB_ST 64
#endif


using namespace fps;

namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int SB_WAVES = 4;     // waves per workgroup
constexpr int SB_ITEMS = 1024;  // most items per workgroup (32 MFMA blocks of 32); fewer on short segments
constexpr int SB_SLOTS = 16;    // LDS candidate slots per (query block, lane)

__device__ __forceinline__ uint32_t sb_key(float f) {  // order-preserving float -> uint32 (as topk.hip)
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// LEMP COORD bound of one (query, 32-item block) pair (M/matrix/factorization/
// pruning/LEMPPruningFunctions.scala:36-49 with the block's longest item as the
// bucket head): an item x can beat theta > 0 only if its normalised focus
// coordinate x_f / |x| lies in [lf, uf]; cb holds the min / max of x_c / |x| over
// the block's items for every coordinate c, so the block is skipped when that range
// misses [lf, uf] (widened by kCoordSlack for fp32 rounding) -- exact.
constexpr float kCoordSlack = 1e-4f;

__device__ __forceinline__ bool coord_pass(float theta, float ql, float bm, float qbf, float2 mm) {
  if (!(theta > 0.f) || !(ql > 0.f)) return true;  // no positive k-th best yet: nothing pruned
  if (!(bm > 0.f)) return false;                   // zero-length block: every score is 0 < theta
  const float tbq = fminf(theta / (bm * ql), 1.f);
  const float a = qbf * tbq;
  const float b = sqrtf(fmaxf((1.f - tbq * tbq) * (1.f - qbf * qbf), 0.f));
  const float lfp = a - b, ufp = a + b;
  const float ratio = qbf != 0.f ? tbq / qbf : INFINITY;
  const float lf = (qbf >= 0.f || lfp > ratio) ? lfp : -1.f;
  const float uf = (qbf <= 0.f || ufp < ratio) ? ufp : 1.f;
  return !(mm.y < lf - kCoordSlack || mm.x > uf + kCoordSlack);
}

// QB 32-query blocks per wave; a workgroup covers SB_WAVES * QB * 32 queries x
// SB_ITEMS items.  COORD: the LEMP coordinate bound per (32-query block, 32-item
// block) before the MFMAs (qf / qbf: each query's focus coordinate argmax q_c^2 and
// q_f / |q|; cb: [N / 32][D] coordinate ranges); stats[0] / [1] count the (query
// block, item block) pairs scored / skipped by the coordinate bound (pairs the length
// bound skips by itself are in neither).
template <int D, int QB, bool MASK = false, bool COORD = false, bool ILV = false, int PD = 1, bool CUR2 = false>
__global__ void __launch_bounds__(256, COORD ? 2 : (CUR2 ? 4 : 3)) score_filter_bf16_kernel(
    const uint16_t* __restrict__ Qb, const uint16_t* __restrict__ Xb, int B, int N,
    const float* __restrict__ best_s, int k, const float* __restrict__ qlen, const float* __restrict__ xbm,
    float margin, float slack, int64_t* __restrict__ cand_pos, int32_t* __restrict__ cnt, int cap,
    const int32_t* __restrict__ qf, const float* __restrict__ qbf, const float2* __restrict__ cb,
    int32_t* __restrict__ stats, const int32_t* __restrict__ gate, int ipw) {
  constexpr int S = D / 16;   // k-steps of 16; also 16-B loads per lane per row
  // COORD gate (device flag, nullable): off when the bound stopped paying on earlier
  // segments of this scan (coord_gate_kernel) -- the bound costs VALU per block pair
  const bool use_coord = COORD && (gate == nullptr || gate[0] > 0);
  constexpr int HALF = D / 2;
  constexpr int WQ = 32 * QB;
  constexpr int GQ = SB_WAVES * WQ;
  __shared__ float red[SB_WAVES];
  const int nqt = (B + GQ - 1) / GQ;
  const int nit = (N + ipw - 1) / ipw;  // ipw: items per workgroup, a multiple of 64, <= SB_ITEMS
  // query tiles fastest: the workgroups reading one item range are consecutive
  // logical ids, i.e. on one XCD (one L2 holds the range)
  const int wg = xcd_remap(blockIdx.x, nqt * nit);
  const int qt = wg % nqt, it = wg / nqt;
  const int i_begin = it * ipw, i_end = min(N, i_begin + ipw);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;

  // LEMP bound per workgroup: no query of the tile can be beaten by the range's
  // longest item -> the whole workgroup leaves before any load of X.  xbm[b] = the
  // longest item of 32-item block b (one value per MFMA block: a scalar load in the
  // loop below instead of a per-lane length load and a 64-lane max per block)
  float xm = 0.f;
  for (int b = (i_begin >> 5) + tid; b < ((i_end + 31) >> 5); b += 256) xm = fmaxf(xm, xbm[b]);
  xm = group_max<64>(xm);
  if (lane == 0) red[wave] = xm;
  __syncthreads();
  xm = red[0];
#pragma unroll
  for (int w = 1; w < SB_WAVES; ++w) xm = fmaxf(xm, red[w]);

  float theta[QB], ql[QB];
  int qrow[QB];
  uint4 qv[QB][S];
  int fq[QB];
  float qb[QB];
  int live = 0;
#pragma unroll
  for (int b = 0; b < QB; ++b) {
    const int q = qt * GQ + wave * WQ + b * 32 + r;
    qrow[b] = q;
    theta[b] = INFINITY;  // rows past B never pass
    ql[b] = 0.f;
    fq[b] = 0;
    qb[b] = 0.f;
    if (q < B) {
      theta[b] = best_s[(int64_t)q * k + k - 1];
      ql[b] = qlen[q];
      live |= !(theta[b] > -INFINITY && ql[b] * xm * slack <= theta[b]);
      if (COORD) {
        fq[b] = qf[q];
        qb[b] = qbf[q];
      }
    }
  }
  if (!__syncthreads_or(live)) return;  // uniform
#pragma unroll
  for (int b = 0; b < QB; ++b) {
    const uint4* src = reinterpret_cast<const uint4*>(Qb + (int64_t)qrow[b] * D + h * HALF);
#pragma unroll
    for (int s = 0; s < S; ++s) qv[b][s] = qrow[b] < B ? src[s] : make_uint4(0, 0, 0, 0);
  }

  // candidates of each (query block, lane) collect in a private LDS list of item
  // offsets and leave with ONE count atomic per query and workgroup at the end: a
  // returning atomic per passing score made every 32 x 32 block with a candidate
  // (most of them) wait a full memory round trip.  A full list falls back to the
  // per-candidate atomic (dense segments, theta = -inf).
  __shared__ uint16_t lst[SB_WAVES][QB][SB_SLOTS][64];
  int lc[QB];
#pragma unroll
  for (int b = 0; b < QB; ++b) lc[b] = 0;
  int scored = 0, skipped = 0;
  // Item tiles are staged in LDS, double-buffered: the workgroup loads each stage of
  // ST items ONCE (16-B loads, every thread 2 at D = 64) and its four waves read their
  // MFMA A operands from LDS.  Before, every wave loaded the same item rows from L2
  // itself (4x the L2 traffic of the workgroup) and half the waves stood waiting on
  // them (r4 counters: ~23 % MFMA busy, profiles/r4_counters_late.md).  The next
  // stage's loads are issued before this stage's MFMAs and land in the other buffer
  // after them; one barrier per stage.  Rows are padded to 2D + 16 bytes: the 16
  // lanes of each ds_read_b128 group then hit 16 distinct 4-bank groups (row stride
  // / 16 is odd).
  constexpr int ST = FPS_SB_ST;        // items per stage: ST / 32 32-item MFMA blocks
  constexpr int NB = ST / 32;
  constexpr int ROWB = 2 * D + 16;     // padded bytes per bf16 item row in LDS
  constexpr int CPR = D / 8;           // 16-B chunks per row
  constexpr int LPT = ST * CPR / 256;  // chunks per thread per stage
  static_assert(ST * CPR % 256 == 0, "stage chunks must divide over the workgroup");
  __shared__ __attribute__((aligned(16))) unsigned char xs[2][ST * ROWB];
  const uint4* __restrict__ X16 = reinterpret_cast<const uint4*>(Xb);
  // PD = prefetch distance in stages: 1 = the next stage's rows are loaded during this
  // stage's MFMAs (one register set); 2 = two register sets, the rows of stage st + 2
  // are issued at the start of stage st and stored to LDS at the end of stage st + 1 --
  // a stage (~16 MFMAs per wave) is shorter than an L2-miss round trip
  uint4 ldA[LPT], ldB[LPT];
  auto gload = [&](int s0, uint4 (&dst)[LPT]) {
#pragma unroll
    for (int u = 0; u < LPT; ++u) {
      const int c = tid + 256 * u, row = c / CPR, col = c % CPR;
      const int i = s0 + row;
      dst[u] = i < i_end ? X16[(int64_t)i * CPR + col] : make_uint4(0, 0, 0, 0);
    }
  };
  auto lstore = [&](int buf, const uint4 (&src)[LPT]) {
#pragma unroll
    for (int u = 0; u < LPT; ++u) {
      const int c = tid + 256 * u, row = c / CPR, col = c % CPR;
      *reinterpret_cast<uint4*>(&xs[buf][row * ROWB + col * 16]) = src[u];
    }
  };
  // the longest item of each of a stage's two blocks and (COORD) their coordinate
  // ranges, prefetched one stage ahead with the rows
  float2 cbs[NB][QB], cbn[NB][QB];
  float bms[NB], bmn[NB];
  auto cload = [&](int s0, float2 (&dst)[NB][QB]) {
#pragma unroll
    for (int bi = 0; bi < NB; ++bi) bmn[bi] = xbm[min((s0 + 32 * bi) >> 5, (N - 1) >> 5)];
    if (COORD && use_coord) {
#pragma unroll
      for (int bi = 0; bi < NB; ++bi) {
        const int blk = min((s0 + 32 * bi) / 32, (N - 1) / 32);
#pragma unroll
        for (int b = 0; b < QB; ++b) dst[bi][b] = cb[(int64_t)blk * D + fq[b]];
      }
    }
  };
  gload(i_begin, ldA);
  cload(i_begin, cbn);
  if (PD == 2 && i_begin + ST < i_end) gload(i_begin + ST, ldB);
  lstore(0, ldA);
  __syncthreads();
  // one stage: the MFMAs over LDS buffer `buf` (items s0 .. s0 + ST); nxt = the register
  // set that receives (PD = 1) or already holds (PD = 2) stage s0 + ST, far (PD = 2) the
  // free set that receives stage s0 + 2 ST
  auto stage = [&](const int s0, const int buf, uint4 (&nxt)[LPT], uint4 (&far)[LPT]) {
    const bool more = s0 + ST < i_end;
#pragma unroll
    for (int bi = 0; bi < NB; ++bi) bms[bi] = bmn[bi];
    if (COORD && use_coord) {
#pragma unroll
      for (int bi = 0; bi < NB; ++bi)
#pragma unroll
        for (int b = 0; b < QB; ++b) cbs[bi][b] = cbn[bi][b];
    }
    if (more) cload(s0 + ST, cbn);  // block bounds first: the next stage waits for them only
    if (PD == 1) {
      if (more) gload(s0 + ST, nxt);  // the next stage's rows are in flight during this stage's MFMAs
    } else if (s0 + 2 * ST < i_end) {
      gload(s0 + 2 * ST, far);
    }
    // CUR2: every block's A operands read from LDS at the start of the stage (the reads of
    // block bi + 1 in flight during block bi's MFMAs) instead of right before each block
    uint4 cur_all[CUR2 ? NB : 1][S];
    if constexpr (CUR2) {
#pragma unroll
      for (int bi = 0; bi < NB; ++bi) {
        const unsigned char* rowp = &xs[buf][(32 * bi + r) * ROWB + h * D];
#pragma unroll
        for (int s = 0; s < S; ++s) cur_all[bi][s] = *reinterpret_cast<const uint4*>(rowp + 16 * s);
      }
    }
#pragma unroll
    for (int bi = 0; bi < NB; ++bi) {
      const int i0 = s0 + 32 * bi;
      if (i0 >= i_end) break;  // uniform
      uint4 cur[S];
      if constexpr (CUR2) {
#pragma unroll
        for (int s = 0; s < S; ++s) cur[s] = cur_all[bi][s];
      } else {
        const unsigned char* rowp = &xs[buf][(32 * bi + r) * ROWB + h * D];  // half h = bytes [h D, h D + D)
#pragma unroll
        for (int s = 0; s < S; ++s) cur[s] = *reinterpret_cast<const uint4*>(rowp + 16 * s);
      }
      const float bm = bms[bi];  // longest item of this block
      // the passing scores of one (query block, 32-item block) into the block's LDS list
      auto emit = [&](int b, const floatx16& acc, float thr) {
        if (MASK) {  // passing registers as a bit mask, walked by ctz
          uint32_t bits = 0;
#pragma unroll
          for (int j = 0; j < 16; ++j) bits |= acc[j] > thr ? (1u << j) : 0u;
          while (bits) {
            const int j = __builtin_ctz(bits);
            bits &= bits - 1;
            const int item = i0 + (j & 3) + 8 * (j >> 2) + 4 * h;
            if (item < i_end) {
              if (lc[b] < SB_SLOTS) {
                lst[wave][b][lc[b]][lane] = (uint16_t)(item - i_begin);
                ++lc[b];
              } else {
                const int q = qrow[b];
                const int slot = atomicAdd(cnt + q, 1);
                if (slot < cap) cand_pos[(int64_t)q * cap + slot] = item;
              }
            }
          }
        } else {  // ~k ln(1 + n / s) passes per query and segment
#pragma unroll
          for (int j = 0; j < 16; ++j) {
            const int item = i0 + (j & 3) + 8 * (j >> 2) + 4 * h;
            if (acc[j] > thr && item < i_end) {
              if (lc[b] < SB_SLOTS) {
                lst[wave][b][lc[b]][lane] = (uint16_t)(item - i_begin);
                ++lc[b];
              } else {
                const int q = qrow[b];
                const int slot = atomicAdd(cnt + q, 1);
                if (slot < cap) cand_pos[(int64_t)q * cap + slot] = item;
              }
            }
          }
        }
      };
      // LEMP length + coordinate bounds of one 32 x 32 pair of blocks: false = skip
      // (wave-uniform)
      auto block_live = [&](int b) {
        if (!(COORD && use_coord)) return true;
        const bool lpass = qrow[b] < B && !(theta[b] > -INFINITY && ql[b] * bm * slack <= theta[b]);
        const bool pass = lpass && coord_pass(theta[b], ql[b], bm, qb[b], cbs[bi][b]);
        if (!__any(pass)) {
          // counted only when the length bound alone would have scored the pair: the
          // gates (coord_gate_kernel, LempTopK's per-batch switch) weigh what COORD
          // adds over LENGTH, not what the length bound skips anyway
          if (__any(lpass)) ++skipped;
          return false;
        }
        ++scored;
        return true;
      };
      auto mfma_block = [&](int b) {
        floatx16 acc = {0};
#pragma unroll
        for (int s = 0; s < S; ++s)
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, cur[s]),
                                                        __builtin_bit_cast(bf16x8, qv[b][s]), acc, 0, 0, 0);
        return acc;
      };
      auto filter = [&](int b, const floatx16& acc) {
        const float thr = theta[b] - margin * ql[b] * bm;
        float m = acc[0];
#pragma unroll
        for (int j = 1; j < 16; ++j) m = fmaxf(m, acc[j]);
        if (m > thr) emit(b, acc, thr);
      };
      bool lv[QB];
      bool all_live = true;
#pragma unroll
      for (int b = 0; b < QB; ++b) {
        lv[b] = block_live(b);
        all_live = all_live && lv[b];
      }
      if (ILV && QB > 1 && all_live) {
        // the QB chains interleaved k-step by k-step: independent MFMAs issue back to
        // back instead of each waiting for its predecessor's result, and every block's
        // filter runs after all the MFMAs (one chain + its max / emit at a time left the
        // matrix core idle through each dependency and each epilogue)
        floatx16 acc[QB];
#pragma unroll
        for (int b = 0; b < QB; ++b) acc[b] = floatx16{0};
#pragma unroll
        for (int s = 0; s < S; ++s)
#pragma unroll
          for (int b = 0; b < QB; ++b)
            acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, cur[s]),
                                                             __builtin_bit_cast(bf16x8, qv[b][s]), acc[b], 0, 0, 0);
#pragma unroll
        for (int b = 0; b < QB; ++b) filter(b, acc[b]);
      } else {
#pragma unroll
        for (int b = 0; b < QB; ++b)
          if (lv[b]) filter(b, mfma_block(b));
      }
    }
    if (more) lstore(buf ^ 1, nxt);  // every wave finished reading buf ^ 1 at the previous barrier
    __syncthreads();
  };
  if (PD == 1) {
    for (int s0 = i_begin, st = 0; s0 < i_end; s0 += ST, ++st) stage(s0, st & 1, ldA, ldB);
  } else {
    for (int s0 = i_begin; s0 < i_end; s0 += 2 * ST) {  // the register sets alternate: unrolled by 2
      stage(s0, 0, ldB, ldA);
      if (s0 + ST < i_end) stage(s0 + ST, 1, ldA, ldB);
    }
  }
  if (COORD && use_coord && stats != nullptr && lane == 0) {
    atomicAdd(stats, scored);
    atomicAdd(stats + 1, skipped);
  }
  // flush: both lane halves hold the same query; half 0 reserves for the pair
#pragma unroll
  for (int b = 0; b < QB; ++b) {
    const int q = qrow[b];
    const int c = lc[b];
    const int other = __shfl_xor(c, 32, 64);
    int base = 0;
    if (h == 0 && c + other > 0) base = atomicAdd(cnt + q, c + other);  // c + other > 0 implies q < B
    base = __shfl(base, r, 64);
    const int off = base + (h ? other : 0);
    for (int t = 0; t < c; ++t)
      if (off + t < cap) cand_pos[(int64_t)q * cap + off + t] = i_begin + lst[wave][b][t][lane];
  }
}

// Exact fp32 re-score of the candidates of one query per wave (4 queries per
// workgroup), 32 candidates per MFMA chain.  A = the query broadcast to all 32 rows
// (lane l supplies q[kk + (l >> 5)]), B = the 32 candidates' rows (lane l supplies
// x_{l & 31}[kk + (l >> 5)]); the k pairs run in score_tile's order, so acc[0]
// (row 0 or 4: every row is the same dot product) is bit-identical to the fp32
// scorer's value for that (query, item).
template <int D>
__global__ void __launch_bounds__(256) cand_rescore_kernel(const float* __restrict__ Q, const float* __restrict__ X,
                                                           const int64_t* __restrict__ ids, int B,
                                                           const float* __restrict__ best_s, int k,
                                                           const int32_t* __restrict__ cnt, int cap,
                                                           uint32_t* __restrict__ cand_key,
                                                           int64_t* __restrict__ cand_id) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = blockIdx.x * SB_WAVES + wave;
  if (q >= B) return;
  const int n = min(cnt[q], cap);
  if (n == 0) return;
  const int c = lane & 31, h = lane >> 5;
  // k pair t = (2t, 2t + 1): lane half h supplies element 2t + h.  Rows are read as
  // float4 (elements 4m .. 4m + 3 = pairs 2m and 2m + 1), a quarter of the load
  // instructions of one float per pair
  const float4* qr = reinterpret_cast<const float4*>(Q + (int64_t)q * D);
  float qh[D / 2];
#pragma unroll
  for (int m = 0; m < D / 4; ++m) {
    const float4 v = qr[m];
    qh[2 * m] = h ? v.y : v.x;
    qh[2 * m + 1] = h ? v.w : v.z;
  }
  const uint32_t ktau = sb_key(best_s[(int64_t)q * k + k - 1]);
  // every load of a chunk is unconditional (a clamped candidate for lanes past n, whose
  // column is computed and dropped): the guarded row loads compiled to a branch and a
  // full memory wait each -- 16 dependent round trips per 32 candidates
  for (int c0 = 0; c0 < n; c0 += 32) {
    const bool ok = c0 + c < n;
    const int64_t pos = cand_id[(int64_t)q * cap + min(c0 + c, n - 1)];
    const int64_t id = ids[pos];
    const float4* xr = reinterpret_cast<const float4*>(X + pos * D);
    float4 xv[D / 4];
#pragma unroll
    for (int m = 0; m < D / 4; ++m) xv[m] = xr[m];
    floatx16 acc = {0};
#pragma unroll
    for (int m = 0; m < D / 4; ++m) {
      const float4 v = xv[m];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(qh[2 * m], h ? v.y : v.x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(qh[2 * m + 1], h ? v.w : v.z, acc, 0, 0, 0);
    }
    if (ok && h == 0) {  // lanes 0..31: column c
      const uint32_t key = sb_key(acc[0]);
      cand_key[(int64_t)q * cap + c0 + c] = key > ktau ? key : 0u;
      cand_id[(int64_t)q * cap + c0 + c] = id;
    }
  }
}

}  // namespace

// COORD gate of a scan (evaluated while gate > 0): stats = cumulative (scored,
// skipped) block pairs, prev = their values at the previous update.  After a segment
// that evaluated the bound: on (1) if it skipped at least num / den of the block pairs,
// else off for the next `rest` segments (gate = -rest + 1 .. 0), after which the bound
// is probed again -- later LEMP buckets hold shorter items, where it prunes more.
// One thread; no host sync.
namespace {
__global__ void coord_gate_kernel(const int32_t* __restrict__ stats, int32_t* __restrict__ prev,
                                  int32_t* __restrict__ gate, int num, int den, int rest) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const int64_t ds = (int64_t)stats[0] - prev[0], dk = (int64_t)stats[1] - prev[1];
  if (ds + dk > 0) gate[0] = dk * den >= (ds + dk) * num ? 1 : 1 - rest;
  else gate[0] += 1;
  prev[0] = stats[0];
  prev[1] = stats[1];
}
}  // namespace

FPS_API int fps_coord_gate(const int32_t* stats, int32_t* prev, int32_t* gate, int num, int den, int rest,
                           void* stream) {
  hipLaunchKernelGGL(coord_gate_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, stats, prev, gate, num, den,
                     rest);
  FPS_CHECK_LAUNCH();
  return 0;
}

// Qb [B, D], Xb [N, D] bf16 (uint16 storage, RNE from the fp32 vectors); qlen [B] the
// fp32 query norms, xbm [ceil(N / 32)] the longest fp32 item norm of every 32-item block; cand_pos [B, cap] int64 receives item positions (0..N-1),
// cnt [B] (zeroed by the caller) counts every candidate.  D in {32, 64, 128}.
// COORD bound (optional, all or none): qf [B] focus coordinates, qbf [B] = q_f / |q|,
// cb [N / 32][D] float2 coordinate ranges of the 32-item blocks (N a multiple of 32
// or the last block's range over its items); stats (optional) = 2 counters.
// fewest workgroups a scorer launch aims for (items per workgroup shrink to reach it);
// 0: always SB_ITEMS items per workgroup (A/B knob, FPS_SB_MIN_WGS)
static int g_sb_min_wgs = 512;
FPS_API void fps_score_set_min_wgs(int v) { g_sb_min_wgs = v; }
// interleaved MFMA chains of a wave's query blocks (ILV; A/B knob FPS_SB_ILV=1): measured equal to one chain at a
// time (MFMA busy 33.8 vs 33.6 %, profiles/r6_scorer_ilv_ab.txt) -- other waves already hide the dependency -- at
// 8 more VGPRs, so off
static int g_sb_ilv = 0;
FPS_API void fps_score_set_ilv(int v) { g_sb_ilv = v; }
// prefetch distance of the LDS item stages (PD above; A/B knob FPS_SB_PD): 1 or 2
#ifndef FPS_SB_PD_DEFAULT
#define FPS_SB_PD_DEFAULT 1
#endif
static int g_sb_pd = FPS_SB_PD_DEFAULT;
FPS_API void fps_score_set_pd(int v) { g_sb_pd = v == 2 ? 2 : 1; }
// every block's LDS operand reads at the start of the stage (CUR2 above; A/B knob FPS_SB_CUR2=1, no COORD)
static int g_sb_cur2 = 0;
FPS_API void fps_score_set_cur2(int v) { g_sb_cur2 = v != 0; }

FPS_API int fps_score_filter_bf16(const uint16_t* Qb, const uint16_t* Xb, int B, int N, int D, const float* best_s,
                                  int k, const float* qlen, const float* xbm, float margin, float slack,
                                  int64_t* cand_pos, int32_t* cnt, int cap, const int32_t* qf, const float* qbf,
                                  const float2* cb, int32_t* stats, const int32_t* gate, void* stream) {
  if (B <= 0 || N <= 0) return 0;
  if (k <= 0 || cap <= 0 || qlen == nullptr || xbm == nullptr) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  const bool coord = qf != nullptr && qbf != nullptr && cb != nullptr;
  // items per workgroup: 1024, halved (down to one 64-item stage) while the launch would
  // have fewer than g_sb_min_wgs (512: best of 256 / 384 / 512 / 768 / 1024 / 1536 / 2304) workgroups -- the short first segments of a geometric
  // scan ran on 32-256 workgroups, 98 / 70 / 63 / 56 us on a mostly idle GPU
  // (profiles/r5_topk_segments.md)
#define FPS_SB(D_, QB_, MASK_)                                                                              \
  {                                                                                                         \
    const int64_t nqt = (B + SB_WAVES * 32 * QB_ - 1) / (SB_WAVES * 32 * QB_);                              \
    int ipw = SB_ITEMS;                                                                                     \
    while (ipw > 64 && nqt * ((N + ipw - 1) / ipw) < g_sb_min_wgs) ipw >>= 1;                             \
    const int64_t nit = (N + ipw - 1) / ipw;                                                                \
    if (nqt * nit > INT32_MAX) return (int)hipErrorInvalidValue;                                            \
    const dim3 grid((unsigned)(nqt * nit));                                                                 \
    if (coord && g_sb_ilv)                                                                                  \
      hipLaunchKernelGGL((score_filter_bf16_kernel<D_, QB_, MASK_, true, true>), grid, dim3(256), 0, s, Qb, \
                         Xb, B, N, best_s, k, qlen, xbm, margin, slack, cand_pos, cnt, cap, qf, qbf, cb,     \
                         stats, gate, ipw);                                                                 \
    else if (coord && g_sb_pd == 2)                                                                         \
      hipLaunchKernelGGL((score_filter_bf16_kernel<D_, QB_, MASK_, true, false, 2>), grid, dim3(256), 0, s,  \
                         Qb, Xb, B, N, best_s, k, qlen, xbm, margin, slack, cand_pos, cnt, cap, qf, qbf, cb, \
                         stats, gate, ipw);                                                                 \
    else if (coord)                                                                                         \
      hipLaunchKernelGGL((score_filter_bf16_kernel<D_, QB_, MASK_, true, false>), grid, dim3(256), 0, s, Qb,\
                         Xb, B, N, best_s, k, qlen, xbm, margin, slack, cand_pos, cnt, cap, qf, qbf, cb,     \
                         stats, gate, ipw);                                                                 \
    else if (g_sb_ilv)                                                                                      \
      hipLaunchKernelGGL((score_filter_bf16_kernel<D_, QB_, MASK_, false, true>), grid, dim3(256), 0, s,    \
                         Qb, Xb, B, N, best_s, k, qlen, xbm, margin, slack, cand_pos, cnt, cap, qf, qbf, cb, \
                         stats, gate, ipw);                                                                 \
    else if (g_sb_cur2)                                                                                     \
      hipLaunchKernelGGL((score_filter_bf16_kernel<D_, QB_, MASK_, false, false, 1, true>), grid, dim3(256), \
                         0, s, Qb, Xb, B, N, best_s, k, qlen, xbm, margin, slack, cand_pos, cnt, cap, qf, qbf,  \
                         cb, stats, gate, ipw);                                                             \
    else if (g_sb_pd == 2)                                                                                  \
      hipLaunchKernelGGL((score_filter_bf16_kernel<D_, QB_, MASK_, false, false, 2>), grid, dim3(256), 0, s,\
                         Qb, Xb, B, N, best_s, k, qlen, xbm, margin, slack, cand_pos, cnt, cap, qf, qbf, cb, \
                         stats, gate, ipw);                                                                 \
    else                                                                                                    \
      hipLaunchKernelGGL((score_filter_bf16_kernel<D_, QB_, MASK_, false, false>), grid, dim3(256), 0, s,   \
                         Qb, Xb, B, N, best_s, k, qlen, xbm, margin, slack, cand_pos, cnt, cap, qf, qbf, cb, \
                         stats, gate, ipw);                                                                 \
  }
  // D = 64: FPS_SB_QB64 query blocks per wave + the bit-mask epilogue (round 2: 4
  // blocks, the fastest of 1/2/4 with branch or mask epilogues, profiles/r2_bf16_topk.md;
  // round 5, with the LDS-staged items and the workgroup floor: 2,
  // profiles/r5_scorer_qb_ab.txt)
  switch (D) {
    case 32: FPS_SB(32, 2, true); break;
    case 64: FPS_SB(64, FPS_SB_QB64, true); break;
    case 128: FPS_SB(128, 1, true); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef FPS_SB
  FPS_CHECK_LAUNCH();
  return 0;
}

// Q [B, D], X [N, D] fp32 (the rows Qb / Xb were rounded from); cand_id holds the
// positions written by fps_score_filter_bf16 and receives ids[pos]; cand_key the
// exact keys (0 for candidates not strictly above best_s[q, k-1]).
FPS_API int fps_cand_rescore(const float* Q, const float* X, const int64_t* ids, int B, int D, const float* best_s,
                             int k, const int32_t* cnt, int cap, uint32_t* cand_key, int64_t* cand_id, void* stream) {
  if (B <= 0) return 0;
  if (k <= 0 || cap <= 0) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  const int grid = (B + SB_WAVES - 1) / SB_WAVES;
  switch (D) {
    case 32: hipLaunchKernelGGL((cand_rescore_kernel<32>), dim3(grid), dim3(256), 0, s, Q, X, ids, B, best_s, k, cnt, cap,
                                cand_key, cand_id); break;
    case 64: hipLaunchKernelGGL((cand_rescore_kernel<64>), dim3(grid), dim3(256), 0, s, Q, X, ids, B, best_s, k, cnt, cap,
                                cand_key, cand_id); break;
    case 128: hipLaunchKernelGGL((cand_rescore_kernel<128>), dim3(grid), dim3(256), 0, s, Q, X, ids, B, best_s, k, cnt,
                                 cap, cand_key, cand_id); break;
    default: return (int)hipErrorInvalidValue;
  }
  FPS_CHECK_LAUNCH();
  return 0;
}

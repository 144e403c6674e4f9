// Word2vec skip-gram negative-sampling step on MFMA (gfx950).  Kernel K6.
//
// Block-shared negatives (Ji et al., "Parallelizing Word2Vec in Shared and
// Distributed Memory"): a workgroup takes M = 32 (center, context) pairs and
// K = 32 negatives shared by all of them, which turns the negative side of
// SGNS into three small GEMMs that run on the matrix cores:
//
//   S  = H . N^T            [M x K]   scores of every center against every negative
//   dH = G . N + g+ (x) O   [M x D]   center gradients      (G = -lr*w*sigmoid(S))
//   dN = G^T . H            [K x D]   negative-row gradients
//   dO = g+ (x) H           [M x D]   positive-context gradients (VALU)
//
// with g+ = lr * (1 - sigmoid(h.o)) and w = neg_per_pair / K so the expected
// gradient equals classic SGNS with ``neg_per_pair`` negatives per pair.
// fp32 in / fp32 accumulate: v_mfma_f32_32x32x2_f32 (exact f32 FMA chain,
// cdna_hip_programming.md §3).  H and N are staged in LDS with rows padded
// to an odd dword stride (conflict-free row-strided operand reads, §2 bank
// rule), 16-B loads, every load of a wave's 4 rows issued before its first
// LDS store (v1 staged one row per wave at a time: latency-bound at one
// block per CU).  S = H N^T is four 16x16x4 MFMA tiles, one per wave, over
// the full K (no cross-wave partial-score buffer) while the other 12 waves
// compute the positive scores.  The context rows O are not staged: they are
// read once, coalesced, for h.o and again in the dH epilogue.  1024-thread
// blocks (16 waves) at one block per CU (87 KB of LDS at D = 300).
// Gradients are accumulated with no-return float atomics straight from the
// MFMA accumulator layout: one register = two rows x 32 consecutive floats,
// the full-rate atomic shape (MI355X_MICROARCH.md "Global float atomics").
//
// Inputs are the pulled rows of the two tables (rows_in for centers,
// rows_out for contexts and negatives, fp32 or bf16) and per-pair row
// positions; outputs are per-unique-row deltas pushed back to the PS.
#include "common.h"

using namespace fps;

typedef float floatx16 __attribute__((ext_vector_type(16)));

namespace {

constexpr int M = 32;    // pairs per block
constexpr int K = 32;    // shared negatives per block
constexpr int NT = 1024; // threads per block (16 waves: one block per CU holds 87 KB of LDS)
constexpr int NW = NT / 64;

template <bool BF16>
__device__ __forceinline__ float ld1(const void* rows, int64_t idx) {
  if (BF16) return bf16_to_f32(((const uint16_t*)rows)[idx]);
  return ((const float*)rows)[idx];
}

// 4 consecutive elements of a row (c..c+3), zero beyond D
template <bool BF16>
__device__ __forceinline__ float4 ld4(const void* rows, int64_t row, int D, int c) {
  const int64_t o = row * D + c;
  float v[4];
  if (c + 3 < D && ((o & 3) == 0)) {
    if (BF16) {
      const uint2 u = *(const uint2*)((const uint16_t*)rows + o);
      return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                         __uint_as_float(u.y & 0xffff0000u));
    }
    return *(const float4*)((const float*)rows + o);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = (c + j < D) ? ld1<BF16>(rows, o + j) : 0.f;
  return make_float4(v[0], v[1], v[2], v[3]);
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }

// C/D map of the 32x32 MFMA: lane l, reg r -> row (col = l & 31)
__device__ __forceinline__ int acc_row(int lane, int r) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

typedef float floatx4 __attribute__((ext_vector_type(4)));

template <bool BF16>
__global__ void __launch_bounds__(NT) sgns_block_kernel(const void* __restrict__ rows_in,
                                                        const void* __restrict__ rows_out,
                                                        const int32_t* __restrict__ pos_c,
                                                        const int32_t* __restrict__ pos_o,
                                                        const int32_t* __restrict__ pos_neg, int64_t n_pairs,
                                                        int D, float lr, float neg_weight,
                                                        float* __restrict__ d_in, float* __restrict__ d_out,
                                                        float* __restrict__ loss_out) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int Dp = (D + 31) & ~31;   // output tiles of 32 columns
  const int LD = Dp + 1;           // odd dword stride
  float* Hs = smem;                // [M][LD]
  float* Ns = Hs + M * LD;         // [K][LD]
  float* Gs = Ns + K * LD;         // [M][K+1]
  float* gpos = Gs + M * (K + 1);  // [M]
  int32_t* pc = (int32_t*)(gpos + M);  // [M]
  int32_t* po = pc + M;                // [M]
  int32_t* pn = po + M;                // [K]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float* scr = (float*)(pn + K) + (size_t)wave * 32 * 33;  // [NW][32][33] wave-private dH tile scratch
  const int64_t n_blocks = (n_pairs + M - 1) / M;
  constexpr int RPW = (M + K) / NW;  // staged rows per wave (4)

  for (int64_t blk = blockIdx.x; blk < n_blocks; blk += gridDim.x) {
    const int64_t p0 = blk * M;
    const int npairs = (int)((n_pairs - p0) < M ? (n_pairs - p0) : M);
    if (tid < M) {
      pc[tid] = tid < npairs ? pos_c[p0 + tid] : -1;
      po[tid] = tid < npairs ? pos_o[p0 + tid] : -1;
    } else if (tid < M + K) {
      pn[tid - M] = pos_neg[blk * K + (tid - M)];
    }
    __syncthreads();
    // ---- stage H and N: RPW rows per wave, every 16-B load of the wave's rows
    // issued before the first LDS store (latency paid once per block, not per row)
    {
      float4 v[RPW][2];
#pragma unroll
      for (int j = 0; j < RPW; ++j) {
        const int r = wave + NW * j;
        const bool is_h = r < M;
        const int32_t rr = is_h ? pc[r] : pn[r - M];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int c = lane * 4 + 256 * h;
          v[j][h] = (rr >= 0 && c < Dp) ? ld4<BF16>(is_h ? rows_in : rows_out, rr, D, c)
                                        : make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
#pragma unroll
      for (int j = 0; j < RPW; ++j) {
        const int r = wave + NW * j;
        float* dst = r < M ? Hs + r * LD : Ns + (r - M) * LD;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int c = lane * 4 + 256 * h;
          if (c < Dp) { dst[c] = v[j][h].x; dst[c + 1] = v[j][h].y; dst[c + 2] = v[j][h].z; dst[c + 3] = v[j][h].w; }
        }
      }
    }
    __syncthreads();
    if (wave < 4) {
      // ---- S = H N^T: four 16x16 tiles, one per wave, full K (no cross-wave reduction)
      const int ti = wave >> 1, tj = wave & 1;
      const int i = lane & 15, kq = lane >> 4;
      floatx4 acc = {0.f, 0.f, 0.f, 0.f};
      const float* hrow = Hs + (16 * ti + i) * LD + kq;
      const float* nrow = Ns + (16 * tj + i) * LD + kq;
      for (int k = 0; k < Dp; k += 4) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(hrow[k], nrow[k], acc, 0, 0, 0);
      // C/D: col = lane & 15, row = 4 * (lane >> 4) + r
      float lsum = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = 16 * ti + 4 * kq + r, kk = 16 * tj + i;
        const bool ok = m < npairs;
        const float sg = sigmoidf_(acc[r]);
        Gs[m * (K + 1) + kk] = ok ? -lr * neg_weight * sg : 0.f;
        if (ok) lsum += -neg_weight * __logf(1.f - sg + 1e-12f);
      }
      if (loss_out) {
        lsum = group_sum<64>(lsum);
        if (lane == 0) atomicAdd(loss_out, lsum);
      }
    } else {
      // ---- positive scores h.o (O read from global, coalesced), waves 4..15
      for (int m = wave - 4; m < M; m += NW - 4) {
        float p = 0.f;
        if (m < npairs) {
#pragma unroll 5
          for (int c = lane; c < D; c += 64) p = fmaf(Hs[m * LD + c], ld1<BF16>(rows_out, (int64_t)po[m] * D + c), p);
        }
        p = group_sum<64>(p);
        if (lane == 0) {
          const bool ok = m < npairs;
          gpos[m] = ok ? lr * (1.f - sigmoidf_(p)) : 0.f;
          if (ok && loss_out) atomicAdd(loss_out, -__logf(sigmoidf_(p) + 1e-12f));
        }
      }
    }
    __syncthreads();
    // ---- dH = G N (+ g+ O) and dN = G^T H: 2 * Dp/32 output tiles over NW waves
    const int ntile = Dp / 32;
    for (int t = wave; t < 2 * ntile; t += NW) {
      const bool is_h = t < ntile;
      const int c0 = (is_h ? t : t - ntile) * 32;
      floatx16 acc = {0};
      const int i = lane & 31, kh = lane >> 5;
#pragma unroll 4
      for (int kk = 0; kk < 32; kk += 2) {
        const int k = kk + kh;
        const float a = is_h ? Gs[i * (K + 1) + k] : Gs[k * (K + 1) + i];
        const float b = is_h ? Ns[k * LD + c0 + i] : Hs[k * LD + c0 + i];
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
      }
      const int col = c0 + (lane & 31);
      if (is_h) {
        // dH rows of pairs that share a center (center-major pair order:
        // skipgram_pairs) are summed through LDS first -- one atomic row per
        // run of equal centers instead of one per pair
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = acc_row(lane, r);
          float v = acc[r];
          if (row < npairs && col < D) v += gpos[row] * ld1<BF16>(rows_out, (int64_t)po[row] * D + col);
          scr[row * 33 + (lane & 31)] = v;
        }
        // wave-private scratch: the wave's own LDS writes are visible to it after
        // the LDS counter drains (no block barrier needed)
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
        if (col < D) {
          const int r0 = 16 * (lane >> 5), r1 = min(r0 + 16, npairs);
          float run = 0.f;
          for (int row = r0; row < r1; ++row) {
            run += scr[row * 33 + (lane & 31)];
            if (row + 1 == r1 || pc[row + 1] != pc[row]) {
              atomic_add_noret(d_in + (int64_t)pc[row] * D + col, run);
              run = 0.f;
            }
          }
        }
      } else if (col < D) {
#pragma unroll
        for (int r = 0; r < 16; ++r) atomic_add_noret(d_out + (int64_t)pn[acc_row(lane, r)] * D + col, acc[r]);
      }
    }
    // ---- dO = g+ H: one wave per row, 256-B atomic wave-instructions
    for (int m = wave; m < npairs; m += NW) {
      const float g = gpos[m];
      float* dst = d_out + (int64_t)po[m] * D;
      for (int c = lane; c < D; c += 64) atomic_add_noret(dst + c, g * Hs[m * LD + c]);
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------- v4
// M = 32 pairs x K4 = 16 shared negatives per block, 512-thread blocks, ~64 KB
// of LDS: two blocks per CU, so one block's float atomics drain while the
// other stages rows and runs its MFMAs (v3 held one 1024-thread block per CU at
// 154 KB: its waves waited ~81 % of their cycles, SQ_WAIT_ANY / SQ_WAVE_CYCLES,
// profiles/r1_w2v_v4.md).  The dH run reduction gathers a tile column's 32
// rows in registers with one half-wave swap instead of a wave-private LDS tile,
// and dN = G^T H is a 32x32x2 MFMA whose rows 16-31 are zero.
constexpr int K4 = 16;
constexpr int NT4 = 512;
constexpr int NW4 = NT4 / 64;

// GROUP > 1: GROUP consecutive blocks of 32 pairs share one set of K4 negatives
// (pos_neg holds K4 rows per 32 * GROUP pairs).  The negative rows are staged once
// per group and their gradient dN = sum over the group's blocks of G^T H stays in
// registers until the group ends: per 32 pairs the dN float atomics (16 of the
// ~33 rows a v4 block pushes) and the N staging loads shrink by 1 / GROUP.  Each
// pair still sees K4 negatives of weight negatives / K4 (same expected gradient).
template <bool BF16, int GROUP>
__global__ void __launch_bounds__(NT4) __attribute__((amdgpu_waves_per_eu(4, 8))) sgns_v4_kernel(const void* __restrict__ rows_in,
                                                      const void* __restrict__ rows_out,
                                                      const int32_t* __restrict__ pos_c,
                                                      const int32_t* __restrict__ pos_o,
                                                      const int32_t* __restrict__ pos_neg, int64_t n_pairs, int D,
                                                      float lr, float neg_weight, float* __restrict__ d_in,
                                                      float* __restrict__ d_out, float* __restrict__ loss_out) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int Dp = (D + 31) & ~31;
  const int LD = Dp + 1;
  float* Hs = smem;                 // [M][LD]
  float* Ns = Hs + M * LD;          // [K4][LD]
  float* Gs = Ns + K4 * LD;         // [M][K4+1]
  float* gpos = Gs + M * (K4 + 1);  // [M]
  int32_t* pc = (int32_t*)(gpos + M);
  int32_t* po = pc + M;
  int32_t* pn = po + M;             // [K4]
  int32_t* lead = pn + K4;          // [M] first pair of the block with the same context
  int32_t* nxt = lead + M;          // [M] next pair with the same context (-1: none)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t n_groups = (n_pairs + M * GROUP - 1) / (M * GROUP);
  constexpr int RPW = (M + K4) / NW4;  // staged rows per wave (6)
  const int ntile = Dp / 32;
  const int i = lane & 31, kh = lane >> 5;

  // a block's pair / negative indices (wave 0: lanes < 32 the pairs, 32..47 the negatives)
  // are requested one block ahead, before the current block's float atomics: vmcnt
  // retires in issue order, so loads issued after them would wait for the atomics
  auto fetch_idx = [&](int64_t g, int sb, int32_t& a, int32_t& b) {
    const int64_t q0 = (g * GROUP + sb) * M;
    a = -1;
    b = -1;
    if (g >= n_groups || q0 >= n_pairs) return;
    if (tid < M) {
      if (q0 + tid < n_pairs) { a = pos_c[q0 + tid]; b = pos_o[q0 + tid]; }
    } else if (sb == 0 && tid < M + K4) {
      a = pos_neg[g * K4 + (tid - M)];
    }
  };
  int32_t nx_a = -1, nx_b = -1;
  if (wave == 0) fetch_idx(blockIdx.x, 0, nx_a, nx_b);
  for (int64_t grp = blockIdx.x; grp < n_groups; grp += gridDim.x) {
    // dN accumulators of this wave's (<= 2) negative-gradient column tiles t = wave + 8 j,
    // t >= ntile, kept across the group's blocks
    floatx16 dn0 = {0}, dn1 = {0};
    for (int sb = 0; sb < GROUP; ++sb) {
      const int64_t p0 = (grp * GROUP + sb) * M;
      if (p0 >= n_pairs) break;  // uniform: the group's tail
      const int npairs = (int)((n_pairs - p0) < M ? (n_pairs - p0) : M);
      if (tid < M) {
        pc[tid] = nx_a;
        po[tid] = nx_b;
      } else if (sb == 0 && tid < M + K4) {
        pn[tid - M] = nx_a;
      }
      __syncthreads();
      if (wave == 0) {  // the next block's indices, in flight during this block
        const bool last = sb + 1 == GROUP || (grp * GROUP + sb + 1) * M >= n_pairs;
        fetch_idx(last ? grp + gridDim.x : grp, last ? 0 : sb + 1, nx_a, nx_b);
      }
      if (wave == 0) {  // adjacent centers share most of their window: one dO row per distinct
                        // context (12.9 distinct contexts per 32 pairs on the bench corpus).
                        // Lane t < 32 finds the pairs with its context by register shuffles
                        // (the LDS scan it replaces was two dependent 32-step loops).
        const int mine = lane < M ? po[lane] : -2;
        uint32_t same = 0u;
#pragma unroll
        for (int j = 0; j < M; ++j) same |= (uint32_t)(__shfl(mine, j, 64) == mine) << j;
        if (lane < M) {
          const uint32_t above = same & ~((2u << lane) - 1u);  // matches after this pair
          lead[lane] = __ffs(same) - 1;                        // first match (itself at the latest)
          nxt[lane] = above ? __ffs(above) - 1 : -1;
        }
      }
      {
        float4 v[RPW][2];
#pragma unroll
        for (int j = 0; j < RPW; ++j) {
          const int r = wave + NW4 * j;
          const bool is_h = r < M;
          const int32_t rr = is_h ? pc[r] : (sb == 0 ? pn[r - M] : -1);  // N rows: once per group
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int c = lane * 4 + 256 * h;
            v[j][h] = (rr >= 0 && c < Dp) ? ld4<BF16>(is_h ? rows_in : rows_out, rr, D, c)
                                          : make_float4(0.f, 0.f, 0.f, 0.f);
          }
        }
#pragma unroll
        for (int j = 0; j < RPW; ++j) {
          const int r = wave + NW4 * j;
          if (r >= M && sb > 0) continue;  // keep the group's staged negatives
          float* dst = r < M ? Hs + r * LD : Ns + (r - M) * LD;
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int c = lane * 4 + 256 * h;
            if (c < Dp) { dst[c] = v[j][h].x; dst[c + 1] = v[j][h].y; dst[c + 2] = v[j][h].z; dst[c + 3] = v[j][h].w; }
          }
        }
      }
      __syncthreads();
      if (wave < 2) {
        // ---- S = H N^T [32 x 16]: one 16x16 tile per wave over the full D
        const int ii = lane & 15, kq = lane >> 4;
        floatx4 acc = {0.f, 0.f, 0.f, 0.f};
        const float* hrow = Hs + (16 * wave + ii) * LD + kq;
        const float* nrow = Ns + ii * LD + kq;
        for (int k = 0; k < Dp; k += 4) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(hrow[k], nrow[k], acc, 0, 0, 0);
        float lsum = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = 16 * wave + 4 * kq + r;
          const bool ok = m < npairs;
          const float sg = sigmoidf_(acc[r]);
          Gs[m * (K4 + 1) + ii] = ok ? -lr * neg_weight * sg : 0.f;
          if (ok) lsum += -neg_weight * __logf(1.f - sg + 1e-12f);
        }
        if (loss_out) {
          lsum = group_sum<64>(lsum);
          if (lane == 0) atomicAdd(loss_out, lsum);
        }
      } else if (Dp <= 320) {
        // ---- positive scores h.o, waves 2..7: every O value this wave needs (its <= 6
        // pairs x 5 columns per lane) is loaded before the first is used -- one global
        // latency per block instead of one per pair
        constexpr int KP = (M + NW4 - 3) / (NW4 - 2), JP = 5;
        const int w2 = wave - 2;
        float ov[KP][JP];
#pragma unroll
        for (int k = 0; k < KP; ++k) {
          const int m = w2 + (NW4 - 2) * k;
#pragma unroll
          for (int j = 0; j < JP; ++j) {
            const int c = lane + 64 * j;
            ov[k][j] = (m < npairs && c < D) ? ld1<BF16>(rows_out, (int64_t)po[m] * D + c) : 0.f;
          }
        }
#pragma unroll
        for (int k = 0; k < KP; ++k) {
          const int m = w2 + (NW4 - 2) * k;
          if (m >= M) break;  // uniform in the wave
          float p = 0.f;
#pragma unroll
          for (int j = 0; j < JP; ++j) {
            const int c = lane + 64 * j;
            if (c < D) p = fmaf(Hs[m * LD + c], ov[k][j], p);
          }
          p = group_sum<64>(p);
          if (lane == 0) {
            const bool ok = m < npairs;
            gpos[m] = ok ? lr * (1.f - sigmoidf_(p)) : 0.f;
            if (ok && loss_out) atomicAdd(loss_out, -__logf(sigmoidf_(p) + 1e-12f));
          }
        }
      } else {
        // ---- positive scores h.o (O read from global, coalesced), waves 2..7
        for (int m = wave - 2; m < M; m += NW4 - 2) {
          float p = 0.f;
          if (m < npairs) {
#pragma unroll 5
            for (int c = lane; c < D; c += 64) p = fmaf(Hs[m * LD + c], ld1<BF16>(rows_out, (int64_t)po[m] * D + c), p);
          }
          p = group_sum<64>(p);
          if (lane == 0) {
            const bool ok = m < npairs;
            gpos[m] = ok ? lr * (1.f - sigmoidf_(p)) : 0.f;
            if (ok && loss_out) atomicAdd(loss_out, -__logf(sigmoidf_(p) + 1e-12f));
          }
        }
      }
      __syncthreads();
      // ---- dH = G N + g+ O [32 x 32 cols] (pushed) and dN += G^T H [16 (of 32) x 32 cols]
      int slot = 0;
      for (int t = wave; t < 2 * ntile; t += NW4) {
        const bool is_h = t < ntile;
        const int c0 = (is_h ? t : t - ntile) * 32;
        const int col = c0 + i;
        if (is_h) {
          floatx16 acc = {0};
#pragma unroll
          for (int kk = 0; kk < K4; kk += 2) {
            const int k = kk + kh;
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(Gs[i * (K4 + 1) + k], Ns[k * LD + c0 + i], acc, 0, 0, 0);
          }
          float v[16], o[16];
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = acc_row(lane, r);
            v[r] = acc[r];
            if (row < npairs && col < D) v[r] += gpos[row] * ld1<BF16>(rows_out, (int64_t)po[row] * D + col);
          }
#pragma unroll
          for (int r = 0; r < 16; ++r) o[r] = __shfl_xor(v[r], 32, 64);
          // this half-wave (kh) owns rows 16*kh .. 16*kh+15 of column col; row q sits in
          // register (q&3) + 4*(q>>3) of the lane half whose (q>>2)&1 matches
          const int r1 = min(16, npairs - 16 * kh);
          float run = 0.f;
#pragma unroll
          for (int j = 0; j < 16; ++j) {
            const int ri0 = (j & 3) + 4 * (j >> 3);         // q = j      (kh = 0)
            const int ri1 = (j & 3) + 4 * (2 + (j >> 3));   // q = 16 + j (kh = 1)
            const float a0 = (j & 4) ? o[ri0] : v[ri0];
            const float a1 = (j & 4) ? v[ri1] : o[ri1];
            const float val = kh ? a1 : a0;
            if (j < r1) {
              const int q = 16 * kh + j;
              run += val;
              if (j + 1 == r1 || pc[q + 1] != pc[q]) {
                if (col < D) atomic_add_noret(d_in + (int64_t)pc[q] * D + col, run);
                run = 0.f;
              }
            }
          }
        } else {
          floatx16 acc = {0};
          if constexpr (GROUP > 1) acc = slot == 0 ? dn0 : dn1;
#pragma unroll
          for (int kk = 0; kk < M; kk += 2) {
            const int k = kk + kh;
            const float a = i < K4 ? Gs[k * (K4 + 1) + i] : 0.f;
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, Hs[k * LD + c0 + i], acc, 0, 0, 0);
          }
          if constexpr (GROUP == 1) {  // v4: pushed at once
            if (col < D) {
#pragma unroll
              for (int r = 0; r < 8; ++r) atomic_add_noret(d_out + (int64_t)pn[acc_row(lane, r)] * D + col, acc[r]);
            }
          } else {
            if (slot == 0) dn0 = acc; else dn1 = acc;
            ++slot;
          }
        }
      }
      // ---- dO = g+ H summed over the pairs of one context: one wave per distinct
      // context, 256-B atomic wave-instructions
      for (int m = wave; m < npairs; m += NW4) {
        if (lead[m] != m) continue;  // uniform in the wave
        float a[(512 + 63) / 64];
#pragma unroll
        for (int u = 0; u < 8; ++u) a[u] = 0.f;
        for (int q = m; q >= 0 && q < npairs; q = nxt[q]) {
          const float g = gpos[q];
#pragma unroll
          for (int u = 0; u < 8; ++u)
            if (lane + 64 * u < D) a[u] += g * Hs[q * LD + lane + 64 * u];
        }
        float* dst = d_out + (int64_t)po[m] * D;
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (lane + 64 * u < D) atomic_add_noret(dst + lane + 64 * u, a[u]);
      }
      __syncthreads();
    }
    if constexpr (GROUP > 1) {
      // ---- the group's negative gradients, once
      int slot = 0;
      for (int t = wave; t < 2 * ntile; t += NW4) {
        if (t < ntile) continue;
        const int col = (t - ntile) * 32 + i;
        const floatx16 acc = slot == 0 ? dn0 : dn1;
        if (col < D) {
#pragma unroll
          for (int r = 0; r < 8; ++r) atomic_add_noret(d_out + (int64_t)pn[acc_row(lane, r)] * D + col, acc[r]);
        }
        ++slot;
      }
      __syncthreads();  // pn is rewritten by the next group
    }
  }
}

}  // namespace

FPS_API size_t fps_sgns_smem_bytes(int D) {
  const int Dp = (D + 31) & ~31, LD = Dp + 1;
  return sizeof(float) * ((size_t)2 * 32 * LD + 32 * 33 + 32 + (size_t)NW * 32 * 33) + sizeof(int32_t) * 96;
}

FPS_API size_t fps_sgns_v4_smem_bytes(int D) {
  const int Dp = (D + 31) & ~31, LD = Dp + 1;
  return sizeof(float) * ((size_t)(32 + K4) * LD + 32 * (K4 + 1) + 32) + sizeof(int32_t) * (128 + K4);
}

// v4: pos_neg holds 16 negative rows per block of 32 pairs
// group: blocks of 32 pairs sharing one set of 16 negatives (1, 2 or 4); pos_neg
// holds 16 rows per 32 * group pairs
FPS_API int fps_sgns_step_v4g(const void* rows_in, const void* rows_out, int rows_bf16, const int32_t* pos_c,
                              const int32_t* pos_o, const int32_t* pos_neg, int64_t n_pairs, int D, float lr,
                              float neg_weight, float* d_in, float* d_out, float* loss_out, int group, void* stream) {
  if (n_pairs <= 0) return 0;
  if (((D + 31) & ~31) > 512) return (int)hipErrorInvalidValue;
  if (group != 1 && group != 2 && group != 4) return (int)hipErrorInvalidValue;
  const size_t smem = fps_sgns_v4_smem_bytes(D);
  if (smem > 80 * 1024) return (int)hipErrorInvalidValue;  // two blocks per CU
  const int64_t ng = (n_pairs + 32 * group - 1) / (32 * group);
  const int grid = (int)(ng < 256 * 2 * 4 ? ng : 256 * 2 * 4);
  hipStream_t s = (hipStream_t)stream;
#define FPS_SGNS_V4(BF, G)                                                                                            \
  do {                                                                                                               \
    (void)hipFuncSetAttribute((const void*)sgns_v4_kernel<BF, G>, hipFuncAttributeMaxDynamicSharedMemorySize,        \
                              (int)smem);                                                                            \
    hipLaunchKernelGGL((sgns_v4_kernel<BF, G>), dim3(grid), dim3(NT4), smem, s, rows_in, rows_out, pos_c, pos_o,     \
                       pos_neg, n_pairs, D, lr, neg_weight, d_in, d_out, loss_out);                                  \
  } while (0)
  if (rows_bf16) {
    if (group == 1) FPS_SGNS_V4(true, 1);
    else if (group == 2) FPS_SGNS_V4(true, 2);
    else FPS_SGNS_V4(true, 4);
  } else {
    if (group == 1) FPS_SGNS_V4(false, 1);
    else if (group == 2) FPS_SGNS_V4(false, 2);
    else FPS_SGNS_V4(false, 4);
  }
#undef FPS_SGNS_V4
  FPS_CHECK_LAUNCH();
  return 0;
}

// pos_neg holds K = 32 negative rows per block of 32 pairs (ceil(n_pairs/32) blocks)
FPS_API int fps_sgns_step(const void* rows_in, const void* rows_out, int rows_bf16, const int32_t* pos_c,
                          const int32_t* pos_o, const int32_t* pos_neg, int64_t n_pairs, int D, float lr,
                          float neg_weight, float* d_in, float* d_out, float* loss_out, void* stream) {
  if (n_pairs <= 0) return 0;
  if (((D + 31) & ~31) > 512) return (int)hipErrorInvalidValue;  // staging covers 2 x 256 columns
  const size_t smem = fps_sgns_smem_bytes(D);
  if (smem > 160 * 1024) return (int)hipErrorInvalidValue;
  const int64_t nb = (n_pairs + 31) / 32;
  const int grid = (int)(nb < 256 * 16 ? nb : 256 * 16);
  hipStream_t s = (hipStream_t)stream;
  if (rows_bf16) {
    (void)hipFuncSetAttribute((const void*)sgns_block_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    hipLaunchKernelGGL(sgns_block_kernel<true>, dim3(grid), dim3(NT), smem, s, rows_in, rows_out, pos_c, pos_o,
                       pos_neg, n_pairs, D, lr, neg_weight, d_in, d_out, loss_out);
  } else {
    (void)hipFuncSetAttribute((const void*)sgns_block_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    hipLaunchKernelGGL(sgns_block_kernel<false>, dim3(grid), dim3(NT), smem, s, rows_in, rows_out, pos_c, pos_o,
                       pos_neg, n_pairs, D, lr, neg_weight, d_in, d_out, loss_out);
  }
  FPS_CHECK_LAUNCH();
  return 0;
}

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
// rule), one wave per row with 16-B loads (a 1 KiB coalesced transaction
// per wave-instruction).  The context rows O are not staged: they are read
// once, coalesced, for h.o and again in the dH epilogue.  512-thread blocks
// (8 waves) keep enough loads in flight at one block per CU.
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

constexpr int M = 32;   // pairs per block
constexpr int K = 32;   // shared negatives per block
constexpr int NT = 512; // threads per block
constexpr int NW = NT / 64;

template <bool BF16>
__device__ __forceinline__ float ld1(const void* rows, int64_t idx) {
  if (BF16) return bf16_to_f32(((const uint16_t*)rows)[idx]);
  return ((const float*)rows)[idx];
}

// 4 consecutive elements of a row (c..c+3), zero beyond D
template <bool BF16>
__device__ __forceinline__ void ld4(const void* rows, int64_t row, int D, int c, float (&v)[4]) {
  const int64_t o = row * D + c;
  if (c + 3 < D && ((o & 3) == 0)) {
    if (BF16) {
      const uint2 u = *(const uint2*)((const uint16_t*)rows + o);
      v[0] = __uint_as_float(u.x << 16); v[1] = __uint_as_float(u.x & 0xffff0000u);
      v[2] = __uint_as_float(u.y << 16); v[3] = __uint_as_float(u.y & 0xffff0000u);
    } else {
      const float4 f = *(const float4*)((const float*)rows + o);
      v[0] = f.x; v[1] = f.y; v[2] = f.z; v[3] = f.w;
    }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = (c + j < D) ? ld1<BF16>(rows, o + j) : 0.f;
  }
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }

// C/D map of the 32x32 MFMA: lane l, reg r -> row (col = l & 31)
__device__ __forceinline__ int acc_row(int lane, int r) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

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
  float* Sred = Gs + M * (K + 1);  // [NW][M][K] per-wave partial scores
  float* gpos = Sred + NW * M * K; // [M]
  int32_t* pc = (int32_t*)(gpos + M);  // [M]
  int32_t* po = pc + M;                // [M]
  int32_t* pn = po + M;                // [K]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t n_blocks = (n_pairs + M - 1) / M;

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
    // ---- stage H and N: one wave per row, 16-B loads, zero padded
    for (int r = wave; r < M + K; r += NW) {
      const bool is_h = r < M;
      const int32_t rr = is_h ? pc[r] : pn[r - M];
      float* dst = is_h ? Hs + r * LD : Ns + (r - M) * LD;
      for (int c = lane * 4; c < Dp; c += 256) {
        float v[4] = {0.f, 0.f, 0.f, 0.f};
        if (rr >= 0) ld4<BF16>(is_h ? rows_in : rows_out, rr, D, c, v);
#pragma unroll
        for (int j = 0; j < 4; ++j) dst[c + j] = v[j];
      }
    }
    __syncthreads();
    // ---- S = H N^T: each wave 1/NW of the k range (k-steps of 2)
    {
      floatx16 acc = {0};
      const int ksteps = Dp / 2;
      const int per = (ksteps + NW - 1) / NW;
      const int k_beg = wave * per, k_end = min(ksteps, k_beg + per);
      const int i = lane & 31, kh = lane >> 5;
      for (int ks = k_beg; ks < k_end; ++ks) {
        const int k = 2 * ks + kh;
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(Hs[i * LD + k], Ns[i * LD + k], acc, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) Sred[(wave * M + acc_row(lane, r)) * K + (lane & 31)] = acc[r];
    }
    // ---- positive scores h.o, O read straight from global (coalesced)
    for (int m = wave; m < M; m += NW) {
      float p = 0.f;
      if (m < npairs) {
        for (int c = lane; c < D; c += 64) p = fmaf(Hs[m * LD + c], ld1<BF16>(rows_out, (int64_t)po[m] * D + c), p);
      }
      p = group_sum<64>(p);
      if (lane == 0) {
        const bool ok = m < npairs;
        gpos[m] = ok ? lr * (1.f - sigmoidf_(p)) : 0.f;
        if (ok && loss_out) atomicAdd(loss_out, -__logf(sigmoidf_(p) + 1e-12f));
      }
    }
    __syncthreads();
    for (int e = tid; e < M * K; e += NT) {
      const int m = e / K;
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) s += Sred[w * M * K + e];
      const bool ok = m < npairs;
      Gs[m * (K + 1) + (e % K)] = ok ? -lr * neg_weight * sigmoidf_(s) : 0.f;
      if (ok && loss_out) atomicAdd(loss_out, -neg_weight * __logf(1.f - sigmoidf_(s) + 1e-12f));
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
      if (col < D) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = acc_row(lane, r);
          if (is_h) {
            if (row < npairs) {
              const float v = acc[r] + gpos[row] * ld1<BF16>(rows_out, (int64_t)po[row] * D + col);
              atomic_add_noret(d_in + (int64_t)pc[row] * D + col, v);
            }
          } else {
            atomic_add_noret(d_out + (int64_t)pn[row] * D + col, acc[r]);
          }
        }
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

}  // namespace

FPS_API size_t fps_sgns_smem_bytes(int D) {
  const int Dp = (D + 31) & ~31, LD = Dp + 1;
  return sizeof(float) * ((size_t)2 * 32 * LD + 32 * 33 + NW * 32 * 32 + 32) + sizeof(int32_t) * 96;
}

// pos_neg holds K = 32 negative rows per block of 32 pairs (ceil(n_pairs/32) blocks)
FPS_API int fps_sgns_step(const void* rows_in, const void* rows_out, int rows_bf16, const int32_t* pos_c,
                          const int32_t* pos_o, const int32_t* pos_neg, int64_t n_pairs, int D, float lr,
                          float neg_weight, float* d_in, float* d_out, float* loss_out, void* stream) {
  if (n_pairs <= 0) return 0;
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

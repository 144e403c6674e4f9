// Inner-product scoring on MFMA for top-K retrieval (gfx950).  Kernel K8 (scoring part).
//
//   S[b, i] = <Q[b, :], X[i, :]>      Q [B, D] fp32, X [N, D] fp32, S [B, N] fp32
//
// The LEMP top-K worker scores each query user against a length-sorted bucket
// of item vectors (M/matrix/factorization/workers/PSTopKGeneratorWorker.scala:46-110);
// on the GPU a bucket is a [B x bucket] GEMM.  fp32 in / fp32 accumulate with
// v_mfma_f32_32x32x2_f32 (exact f32 FMA chain, so scores match the CPU
// reference bit-for-bit up to summation order).  Workgroup tile 64 x 64,
// 4 waves in a 2 x 2 grid of 32 x 32 MFMA tiles; K staged through LDS in
// 32-wide slabs with rows padded to an odd dword stride (conflict-free
// row-strided operand reads); 16-B global loads; XCD-aware block remap so the
// blocks sharing an item panel run on one XCD's L2.
#include "common.h"

using namespace fps;

typedef float floatx16 __attribute__((ext_vector_type(16)));

namespace {

constexpr int TB = 64;   // tile rows (queries) and cols (items)
constexpr int KB = 32;   // k slab
constexpr int LDK = KB + 1;

__device__ __forceinline__ int acc_row(int lane, int r) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

// The 64 x 64 score tile (q0.., i0..) of this workgroup: wave (wr, wc) holds the
// 32 x 32 sub-tile in acc (row wr*32 + acc_row(lane, r), column wc*32 + lane%32).
__device__ __forceinline__ floatx16 score_tile(const float* __restrict__ Q, const float* __restrict__ X, int B,
                                               int N, int D, int q0, int i0, float* Qs, float* Xs) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  floatx16 acc = {0};
  for (int k0 = 0; k0 < D; k0 += KB) {
    // stage 64 rows x 32 floats of Q and X: 256 threads x 4 floats x 2 passes each
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      const int e = (pass * 256 + tid);  // 0..511 -> (row, float4 column)
      const int r = e >> 3, c4 = (e & 7) * 4;
      const int kq = k0 + c4;
      float qv[4] = {0.f, 0.f, 0.f, 0.f}, xv[4] = {0.f, 0.f, 0.f, 0.f};
      const int qrow = q0 + r, xrow = i0 + r;
      if (qrow < B) {
        if (kq + 3 < D && ((((int64_t)qrow * D + kq) & 3) == 0)) {
          const float4 f = *(const float4*)(Q + (int64_t)qrow * D + kq);
          qv[0] = f.x; qv[1] = f.y; qv[2] = f.z; qv[3] = f.w;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) qv[j] = kq + j < D ? Q[(int64_t)qrow * D + kq + j] : 0.f;
        }
      }
      if (xrow < N) {
        if (kq + 3 < D && ((((int64_t)xrow * D + kq) & 3) == 0)) {
          const float4 f = *(const float4*)(X + (int64_t)xrow * D + kq);
          xv[0] = f.x; xv[1] = f.y; xv[2] = f.z; xv[3] = f.w;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) xv[j] = kq + j < D ? X[(int64_t)xrow * D + kq + j] : 0.f;
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        Qs[r * LDK + c4 + j] = qv[j];
        Xs[r * LDK + c4 + j] = xv[j];
      }
    }
    __syncthreads();
    const int ar = wr * 32 + (lane & 31), br = wc * 32 + (lane & 31), kh = lane >> 5;
#pragma unroll
    for (int kk = 0; kk < KB; kk += 2)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(Qs[ar * LDK + kk + kh], Xs[br * LDK + kk + kh], acc, 0, 0, 0);
    __syncthreads();
  }
  return acc;
}

// workgroup -> (query tile, item tile): query tiles fastest, so the (few) blocks
// that read one item panel are consecutive logical ids, i.e. on one XCD, and X
// is fetched into one L2
__device__ __forceinline__ void tile_of(int B, int N, int& q0, int& i0) {
  const int nbx = (N + TB - 1) / TB, nby = (B + TB - 1) / TB;
  const int wg = xcd_remap(blockIdx.x, nbx * nby);
  q0 = (wg % nby) * TB;
  i0 = (wg / nby) * TB;
}

__global__ void __launch_bounds__(256) score_gemm_kernel(const float* __restrict__ Q, const float* __restrict__ X,
                                                         float* __restrict__ S, int B, int N, int D, int64_t ldS) {
  __shared__ float Qs[TB * LDK];
  __shared__ float Xs[TB * LDK];
  int q0, i0;
  tile_of(B, N, q0, i0);
  const floatx16 acc = score_tile(Q, X, B, N, D, q0, i0, Qs, Xs);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int col = i0 + wc * 32 + (lane & 31);
  if (col < N) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = q0 + wr * 32 + acc_row(lane, r);
      if (row < B) S[(int64_t)row * ldS + col] = acc[r];
    }
  }
}

__device__ __forceinline__ uint32_t score_key(float f) {  // order-preserving float -> uint32 (as topk.hip)
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// Scoring fused with the top-K threshold filter: scores are never stored; each
// one strictly above its query's current k-th best (best_s[q, k-1]) is appended
// to the query's candidate list (key, item id) -- after the first items of a
// length-sorted scan, only a few hundred of a bucket's 64k items per query pass.
// cnt[q] counts every passing score; entries beyond cap are dropped (the caller
// sees cnt > cap and rescans the segment unfused).
//
// With qlen / xlen (vector norms) the LEMP length bound is applied per tile on
// the device: a tile none of whose 64 queries can be beaten by its longest item
// (|q| * max|x| * slack <= theta_q) exits before loading anything -- exact, and
// it replaces the host-side "every query settled" test per bucket (a host sync).

__global__ void __launch_bounds__(256) score_filter_kernel(const float* __restrict__ Q, const float* __restrict__ X,
                                                           const int64_t* __restrict__ ids, int B, int N, int D,
                                                           const float* __restrict__ best_s, int k,
                                                           const float* __restrict__ qlen,
                                                           const float* __restrict__ xlen, float slack,
                                                           uint32_t* __restrict__ cand_key,
                                                           int64_t* __restrict__ cand_id, int32_t* __restrict__ cnt,
                                                           int cap) {
  __shared__ float Qs[TB * LDK];
  __shared__ float Xs[TB * LDK];
  __shared__ uint32_t ktau[TB];
  int q0, i0;
  tile_of(B, N, q0, i0);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float theta = INFINITY;
  if (tid < TB && q0 + tid < B) theta = best_s[(int64_t)(q0 + tid) * k + k - 1];
  if (xlen != nullptr) {
    float xl = (tid < TB && i0 + tid < N) ? xlen[i0 + tid] : 0.f;
    xl = group_max<64>(xl);  // wave 0 holds the tile's 64 items
    int live = 0;
    if (tid < TB && q0 + tid < B) live = !(theta > -INFINITY && qlen[q0 + tid] * xl * slack <= theta);
    if (!__syncthreads_or(live)) return;  // uniform: the whole workgroup leaves
  }
  if (tid < TB) ktau[tid] = q0 + tid < B ? score_key(theta) : 0xffffffffu;
  // (score_tile's first __syncthreads orders the ktau stores before the reads below)
  const floatx16 acc = score_tile(Q, X, B, N, D, q0, i0, Qs, Xs);
  const int wr = wave >> 1, wc = wave & 1;
  const int col = i0 + wc * 32 + (lane & 31);
  if (col >= N) return;
  const int64_t id = ids[col];
  // (one counter atomic per passing score: a per-wave aggregated reservation was
  // measured slower -- its registers cost occupancy, 8 -> 6 waves/SIMD)
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int rl = wr * 32 + acc_row(lane, r);
    const uint32_t key = score_key(acc[r]);
    if (key > ktau[rl]) {  // rows past B have ktau = max: never pass
      const int q = q0 + rl;
      const int slot = atomicAdd(cnt + q, 1);
      if (slot < cap) {
        cand_key[(int64_t)q * cap + slot] = key;
        cand_id[(int64_t)q * cap + slot] = id;
      }
    }
  }
}

}  // namespace

FPS_API int fps_score_filter(const float* Q, const float* X, const int64_t* ids, int B, int N, int D,
                             const float* best_s, int k, uint32_t* cand_key, int64_t* cand_id, int32_t* cnt, int cap,
                             void* stream) {
  if (B <= 0 || N <= 0) return 0;
  if (k <= 0 || cap <= 0) return (int)hipErrorInvalidValue;
  const int nwg = ((N + TB - 1) / TB) * ((B + TB - 1) / TB);
  hipLaunchKernelGGL(score_filter_kernel, dim3(nwg), dim3(256), 0, (hipStream_t)stream, Q, X, ids, B, N, D, best_s, k,
                     nullptr, nullptr, 1.f, cand_key, cand_id, cnt, cap);
  FPS_CHECK_LAUNCH();
  return 0;
}

// the same with the per-tile LEMP length bound (qlen [B], xlen [N]; both or neither)
FPS_API int fps_score_filter_lemp(const float* Q, const float* X, const int64_t* ids, int B, int N, int D,
                                  const float* best_s, int k, const float* qlen, const float* xlen, float slack,
                                  uint32_t* cand_key, int64_t* cand_id, int32_t* cnt, int cap, void* stream) {
  if (B <= 0 || N <= 0) return 0;
  if (k <= 0 || cap <= 0 || D <= 0) return (int)hipErrorInvalidValue;
  if ((qlen == nullptr) != (xlen == nullptr)) return (int)hipErrorInvalidValue;
  const int64_t nwg = (int64_t)((N + TB - 1) / TB) * ((B + TB - 1) / TB);
  if (nwg > INT32_MAX) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(score_filter_kernel, dim3((unsigned)nwg), dim3(256), 0, (hipStream_t)stream, Q, X, ids, B, N, D,
                     best_s, k, qlen, xlen, slack, cand_key, cand_id, cnt, cap);
  FPS_CHECK_LAUNCH();
  return 0;
}

FPS_API int fps_score_gemm(const float* Q, const float* X, float* S, int B, int N, int D, int64_t ldS, void* stream) {
  if (B <= 0 || N <= 0) return 0;
  const int nwg = ((N + TB - 1) / TB) * ((B + TB - 1) / TB);
  hipLaunchKernelGGL(score_gemm_kernel, dim3(nwg), dim3(256), 0, (hipStream_t)stream, Q, X, S, B, N, D, ldS);
  FPS_CHECK_LAUNCH();
  return 0;
}

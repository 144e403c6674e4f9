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

template <int NPL>
__global__ void __launch_bounds__(256) sgns_std_kernel(const float* __restrict__ rows_in,
                                                       const float* __restrict__ rows_out,
                                                       const int32_t* __restrict__ pos_c,
                                                       const int32_t* __restrict__ pos_o,
                                                       const int32_t* __restrict__ pos_neg, int64_t P, int D, int k,
                                                       float lr, float* __restrict__ d_in, float* __restrict__ d_out,
                                                       float* __restrict__ loss, int chunk) {
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
    float* dst = d_in + (int64_t)cur * D;
#pragma unroll
    for (int m = 0; m < NPL; ++m) {
      const int j = lane + 64 * m;
      if (j < D) atomic_add_noret(dst + j, h[m] - h0[m]);
    }
  };
  for (int64_t p = p0; p < p1; ++p) {
    const int32_t c = pos_c[p];
    if (c != cur) {  // a new center run: push the previous run's change, load this center
      flush();
      cur = c;
      const float* src = rows_in + (int64_t)c * D;
#pragma unroll
      for (int m = 0; m < NPL; ++m) {
        const int j = lane + 64 * m;
        h[m] = j < D ? src[j] : 0.f;
        h0[m] = h[m];
      }
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
      for (int q = 0; q < SG; ++q) {  // all loads of the group in flight
        const float* src = rows_out + (int64_t)(row[q] < 0 ? 0 : row[q]) * D;
#pragma unroll
        for (int m = 0; m < NPL; ++m) {
          const int j = lane + 64 * m;
          xv[q][m] = (row[q] >= 0 && j < D) ? src[j] : 0.f;
        }
      }
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
        float* dst = d_out + (int64_t)row[q] * D;
#pragma unroll
        for (int m = 0; m < NPL; ++m) {
          const int j = lane + 64 * m;
          if (j < D) atomic_add_noret(dst + j, g * h[m]);
          dh[m] += g * xv[q][m];
        }
      }
    }
#pragma unroll
    for (int m = 0; m < NPL; ++m) h[m] += dh[m];
  }
  flush();
  if (loss != nullptr && lane == 0) atomicAdd(loss, lsum);
}

}  // namespace

// P pairs: centers pos_c[P] (rows of rows_in / d_in), contexts pos_o[P] and
// k negatives per pair pos_neg[P * k] (rows of rows_out / d_out); fp32 rows,
// D <= 512.  loss (optional, zeroed by the caller) receives the summed loss.
FPS_API int fps_sgns_standard(const float* rows_in, const float* rows_out, const int32_t* pos_c,
                              const int32_t* pos_o, const int32_t* pos_neg, int64_t P, int D, int k, float lr,
                              float* d_in, float* d_out, float* loss, void* stream) {
  if (P <= 0) return 0;
  if (D <= 0 || D > 512 || k < 0) return (int)hipErrorInvalidValue;
  // ~16 pairs per wave: long enough to reuse a center across its window, short
  // enough for >= 32k waves at 1M pairs (the GPU holds ~8k)
  const int chunk = 16;
  const int64_t waves = (P + chunk - 1) / chunk;
  const int64_t blocks = (waves + 3) / 4;
  if (blocks > INT32_MAX) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
#define FPS_SGS(NPL_)                                                                                            \
  hipLaunchKernelGGL(sgns_std_kernel<NPL_>, dim3((unsigned)blocks), dim3(256), 0, s, rows_in, rows_out, pos_c,    \
                     pos_o, pos_neg, P, D, k, lr, d_in, d_out, loss, chunk)
  if (D <= 64) FPS_SGS(1);
  else if (D <= 128) FPS_SGS(2);
  else if (D <= 256) FPS_SGS(4);
  else if (D <= 320) FPS_SGS(5);
  else FPS_SGS(8);
#undef FPS_SGS
  FPS_CHECK_LAUNCH();
  return 0;
}

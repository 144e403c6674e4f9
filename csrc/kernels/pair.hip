// Pairwise embedding SGD on pulled rows (gfx950).  The compute kernel of the
// sparse-embedding workload (BASELINE config #5: a 100B-parameter table
// sharded over the PS, SURVEY §7 item 4 "capacity / bounded staleness").
//
// Every example is a pair of ids (a, b) of ONE sharded table plus a label;
// both rows were pulled (rows[pa[i]], rows[pb[i]], wire fp32 or bf16) and the
// updates accumulate into the per-unique-key delta buffer that is pushed back
// to the owners -- the push/pull shape of the reference's MF worker
// (M/matrix/factorization/workers/PSOnlineMatrixFactorizationWorker.scala:41-55)
// with both sides served by the PS, like its word2vec-style uses.
//
//   s = <ea, eb>
//   loss 0 (logistic, label in {0,1}):  g = label - sigmoid(s)
//   loss 1 (squared):                   g = label - s
//   delta[pa] += lr * g * eb ;  delta[pb] += lr * g * ea
//
// Layout: TPR lanes per pair (one fp32 per lane at D = 64), UNR pairs in
// flight per lane group, no-return float atomics into the delta rows (the
// 4*D-byte contiguous shape).  Optional loss sum (double, one atomic per block).
#include "common.h"

using namespace fps;

namespace {

template <int TPR, int NV, int UNR, bool ROWS_BF16>
__global__ void __launch_bounds__(256) pair_sgd_pulled_kernel(const void* __restrict__ rows,
                                                              const int32_t* __restrict__ pa,
                                                              const int32_t* __restrict__ pb,
                                                              const float* __restrict__ label,
                                                              float* __restrict__ delta, int64_t B, int D, float lr,
                                                              int loss_kind, double* __restrict__ loss_out) {
  constexpr int RPW = 64 / TPR;
  __shared__ float red[4];
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int64_t first = wave * RPW + lane / TPR, step = nwaves * RPW;
  const int j0 = lane % TPR;
  float lacc = 0.f;
  for (int64_t base = first; base < B; base += step * UNR) {
    float av[UNR][NV], bv[UNR][NV], yv[UNR];
    int64_t ra[UNR], rb[UNR];
    bool ok[UNR];
#pragma unroll
    for (int q = 0; q < UNR; ++q) {
      const int64_t i = base + (int64_t)q * step;
      ok[q] = i < B;
      ra[q] = ok[q] ? (int64_t)pa[i] * D : 0;
      rb[q] = ok[q] ? (int64_t)pb[i] * D : 0;
      yv[q] = ok[q] ? label[i] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < UNR; ++q) {
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const int j = j0 + v * TPR;
        const bool in = ok[q] && j < D;
        if (ROWS_BF16) {
          av[q][v] = in ? bf16_to_f32(((const uint16_t*)rows)[ra[q] + j]) : 0.f;
          bv[q][v] = in ? bf16_to_f32(((const uint16_t*)rows)[rb[q] + j]) : 0.f;
        } else {
          av[q][v] = in ? ((const float*)rows)[ra[q] + j] : 0.f;
          bv[q][v] = in ? ((const float*)rows)[rb[q] + j] : 0.f;
        }
      }
    }
#pragma unroll
    for (int q = 0; q < UNR; ++q) {
      float p = 0.f;
#pragma unroll
      for (int v = 0; v < NV; ++v) p = fmaf(av[q][v], bv[q][v], p);
      const float s = group_sum<TPR>(p);
      float g;
      if (loss_kind == 0) {
        const float sig = 1.f / (1.f + __expf(-s));
        g = yv[q] - sig;
        // -log(sigmoid(s)) for positives, -log(1 - sigmoid(s)) for negatives (stable form)
        const float z = yv[q] > 0.5f ? s : -s;
        if (ok[q] && j0 == 0) lacc += fmaxf(-z, 0.f) + log1pf(__expf(-fabsf(z)));
      } else {
        g = yv[q] - s;
        if (ok[q] && j0 == 0) lacc += 0.5f * g * g;
      }
      if (!ok[q]) continue;
      const float c = lr * g;
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const int j = j0 + v * TPR;
        if (j >= D) break;
        atomic_add_noret(delta + ra[q] + j, c * bv[q][v]);
        atomic_add_noret(delta + rb[q] + j, c * av[q][v]);
      }
    }
  }
  if (loss_out != nullptr) {
    lacc = group_sum<64>(lacc);
    if (lane == 0) red[threadIdx.x >> 6] = lacc;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(loss_out, (double)(red[0] + red[1] + red[2] + red[3]));
  }
}

}  // namespace

#define PAIR_TPR_SWITCH(D, ...)                                                 \
  do {                                                                          \
    if ((D) <= 8) { constexpr int TPR = 8, NV = 1; __VA_ARGS__; }               \
    else if ((D) <= 16) { constexpr int TPR = 16, NV = 1; __VA_ARGS__; }        \
    else if ((D) <= 32) { constexpr int TPR = 32, NV = 1; __VA_ARGS__; }        \
    else if ((D) <= 64) { constexpr int TPR = 64, NV = 1; __VA_ARGS__; }        \
    else if ((D) <= 128) { constexpr int TPR = 64, NV = 2; __VA_ARGS__; }       \
    else if ((D) <= 256) { constexpr int TPR = 64, NV = 4; __VA_ARGS__; }       \
    else if ((D) <= 512) { constexpr int TPR = 64, NV = 8; __VA_ARGS__; }       \
    else { return (int)hipErrorInvalidValue; }                                  \
  } while (0)

FPS_API int fps_pair_sgd_pulled(const void* rows, int rows_bf16, const int32_t* pa, const int32_t* pb,
                                const float* label, float* delta, int64_t B, int D, float lr, int loss_kind,
                                double* loss_out, void* stream) {
  if (B <= 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  constexpr int UNR = 4;
  PAIR_TPR_SWITCH(D, {
    const int g = grid_for(B, 4 * (64 / TPR) * UNR, 256 * 8);
    if (rows_bf16)
      hipLaunchKernelGGL((pair_sgd_pulled_kernel<TPR, NV, UNR, true>), dim3(g), dim3(256), 0, s, rows, pa, pb, label,
                         delta, B, D, lr, loss_kind, loss_out);
    else
      hipLaunchKernelGGL((pair_sgd_pulled_kernel<TPR, NV, UNR, false>), dim3(g), dim3(256), 0, s, rows, pa, pb, label,
                         delta, B, D, lr, loss_kind, loss_out);
  });
  FPS_CHECK_LAUNCH();
  return 0;
}

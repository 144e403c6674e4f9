// Item-grouped MF SGD (gfx950): one lane group per item, the item's ratings
// processed sequentially against a register-resident item row.
//
// Why: the flat kernel (mf.hip) issues one 256-B float-atomic add per rating
// into the item table; at ~1 KiB of traffic per rating it sits near the
// chip-wide ~1.3 TB/s atomic ceiling (profiles/README.md).  Grouping a
// micro-batch by item (a counting sort, csr_* below) lets each item row be
// read once, updated in registers across all its ratings of the batch, and
// written back once with a plain store -- no item atomics at all.  Per rating
// only the user row moves (256 B read + 256 B write).
//
// Semantics: inside a micro-batch an item's ratings are applied sequentially
// (exact per-item SGD, like the reference worker processing one item's
// FIFO); user rows are Hogwild across items, as in the flat kernel.
//   local mode  : I is the local PS shard; the row is updated in place.
//   pulled mode : I is the pulled-rows buffer (read only); the kernel writes
//                 delta[g] = (final row - pulled row) for the push.
#include "common.h"

using namespace fps;

namespace {

__global__ void csr_count_kernel(const int32_t* __restrict__ key, int64_t n, int32_t* __restrict__ cnt) {
  for (int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; b < n; b += (int64_t)gridDim.x * blockDim.x)
    atomicAdd(cnt + key[b], 1);
}

// ptr = exclusive prefix of cnt (computed by the caller); cursor zeroed
__global__ void csr_scatter_kernel(const int32_t* __restrict__ key, int64_t n, const int32_t* __restrict__ ptr,
                                   int32_t* __restrict__ cursor, int32_t* __restrict__ order) {
  for (int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; b < n; b += (int64_t)gridDim.x * blockDim.x) {
    const int32_t k = key[b];
    const int32_t s = atomicAdd(cursor + k, 1);
    order[ptr[k] + s] = (int32_t)b;
  }
}

// PF: user rows prefetched per batch of the group's ratings
template <int TPR, int NV, int PF, bool PULLED, bool ROWS_BF16>
__global__ void __launch_bounds__(256) mf_sgd_grouped_kernel(float* __restrict__ U, void* __restrict__ I,
                                                             const int32_t* __restrict__ uid,
                                                             const float* __restrict__ rating,
                                                             const int32_t* __restrict__ ptr,
                                                             const int32_t* __restrict__ order, int64_t G, int D,
                                                             float lr, float lambda, float* __restrict__ delta) {
  constexpr int RPW = 64 / TPR;
  const int lane = threadIdx.x & 63;
  const int j0 = lane % TPR;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t g = wave * RPW + lane / TPR; g < G; g += nwaves * RPW) {
    const int32_t beg = ptr[g], end = ptr[g + 1];
    if (beg == end) continue;  // uniform inside the lane group
    float iv[NV], i0[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int j = j0 + v * TPR;
      float x = 0.f;
      if (j < D) {
        if (ROWS_BF16) x = bf16_to_f32(((const uint16_t*)I)[g * D + j]);
        else x = ((const float*)I)[g * D + j];
      }
      iv[v] = x;
      i0[v] = x;
    }
    for (int32_t s = beg; s < end; s += PF) {
      float uv[PF][NV], rv[PF];
      int64_t urow[PF];
#pragma unroll
      for (int q = 0; q < PF; ++q) {
        const bool ok = s + q < end;
        const int32_t b = ok ? order[s + q] : 0;
        urow[q] = ok ? (int64_t)uid[b] * D : -1;
        rv[q] = ok ? rating[b] : 0.f;
      }
#pragma unroll
      for (int q = 0; q < PF; ++q) {
#pragma unroll
        for (int v = 0; v < NV; ++v) {
          const int j = j0 + v * TPR;
          uv[q][v] = (urow[q] >= 0 && j < D) ? U[urow[q] + j] : 0.f;
        }
      }
#pragma unroll
      for (int q = 0; q < PF; ++q) {
        if (urow[q] < 0) break;  // uniform inside the group
        float p = 0.f;
#pragma unroll
        for (int v = 0; v < NV; ++v) p = fmaf(uv[q][v], iv[v], p);
        const float e = rv[q] - group_sum<TPR>(p);
#pragma unroll
        for (int v = 0; v < NV; ++v) {
          const int j = j0 + v * TPR;
          const float u = uv[q][v], it = iv[v];
          if (j < D) U[urow[q] + j] = u + lr * (e * it - lambda * u);
          iv[v] = it + lr * (e * u - lambda * it);
        }
      }
    }
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int j = j0 + v * TPR;
      if (j >= D) continue;
      if (PULLED) delta[g * D + j] = iv[v] - i0[v];
      else ((float*)I)[g * D + j] = iv[v];
    }
  }
}

}  // namespace

#define NV_TPR_SWITCH_G(D, ...)                                                 \
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

FPS_API int fps_csr_count(const int32_t* key, int64_t n, int32_t* cnt, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(csr_count_kernel, dim3(grid_for(n, 256, 256 * 16)), dim3(256), 0, (hipStream_t)stream, key, n,
                     cnt);
  FPS_CHECK_LAUNCH();
  return 0;
}

FPS_API int fps_csr_scatter(const int32_t* key, int64_t n, const int32_t* ptr, int32_t* cursor, int32_t* order,
                            void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(csr_scatter_kernel, dim3(grid_for(n, 256, 256 * 16)), dim3(256), 0, (hipStream_t)stream, key,
                     n, ptr, cursor, order);
  FPS_CHECK_LAUNCH();
  return 0;
}

// rows_mode: 0 = local fp32 table updated in place, 1 = pulled fp32 rows, 2 = pulled bf16 rows
FPS_API int fps_mf_sgd_grouped(float* U, void* I, int rows_mode, const int32_t* uid, const float* r,
                               const int32_t* ptr, const int32_t* order, int64_t G, int D, float lr, float lambda,
                               float* delta, void* stream) {
  if (G <= 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  constexpr int PF = 4;
  NV_TPR_SWITCH_G(D, {
    const int g = grid_for(G, 4 * (64 / TPR), 256 * 16);
    if (rows_mode == 0)
      hipLaunchKernelGGL((mf_sgd_grouped_kernel<TPR, NV, PF, false, false>), dim3(g), dim3(256), 0, s, U, I, uid, r, ptr, order, G, D, lr, lambda, delta);
    else if (rows_mode == 1)
      hipLaunchKernelGGL((mf_sgd_grouped_kernel<TPR, NV, PF, true, false>), dim3(g), dim3(256), 0, s, U, I, uid, r, ptr, order, G, D, lr, lambda, delta);
    else
      hipLaunchKernelGGL((mf_sgd_grouped_kernel<TPR, NV, PF, true, true>), dim3(g), dim3(256), 0, s, U, I, uid, r, ptr, order, G, D, lr, lambda, delta);
  });
  FPS_CHECK_LAUNCH();
  return 0;
}

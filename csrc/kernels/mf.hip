// Matrix-factorization SGD kernels (gfx950).  K4 (fused SGD step) + K14 (RMSE).
//
// Reference math (FactorUpdater / SGDUpdater,
// M/matrix/factorization/factors/SGDUpdater.scala:3-13, applied by the online
// worker M/matrix/factorization/workers/PSOnlineMatrixFactorizationWorker.scala:41-55):
//   e = r - u.i ; du = lr*e*i ; di = lr*e*u ; u += du (worker) ; push(item, di)
// Optional L2 term ``lambda`` (the reference leaves "fixme add lambda").
//
// Two forms:
//  * mf_sgd_local  -- the PS shard holding the items is on this GPU: the
//    "pull" is a direct read of the item row and the "push" a no-return
//    global_atomic_add_f32 of di into it (one fused pass, no wire buffers).
//  * mf_sgd_pulled -- items arrived from remote PS shards (all-to-all):
//    rows[pos[b]] is the pulled value, di is accumulated (atomically, the
//    batch may hit an item many times) into the per-unique-key delta buffer
//    that is pushed back to the owners.
// In both, user rows live in this worker's HBM table (ratings are
// partitioned by user, M/matrix/factorization/PSOnlineMatrixFactorization.scala:62-64).
//
// Each rating is handled by TPR lanes (TPR = D for D = 64); UNR ratings are
// in flight per lane group to hide HBM latency (4 rows/wave in flight is the
// measured sweet spot for random-row gathers, MI355X_MICROARCH.md).
#include "common.h"

using namespace fps;

namespace {

template <int TPR>
__device__ __forceinline__ void group_coords(int64_t& first, int64_t& step, int& j0) {
  constexpr int RPW = 64 / TPR;
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  first = wave * RPW + lane / TPR;
  step = nwaves * RPW;
  j0 = lane % TPR;
}

// seg != nullptr: the batch is the segment [seg[0], seg[1]) of uid/iid/rating,
// read on the device (item-block rotation: segment sizes never visit the host)
template <int TPR, int NV, int UNR, bool USER_ATOMIC>
__global__ void __launch_bounds__(256) mf_sgd_local_kernel(float* __restrict__ U, float* __restrict__ I,
                                                           const int32_t* __restrict__ uid,
                                                           const int32_t* __restrict__ iid,
                                                           const float* __restrict__ rating, int64_t B, int D,
                                                           float lr, float lambda,
                                                           const int32_t* __restrict__ seg) {
  if (seg != nullptr) {
    const int32_t beg = seg[0];
    B = seg[1] - beg;
    uid += beg; iid += beg; rating += beg;
  }
  int64_t first, step; int j0;
  group_coords<TPR>(first, step, j0);
  for (int64_t base = first; base < B; base += step * UNR) {
    float uv[UNR][NV], iv[UNR][NV], rv[UNR];
    int64_t urow[UNR], irow[UNR];
    bool ok[UNR];
#pragma unroll
    for (int q = 0; q < UNR; ++q) {
      const int64_t b = base + (int64_t)q * step;
      ok[q] = b < B;
      urow[q] = ok[q] ? (int64_t)uid[b] * D : 0;
      irow[q] = ok[q] ? (int64_t)iid[b] * D : 0;
      rv[q] = ok[q] ? rating[b] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < UNR; ++q) {
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const int j = j0 + v * TPR;
        const bool in = ok[q] && j < D;
        uv[q][v] = in ? U[urow[q] + j] : 0.f;
        iv[q][v] = in ? I[irow[q] + j] : 0.f;
      }
    }
#pragma unroll
    for (int q = 0; q < UNR; ++q) {
      float p = 0.f;
#pragma unroll
      for (int v = 0; v < NV; ++v) p = fmaf(uv[q][v], iv[q][v], p);
      const float dot = group_sum<TPR>(p);
      const float e = rv[q] - dot;
      if (!ok[q]) continue;
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const int j = j0 + v * TPR;
        if (j >= D) break;
        const float du = lr * (e * iv[q][v] - lambda * uv[q][v]);
        const float di = lr * (e * uv[q][v] - lambda * iv[q][v]);
        if (USER_ATOMIC) atomic_add_noret(U + urow[q] + j, du);
        else U[urow[q] + j] = uv[q][v] + du;
        atomic_add_noret(I + irow[q] + j, di);
      }
    }
  }
}

template <int TPR, int NV, int UNR, bool ROWS_BF16>
__global__ void __launch_bounds__(256) mf_sgd_pulled_kernel(float* __restrict__ U, const int32_t* __restrict__ uid,
                                                            const float* __restrict__ rating,
                                                            const void* __restrict__ rows,
                                                            const int32_t* __restrict__ pos,
                                                            float* __restrict__ delta, int64_t B, int D, float lr,
                                                            float lambda, int user_atomic) {
  int64_t first, step; int j0;
  group_coords<TPR>(first, step, j0);
  for (int64_t base = first; base < B; base += step * UNR) {
    float uv[UNR][NV], iv[UNR][NV], rv[UNR];
    int64_t urow[UNR], prow[UNR];
    bool ok[UNR];
#pragma unroll
    for (int q = 0; q < UNR; ++q) {
      const int64_t b = base + (int64_t)q * step;
      ok[q] = b < B;
      urow[q] = ok[q] ? (int64_t)uid[b] * D : 0;
      prow[q] = ok[q] ? (int64_t)pos[b] * D : 0;
      rv[q] = ok[q] ? rating[b] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < UNR; ++q) {
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const int j = j0 + v * TPR;
        const bool in = ok[q] && j < D;
        uv[q][v] = in ? U[urow[q] + j] : 0.f;
        if (ROWS_BF16) iv[q][v] = in ? bf16_to_f32(((const uint16_t*)rows)[prow[q] + j]) : 0.f;
        else iv[q][v] = in ? ((const float*)rows)[prow[q] + j] : 0.f;
      }
    }
#pragma unroll
    for (int q = 0; q < UNR; ++q) {
      float p = 0.f;
#pragma unroll
      for (int v = 0; v < NV; ++v) p = fmaf(uv[q][v], iv[q][v], p);
      const float dot = group_sum<TPR>(p);
      const float e = rv[q] - dot;
      if (!ok[q]) continue;
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const int j = j0 + v * TPR;
        if (j >= D) break;
        const float du = lr * (e * iv[q][v] - lambda * uv[q][v]);
        const float di = lr * (e * uv[q][v] - lambda * iv[q][v]);
        if (user_atomic) atomic_add_noret(U + urow[q] + j, du);
        else U[urow[q] + j] = uv[q][v] + du;
        atomic_add_noret(delta + prow[q] + j, di);
      }
    }
  }
}

// sum of squared errors over (uid, iid, r) with both tables local
template <int TPR, int NV>
__global__ void __launch_bounds__(256) mf_sq_err_kernel(const float* __restrict__ U, const float* __restrict__ I,
                                                        const int32_t* __restrict__ uid,
                                                        const int32_t* __restrict__ iid,
                                                        const float* __restrict__ rating, int64_t B, int D,
                                                        double* __restrict__ out) {
  __shared__ float red[4];
  int64_t first, step; int j0;
  group_coords<TPR>(first, step, j0);
  float acc = 0.f;
  for (int64_t b = first; b < B; b += step) {
    const int64_t ur = (int64_t)uid[b] * D, ir = (int64_t)iid[b] * D;
    float p = 0.f;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int j = j0 + v * TPR;
      if (j < D) p = fmaf(U[ur + j], I[ir + j], p);
    }
    const float dot = group_sum<TPR>(p);
    const float e = rating[b] - dot;
    if (j0 == 0) acc += e * e;
  }
  acc = group_sum<64>(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(out, (double)(red[0] + red[1] + red[2] + red[3]));
}

}  // namespace

#define NV_TPR_SWITCH(D, ...)                                                   \
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

static inline int sgd_grid(int64_t B, int TPR, int UNR) {
  const int64_t per_block = (int64_t)4 * (64 / TPR) * UNR;
  return grid_for(B, (int)per_block, 256 * 8);
}

FPS_API int fps_mf_sgd_local(float* U, float* I, const int32_t* uid, const int32_t* iid, const float* r, int64_t B,
                             int D, float lr, float lambda, int user_atomic, void* stream) {
  if (B <= 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  constexpr int UNR = 4;
  NV_TPR_SWITCH(D, {
    const int g = sgd_grid(B, TPR, UNR);
    if (user_atomic) hipLaunchKernelGGL((mf_sgd_local_kernel<TPR, NV, UNR, true>), dim3(g), dim3(256), 0, s, U, I, uid, iid, r, B, D, lr, lambda, (const int32_t*)nullptr);
    else hipLaunchKernelGGL((mf_sgd_local_kernel<TPR, NV, UNR, false>), dim3(g), dim3(256), 0, s, U, I, uid, iid, r, B, D, lr, lambda, (const int32_t*)nullptr);
  });
  FPS_CHECK_LAUNCH();
  return 0;
}

// Segment form: ratings [seg[0], seg[1]) with seg a DEVICE pointer; max_B only
// sizes the grid (grid-stride loop, any segment length is handled).
FPS_API int fps_mf_sgd_local_seg(float* U, float* I, const int32_t* uid, const int32_t* iid, const float* r,
                                 const int32_t* seg, int64_t max_B, int D, float lr, float lambda, int user_atomic,
                                 void* stream) {
  if (max_B <= 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  constexpr int UNR = 4;
  NV_TPR_SWITCH(D, {
    const int g = sgd_grid(max_B, TPR, UNR);
    if (user_atomic) hipLaunchKernelGGL((mf_sgd_local_kernel<TPR, NV, UNR, true>), dim3(g), dim3(256), 0, s, U, I, uid, iid, r, (int64_t)0, D, lr, lambda, seg);
    else hipLaunchKernelGGL((mf_sgd_local_kernel<TPR, NV, UNR, false>), dim3(g), dim3(256), 0, s, U, I, uid, iid, r, (int64_t)0, D, lr, lambda, seg);
  });
  FPS_CHECK_LAUNCH();
  return 0;
}

FPS_API int fps_mf_sgd_pulled(float* U, const int32_t* uid, const float* r, const void* rows, int rows_bf16,
                              const int32_t* pos, float* delta, int64_t B, int D, float lr, float lambda,
                              int user_atomic, void* stream) {
  if (B <= 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  constexpr int UNR = 4;
  NV_TPR_SWITCH(D, {
    const int g = sgd_grid(B, TPR, UNR);
    if (rows_bf16) hipLaunchKernelGGL((mf_sgd_pulled_kernel<TPR, NV, UNR, true>), dim3(g), dim3(256), 0, s, U, uid, r, rows, pos, delta, B, D, lr, lambda, user_atomic);
    else hipLaunchKernelGGL((mf_sgd_pulled_kernel<TPR, NV, UNR, false>), dim3(g), dim3(256), 0, s, U, uid, r, rows, pos, delta, B, D, lr, lambda, user_atomic);
  });
  FPS_CHECK_LAUNCH();
  return 0;
}

FPS_API int fps_mf_sq_err(const float* U, const float* I, const int32_t* uid, const int32_t* iid, const float* r,
                          int64_t B, int D, double* out, void* stream) {
  if (B <= 0) return 0;
  NV_TPR_SWITCH(D, {
    const int g = grid_for(B, 4 * (64 / TPR), 256 * 8);
    hipLaunchKernelGGL((mf_sq_err_kernel<TPR, NV>), dim3(g), dim3(256), 0, (hipStream_t)stream, U, I, uid, iid, r, B, D, out);
  });
  FPS_CHECK_LAUNCH();
  return 0;
}

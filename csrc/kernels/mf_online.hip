// Online MF + top-K worker, learning side (gfx950): the per-batch SGD of
// PSOnlineMatrixFactorizationAndTopKGeneratorWorker
// (M/matrix/factorization/workers/PSOnlineMatrixFactorizationAndTopKGeneratorWorker.scala:120-166)
// and the in-place refresh of the worker's LEMP index (models/mf/topk_tensor.py
// OnlineMFTopKWorker).  The torch form issued ~12 launches per SGD phase and ~12 for
// the refresh (gather, dot, two index_adds, masks, counters); at 4096 ratings per
// micro-batch those launches, not the bytes, set the batch time.
//
//   mf_online_grad_kernel + mf_online_apply_kernel -- one SGD phase (a negative j of
//       every rating, or the ratings themselves) in two passes, one wave per entry t,
//       lanes over the factors.  Pass 1 reads the entry's user vector U[urow[t]] (the
//       pulled row, fixed over the phases) and its local item row W[irow[t]],
//       g = lr (target - <u, w>), du[urow] += g w (entries are distinct rows of du)
//       and keeps g; pass 2 adds g u to W[irow] (float atomics: entries share items).
//       The split keeps the torch form's batch semantics: every entry of a phase reads
//       the item rows as the phase starts (one fused pass let an entry read a row
//       another entry of the same phase was updating: 46 % of the item values off
//       after 6 batches in tests/test_topk_seen_merge_gpu.py).  irow < 0 skips the
//       entry (a failed negative draw, a rating owned by another rank).
//   index_refresh_kernel    -- the touched item rows into the LEMP index copies
//       (fp32 vectors, bf16 shadow, lengths) at their index positions (pos[row] < 0:
//       not in the index).  Repeated rows write the same value.
#include "common.h"

using namespace fps;

namespace {

// pass 1 of a phase: reads only (every entry sees the item rows as the phase starts)
template <int NPL>
__global__ void __launch_bounds__(256) mf_online_grad_kernel(const float* __restrict__ U,
                                                             const int64_t* __restrict__ urow,
                                                             const int64_t* __restrict__ irow,
                                                             const float* __restrict__ target, int64_t n, int D,
                                                             float lr, const float* __restrict__ W,
                                                             float* __restrict__ du, float* __restrict__ gbuf,
                                                             unsigned long long* __restrict__ trained) {
  __shared__ unsigned long long s_done;
  if (threadIdx.x == 0) s_done = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  unsigned long long done = 0;
  for (int64_t t = wave; t < n; t += nwaves) {
    const int64_t il = irow[t];
    if (il < 0) continue;  // wave-uniform
    const int64_t r = urow != nullptr ? urow[t] : t;
    float w[NPL];
    float dot = 0.f;
#pragma unroll
    for (int m = 0; m < NPL; ++m) {
      const int j = lane + 64 * m;
      const float u = j < D ? U[r * D + j] : 0.f;
      w[m] = j < D ? W[il * D + j] : 0.f;
      dot += u * w[m];
    }
    dot = group_sum<64>(dot);
    const float g = lr * ((target != nullptr ? target[t] : 0.f) - dot);
#pragma unroll
    for (int m = 0; m < NPL; ++m) {
      const int j = lane + 64 * m;
      if (j < D) du[r * D + j] += g * w[m];
    }
    if (lane == 0) gbuf[t] = g;
    ++done;
  }
  // one global atomic per workgroup (one per wave on a single counter serialised
  // ~4k same-address atomics: 52 us per phase at 4096 entries)
  if (lane == 0 && done) atomicAdd(&s_done, done);
  __syncthreads();
  if (trained != nullptr && threadIdx.x == 0 && s_done) atomicAdd(trained, s_done);
}

// pass 2: the item updates (float atomics: entries share items)
template <int NPL>
__global__ void __launch_bounds__(256) mf_online_apply_kernel(const float* __restrict__ U,
                                                              const int64_t* __restrict__ urow,
                                                              const int64_t* __restrict__ irow, int64_t n, int D,
                                                              const float* __restrict__ gbuf, float* __restrict__ W) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t t = wave; t < n; t += nwaves) {
    const int64_t il = irow[t];
    if (il < 0) continue;
    const int64_t r = urow != nullptr ? urow[t] : t;
    const float g = gbuf[t];
#pragma unroll
    for (int m = 0; m < NPL; ++m) {
      const int j = lane + 64 * m;
      if (j < D) atomic_add_noret(W + il * D + j, g * U[r * D + j]);
    }
  }
}

template <int NPL>
__global__ void __launch_bounds__(256) index_refresh_kernel(const int64_t* __restrict__ rows, int64_t n,
                                                            const int64_t* __restrict__ pos,
                                                            const float* __restrict__ W, int D,
                                                            float* __restrict__ vecs, uint16_t* __restrict__ vecs_bf,
                                                            float* __restrict__ lengths) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t t = wave; t < n; t += nwaves) {
    const int64_t row = rows[t];
    if (row < 0) continue;
    const int64_t p = pos[row];
    if (p < 0) continue;  // wave-uniform
    float ss = 0.f;
#pragma unroll
    for (int m = 0; m < NPL; ++m) {
      const int j = lane + 64 * m;
      if (j < D) {
        const float v = W[row * D + j];
        vecs[p * D + j] = v;
        if (vecs_bf != nullptr) vecs_bf[p * D + j] = f32_to_bf16(v);
        ss += v * v;
      }
    }
    ss = group_sum<64>(ss);
    if (lane == 0) lengths[p] = sqrtf(ss);
  }
}

}  // namespace

#define FPS_NPL_SWITCH(D, ...)                                   \
  do {                                                           \
    if ((D) <= 64) { constexpr int NPL = 1; __VA_ARGS__; }       \
    else if ((D) <= 128) { constexpr int NPL = 2; __VA_ARGS__; } \
    else { constexpr int NPL = 4; __VA_ARGS__; }                 \
  } while (0)

// U [*, D] pulled user rows (row urow[t], or t when urow is null); irow [n] local item
// rows (< 0: skip); target [n] (null: 0, a negative); W [n_local, D] item shard; du
// [*, D] user deltas (rows distinct across the n entries); trained (nullable) counts
// the entries applied.  D <= 256.
FPS_API int fps_mf_online_phase(const float* U, const int64_t* urow, const int64_t* irow, const float* target,
                                int64_t n, int D, float lr, float* W, float* du, float* gbuf,
                                unsigned long long* trained, void* stream) {
  if (n <= 0) return 0;
  if (D <= 0 || D > 256) return (int)hipErrorInvalidValue;
  const int g = grid_for(n, 4, 512);
  hipStream_t s = (hipStream_t)stream;
  FPS_NPL_SWITCH(D, {
    hipLaunchKernelGGL(mf_online_grad_kernel<NPL>, dim3(g), dim3(256), 0, s, U, urow, irow, target, n, D, lr,
                       (const float*)W, du, gbuf, trained);
    hipLaunchKernelGGL(mf_online_apply_kernel<NPL>, dim3(g), dim3(256), 0, s, U, urow, irow, n, D,
                       (const float*)gbuf, W);
  });
  FPS_CHECK_LAUNCH();
  return 0;
}

// rows [n] local item rows (< 0: skip), pos [n_local] index position of a local row
// (< 0: not indexed); vecs [N, D] fp32 / vecs_bf [N, D] bf16 (nullable) / lengths [N]
FPS_API int fps_index_refresh(const int64_t* rows, int64_t n, const int64_t* pos, const float* W, int D, float* vecs,
                              uint16_t* vecs_bf, float* lengths, void* stream) {
  if (n <= 0) return 0;
  if (D <= 0 || D > 256) return (int)hipErrorInvalidValue;
  const int g = grid_for(n, 4, 256 * 16);
  FPS_NPL_SWITCH(D, hipLaunchKernelGGL(index_refresh_kernel<NPL>, dim3(g), dim3(256), 0, (hipStream_t)stream, rows, n,
                                       pos, W, D, vecs, vecs_bf, lengths));
  FPS_CHECK_LAUNCH();
  return 0;
}

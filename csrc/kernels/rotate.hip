// Rating partition for the item-block rotation (stratified SGD over the xGMI ring).
//
// Items are hash-sharded ``i % W`` (the PS layout, M/matrix/factorization/
// PSOnlineMatrixFactorization.scala:58-60); each shard q is split into two
// halves by local row (``i // W < half[q]``), giving K = 2W item blocks
// b = 2q + h.  A worker's micro-batch (its users' ratings) is partitioned by
// block so that sub-step t touches exactly one block, the one resident on the
// GPU at that time (models/mf/fast.py, parallel/rotation.py).
//
//   rot_count   : per-block counts (LDS histogram, one global atomic per
//                 (workgroup, block))
//   rot_scatter : (uid, row-in-block, rating) written grouped by block; each
//                 workgroup reserves its range of every block with one global
//                 atomic, items take LDS-atomic slots inside it (order inside a
//                 block is arbitrary: Hogwild SGD inside a block, as the flat kernel)
#include "common.h"

using namespace fps;

namespace {

constexpr int ROT_MAX_K = 128;
constexpr int ROT_ITEMS = 16;  // ratings per thread per workgroup chunk

__device__ __forceinline__ void item_block(int32_t i, int W, const int32_t* __restrict__ half, int& b, int32_t& row) {
  const int q = i % W;
  const int32_t loc = i / W;
  const int32_t hq = half[q];
  const int h = loc >= hq;
  b = 2 * q + h;
  row = loc - (h ? hq : 0);
}

__global__ void __launch_bounds__(256) rot_count_kernel(const int32_t* __restrict__ iid, int64_t n, int W,
                                                        const int32_t* __restrict__ half, int32_t* __restrict__ counts,
                                                        uint8_t* __restrict__ seen) {
  __shared__ int32_t h[ROT_MAX_K];
  const int K = 2 * W;
  for (int k = threadIdx.x; k < K; k += blockDim.x) h[k] = 0;
  __syncthreads();
  for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n; x += (int64_t)gridDim.x * blockDim.x) {
    int b; int32_t row;
    const int32_t i = iid[x];
    item_block(i, W, half, b, row);
    atomicAdd(h + b, 1);
    if (seen != nullptr) seen[i] = 1;  // touched-item marks for the close-time dump
  }
  __syncthreads();
  for (int k = threadIdx.x; k < K; k += blockDim.x)
    if (h[k]) atomicAdd(counts + k, h[k]);
}

// ptr[K+1]: exclusive prefix of counts; cursor[K] zeroed by the caller
__global__ void __launch_bounds__(256) rot_scatter_kernel(const int32_t* __restrict__ uid,
                                                          const int32_t* __restrict__ iid,
                                                          const float* __restrict__ rating, int64_t n, int W,
                                                          const int32_t* __restrict__ half,
                                                          const int32_t* __restrict__ ptr,
                                                          int32_t* __restrict__ cursor, int32_t* __restrict__ uid_out,
                                                          int32_t* __restrict__ row_out, float* __restrict__ r_out) {
  __shared__ int32_t cnt[ROT_MAX_K];
  __shared__ int32_t base[ROT_MAX_K];
  const int K = 2 * W;
  for (int k = threadIdx.x; k < K; k += blockDim.x) cnt[k] = 0;
  __syncthreads();
  const int64_t chunk0 = (int64_t)blockIdx.x * blockDim.x * ROT_ITEMS;
  int bb[ROT_ITEMS];
  int32_t slot[ROT_ITEMS], rows[ROT_ITEMS];
#pragma unroll
  for (int it = 0; it < ROT_ITEMS; ++it) {
    const int64_t x = chunk0 + (int64_t)it * blockDim.x + threadIdx.x;
    bb[it] = -1;
    if (x < n) {
      item_block(iid[x], W, half, bb[it], rows[it]);
      slot[it] = atomicAdd(cnt + bb[it], 1);
    }
  }
  __syncthreads();
  for (int k = threadIdx.x; k < K; k += blockDim.x) base[k] = cnt[k] ? ptr[k] + atomicAdd(cursor + k, cnt[k]) : 0;
  __syncthreads();
#pragma unroll
  for (int it = 0; it < ROT_ITEMS; ++it) {
    if (bb[it] < 0) continue;
    const int64_t x = chunk0 + (int64_t)it * blockDim.x + threadIdx.x;
    const int32_t o = base[bb[it]] + slot[it];
    uid_out[o] = uid[x];
    row_out[o] = rows[it];
    r_out[o] = rating[x];
  }
}

// exclusive prefix of K counts into ptr[K+1] (tiny)
__global__ void rot_scan_kernel(const int32_t* __restrict__ counts, int K, int32_t* __restrict__ ptr) {
  if (threadIdx.x == 0) {
    int32_t acc = 0;
    for (int k = 0; k < K; ++k) { ptr[k] = acc; acc += counts[k]; }
    ptr[K] = acc;
  }
}

}  // namespace

// counts[K] and cursor[K] must be zeroed by the caller; ptr has K+1 entries;
// seen (optional, num_items bytes) gets seen[i] = 1 for every rated item.
FPS_API int fps_rot_partition(const int32_t* uid, const int32_t* iid, const float* rating, int64_t n, int W,
                              const int32_t* half, int32_t* counts, int32_t* ptr, int32_t* cursor, int32_t* uid_out,
                              int32_t* row_out, float* r_out, uint8_t* seen, void* stream) {
  if (2 * W > ROT_MAX_K) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  if (n > 0) hipLaunchKernelGGL(rot_count_kernel, dim3(grid_for(n, 256 * 8, 256 * 8)), dim3(256), 0, s, iid, n, W,
                                half, counts, seen);
  hipLaunchKernelGGL(rot_scan_kernel, dim3(1), dim3(64), 0, s, (const int32_t*)counts, 2 * W, ptr);
  if (n > 0) {
    const int64_t g = (n + 256 * ROT_ITEMS - 1) / (256 * ROT_ITEMS);
    hipLaunchKernelGGL(rot_scatter_kernel, dim3((unsigned)g), dim3(256), 0, s, uid, iid, rating, n, W, half,
                       (const int32_t*)ptr, cursor, uid_out, row_out, r_out);
  }
  FPS_CHECK_LAUNCH();
  return 0;
}

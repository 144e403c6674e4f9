// Negative sampling kernels (gfx950).  K5.
//
// * uniform_reject -- MF negatives (PSOnlineMatrixFactorizationWorker.scala:70-79,
//   PSOnlineMatrixFactorizationAndTopKGeneratorWorker.scala:141-156): k items per
//   rating, uniform over [0, n_items), redrawn (<= 32 tries, the reference's
//   bound) while equal to the rating's own item or present in the user's
//   recent-items ring (``ring[user * mem .. + mem)``, -1 = empty, optional).
// * alias -- word2vec unigram^0.75 sampling with Walker's alias table.
// Stateless counter-based RNG (hash of seed, counter, index): a step is
// reproducible and needs no per-thread generator state.
#include "common.h"

using namespace fps;

namespace {

__device__ __forceinline__ uint32_t rnd(uint32_t seed, uint64_t counter, uint64_t i, uint32_t salt) {
  uint32_t h = fmix32(seed ^ 0x68bc21ebu);
  h = fmix32(h ^ (uint32_t)counter);
  h = fmix32(h ^ (uint32_t)(counter >> 32) ^ (uint32_t)i);
  h = fmix32(h ^ (uint32_t)(i >> 32) ^ (salt * 0x9e3779b9u));
  return h;
}

// known != nullptr: draw from the worker's known items known[0 .. *known_count)
// (the reference samples among the item ids the worker has seen,
// PSOnlineMatrixFactorizationWorker.scala:70-79) instead of [0, n_items)
__global__ void uniform_reject_kernel(int64_t n, int k, int32_t n_items, const int32_t* __restrict__ positive,
                                      const int32_t* __restrict__ user, const int32_t* __restrict__ ring, int mem,
                                      const int32_t* __restrict__ known, const int32_t* __restrict__ known_count,
                                      uint32_t seed, uint64_t counter, int32_t* __restrict__ out) {
  const int64_t total = n * k;
  const uint32_t span = known ? (uint32_t)max(*known_count, 1) : (uint32_t)n_items;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = t / k;
    const int32_t pos = positive ? positive[b] : -1;
    const int32_t* r = (ring && user) ? ring + (int64_t)user[b] * mem : nullptr;
    int32_t cand = 0;
    for (uint32_t tries = 0; tries < 32; ++tries) {
      const int32_t j = (int32_t)(((uint64_t)rnd(seed, counter, t, tries) * (uint64_t)span) >> 32);
      cand = known ? known[j] : j;
      bool bad = cand == pos;
      if (r) for (int m = 0; m < mem && !bad; ++m) bad = r[m] == cand;
      if (!bad) break;
    }
    out[t] = cand;
  }
}

__global__ void alias_kernel(const float* __restrict__ prob, const int32_t* __restrict__ alias, int32_t V, int64_t n,
                             uint32_t seed, uint64_t counter, int32_t* __restrict__ out) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t h1 = rnd(seed, counter, t, 1), h2 = rnd(seed, counter, t, 2);
    const int32_t col = (int32_t)(((uint64_t)h1 * (uint64_t)V) >> 32);
    const float u = (float)(h2 >> 8) * (1.0f / 16777216.0f);
    out[t] = u < prob[col] ? col : alias[col];
  }
}

// per-user ring of the last ``mem`` rated items (the reference's userMemory
// FIFO of seen items); slots inside one batch are taken in arrival order of
// the atomics
__global__ void ring_push_kernel(int32_t* __restrict__ ring, int32_t* __restrict__ cursor,
                                 const int32_t* __restrict__ uid, const int32_t* __restrict__ iid, int64_t n,
                                 int mem) {
  for (int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; b < n; b += (int64_t)gridDim.x * blockDim.x) {
    const int32_t u = uid[b];
    const uint32_t slot = (uint32_t)atomicAdd(cursor + u, 1) % (uint32_t)mem;
    ring[(int64_t)u * mem + slot] = iid[b];
  }
}

// append first-seen items to the worker's known-item list
__global__ void known_append_kernel(int32_t* __restrict__ flag, int32_t* __restrict__ list,
                                    int32_t* __restrict__ count, const int32_t* __restrict__ iid, int64_t n) {
  for (int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; b < n; b += (int64_t)gridDim.x * blockDim.x) {
    const int32_t i = iid[b];
    if (flag[i] == 0 && atomicExch(flag + i, 1) == 0) list[atomicAdd(count, 1)] = i;
  }
}

}  // namespace

FPS_API int fps_ring_push(int32_t* ring, int32_t* cursor, const int32_t* uid, const int32_t* iid, int64_t n, int mem,
                          void* stream) {
  if (n <= 0 || mem <= 0) return 0;
  hipLaunchKernelGGL(ring_push_kernel, dim3(grid_for(n, 256, 256 * 16)), dim3(256), 0, (hipStream_t)stream, ring,
                     cursor, uid, iid, n, mem);
  FPS_CHECK_LAUNCH();
  return 0;
}

FPS_API int fps_known_append(int32_t* flag, int32_t* list, int32_t* count, const int32_t* iid, int64_t n,
                             void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(known_append_kernel, dim3(grid_for(n, 256, 256 * 16)), dim3(256), 0, (hipStream_t)stream, flag,
                     list, count, iid, n);
  FPS_CHECK_LAUNCH();
  return 0;
}

FPS_API int fps_sample_uniform_reject(int64_t n, int k, int32_t n_items, const int32_t* positive, const int32_t* user,
                                      const int32_t* ring, int mem, const int32_t* known, const int32_t* known_count,
                                      uint32_t seed, uint64_t counter, int32_t* out, void* stream) {
  if (n <= 0 || k <= 0) return 0;
  if ((known == nullptr) != (known_count == nullptr)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(uniform_reject_kernel, dim3(grid_for(n * k, 256, 256 * 16)), dim3(256), 0, (hipStream_t)stream,
                     n, k, n_items, positive, user, ring, mem, known, known_count, seed, counter, out);
  FPS_CHECK_LAUNCH();
  return 0;
}

FPS_API int fps_sample_alias(const float* prob, const int32_t* alias, int32_t V, int64_t n, uint32_t seed,
                             uint64_t counter, int32_t* out, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(alias_kernel, dim3(grid_for(n, 256, 256 * 16)), dim3(256), 0, (hipStream_t)stream, prob, alias,
                     V, n, seed, counter, out);
  FPS_CHECK_LAUNCH();
  return 0;
}

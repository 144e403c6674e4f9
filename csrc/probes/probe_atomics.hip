// Probe: the price of per-user atomics on gfx950 (design input for exact user rows).
// 64M ratings with uniform user ids over 10M users; one rating per thread.
#include <hip/hip_runtime.h>
#include <stdint.h>
#define API extern "C" __attribute__((visibility("default")))

__global__ void k_load(const int32_t* __restrict__ uid, const int32_t* __restrict__ cnt, int32_t* __restrict__ ord,
                       int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    ord[i] = cnt[uid[i]];
}
__global__ void k_ret(const int32_t* __restrict__ uid, int32_t* __restrict__ cnt, int32_t* __restrict__ ord,
                      int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    ord[i] = atomicAdd(cnt + uid[i], 1);
}
__global__ void k_noret(const int32_t* __restrict__ uid, int32_t* __restrict__ cnt, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    __hip_atomic_fetch_add(cnt + uid[i], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// lock + release: CAS 0 -> 1 until it succeeds, then an atomic exchange back to 0
__global__ void k_lock(const int32_t* __restrict__ uid, int32_t* __restrict__ lk, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int32_t* p = lk + uid[i];
    int spins = 0;
    while (atomicCAS(p, 0, 1) != 0 && ++spins < (1 << 20)) __builtin_amdgcn_s_sleep(1);
    atomicExch(p, 0);
  }
}
// one rating per 16-lane group (the SGD kernel's shape): lane 0 of the group does the atomic
__global__ void k_ret16(const int32_t* __restrict__ uid, int32_t* __restrict__ cnt, int32_t* __restrict__ ord,
                        int64_t n) {
  const int64_t g0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4;
  const int64_t ng = ((int64_t)gridDim.x * blockDim.x) >> 4;
  for (int64_t i = g0; i < n; i += ng)
    if ((threadIdx.x & 15) == 0) ord[i] = atomicAdd(cnt + uid[i], 1);
}

API int probe_run(int which, const int32_t* uid, int32_t* cnt, int32_t* ord, int64_t n, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int grid = 256 * 16, block = 256;
  switch (which) {
    case 0: hipLaunchKernelGGL(k_load, dim3(grid), dim3(block), 0, s, uid, cnt, ord, n); break;
    case 1: hipLaunchKernelGGL(k_ret, dim3(grid), dim3(block), 0, s, uid, cnt, ord, n); break;
    case 2: hipLaunchKernelGGL(k_noret, dim3(grid), dim3(block), 0, s, uid, cnt, n); break;
    case 3: hipLaunchKernelGGL(k_lock, dim3(grid), dim3(block), 0, s, uid, cnt, n); break;
    case 4: hipLaunchKernelGGL(k_ret16, dim3(grid * 4), dim3(block), 0, s, uid, cnt, ord, n); break;
    default: return -1;
  }
  return (int)hipGetLastError();
}

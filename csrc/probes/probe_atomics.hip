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

// ---- row updates (the tile SGD's user-row write, 64 floats = 256 B per rating), one
// wave per update: lane l owns float l.  tab[rows][64]; uid[i] picks the row.
__device__ __forceinline__ int xcc_id() {
  int x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
  return x & 7;
}
// MODE 0: plain load + add + store (Hogwild); 1: device-scope float atomic add (memory side);
// 2: workgroup-scope float atomic add; 3 / 4: as 1 / 2, the row index remapped so every XCD
// touches only its own eighth of the rows (XCD-owned rows: one L2 holds each)
template <int MODE>
__global__ void __launch_bounds__(256) k_rows(const int32_t* __restrict__ uid, float* __restrict__ tab, int64_t n,
                                              int32_t rows) {
  const int lane = threadIdx.x & 63;
  const int64_t w0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int x = (MODE >= 3) ? xcc_id() : 0;
  for (int64_t i = w0; i < n; i += nw) {
    int32_t u = uid[i];
    if (MODE >= 3) u = (u & ~7) | x;
    if (u >= rows) u -= 8;
    float* p = tab + (int64_t)u * 64 + lane;
    const float d = 1e-7f * (float)(lane + 1);
    if (MODE == 0) {
      *p = *p + d;
    } else if (MODE == 1 || MODE == 3) {
      __hip_atomic_fetch_add(p, d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      __hip_atomic_fetch_add(p, d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
}

API int probe_rows(int mode, const int32_t* uid, float* tab, int64_t n, int32_t rows, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int grid = 256 * 8, block = 256;
  switch (mode) {
    case 0: hipLaunchKernelGGL(k_rows<0>, dim3(grid), dim3(block), 0, s, uid, tab, n, rows); break;
    case 1: hipLaunchKernelGGL(k_rows<1>, dim3(grid), dim3(block), 0, s, uid, tab, n, rows); break;
    case 2: hipLaunchKernelGGL(k_rows<2>, dim3(grid), dim3(block), 0, s, uid, tab, n, rows); break;
    case 3: hipLaunchKernelGGL(k_rows<3>, dim3(grid), dim3(block), 0, s, uid, tab, n, rows); break;
    case 4: hipLaunchKernelGGL(k_rows<4>, dim3(grid), dim3(block), 0, s, uid, tab, n, rows); break;
    default: return -1;
  }
  return (int)hipGetLastError();
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

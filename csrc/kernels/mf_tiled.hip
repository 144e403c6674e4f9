// LDS-tiled MF SGD (gfx950): item rows live in LDS, no global item atomics.
//
// Why: the flat kernel (mf.hip) pushes every rating's item delta with a
// 256-B global float-atomic wave-instruction; those execute at the memory
// side at ~1.3 TB/s chip-wide (MI355X_MICROARCH.md "Global float atomics"),
// so a rating costs >= 256 B / 1.3 TB/s of atomic time on top of its 768 B
// of plain traffic -- the measured 3.9e9 ratings/s sits on that ceiling
// (profiles/README.md).  Here the item table (or the rotating item block,
// parallel/rotation.py) is cut into tiles of R rows; the ratings of a
// micro-batch are bucketed by tile (tile_partition below); one workgroup loads
// its tile into LDS (R x D fp32, 32 KiB at R = 128, D = 64), runs the SGD of
// every rating of the tile with the item row read from LDS and the item delta
// added with LDS float atomics (ds_add_f32, exact), and writes the tile back
// once.  Global traffic per rating: user row read + write (512 B) + 12 B of
// rating; the item table moves twice per micro-batch.
//
// Semantics are those of the flat kernel: every rating reads the item row as
// it is at that moment and its delta is added atomically; user rows are
// updated Hogwild (plain store) -- M/matrix/factorization/workers/
// PSOnlineMatrixFactorizationWorker.scala:41-55 with the PS add of
// M/matrix/factorization/PSOnlineMatrixFactorization.scala:58-60.
//
// Lane layout: TPR lanes per rating, each holding V float4 of the rows
// (D = 4 * TPR * V; D = 64 -> 16 lanes x 1 float4, 4 ratings per wave
// instruction, UNR = 4 in flight per lane group = 16 user rows per wave).
// LDS row stride = D floats (no padding): a ds_read_b128 lane group then
// covers each row's 64 banks exactly once (MI355X_MICROARCH.md "LDS").
#include "common.h"

using namespace fps;

namespace {

// ---------------------------------------------------------------- partition
// bucket of a rating = block * T + row_in_block / R (block layout of rotate.hip:
// b = 2q + h, q = i % W, h = (i / W >= half[q])); W = 1 with half[0] = num_items
// gives a single block (the whole local table).
__device__ __forceinline__ void tile_bucket(int32_t i, int W, const int32_t* __restrict__ half, int R, int T,
                                            int& bucket, int32_t& row) {
  const int q = i % W;
  const int32_t loc = i / W;
  const int32_t hq = half[q];
  const int h = loc >= hq;
  row = loc - (h ? hq : 0);
  bucket = (2 * q + h) * T + row / R;
}

constexpr int TP_MAX_BUCKETS = 16384;  // 64 KiB of LDS counters

// K1: per-workgroup histogram H[w][KT] (plain stores, no global atomics)
__global__ void __launch_bounds__(1024) tile_hist_kernel(const int32_t* __restrict__ iid, int64_t n, int64_t chunk,
                                                         int W, const int32_t* __restrict__ half, int R, int T,
                                                         int KT, int32_t* __restrict__ H, uint8_t* __restrict__ seen) {
  __shared__ int32_t cnt[TP_MAX_BUCKETS];
  for (int k = threadIdx.x; k < KT; k += blockDim.x) cnt[k] = 0;
  __syncthreads();
  const int64_t lo = (int64_t)blockIdx.x * chunk, hi = min(n, lo + chunk);
  for (int64_t x = lo + threadIdx.x; x < hi; x += blockDim.x) {
    const int32_t i = iid[x];
    int bk; int32_t row;
    tile_bucket(i, W, half, R, T, bk, row);
    atomicAdd(cnt + bk, 1);
    if (seen != nullptr) seen[i] = 1;
  }
  __syncthreads();
  int32_t* Hw = H + (int64_t)blockIdx.x * KT;
  for (int k = threadIdx.x; k < KT; k += blockDim.x) Hw[k] = cnt[k];
}

// K2: per bucket, exclusive scan over the G workgroups (coalesced across buckets)
__global__ void tile_colscan_kernel(int32_t* __restrict__ H, int G, int KT, int32_t* __restrict__ totals) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= KT) return;
  int32_t run = 0;
  for (int w = 0; w < G; ++w) {
    const int32_t v = H[(int64_t)w * KT + k];
    H[(int64_t)w * KT + k] = run;
    run += v;
  }
  totals[k] = run;
}

// K3: exclusive scan of KT totals into ptr[KT+1] (one 1024-thread workgroup)
__global__ void __launch_bounds__(1024) tile_scan_kernel(const int32_t* __restrict__ totals, int KT,
                                                         int32_t* __restrict__ ptr) {
  __shared__ int32_t part[1024];
  const int per = (KT + 1023) / 1024;
  const int k0 = threadIdx.x * per;
  int32_t s = 0;
  for (int k = k0; k < min(KT, k0 + per); ++k) s += totals[k];
  part[threadIdx.x] = s;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {  // Hillis-Steele inclusive scan
    const int32_t v = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  int32_t run = threadIdx.x ? part[threadIdx.x - 1] : 0;
  for (int k = k0; k < min(KT, k0 + per); ++k) { ptr[k] = run; run += totals[k]; }
  if (threadIdx.x == 1023) ptr[KT] = part[1023];
}

// K4: scatter packed 16-B records {uid, row-in-block, rating bits, 0} to
// ptr[bucket] + H[w][bucket] + LDS slot (one 16-B store per rating instead of
// three scattered 4-B stores)
__global__ void __launch_bounds__(1024) tile_scatter_kernel(const int32_t* __restrict__ uid,
                                                            const int32_t* __restrict__ iid,
                                                            const float* __restrict__ rating, int64_t n,
                                                            int64_t chunk, int W, const int32_t* __restrict__ half,
                                                            int R, int T, int KT, const int32_t* __restrict__ H,
                                                            const int32_t* __restrict__ ptr,
                                                            int4* __restrict__ rec) {
  __shared__ int32_t cur[TP_MAX_BUCKETS];
  const int32_t* Hw = H + (int64_t)blockIdx.x * KT;
  for (int k = threadIdx.x; k < KT; k += blockDim.x) cur[k] = ptr[k] + Hw[k];
  __syncthreads();
  const int64_t lo = (int64_t)blockIdx.x * chunk, hi = min(n, lo + chunk);
  for (int64_t x = lo + threadIdx.x; x < hi; x += blockDim.x) {
    int bk; int32_t row;
    tile_bucket(iid[x], W, half, R, T, bk, row);
    const int32_t o = atomicAdd(cur + bk, 1);
    rec[o] = make_int4(uid[x], row, __float_as_int(rating[x]), 0);
  }
}

// ---------------------------------------------------------------- SGD
template <int TPR, int V, int UNR>
__global__ void __launch_bounds__(512) mf_sgd_tiled_kernel(float* __restrict__ U, float* __restrict__ I,
                                                           const int4* __restrict__ rec,
                                                           const int32_t* __restrict__ ptr, int R,
                                                           int64_t block_rows, float lr, float lambda) {
  extern __shared__ float4 tile[];
  constexpr int D4 = TPR * V;  // float4 per row
  constexpr int RPW = 64 / TPR;
  const int t = blockIdx.x;
  const int64_t r0 = (int64_t)t * R;
  const int nr = (int)min((int64_t)R, block_rows - r0);
  float4* Ig = reinterpret_cast<float4*>(I) + r0 * D4;
  {  // tile load: all of a thread's loads in flight before its LDS writes
    constexpr int LPT = 8;  // float4 per thread per round (<= 64 KiB tiles at 512 threads)
    const int tot = nr * D4;
    for (int x0 = threadIdx.x; x0 < tot; x0 += blockDim.x * LPT) {
      float4 v[LPT];
#pragma unroll
      for (int k = 0; k < LPT; ++k) {
        const int x = x0 + k * blockDim.x;
        if (x < tot) v[k] = Ig[x];
      }
#pragma unroll
      for (int k = 0; k < LPT; ++k) {
        const int x = x0 + k * blockDim.x;
        if (x < tot) tile[x] = v[k];
      }
    }
  }
  __syncthreads();
  const int32_t beg = ptr[t], end = ptr[t + 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int g = lane / TPR, j = lane % TPR;
  const int stride = nw * RPW;
  const float4* Ug = reinterpret_cast<const float4*>(U);
  // records of the first round; every load is unconditional (index clamped to
  // the segment) so the UNR loads issue back to back
  int4 cur[UNR];
  int32_t base = beg + wave * RPW + g;
  const int32_t last = end - 1;  // records are only read when the tile has ratings (beg < end)
  if (beg < end) {
#pragma unroll
    for (int q = 0; q < UNR; ++q) cur[q] = rec[min(base + q * stride, last)];
  }
  for (; base < end; base += stride * UNR) {
    int4 nxt[UNR];
#pragma unroll
    for (int q = 0; q < UNR; ++q)  // prefetch the next round's records
      nxt[q] = rec[min(base + (UNR + q) * stride, last)];
    float4 uv[UNR][V], iv[UNR][V];
#pragma unroll
    for (int q = 0; q < UNR; ++q) {
      const int64_t ur = (int64_t)cur[q].x * D4;
      const int tr = (int)(cur[q].y - r0) * D4;
#pragma unroll
      for (int v = 0; v < V; ++v) {
        uv[q][v] = Ug[ur + j + v * TPR];
        iv[q][v] = tile[tr + j + v * TPR];
      }
    }
#pragma unroll
    for (int q = 0; q < UNR; ++q) {
      float p = 0.f;
#pragma unroll
      for (int v = 0; v < V; ++v)
        p += uv[q][v].x * iv[q][v].x + uv[q][v].y * iv[q][v].y + uv[q][v].z * iv[q][v].z + uv[q][v].w * iv[q][v].w;
      const float e = __int_as_float(cur[q].z) - group_sum<TPR>(p);
      if (base + q * stride >= end) continue;  // uniform in the lane group
      const int64_t ur = (int64_t)cur[q].x * D4;
      const int tr = (int)(cur[q].y - r0) * D4;
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const float4 u = uv[q][v], i = iv[q][v];
        float4 nu;
        nu.x = u.x + lr * (e * i.x - lambda * u.x);
        nu.y = u.y + lr * (e * i.y - lambda * u.y);
        nu.z = u.z + lr * (e * i.z - lambda * u.z);
        nu.w = u.w + lr * (e * i.w - lambda * u.w);
        reinterpret_cast<float4*>(U)[ur + j + v * TPR] = nu;
        float* ti = reinterpret_cast<float*>(tile + tr + j + v * TPR);
        atomicAdd(ti + 0, lr * (e * u.x - lambda * i.x));
        atomicAdd(ti + 1, lr * (e * u.y - lambda * i.y));
        atomicAdd(ti + 2, lr * (e * u.z - lambda * i.z));
        atomicAdd(ti + 3, lr * (e * u.w - lambda * i.w));
      }
    }
#pragma unroll
    for (int q = 0; q < UNR; ++q) cur[q] = nxt[q];
  }
  __syncthreads();
  for (int x = threadIdx.x; x < nr * D4; x += blockDim.x) Ig[x] = tile[x];
}

}  // namespace

// Workspace: H holds G * KT int32 (G = fps_tile_partition_groups(n)), totals KT.
FPS_API int fps_tile_partition_groups(int64_t n) {
  int64_t g = (n + 65535) / 65536;  // >= 64 Ki ratings per workgroup
  if (g < 1) g = 1;
  if (g > 512) g = 512;
  return (int)g;
}

// rec: n packed records {uid, row-in-block, rating bits, 0} grouped by bucket
FPS_API int fps_tile_partition(const int32_t* uid, const int32_t* iid, const float* rating, int64_t n, int W,
                               const int32_t* half, int R, int T, int32_t* H, int32_t* totals, int32_t* ptr,
                               int4* rec, uint8_t* seen, void* stream) {
  const int KT = 2 * W * T;
  if (KT > TP_MAX_BUCKETS || R <= 0 || T <= 0) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  const int G = fps_tile_partition_groups(n);
  const int64_t chunk = (n + G - 1) / G;
  hipLaunchKernelGGL(tile_hist_kernel, dim3(G), dim3(1024), 0, s, iid, n, chunk, W, half, R, T, KT, H, seen);
  hipLaunchKernelGGL(tile_colscan_kernel, dim3((KT + 255) / 256), dim3(256), 0, s, H, G, KT, totals);
  hipLaunchKernelGGL(tile_scan_kernel, dim3(1), dim3(1024), 0, s, (const int32_t*)totals, KT, ptr);
  if (n > 0)
    hipLaunchKernelGGL(tile_scatter_kernel, dim3(G), dim3(1024), 0, s, uid, iid, rating, n, chunk, W, half, R, T,
                       KT, (const int32_t*)H, (const int32_t*)ptr, rec);
  FPS_CHECK_LAUNCH();
  return 0;
}

// One launch per block: T tiles of R rows of I[block_rows, D]; ptr = the
// block's T+1 tile offsets (device).  D must be 16, 32, 64, 128 or 256.
FPS_API int fps_mf_sgd_tiled(float* U, float* I, const int4* rec, const int32_t* ptr, int T, int R,
                             int64_t block_rows, int D, float lr, float lambda, void* stream) {
  if (T <= 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const size_t lds = (size_t)R * D * sizeof(float);
  if (lds > 64 * 1024) return (int)hipErrorInvalidValue;
  constexpr int UNR = 4;
#define FPS_TILED(TPR_, V_)                                                                                      \
  hipLaunchKernelGGL((mf_sgd_tiled_kernel<TPR_, V_, UNR>), dim3(T), dim3(512), lds, s, U, I, rec, ptr, R,      \
                     block_rows, lr, lambda)
  switch (D) {
    case 16: FPS_TILED(4, 1); break;
    case 32: FPS_TILED(8, 1); break;
    case 64: FPS_TILED(16, 1); break;
    case 128: FPS_TILED(16, 2); break;
    case 256: FPS_TILED(16, 4); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef FPS_TILED
  FPS_CHECK_LAUNCH();
  return 0;
}

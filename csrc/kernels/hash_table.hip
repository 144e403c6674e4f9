// Persistent device hash-table PS shard (gfx950): the HBM counterpart of
// SimplePSLogic's HashMap[Integer, P] over the FULL signed 32-bit id space
// with lazy init on first touch (M/server/SimplePSLogic.scala:7-26).
//
// Layout (one shard per rank, all in HBM):
//   tab[cap]     u64  0 = empty, (1 << 32) | (uint32)key = occupied; linear
//                     probing from fmix32(key ^ SALT) & (cap - 1)
//   rowmap[cap]  i32  row of an occupied slot
//   rowkey[rcap] i32  key of a row (dump / global ids)
//   rows         [rcap, D] parameters, COMPACT: rows are handed out in insert
//                     order by one counter, so a dump is rows[0:count] and a
//                     rehash of tab never moves a row (cached row indices of
//                     in-flight plans stay valid).
//
// A lookup-or-insert is three launches (kernel boundaries replace any spin
// wait: a lane never waits on another lane's write inside one kernel):
//   1. find/insert: CAS the key into tab; the CAS winner is the key's unique
//      inserter ("fresh") -- also across the source segments of one call;
//   2. assign: fresh lanes take rows (one atomicAdd per block tile, block scan)
//      and publish rowmap[slot] / rowkey[row];
//   3. resolve: every request reads rowmap[slot];
//   4. (optional) init of the fresh rows: zeros / const / hash-uniform by id.
// The host keeps cap >= 2 * (rows + incoming keys) and rcap >= rows + incoming
// (ops.HashShardTable.reserve), so every probe sequence ends at a free slot;
// a full table still terminates (probe count <= cap) and raises `overflow`.
#include "common.h"

using namespace fps;

namespace {

constexpr uint32_t kSalt = 0x2545f491u;
constexpr unsigned long long kOcc = 1ull << 32;

__device__ __forceinline__ unsigned long long tagged(int32_t k) { return kOcc | (unsigned long long)(uint32_t)k; }

__global__ void __launch_bounds__(256) ht_find_insert_kernel(const int32_t* __restrict__ keys, int64_t n,
                                                             unsigned long long* __restrict__ tab, uint32_t mask,
                                                             int insert, int32_t* __restrict__ slot,
                                                             uint8_t* __restrict__ fresh,
                                                             int32_t* __restrict__ overflow) {
  for (int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; b < n; b += (int64_t)gridDim.x * blockDim.x) {
    const int32_t k = keys[b];
    const unsigned long long want = tagged(k);
    uint32_t h = fmix32((uint32_t)k ^ kSalt) & mask;
    int32_t s = -1;
    uint8_t ins = 0;
    for (uint32_t probe = 0; probe <= mask; ++probe) {
      const unsigned long long cur = tab[h];
      if (cur == want) { s = (int32_t)h; break; }
      if (cur == 0ull) {
        if (!insert) break;  // lookup only: an empty slot ends the probe sequence
        const unsigned long long old = atomicCAS(tab + h, 0ull, want);
        if (old == 0ull) { s = (int32_t)h; ins = 1; break; }  // this request inserted the key
        if (old == want) { s = (int32_t)h; break; }           // a racing request inserted it
      }
      h = (h + 1) & mask;
    }
    if (s < 0 && insert) overflow[0] = 1;
    slot[b] = s;
    fresh[b] = ins;
  }
}

// fresh requests take compact rows: one atomicAdd on the row counter per block
// and tile of 256 x HT_AU requests (a block scan hands out the rows inside the
// tile).  One atomic per wave serialised ~65k same-address atomics per 4M-key
// call at the L2 (471 us, 3 % of HBM rate: profiles/r4_counters.md).
constexpr int HT_AU = 8;

__global__ void __launch_bounds__(256) ht_assign_kernel(const int32_t* __restrict__ keys, int64_t n,
                                                        const int32_t* __restrict__ slot,
                                                        const uint8_t* __restrict__ fresh,
                                                        int32_t* __restrict__ rowmap, int32_t* __restrict__ rowkey,
                                                        int32_t* __restrict__ count, int64_t rcap,
                                                        int32_t* __restrict__ overflow) {
  __shared__ int32_t s_wave[4];
  __shared__ int32_t s_base;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  constexpr int TILE = 256 * HT_AU;
  for (int64_t t0 = (int64_t)blockIdx.x * TILE; t0 < n; t0 += (int64_t)gridDim.x * TILE) {  // block-uniform
    uint32_t fm = 0;  // which of this thread's HT_AU requests are fresh (coalesced: stride 256)
    uint8_t fv[HT_AU];  // unconditional clamped loads, all in flight (a guarded one waited each)
#pragma unroll
    for (int j = 0; j < HT_AU; ++j) fv[j] = fresh[min(t0 + j * 256 + threadIdx.x, n - 1)];
#pragma unroll
    for (int j = 0; j < HT_AU; ++j)
      if (t0 + j * 256 + threadIdx.x < n && fv[j]) fm |= 1u << j;
    const int c = __popc(fm);
    int x = c;  // inclusive wave scan
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane == 63) s_wave[wv] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
      const int tot = s_wave[0] + s_wave[1] + s_wave[2] + s_wave[3];
      s_base = tot ? atomicAdd(count, tot) : 0;
    }
    __syncthreads();
    int32_t row = s_base + x - c;
    for (int w = 0; w < wv; ++w) row += s_wave[w];
#pragma unroll
    for (int j = 0; j < HT_AU; ++j) {
      if (!((fm >> j) & 1u)) continue;
      const int64_t b = t0 + j * 256 + threadIdx.x;
      if (row < rcap) {
        rowmap[slot[b]] = row;
        rowkey[row] = keys[b];
      } else {
        overflow[0] = 2;
        rowmap[slot[b]] = -1;
      }
      ++row;
    }
    __syncthreads();  // s_wave / s_base are rewritten by the next tile
  }
}

__global__ void __launch_bounds__(256) ht_resolve_kernel(const int32_t* __restrict__ slot, int64_t n,
                                                         const int32_t* __restrict__ rowmap,
                                                         int32_t* __restrict__ row) {
  for (int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; b < n; b += (int64_t)gridDim.x * blockDim.x) {
    const int32_t s = slot[b];
    row[b] = s >= 0 ? rowmap[s] : -1;
  }
}

// rehash: re-insert rows [0, count) (unique keys) into a fresh tab/rowmap
__global__ void __launch_bounds__(256) ht_rehash_kernel(const int32_t* __restrict__ rowkey, int64_t count,
                                                        unsigned long long* __restrict__ tab, uint32_t mask,
                                                        int32_t* __restrict__ rowmap,
                                                        int32_t* __restrict__ overflow) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < count; r += (int64_t)gridDim.x * blockDim.x) {
    const int32_t k = rowkey[r];
    const unsigned long long want = tagged(k);
    uint32_t h = fmix32((uint32_t)k ^ kSalt) & mask;
    bool done = false;
    for (uint32_t probe = 0; probe <= mask; ++probe) {
      if (atomicCAS(tab + h, 0ull, want) == 0ull) {
        rowmap[h] = (int32_t)r;
        done = true;
        break;
      }
      h = (h + 1) & mask;
    }
    if (!done) overflow[0] = 1;
  }
}

// init of the freshly inserted rows (row-parallel, TPR lanes per row):
// kind 0 = zeros, 1 = const lo, 2 = U[lo, hi) hash-RNG keyed by the id (K9)
template <int TPR>
__global__ void __launch_bounds__(256) ht_init_fresh_kernel(float* __restrict__ rows, int D,
                                                            const int32_t* __restrict__ row,
                                                            const uint8_t* __restrict__ fresh,
                                                            const int32_t* __restrict__ keys, int64_t n, int kind,
                                                            float lo, float hi, uint32_t seed) {
  constexpr int RPW = 64 / TPR;
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int j0 = lane % TPR;
  for (int64_t b = wave * RPW + lane / TPR; b < n; b += nwaves * RPW) {
    if (!fresh[b]) continue;
    const int64_t r = row[b];
    if (r < 0) continue;
    float* dst = rows + r * (int64_t)D;
    const float span = hi - lo;
    for (int j = j0; j < D; j += TPR)
      dst[j] = kind == 0 ? 0.f : (kind == 1 ? lo : lo + span * hash_uniform(seed, (int64_t)keys[b], (uint32_t)j));
  }
}

}  // namespace

// keys[n] -> row[n] (-1: absent on a lookup, or overflow); fresh[n] = 1 for the
// request that inserted its key.  ws: int32[2 * n] scratch (slots).  count is
// the device row counter; overflow[0] is set non-zero on a full table / pool.
FPS_API int fps_ht_lookup(const int32_t* keys, int64_t n, unsigned long long* tab, int64_t cap, int32_t* rowmap,
                          int32_t* rowkey, int32_t* count, int64_t rcap, int insert, int32_t* slot_ws,
                          uint8_t* fresh, int32_t* row, int32_t* overflow, float* rows, int D, int init_kind,
                          float lo, float hi, uint32_t seed, void* stream) {
  if (n <= 0) return 0;
  if (cap <= 0 || (cap & (cap - 1)) != 0 || cap > (1ll << 31)) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  const int g = grid_for(n, 256, 256 * 16);
  hipLaunchKernelGGL(ht_find_insert_kernel, dim3(g), dim3(256), 0, s, keys, n, tab, (uint32_t)(cap - 1), insert,
                     slot_ws, fresh, overflow);
  if (insert)
    hipLaunchKernelGGL(ht_assign_kernel, dim3(grid_for(n, 256 * HT_AU)), dim3(256), 0, s, keys, n, (const int32_t*)slot_ws,
                       (const uint8_t*)fresh, rowmap, rowkey, count, rcap, overflow);
  hipLaunchKernelGGL(ht_resolve_kernel, dim3(g), dim3(256), 0, s, (const int32_t*)slot_ws, n,
                     (const int32_t*)rowmap, row);
  if (insert && rows != nullptr && init_kind >= 0) {
#define HT_INIT(TPR_)                                                                                               \
  hipLaunchKernelGGL(ht_init_fresh_kernel<TPR_>, dim3(grid_for(n, 4 * (64 / TPR_), 256 * 16)), dim3(256), 0, s,     \
                     rows, D, (const int32_t*)row, (const uint8_t*)fresh, keys, n, init_kind, lo, hi, seed)
    if (D <= 1) HT_INIT(1);
    else if (D <= 4) HT_INIT(4);
    else if (D <= 16) HT_INIT(16);
    else if (D <= 32) HT_INIT(32);
    else HT_INIT(64);
#undef HT_INIT
  }
  FPS_CHECK_LAUNCH();
  return 0;
}

// rebuild tab / rowmap (zeroed by the caller, cap a power of two) from rowkey[0:count]
FPS_API int fps_ht_rehash(const int32_t* rowkey, int64_t count, unsigned long long* tab, int64_t cap,
                          int32_t* rowmap, int32_t* overflow, void* stream) {
  if (count <= 0) return 0;
  if (cap <= 0 || (cap & (cap - 1)) != 0 || cap > (1ll << 31) || count > cap) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(ht_rehash_kernel, dim3(grid_for(count, 256, 256 * 16)), dim3(256), 0, (hipStream_t)stream, rowkey,
                     count, tab, (uint32_t)(cap - 1), rowmap, overflow);
  FPS_CHECK_LAUNCH();
  return 0;
}

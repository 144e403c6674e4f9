// PS shard table kernels (gfx950): init, pull-serve gather, push apply,
// per-step key de-duplication + bucketing for the all-to-all.
//
//   K9  init_rows      -- deterministic hash-RNG init by global id
//   K2  gather_rows    -- pull serve: rows of the HBM shard -> wire buffer
//   K3  apply_rows     -- push apply: add / set / sgd / adagrad
//   K1  dedup_*        -- unique keys per destination shard + slot per request
//
// Row layout: a row of D fp32 is owned by TPR lanes (TPR = pow2 >= D, <= 64),
// NV = ceil(D / TPR) values per lane.  D = 64 -> one float per lane, one
// 256-B coalesced transaction per row and per atomic wave-instruction.
#include "common.h"

using namespace fps;

namespace {

template <int TPR>
__device__ __forceinline__ void row_coords(int64_t& first, int64_t& step, int& j0) {
  constexpr int RPW = 64 / TPR;
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  first = wave * RPW + lane / TPR;
  step = nwaves * RPW;
  j0 = lane % TPR;
}

template <int TPR>
__global__ void __launch_bounds__(256) init_rows_kernel(float* __restrict__ table, int64_t n_rows, int D,
                                                        int64_t id_base, int64_t id_stride, float lo, float hi,
                                                        uint32_t seed) {
  int64_t r, step; int j0;
  row_coords<TPR>(r, step, j0);
  const float span = hi - lo;
  for (; r < n_rows; r += step) {
    const int64_t gid = id_base + r * id_stride;
    float* row = table + r * (int64_t)D;
    for (int j = j0; j < D; j += TPR) row[j] = lo + span * hash_uniform(seed, gid, (uint32_t)j);
  }
}

// Untouched-row sentinel (tables with ``touch_sentinel``: zero init, additive rules):
// a row that was never pulled or pushed holds -0.0 (bits 0x80000000) and reads as
// zero; the first serve of it stores +0.0 back (``flip``), and every apply adds
// deltas with -0.0 mapped to +0.0 (``pos0``), so "touched" = "not the sentinel" and
// the close-time dump needs no per-request byte marks -- the flip is a conditional
// store to the cache line the gather just read, and only on a row's first touch.
constexpr uint32_t NEG0_BITS = 0x80000000u;
__device__ __forceinline__ float pos0(float x) { return x == 0.f ? 0.f : x; }  // -0.0 -> +0.0
// the flip is a CAS, never a plain store: a pipelined kernel may already be adding into
// the fresh row (the next batch's gather beside this batch's push), and a +0.0 store
// would overwrite its update; the CAS only replaces a value that is still the sentinel
__device__ __forceinline__ void flip_neg0(float* p) {
  atomicCAS(reinterpret_cast<unsigned int*>(p), NEG0_BITS, 0u);
}

template <int TPR, bool OUT_BF16, typename IDX>
__global__ void __launch_bounds__(256) gather_rows_kernel(const float* __restrict__ table, const IDX* __restrict__ idx,
                                                          int64_t n, int D, void* __restrict__ out,
                                                          uint8_t* __restrict__ touched, float* __restrict__ flip) {
  int64_t r, step; int j0;
  row_coords<TPR>(r, step, j0);
  for (; r < n; r += step) {
    const int64_t row = (int64_t)idx[r];
    if (row < 0) {  // padding slot of a fixed-shape plan: a zero row, nothing marked
      for (int j = j0; j < D; j += TPR) {
        if (OUT_BF16) ((uint16_t*)out)[r * D + j] = 0;
        else ((float*)out)[r * D + j] = 0.f;
      }
      continue;
    }
    const float* src = table + row * D;
    for (int j = j0; j < D; j += TPR) {
      const float v = src[j];
      if (OUT_BF16) ((uint16_t*)out)[r * D + j] = f32_to_bf16(v);
      else ((float*)out)[r * D + j] = v;
      if (flip != nullptr && __float_as_uint(v) == NEG0_BITS) flip_neg0(flip + row * D + j);
    }
    if (touched != nullptr && j0 == 0) touched[row] = 1;
  }
}

// D = 1 rows (PA's weight per feature, 4 B): SC rows per thread, every index and value
// load issued before the first dependent access, so a wave keeps SC random row accesses
// in flight per lane instead of one (the one-row-per-lane loops above issue a dependent
// idx -> row pair per trip: 96 us to gather and 218 us to add 4M scalars at N = 8,
// profiles/r6_ps_paths_hot_owner.md).  Thread t covers rows base + t + k * 256.
constexpr int SC = 8;

template <bool OUT_BF16, typename IDX>
__global__ void __launch_bounds__(256) gather_scalar_kernel(const float* __restrict__ table,
                                                            const IDX* __restrict__ idx, int64_t n,
                                                            void* __restrict__ out, uint8_t* __restrict__ touched,
                                                            float* __restrict__ flip) {
  const int64_t base = (int64_t)blockIdx.x * (256 * SC) + threadIdx.x;
  int64_t row[SC];
#pragma unroll
  for (int k = 0; k < SC; ++k) {
    const int64_t r = base + k * 256;
    row[k] = r < n ? (int64_t)idx[r] : -2;
  }
  float v[SC];
#pragma unroll
  for (int k = 0; k < SC; ++k) v[k] = row[k] >= 0 ? table[row[k]] : 0.f;
#pragma unroll
  for (int k = 0; k < SC; ++k) {
    const int64_t r = base + k * 256;
    if (row[k] == -2) continue;  // past the end (a padding slot, row -1, serves zero)
    if (OUT_BF16) ((uint16_t*)out)[r] = f32_to_bf16(v[k]);
    else ((float*)out)[r] = v[k];
    if (row[k] < 0) continue;
    if (flip != nullptr && __float_as_uint(v[k]) == NEG0_BITS) flip_neg0(flip + row[k]);
    if (touched != nullptr) touched[row[k]] = 1;
  }
}

// OP 0: atomic add (keys may repeat), 4: plain read-modify-write (unique keys), 1: set
template <int OP, bool IN_BF16>
__global__ void __launch_bounds__(256) apply_scalar_kernel(float* __restrict__ table, const int32_t* __restrict__ idx,
                                                           int64_t n, const void* __restrict__ delta,
                                                           uint8_t* __restrict__ touched) {
  const int64_t base = (int64_t)blockIdx.x * (256 * SC) + threadIdx.x;
  int32_t row[SC];
  float g[SC];
#pragma unroll
  for (int k = 0; k < SC; ++k) {
    const int64_t r = base + k * 256;
    row[k] = r < n ? idx[r] : -1;
    g[k] = r < n ? (IN_BF16 ? bf16_to_f32(((const uint16_t*)delta)[r]) : ((const float*)delta)[r]) : 0.f;
  }
  float old[SC];
  if (OP == 4) {
#pragma unroll
    for (int k = 0; k < SC; ++k) old[k] = row[k] >= 0 ? table[row[k]] : 0.f;
  }
#pragma unroll
  for (int k = 0; k < SC; ++k) {
    if (row[k] < 0) continue;
    const float d = pos0(g[k]);  // a -0.0 delta must not keep the sentinel
    if (OP == 0) atomic_add_noret(table + row[k], d);
    else if (OP == 4) table[row[k]] = old[k] + d;
    else table[row[k]] = d;
    if (touched != nullptr) touched[row[k]] = 1;
  }
}

// op: 0 = add (atomic), 1 = set, 2 = sgd w -= lr*g (atomic), 3 = adagrad
// (acc += g^2, w -= lr*g/sqrt(acc+eps); keys must be unique in the launch),
// 4 = add (unique keys, plain RMW), 5 = add + renorm: w += g, then the row's
// euclidean length is recomputed in the epilogue and stored in state[row] (the
// LengthAndVector PS of psOnlineLearnerAndGenerator: attachLength(vectorSum(v, d)),
// M/matrix/factorization/PSOnlineMatrixFactorizationAndTopKGenerator.scala:81-84;
// unique keys in the launch).
template <int TPR, bool IN_BF16, int OP>
__global__ void __launch_bounds__(256) apply_rows_kernel(float* __restrict__ table, float* __restrict__ state,
                                                         const int32_t* __restrict__ idx, int64_t n, int D,
                                                         const void* __restrict__ delta, float lr, float eps,
                                                         uint8_t* __restrict__ touched) {
  int64_t r, step; int j0;
  row_coords<TPR>(r, step, j0);
  for (; r < n; r += step) {
    const int64_t row = (int64_t)idx[r];
    if (row < 0) continue;  // padding slot
    float* dst = table + row * D;
    float ss = 0.f;
    for (int j = j0; j < D; j += TPR) {
      // pos0: a -0.0 delta must not keep an untouched row's -0.0 sentinel (see gather_rows_kernel)
      float g = pos0(IN_BF16 ? bf16_to_f32(((const uint16_t*)delta)[r * D + j]) : ((const float*)delta)[r * D + j]);
      if (OP == 5) {
        const float v = dst[j] + g;
        dst[j] = v;
        ss += v * v;
      } else if (OP == 0) {
        atomic_add_noret(dst + j, g);
      } else if (OP == 1) {
        dst[j] = g;
      } else if (OP == 2) {
        atomic_add_noret(dst + j, pos0(-lr * g));
      } else if (OP == 4) {
        dst[j] += g;  // keys unique within the launch: plain read-modify-write
      } else {
        float* acc = state + row * D + j;
        float a = *acc + g * g;
        *acc = a;
        dst[j] += pos0(-lr * g * rsqrtf(a + eps));
      }
    }
    if (OP == 5) {  // the lane group of the row (TPR lanes, all active together) sums the squares
#pragma unroll
      for (int o = TPR / 2; o > 0; o >>= 1) ss += __shfl_xor(ss, o, TPR);
      if (j0 == 0) state[row] = sqrtf(ss);
    }
    if (touched != nullptr && j0 == 0) touched[row] = 1;
  }
}

// 16-byte variants for fp32 rows with D % 4 == 0 (every table the apps build:
// MF 64, SGNS 300, top-K 64+1 is excluded by the divisibility test).  A lane owns
// NV float4 of its row (TPR lanes per row, D/4 <= TPR * NV) and issues all of its
// loads before any store, so a wave has NV x 16 B in flight per lane instead of one
// dependent 4-B load per loop trip (the scalar kernels above reached ~1.6 TB/s on
// SGNS's 1200-B rows, profiles/r4_w2v_ps_path_kernel_stats.csv).
typedef float to_f4 __attribute__((ext_vector_type(4)));

template <int TPR, int NV, typename IDX>
__global__ void __launch_bounds__(256) gather_rows_v4_kernel(const to_f4* __restrict__ table,
                                                             const IDX* __restrict__ idx, int64_t n, int D4,
                                                             to_f4* __restrict__ out, uint8_t* __restrict__ touched,
                                                             float* __restrict__ flip) {
  int64_t r, step; int j0;
  row_coords<TPR>(r, step, j0);
  for (; r < n; r += step) {
    const int64_t row = (int64_t)idx[r];
    if (row < 0) {  // padding slot of a fixed-shape plan
#pragma unroll
      for (int q = 0; q < NV; ++q) {
        const int j = j0 + q * TPR;
        if (j < D4) out[r * D4 + j] = to_f4{0.f, 0.f, 0.f, 0.f};
      }
      continue;
    }
    const to_f4* src = table + row * D4;
    to_f4 v[NV];
#pragma unroll
    for (int q = 0; q < NV; ++q) {
      const int j = j0 + q * TPR;
      if (j < D4) v[q] = src[j];  // hot rows (Zipf ids) are re-read: keep them cacheable
    }
#pragma unroll
    for (int q = 0; q < NV; ++q) {
      const int j = j0 + q * TPR;
      if (j < D4) {
        out[r * D4 + j] = v[q];
        if (flip != nullptr) {
          float* f = flip + (row * D4 + j) * 4;
          if (__float_as_uint(v[q].x) == NEG0_BITS) flip_neg0(f + 0);
          if (__float_as_uint(v[q].y) == NEG0_BITS) flip_neg0(f + 1);
          if (__float_as_uint(v[q].z) == NEG0_BITS) flip_neg0(f + 2);
          if (__float_as_uint(v[q].w) == NEG0_BITS) flip_neg0(f + 3);
        }
      }
    }
    if (touched != nullptr && j0 == 0) touched[row] = 1;
  }
}

// op 1 (set) and op 4 (add, keys unique in the launch: plain read-modify-write)
template <int TPR, int NV, int OP>
__global__ void __launch_bounds__(256) apply_rows_v4_kernel(to_f4* __restrict__ table, const int32_t* __restrict__ idx,
                                                            int64_t n, int D4, const to_f4* __restrict__ delta,
                                                            uint8_t* __restrict__ touched) {
  int64_t r, step; int j0;
  row_coords<TPR>(r, step, j0);
  for (; r < n; r += step) {
    const int64_t row = (int64_t)idx[r];
    if (row < 0) continue;  // padding slot
    to_f4* dst = table + row * D4;
    to_f4 g[NV], w[NV];
#pragma unroll
    for (int q = 0; q < NV; ++q) {
      const int j = j0 + q * TPR;
      if (j < D4) {
        g[q] = __builtin_nontemporal_load(delta + r * D4 + j);
        if (OP == 4) w[q] = dst[j];
      }
    }
#pragma unroll
    for (int q = 0; q < NV; ++q) {
      const int j = j0 + q * TPR;
      if (j < D4) {
        to_f4 o;
        if (OP == 4) {
          o.x = w[q].x + pos0(g[q].x); o.y = w[q].y + pos0(g[q].y);
          o.z = w[q].z + pos0(g[q].z); o.w = w[q].w + pos0(g[q].w);
        } else {
          o.x = pos0(g[q].x); o.y = pos0(g[q].y); o.z = pos0(g[q].z); o.w = pos0(g[q].w);
        }
        dst[j] = o;
      }
    }
    if (touched != nullptr && j0 == 0) touched[row] = 1;
  }
}

// ---- de-duplication of request keys (one step, epoch-tagged map, no spins)
// map[key] = epoch << 32 | (0xffffffff - owner_request_index); atomicMax makes
// the newest epoch win and, inside it, the smallest request index.
//
// Two addressings of the claim map:
//  * dense  (HASHED = false): map has one entry per id of the table (MF items:
//    1M ids -> 8 MB), map index = key;
//  * hashed (HASHED = true): for id spaces of 1e9+ (PA 1B features, the
//    100B-parameter table) a per-batch open-addressing hash table
//    (dedup_hash_insert_kernel, capacity ~2x the batch) gives every request
//    the slot of its key and marks the one request whose CAS inserted it as
//    the owner -- no claim map, no claim pass.
// Epoch-tagged linear-probing insert: tab[h] = epoch << 32 | key.  Entries of
// older epochs count as empty, so nothing is cleared between steps.  The
// capacity (power of two, >= 2n) bounds every probe sequence.  The request
// whose CAS writes the key owns it; owner_slot is then indexed by hash slot.
//
// HU requests per thread are in flight together (their key loads, slot loads and
// first CASes issue back to back): with one request per iteration the dependent
// key -> slot -> CAS chain left the kernel latency-bound (202 us per 4M keys,
// profiles/r3_pa_ps_path_kernel_stats.csv).  The rare requests whose first slot
// is taken by another key finish with the serial probe loop.
constexpr int DEDUP_HU = 4;

__device__ __forceinline__ bool hash_probe(unsigned long long* __restrict__ tab, uint32_t mask, uint32_t epoch,
                                           unsigned long long mine, uint32_t& h, unsigned long long cur) {
  for (;;) {  // cur = tab[h] as last seen; returns whether this request inserted the key
    if ((uint32_t)(cur >> 32) != epoch) {
      const unsigned long long old = atomicCAS(tab + h, cur, mine);
      if (old == cur) return true;  // claimed the empty slot: this request owns the key
      cur = old;                    // somebody else wrote it first: re-examine
      if ((uint32_t)(cur >> 32) != epoch) continue;
    }
    if (cur == mine) return false;  // our key already lives here
    h = (h + 1) & mask;
    cur = tab[h];
  }
}

__global__ void dedup_hash_insert_kernel(const int32_t* __restrict__ keys, int64_t n,
                                         unsigned long long* __restrict__ tab, uint32_t mask, uint32_t epoch,
                                         int32_t* __restrict__ hslot) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t b0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; b0 < n; b0 += DEDUP_HU * stride) {
    unsigned long long mine[DEDUP_HU], cur[DEDUP_HU];
    uint32_t h[DEDUP_HU];
    bool act[DEDUP_HU], own[DEDUP_HU];
#pragma unroll
    for (int u = 0; u < DEDUP_HU; ++u) {
      const int64_t b = b0 + u * stride;
      act[u] = b < n;
      const uint32_t k = act[u] ? (uint32_t)keys[b] : 0u;
      mine[u] = ((unsigned long long)epoch << 32) | k;
      h[u] = fmix32(k ^ 0x5bd1e995u) & mask;
      own[u] = false;
    }
#pragma unroll
    for (int u = 0; u < DEDUP_HU; ++u) cur[u] = act[u] ? tab[h[u]] : 0ull;
#pragma unroll
    for (int u = 0; u < DEDUP_HU; ++u) {  // first attempt of every request: independent CASes
      if (act[u] && (uint32_t)(cur[u] >> 32) != epoch) {
        const unsigned long long old = atomicCAS(tab + h[u], cur[u], mine[u]);
        if (old == cur[u]) { own[u] = true; act[u] = false; }
        else cur[u] = old;
      }
    }
#pragma unroll
    for (int u = 0; u < DEDUP_HU; ++u) {
      if (act[u]) own[u] = hash_probe(tab, mask, epoch, mine[u], h[u], cur[u]);
      // bit 31 marks the key's owner (the CAS winner: exactly one per key), so no
      // separate claim pass is needed on the hashed path; cap <= 2^31 keeps h < 2^31
      const int64_t b = b0 + u * stride;
      if (b < n) hslot[b] = (int32_t)(h[u] | (own[u] ? 0x80000000u : 0u));
    }
  }
}

// dense path only (the hashed path takes ownership from the insert's CAS)
__global__ void dedup_claim_kernel(const int32_t* __restrict__ keys, int64_t n, unsigned long long* __restrict__ map,
                                   uint32_t epoch) {
  for (int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; b < n; b += (int64_t)gridDim.x * blockDim.x) {
    const unsigned long long v = ((unsigned long long)epoch << 32) | (unsigned long long)(0xffffffffu - (uint32_t)b);
    atomicMax(map + keys[b], v);
  }
}

// owners take a slot inside their destination shard's group
// part_kind 0 = hash (|id| % W, dense local id / W), 1 = range, 2 = sparse hash:
// |id| % W over the full signed 32-bit range (int64 |.|: no Math.abs(Int.MinValue)
// overflow) and the id itself as the key (the owner's device hash
// table maps it to a row, kernels/hash_table.hip)
__device__ __forceinline__ void key_dest(int32_t k, int W, int part_kind, int64_t block, int& d, int32_t& local) {
  if (part_kind == 0) { d = k % W; local = k / W; }
  else if (part_kind == 2) { const int64_t a = k < 0 ? -(int64_t)k : (int64_t)k; d = (int)(a % W); local = k; }
  else { d = (int)(k / block); if (d >= W) d = W - 1; local = (int32_t)(k - (int64_t)d * block); }
}

// Wave-aggregated slot allocation: the lanes of a wave that target the same
// shard take their slots with ONE atomicAdd (leader lane), ranks by popcount.
// A per-lane atomicAdd on W (often 1) counters serialises the whole batch on a
// single address (measured 11 ms for 1M owners on one counter).
__device__ __forceinline__ int32_t wave_alloc(bool want, int d, int32_t* __restrict__ counts) {
  const int lane = threadIdx.x & 63;
  unsigned long long pending = __ballot(want);
  int32_t slot = -1;
  while (pending) {  // uniform: every lane sees the same ballots
    const int leader = __ffsll((long long)pending) - 1;
    const int dd = __shfl(d, leader, 64);
    const unsigned long long m = __ballot(want && d == dd);
    int32_t base = 0;
    if (lane == leader) base = atomicAdd(counts + dd, (int32_t)__popcll(m));
    base = __shfl(base, leader, 64);
    if (want && d == dd) slot = base + (int32_t)__popcll(m & ((1ull << lane) - 1ull));
    pending &= ~m;
  }
  return slot;
}

// Two-level slot allocation: waves aggregate into per-shard LDS counters
// (wave_alloc on LDS), then one global atomicAdd per (block, shard) reserves
// the block's range.  With W = 1 every owner of the batch targets one
// counter; a per-wave global atomic still serialised 65k adds (0.72 ms for
// 4M keys), per-block reservation needs n / (256 * DEDUP_ITEMS) of them.
constexpr int DEDUP_ITEMS = 16;
constexpr int DEDUP_MAX_W = 64;

template <bool HASHED>
__global__ void __launch_bounds__(256) dedup_assign_kernel(const int32_t* __restrict__ keys,
                                                           const int32_t* __restrict__ hslot, int64_t n,
                                                           const unsigned long long* __restrict__ map, int W,
                                                           int part_kind, int64_t block, int32_t* __restrict__ counts,
                                                           int32_t* __restrict__ owner_slot) {
  __shared__ int32_t lds_cnt[DEDUP_MAX_W];
  __shared__ int32_t lds_base[DEDUP_MAX_W];
  for (int d = threadIdx.x; d < W; d += blockDim.x) lds_cnt[d] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * blockDim.x * DEDUP_ITEMS;
  int32_t slot_l[DEDUP_ITEMS];
  int dd[DEDUP_ITEMS];
  // loads first, all in flight (clamped indices, masked after: a load guarded by
  // b < n compiled to a branch and a full wait per item), then the slot allocation
  int32_t kv[DEDUP_ITEMS];
#pragma unroll
  for (int it = 0; it < DEDUP_ITEMS; ++it) kv[it] = keys[min(base + (int64_t)it * blockDim.x + threadIdx.x, n - 1)];
  uint32_t ov[DEDUP_ITEMS];  // dense: the claim's owner; hashed: the hash slot word
  if (HASHED && hslot == nullptr) {
#pragma unroll
    for (int it = 0; it < DEDUP_ITEMS; ++it) ov[it] = 0x80000000u;
  } else {
#pragma unroll
    for (int it = 0; it < DEDUP_ITEMS; ++it) {
      const int64_t bc = min(base + (int64_t)it * blockDim.x + threadIdx.x, n - 1);
      if (HASHED) ov[it] = (uint32_t)hslot[bc];
      else ov[it] = 0xffffffffu - (uint32_t)(map[kv[it]] & 0xffffffffull);
    }
  }
#pragma unroll
  for (int it = 0; it < DEDUP_ITEMS; ++it) {
    const int64_t b = base + (int64_t)it * blockDim.x + threadIdx.x;
    bool own = false;
    int d = 0;
    if (b < n) {
      int32_t local;
      key_dest(kv[it], W, part_kind, block, d, local);
      // hashed without hslot: every request owns its own slot b
      own = HASHED ? (int32_t)ov[it] < 0 : ov[it] == (uint32_t)b;
    }
    dd[it] = own ? d : -1;
    slot_l[it] = wave_alloc(own, d, lds_cnt);  // LDS atomics: cheap
  }
  __syncthreads();
  for (int d = threadIdx.x; d < W; d += blockDim.x)
    lds_base[d] = lds_cnt[d] ? atomicAdd(counts + d, lds_cnt[d]) : 0;
  __syncthreads();
#pragma unroll
  for (int it = 0; it < DEDUP_ITEMS; ++it) {
    if (dd[it] < 0) continue;
    const int64_t b = base + (int64_t)it * blockDim.x + threadIdx.x;
    // dense: indexed by the owner's request index; hashed: by the key's hash slot
    owner_slot[HASHED && hslot != nullptr ? (int64_t)(ov[it] & 0x7fffffffu) : b] = lds_base[dd[it]] + slot_l[it];
  }
}

// exclusive prefix of the W counts (W <= 1024; one tiny block)
__global__ void dedup_scan_kernel(const int32_t* __restrict__ counts, int W, int32_t* __restrict__ prefix) {
  if (threadIdx.x == 0) {
    int32_t acc = 0;
    for (int d = 0; d < W; ++d) { prefix[d] = acc; acc += counts[d]; }
    prefix[W] = acc;
  }
}

// compact position of every request; owners also write their unique local
// key, so uniq[0:total] is grouped by destination shard in ascending order
template <bool HASHED>
__global__ void dedup_resolve_kernel(const int32_t* __restrict__ keys, const int32_t* __restrict__ hslot, int64_t n,
                                     const unsigned long long* __restrict__ map,
                                     int W, int part_kind, int64_t block, const int32_t* __restrict__ prefix,
                                     const int32_t* __restrict__ owner_slot, int32_t* __restrict__ uniq,
                                     int32_t* __restrict__ pos) {
  // DEDUP_HU requests per thread in flight (the owner-slot loads are random)
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t b0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; b0 < n; b0 += DEDUP_HU * stride) {
    int32_t local[DEDUP_HU], p[DEDUP_HU];
    int64_t at[DEDUP_HU];
    bool own[DEDUP_HU], act[DEDUP_HU];
    int d[DEDUP_HU];
    // unconditional loads of clamped indices (masked after): guarded loads compiled to a
    // branch and a full wait each
    int32_t kv[DEDUP_HU];
#pragma unroll
    for (int u = 0; u < DEDUP_HU; ++u) kv[u] = keys[min(b0 + u * stride, n - 1)];
    uint64_t mv[DEDUP_HU];
    int32_t hv[DEDUP_HU];
#pragma unroll
    for (int u = 0; u < DEDUP_HU; ++u) {
      if (HASHED) hv[u] = hslot != nullptr ? hslot[min(b0 + u * stride, n - 1)] : 0;
      else mv[u] = map[kv[u]];
    }
#pragma unroll
    for (int u = 0; u < DEDUP_HU; ++u) {
      const int64_t b = b0 + u * stride;
      act[u] = b < n;
      const int32_t k = act[u] ? kv[u] : 0;
      key_dest(k, W, part_kind, block, d[u], local[u]);
      if (HASHED) {
        const int32_t hs = !act[u] ? 0 : (hslot != nullptr ? hv[u] : (int32_t)((uint32_t)b | 0x80000000u));
        at[u] = hs & 0x7fffffff;
        own[u] = hs < 0;
      } else {
        const uint32_t owner = act[u] ? 0xffffffffu - (uint32_t)(mv[u] & 0xffffffffull) : 0u;
        at[u] = owner;
        own[u] = owner == (uint32_t)b;
      }
    }
#pragma unroll
    for (int u = 0; u < DEDUP_HU; ++u) p[u] = act[u] ? prefix[d[u]] + owner_slot[at[u]] : 0;
#pragma unroll
    for (int u = 0; u < DEDUP_HU; ++u) {
      if (!act[u]) continue;
      pos[b0 + u * stride] = p[u];
      if (own[u]) uniq[p[u]] = local[u];
    }
  }
}

// shard id + per-shard count + stable rank inside the shard, for callers
// that ship raw (non-deduplicated) keys.
__global__ void bucketize_kernel(const int32_t* __restrict__ keys, int64_t n, int W, int part_kind, int64_t block,
                                 int32_t* __restrict__ shard, int32_t* __restrict__ counts) {
  const int lane = threadIdx.x & 63;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t w0 = (int64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63); w0 < n; w0 += stride) {
    const int64_t b = w0 + lane;
    int d = 0;
    if (b < n) {
      const int64_t k = keys[b] < 0 ? -(int64_t)keys[b] : (int64_t)keys[b];
      if (part_kind == 0 || part_kind == 2) d = (int)(k % W);
      else { d = (int)(k / block); if (d >= W) d = W - 1; }
      shard[b] = d;
    }
    wave_alloc(b < n, d, counts);
  }
}

}  // namespace

// D = 1 (PA weights, LEMP norms): one lane per row, 64 independent rows per
// wave instruction (scattered 4-B rows are transaction-bound, not byte-bound)
#define TPR_SWITCH(D, ...)                                   \
  do {                                                       \
    if ((D) <= 1) { constexpr int TPR = 1; __VA_ARGS__; }     \
    else if ((D) <= 2) { constexpr int TPR = 2; __VA_ARGS__; } \
    else if ((D) <= 4) { constexpr int TPR = 4; __VA_ARGS__; } \
    else if ((D) <= 8) { constexpr int TPR = 8; __VA_ARGS__; } \
    else if ((D) <= 16) { constexpr int TPR = 16; __VA_ARGS__; } \
    else if ((D) <= 32) { constexpr int TPR = 32; __VA_ARGS__; } \
    else { constexpr int TPR = 64; __VA_ARGS__; }            \
  } while (0)

static inline int rows_grid(int64_t n, int TPR) {
  const int64_t rows_per_block = 4 * (64 / TPR);  // 256 threads = 4 waves
  return grid_for(n, (int)rows_per_block, 256 * 32);
}

namespace {
// touched[rows[i]] = 1 (close-time dump bookkeeping of the in-place update paths)
__global__ void mark_rows_kernel(uint8_t* __restrict__ touched, const int32_t* __restrict__ rows, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    if (rows[i] >= 0) touched[rows[i]] = 1;  // < 0: a padding slot
}

// identity plans over a sentinel table: flip the -0.0 entries of the rows whose mask
// byte is set (the present keys), one thread per entry; rows without the mask are not
// read (a whole-table masked_fill read and rewrote every row per micro-batch)
__global__ void flip_masked_kernel(float* __restrict__ table, const uint8_t* __restrict__ mask, int64_t n_rows,
                                   int D) {
  const int64_t total = n_rows * D;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x)
    if (mask[i / D] && __float_as_uint(table[i]) == NEG0_BITS) flip_neg0(table + i);
}
}  // namespace

namespace {
// ---- flag dedup: for batches that cover a large part of a dense key space (MF
// items: 64M requests over 1M ids), the claim-map dedup spends its time in
// contended atomicMax / owner lookups (2.5 + 1.75 ms for 64M keys).  Here every
// request just stores the epoch into flag[key] (plain, idempotent), one scan over
// the key space in shard-major order numbers the present keys, and each request
// reads its slot back: no atomics, deterministic layout (unique keys sorted by
// shard, then local key).
constexpr int FLAG_CH = 4096;  // keys of the (virtual) key space per scan workgroup

__global__ void flag_keys_kernel(const int32_t* __restrict__ keys, int64_t n, uint32_t* __restrict__ flag,
                                 uint32_t epoch) {
  for (int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; b < n; b += (int64_t)gridDim.x * blockDim.x) {
    const int32_t k = keys[b];
    if (flag[k] != epoch) flag[k] = epoch;  // repeats of a key (64 per step for MF items) only read
  }
}

// virtual index v (shard-major) -> key; hash: v = d * L + l, key = d + W * l; range: key = v
__device__ __forceinline__ int64_t flag_key_of(int64_t v, int64_t num_ids, int W, int part_kind, int64_t L) {
  if (part_kind != 0) return v;
  const int64_t d = v / L, l = v - d * L;
  return d + (int64_t)W * l;
}

__device__ __forceinline__ int32_t block_exclusive_scan_1024(int32_t x, int32_t* wsum, int32_t& total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int32_t inc = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int32_t y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  int32_t before = 0;
  total = 0;
  for (int q = 0; q < 16; ++q) {
    if (q < w) before += wsum[q];
    total += wsum[q];
  }
  __syncthreads();  // wsum reused by the caller's next scan
  return before + inc - x;
}

// pass 1: present keys per chunk of the virtual key space
__global__ void __launch_bounds__(1024) flag_count_kernel(const uint32_t* __restrict__ flag, int64_t num_ids,
                                                          int64_t V, int W, int part_kind, int64_t L,
                                                          uint32_t epoch, int32_t* __restrict__ bsum) {
  __shared__ int32_t wsum[16];
  const int64_t v0 = (int64_t)blockIdx.x * FLAG_CH + threadIdx.x * 4;
  int32_t c = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int64_t v = v0 + q;
    if (v < V) {
      const int64_t k = flag_key_of(v, num_ids, W, part_kind, L);
      c += (k < num_ids && flag[k] == epoch) ? 1 : 0;
    }
  }
  int32_t total;
  block_exclusive_scan_1024(c, wsum, total);
  if (threadIdx.x == 0) bsum[blockIdx.x] = total;
}

// pass 2 (one workgroup): exclusive scan of the chunk counts in place; bsum[nb] = total
__global__ void __launch_bounds__(1024) flag_scan_kernel(int32_t* __restrict__ bsum, int nb) {
  __shared__ int32_t wsum[16];
  int32_t carry = 0;
  for (int base = 0; base < nb; base += 1024) {
    const int i = base + threadIdx.x;
    const int32_t x = i < nb ? bsum[i] : 0;
    int32_t total;
    const int32_t ex = block_exclusive_scan_1024(x, wsum, total);
    if (i < nb) bsum[i] = carry + ex;
    carry += total;
  }
  if (threadIdx.x == 0) bsum[nb] = carry;
}

// pass 3: slot of every present key, its local key in uniq, shard starts in prefix
__global__ void __launch_bounds__(1024) flag_assign_kernel(const uint32_t* __restrict__ flag, int64_t num_ids,
                                                           int64_t V, int W, int part_kind, int64_t L,
                                                           int64_t block, uint32_t epoch,
                                                           const int32_t* __restrict__ bsum,
                                                           int32_t* __restrict__ slot, int32_t* __restrict__ uniq,
                                                           int32_t* __restrict__ prefix) {
  __shared__ int32_t wsum[16];
  const int64_t v0 = (int64_t)blockIdx.x * FLAG_CH + threadIdx.x * 4;
  bool pres[4];
  int64_t key[4];
  int32_t c = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int64_t v = v0 + q;
    key[q] = v < V ? flag_key_of(v, num_ids, W, part_kind, L) : num_ids;
    pres[q] = key[q] < num_ids && flag[key[q]] == epoch;
    c += pres[q] ? 1 : 0;
  }
  int32_t total;
  int32_t at = bsum[blockIdx.x] + block_exclusive_scan_1024(c, wsum, total);
  const int64_t shard_len = part_kind == 0 ? L : block;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int64_t v = v0 + q;
    if (v < V && v % shard_len == 0 && v / shard_len < W) prefix[v / shard_len] = at;  // first v of shard d
    if (pres[q]) {
      const int64_t k = key[q];
      int64_t local;
      if (part_kind == 0) local = k / W;
      else { int64_t d = k / block; if (d >= W) d = W - 1; local = k - d * block; }
      slot[k] = at;
      uniq[at] = (int32_t)local;
      ++at;
    }
  }
}

__global__ void flag_pos_kernel(const int32_t* __restrict__ keys, int64_t n, const int32_t* __restrict__ slot,
                                int32_t* __restrict__ pos) {
  for (int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; b < n; b += (int64_t)gridDim.x * blockDim.x)
    pos[b] = slot[keys[b]];
}

__global__ void flag_counts_kernel(const int32_t* __restrict__ bsum, int nb, int W, int64_t V, int64_t shard_len,
                                   int32_t* __restrict__ prefix, int32_t* __restrict__ counts) {
  if (threadIdx.x != 0) return;
  prefix[W] = bsum[nb];
  for (int d = 0; d < W; ++d)
    if ((int64_t)d * shard_len >= V) prefix[d] = bsum[nb];  // empty trailing range shard: never scanned
  for (int d = 0; d < W; ++d) counts[d] = prefix[d + 1] - prefix[d];
}
}  // namespace

// Flag dedup (see flag_keys_kernel).  flag / slot: num_ids entries (flag epoch-tagged,
// never cleared); bsum: fps_dedup_flags_ws_ints(num_ids, W) ints.  Same outputs as
// fps_dedup: counts[W], prefix[W+1], uniq (shard-major, ascending local keys), pos[n].
FPS_API int64_t fps_dedup_flags_ws_ints(int64_t num_ids, int W) {
  const int64_t L = (num_ids + W - 1) / W;
  const int64_t V = (int64_t)W * L;
  return (V + FLAG_CH - 1) / FLAG_CH + 1;
}

FPS_API int fps_dedup_flags(const int32_t* keys, int64_t n, uint32_t* flag, int32_t* slot, uint32_t epoch,
                            int64_t num_ids, int W, int part_kind, int64_t block, int32_t* bsum, int32_t* counts,
                            int32_t* prefix, int32_t* uniq, int32_t* pos, void* stream) {
  if (W <= 0 || num_ids <= 0) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  const int64_t L = (num_ids + W - 1) / W;
  const int64_t V = part_kind == 0 ? (int64_t)W * L : num_ids;
  const int nb = (int)((V + FLAG_CH - 1) / FLAG_CH);
  if (part_kind != 0 && block <= 0) return (int)hipErrorInvalidValue;
  if (n > 0)
    hipLaunchKernelGGL(flag_keys_kernel, dim3(grid_for(n, 256, 256 * 16)), dim3(256), 0, s, keys, n, flag, epoch);
  hipLaunchKernelGGL(flag_count_kernel, dim3(nb), dim3(1024), 0, s, (const uint32_t*)flag, num_ids, V, W, part_kind,
                     L, epoch, bsum);
  hipLaunchKernelGGL(flag_scan_kernel, dim3(1), dim3(1024), 0, s, bsum, nb);
  hipLaunchKernelGGL(flag_assign_kernel, dim3(nb), dim3(1024), 0, s, (const uint32_t*)flag, num_ids, V, W, part_kind,
                     L, block, epoch, (const int32_t*)bsum, slot, uniq, prefix);
  hipLaunchKernelGGL(flag_counts_kernel, dim3(1), dim3(64), 0, s, (const int32_t*)bsum, nb, W, V,
                     part_kind == 0 ? L : block, prefix, counts);
  if (n > 0)
    hipLaunchKernelGGL(flag_pos_kernel, dim3(grid_for(n, 256, 256 * 16)), dim3(256), 0, s, keys, n,
                       (const int32_t*)slot, pos);
  FPS_CHECK_LAUNCH();
  return 0;
}

// The world-1 static de-duplicated plan in one launch (it was seven torch ops per
// micro-batch): slot j < nb serves uniq[j] when j < U = prefix[1] (the unique keys)
// and the real key uniq[j mod U] as padding otherwise (valid[j] = j < U); pos_out = a
// copy of the request positions (the dedup workspace reuses pos for the next plan);
// push_rows[j] = gkeys[j] for the real keys, -1 for the padding (the rows a push applies).
__global__ void static_plan_kernel(const int32_t* __restrict__ uniq, const int32_t* __restrict__ prefix,
                                   int64_t nb, const int32_t* __restrict__ pos, int64_t n,
                                   int32_t* __restrict__ gkeys, uint8_t* __restrict__ valid,
                                   int32_t* __restrict__ pos_out, int32_t* __restrict__ push_rows) {
  const int64_t U = prefix[1];
  const int64_t Uc = U > 0 ? U : 1;
  const int64_t m = nb > n ? nb : n;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += (int64_t)gridDim.x * blockDim.x) {
    if (j < nb) {
      const bool v = j < U;
      const int32_t key = uniq[v ? j : j % Uc];
      valid[j] = v;
      gkeys[j] = key;
      push_rows[j] = v ? key : -1;
    }
    if (j < n) pos_out[j] = pos[j];
  }
}

FPS_API int fps_static_plan(const int32_t* uniq, const int32_t* prefix, int64_t nb, const int32_t* pos, int64_t n,
                            int32_t* gkeys, uint8_t* valid, int32_t* pos_out, int32_t* push_rows, void* stream) {
  const int64_t m = nb > n ? nb : n;
  if (m <= 0) return 0;
  hipLaunchKernelGGL(static_plan_kernel, dim3(grid_for(m, 256, 256 * 16)), dim3(256), 0, (hipStream_t)stream, uniq,
                     prefix, nb, pos, n, gkeys, valid, pos_out, push_rows);
  FPS_CHECK_LAUNCH();
  return 0;
}

namespace {
// ---- emulated all-to-all receive (parallel/emulated.py, hot-owner model): segment j of
// the output is rows [0, m_j) of `src` (k rows), tiled as often as m_j needs, i.e.
// out[off_j + i] = src[i mod k].  One launch over the output's 16-B (or smaller) words; the
// segment of a word by a linear search over <= FPS_FILL_MAX_SEGS offsets.  (A torch.cat
// of the prefixes ran at ~0.6 TB/s -- 300 us per SGNS exchange -- so the transfer model
// cost more device time than the receive it models.)
constexpr int FPS_FILL_MAX_SEGS = 64;
struct SegOffsets {
  int64_t off[FPS_FILL_MAX_SEGS + 1];  // output row offsets: off[0] = 0, off[nseg] = rows out
};

// source row of output row `row`: segment by a linear search (<= 64 offsets), then the
// row inside the source (a modulo only where a segment tiles the source)
__device__ __forceinline__ int64_t segment_src_row(const SegOffsets& so, int nseg, int64_t row, int64_t k) {
  int j = 0;
  while (j + 1 < nseg && so.off[j + 1] <= row) ++j;
  int64_t r = row - so.off[j];
  return r < k ? r : r % k;
}

// LPR lanes per row (a power of two covering the row's words, at most 64): a wave
// copies 64 / LPR rows at a time, so a 4-B row (PA's scalar weights) takes one lane,
// a 128-B or 256-B row (config #5's bf16 / fp32 rows) 8 or 16 lanes and a 600-B row
// (SGNS) the whole wave -- every lane busy with one 16-B (or smaller) word per step.
//
// min_ticks > 0 (the emulated link, parallel/emulated.py): the kernel also lasts at least
// min_ticks of the 100 MHz s_memrealtime clock from the start of workgroup 0 -- its
// first wave spins (s_sleep) after its share of the copy.  A transfer that writes its
// receive buffer as the data arrives completes at max(link time, write time), in one
// kernel on one stream.
template <typename T>
__global__ void segment_fill_kernel(const T* __restrict__ src, int64_t k, int64_t wpr, T* __restrict__ out,
                                    SegOffsets so, int nseg, int lpr_shift, uint64_t min_ticks) {
  const bool timer = min_ticks > 0 && blockIdx.x == 0 && threadIdx.x < 64;  // wave-uniform
  const uint64_t t0 = timer ? __builtin_amdgcn_s_memrealtime() : 0;
  const int64_t rows = so.off[nseg];
  const int lane = threadIdx.x & 63;
  const int lpr = 1 << lpr_shift, rpw = 64 >> lpr_shift;
  const int sub = lane >> lpr_shift, c0 = lane & (lpr - 1);
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t waves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int64_t stride = waves * rpw;
  if (wpr <= lpr) {
    // a row is at most one word per lane (PA's 4-B weights, 128-B rows, ...): FILL_UR rows
    // per lane per trip, every load issued before the first store -- one dependent
    // load / store pair per trip left a 256-workgroup launch latency-bound (a 16.8 MB
    // receive of 4-B rows took 117 us beside the owner's gather)
    constexpr int FILL_UR = 8;
    const bool on = c0 < wpr;
    for (int64_t row0 = wave * rpw + sub; row0 < rows; row0 += stride * FILL_UR) {
      int64_t r[FILL_UR];
      T v[FILL_UR];
#pragma unroll
      for (int u = 0; u < FILL_UR; ++u) {
        const int64_t row = row0 + u * stride;
        r[u] = on && row < rows ? segment_src_row(so, nseg, row, k) : -1;
      }
#pragma unroll
      for (int u = 0; u < FILL_UR; ++u)
        if (r[u] >= 0) v[u] = src[r[u] * wpr + c0];
#pragma unroll
      for (int u = 0; u < FILL_UR; ++u)
        if (r[u] >= 0) out[(row0 + u * stride) * wpr + c0] = v[u];
    }
  } else {
    for (int64_t row = wave * rpw + sub; row < rows; row += stride) {
      const int64_t r = segment_src_row(so, nseg, row, k);
      for (int64_t c = c0; c < wpr; c += lpr) out[row * wpr + c] = src[r * wpr + c];
    }
  }
  if (timer)
    while (__builtin_amdgcn_s_memrealtime() - t0 < min_ticks) __builtin_amdgcn_s_sleep(8);
}

// workgroups of a fill that also times a link (A/B knob fps_segment_fill_set_link_wgs)
int g_fill_link_wgs = 256;

template <typename T>
void segment_fill_launch(const void* src, int64_t k, int64_t row_bytes, void* out, const SegOffsets& so, int nseg,
                         hipStream_t st, uint64_t min_ticks) {
  const int64_t wpr = row_bytes / (int64_t)sizeof(T);
  int sh = 0;
  while (sh < 6 && (1ll << sh) < wpr) ++sh;
  const int64_t rows = so.off[nseg];
  const int64_t waves = (rows + (64 >> sh) - 1) / (64 >> sh);
  // a modelled link transfer (min_ticks > 0) writes with at most one workgroup per CU, as
  // RCCL's copy kernels occupy a few CUs, not the whole GPU beside the compute
  const int max_blocks = min_ticks > 0 ? g_fill_link_wgs : 256 * 16;
  hipLaunchKernelGGL(segment_fill_kernel<T>, dim3(grid_for(waves, 4, max_blocks)), dim3(256), 0, st, (const T*)src,
                     k, wpr, (T*)out, so, nseg, sh, min_ticks);
}
}  // namespace

FPS_API void fps_segment_fill_set_link_wgs(int v) { g_fill_link_wgs = v > 0 ? v : 256; }

// rows[nseg]: rows of each output segment (host array); src: k rows of row_bytes;
// min_us > 0: the kernel lasts at least that long (see segment_fill_kernel)
FPS_API int fps_segment_fill(const void* src, int64_t k, int64_t row_bytes, void* out, const int64_t* rows, int nseg,
                             void* stream, double min_us) {
  if (nseg <= 0 || nseg > FPS_FILL_MAX_SEGS || row_bytes <= 0) return (int)hipErrorInvalidValue;
  SegOffsets so;
  so.off[0] = 0;
  for (int j = 0; j < nseg; ++j) {
    if (rows[j] < 0) return (int)hipErrorInvalidValue;
    so.off[j + 1] = so.off[j] + rows[j];
  }
  const uint64_t min_ticks = min_us > 0 ? (uint64_t)(min_us * 100.0) : 0;  // s_memrealtime: 100 MHz
  if (so.off[nseg] == 0 && min_ticks == 0) return 0;
  if (so.off[nseg] > 0 && k <= 0) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  auto fits = [&](int64_t a) {
    return row_bytes % a == 0 && (uintptr_t)src % a == 0 && (uintptr_t)out % a == 0;
  };
  if (fits(16)) segment_fill_launch<uint4>(src, k, row_bytes, out, so, nseg, st, min_ticks);
  else if (fits(8)) segment_fill_launch<uint2>(src, k, row_bytes, out, so, nseg, st, min_ticks);
  else if (fits(4)) segment_fill_launch<uint32_t>(src, k, row_bytes, out, so, nseg, st, min_ticks);
  else if (fits(2)) segment_fill_launch<uint16_t>(src, k, row_bytes, out, so, nseg, st, min_ticks);
  else segment_fill_launch<uint8_t>(src, k, row_bytes, out, so, nseg, st, min_ticks);
  FPS_CHECK_LAUNCH();
  return 0;
}

FPS_API int fps_mark_rows(uint8_t* touched, const int32_t* rows, int64_t n, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(mark_rows_kernel, dim3(grid_for(n, 256, 256 * 16)), dim3(256), 0, (hipStream_t)stream, touched,
                     rows, n);
  FPS_CHECK_LAUNCH();
  return 0;
}

namespace {
// The count message of a dynamic PS plan: row j = (2 counts[j] + request, flag).  One
// launch instead of the cast / scale / offset / fill / concatenate chain (five torch
// kernels and their host calls per micro-batch, TensorPS._pending).
__global__ void pack_counts_kernel(const int32_t* __restrict__ counts, int W, int request, int flag,
                                   int32_t* __restrict__ out) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= W) return;
  out[2 * j] = counts[j] * 2 + request;
  out[2 * j + 1] = flag;
}
}  // namespace

FPS_API int fps_pack_counts(const int32_t* counts, int W, int request, int flag, int32_t* out, void* stream) {
  if (W <= 0) return 0;
  hipLaunchKernelGGL(pack_counts_kernel, dim3((W + 255) / 256), dim3(256), 0, (hipStream_t)stream, counts, W, request,
                     flag, out);
  FPS_CHECK_LAUNCH();
  return 0;
}

FPS_API int fps_flip_masked(float* table, const uint8_t* mask, int64_t n_rows, int D, void* stream) {
  if (n_rows <= 0 || D <= 0) return 0;
  hipLaunchKernelGGL(flip_masked_kernel, dim3(grid_for(n_rows * D, 256, 256 * 16)), dim3(256), 0, (hipStream_t)stream,
                     table, mask, n_rows, D);
  FPS_CHECK_LAUNCH();
  return 0;
}

FPS_API int fps_init_rows(float* table, int64_t n_rows, int D, int64_t id_base, int64_t id_stride, float lo, float hi,
                          uint32_t seed, void* stream) {
  if (n_rows <= 0) return 0;
  TPR_SWITCH(D, hipLaunchKernelGGL(init_rows_kernel<TPR>, dim3(rows_grid(n_rows, TPR)), dim3(256), 0,
                                   (hipStream_t)stream, table, n_rows, D, id_base, id_stride, lo, hi, seed));
  FPS_CHECK_LAUNCH();
  return 0;
}

// (TPR, NV) of the 16-byte kernels for D4 = D / 4 float4 per row; false: use the scalar kernels
static inline bool v4_shape(int D, const void* a, const void* b, int& tpr, int& nv) {
  if (D % 4 != 0 || ((uintptr_t)a & 15) || ((uintptr_t)b & 15)) return false;
  const int D4 = D / 4;
  if (D4 > 256) return false;
  nv = D4 <= 64 ? 1 : D4 <= 128 ? 2 : 4;
  tpr = 1;
  while (tpr * nv < D4) tpr <<= 1;
  return true;
}

#define V4_SWITCH(tpr, nv, ...)                                                                      \
  do {                                                                                               \
    if (nv == 1) {                                                                                   \
      constexpr int NV = 1;                                                                          \
      switch (tpr) {                                                                                 \
        case 1: { constexpr int TPR = 1; __VA_ARGS__; } break;                                      \
        case 2: { constexpr int TPR = 2; __VA_ARGS__; } break;                                      \
        case 4: { constexpr int TPR = 4; __VA_ARGS__; } break;                                      \
        case 8: { constexpr int TPR = 8; __VA_ARGS__; } break;                                      \
        case 16: { constexpr int TPR = 16; __VA_ARGS__; } break;                                    \
        case 32: { constexpr int TPR = 32; __VA_ARGS__; } break;                                    \
        default: { constexpr int TPR = 64; __VA_ARGS__; }                                           \
      }                                                                                              \
    } else if (nv == 2) { constexpr int NV = 2, TPR = 64; __VA_ARGS__; }                             \
    else { constexpr int NV = 4, TPR = 64; __VA_ARGS__; }                                            \
  } while (0)

FPS_API int fps_gather_rows(const float* table, const void* idx, int idx_is_64, int64_t n, int D, void* out,
                            int out_bf16, uint8_t* touched, int flip_sentinel, void* stream) {
  float* flip = flip_sentinel ? const_cast<float*>(table) : nullptr;
  if (n <= 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (D == 1) {  // scalar rows: SC loads in flight per lane
    const int64_t g = (n + 256 * SC - 1) / (256 * SC);
    if (idx_is_64) {
      if (out_bf16) hipLaunchKernelGGL((gather_scalar_kernel<true, int64_t>), dim3(g), dim3(256), 0, s, table, (const int64_t*)idx, n, out, touched, flip);
      else hipLaunchKernelGGL((gather_scalar_kernel<false, int64_t>), dim3(g), dim3(256), 0, s, table, (const int64_t*)idx, n, out, touched, flip);
    } else {
      if (out_bf16) hipLaunchKernelGGL((gather_scalar_kernel<true, int32_t>), dim3(g), dim3(256), 0, s, table, (const int32_t*)idx, n, out, touched, flip);
      else hipLaunchKernelGGL((gather_scalar_kernel<false, int32_t>), dim3(g), dim3(256), 0, s, table, (const int32_t*)idx, n, out, touched, flip);
    }
    FPS_CHECK_LAUNCH();
    return 0;
  }
  int tpr, nv;
  if (!out_bf16 && v4_shape(D, table, out, tpr, nv)) {
    const int D4 = D / 4;
    V4_SWITCH(tpr, nv, {
      const int g = rows_grid(n, TPR);
      if (idx_is_64)
        hipLaunchKernelGGL((gather_rows_v4_kernel<TPR, NV, int64_t>), dim3(g), dim3(256), 0, s, (const to_f4*)table,
                           (const int64_t*)idx, n, D4, (to_f4*)out, touched, flip);
      else
        hipLaunchKernelGGL((gather_rows_v4_kernel<TPR, NV, int32_t>), dim3(g), dim3(256), 0, s, (const to_f4*)table,
                           (const int32_t*)idx, n, D4, (to_f4*)out, touched, flip);
    });
    FPS_CHECK_LAUNCH();
    return 0;
  }
  TPR_SWITCH(D, {
    const int g = rows_grid(n, TPR);
    if (idx_is_64) {
      if (out_bf16) hipLaunchKernelGGL((gather_rows_kernel<TPR, true, int64_t>), dim3(g), dim3(256), 0, s, table, (const int64_t*)idx, n, D, out, touched, flip);
      else hipLaunchKernelGGL((gather_rows_kernel<TPR, false, int64_t>), dim3(g), dim3(256), 0, s, table, (const int64_t*)idx, n, D, out, touched, flip);
    } else {
      if (out_bf16) hipLaunchKernelGGL((gather_rows_kernel<TPR, true, int32_t>), dim3(g), dim3(256), 0, s, table, (const int32_t*)idx, n, D, out, touched, flip);
      else hipLaunchKernelGGL((gather_rows_kernel<TPR, false, int32_t>), dim3(g), dim3(256), 0, s, table, (const int32_t*)idx, n, D, out, touched, flip);
    }
  });
  FPS_CHECK_LAUNCH();
  return 0;
}

template <int TPR>
static void launch_apply(float* table, float* state, const int32_t* idx, int64_t n, int D, const void* delta,
                         int delta_bf16, int op, float lr, float eps, uint8_t* touched, hipStream_t s) {
  const int g = rows_grid(n, TPR);
  if (delta_bf16) {
    switch (op) {
      case 0: hipLaunchKernelGGL((apply_rows_kernel<TPR, true, 0>), dim3(g), dim3(256), 0, s, table, state, idx, n, D, delta, lr, eps, touched); break;
      case 1: hipLaunchKernelGGL((apply_rows_kernel<TPR, true, 1>), dim3(g), dim3(256), 0, s, table, state, idx, n, D, delta, lr, eps, touched); break;
      case 2: hipLaunchKernelGGL((apply_rows_kernel<TPR, true, 2>), dim3(g), dim3(256), 0, s, table, state, idx, n, D, delta, lr, eps, touched); break;
      case 4: hipLaunchKernelGGL((apply_rows_kernel<TPR, true, 4>), dim3(g), dim3(256), 0, s, table, state, idx, n, D, delta, lr, eps, touched); break;
      case 5: hipLaunchKernelGGL((apply_rows_kernel<TPR, true, 5>), dim3(g), dim3(256), 0, s, table, state, idx, n, D, delta, lr, eps, touched); break;
      default: hipLaunchKernelGGL((apply_rows_kernel<TPR, true, 3>), dim3(g), dim3(256), 0, s, table, state, idx, n, D, delta, lr, eps, touched);
    }
  } else {
    switch (op) {
      case 0: hipLaunchKernelGGL((apply_rows_kernel<TPR, false, 0>), dim3(g), dim3(256), 0, s, table, state, idx, n, D, delta, lr, eps, touched); break;
      case 1: hipLaunchKernelGGL((apply_rows_kernel<TPR, false, 1>), dim3(g), dim3(256), 0, s, table, state, idx, n, D, delta, lr, eps, touched); break;
      case 2: hipLaunchKernelGGL((apply_rows_kernel<TPR, false, 2>), dim3(g), dim3(256), 0, s, table, state, idx, n, D, delta, lr, eps, touched); break;
      case 4: hipLaunchKernelGGL((apply_rows_kernel<TPR, false, 4>), dim3(g), dim3(256), 0, s, table, state, idx, n, D, delta, lr, eps, touched); break;
      case 5: hipLaunchKernelGGL((apply_rows_kernel<TPR, false, 5>), dim3(g), dim3(256), 0, s, table, state, idx, n, D, delta, lr, eps, touched); break;
      default: hipLaunchKernelGGL((apply_rows_kernel<TPR, false, 3>), dim3(g), dim3(256), 0, s, table, state, idx, n, D, delta, lr, eps, touched);
    }
  }
}

FPS_API int fps_apply_rows(float* table, float* state, const int32_t* idx, int64_t n, int D, const void* delta,
                           int delta_bf16, int op, float lr, float eps, uint8_t* touched, void* stream) {
  if (n <= 0) return 0;
  if ((op == 3 || op == 5) && state == nullptr) return (int)hipErrorInvalidValue;
  if (D == 1 && (op == 0 || op == 1 || op == 4)) {  // scalar rows: SC loads in flight per lane
    hipStream_t s = (hipStream_t)stream;
    const int64_t g = (n + 256 * SC - 1) / (256 * SC);
#define FPS_APSC(OP_)                                                                                                  \
    if (delta_bf16) hipLaunchKernelGGL((apply_scalar_kernel<OP_, true>), dim3(g), dim3(256), 0, s, table, idx, n, delta, touched); \
    else hipLaunchKernelGGL((apply_scalar_kernel<OP_, false>), dim3(g), dim3(256), 0, s, table, idx, n, delta, touched);
    if (op == 0) { FPS_APSC(0); } else if (op == 4) { FPS_APSC(4); } else { FPS_APSC(1); }
#undef FPS_APSC
    FPS_CHECK_LAUNCH();
    return 0;
  }
  int tpr, nv;
  if (!delta_bf16 && (op == 1 || op == 4) && v4_shape(D, table, delta, tpr, nv)) {
    const int D4 = D / 4;
    hipStream_t s = (hipStream_t)stream;
    V4_SWITCH(tpr, nv, {
      const int g = rows_grid(n, TPR);
      if (op == 4)
        hipLaunchKernelGGL((apply_rows_v4_kernel<TPR, NV, 4>), dim3(g), dim3(256), 0, s, (to_f4*)table, idx, n, D4,
                           (const to_f4*)delta, touched);
      else
        hipLaunchKernelGGL((apply_rows_v4_kernel<TPR, NV, 1>), dim3(g), dim3(256), 0, s, (to_f4*)table, idx, n, D4,
                           (const to_f4*)delta, touched);
    });
    FPS_CHECK_LAUNCH();
    return 0;
  }
  TPR_SWITCH(D, launch_apply<TPR>(table, state, idx, n, D, delta, delta_bf16, op, lr, eps, touched, (hipStream_t)stream));
  FPS_CHECK_LAUNCH();
  return 0;
}

template <bool HASHED>
static int launch_dedup(const int32_t* keys, const int32_t* hslot, int64_t n, unsigned long long* map,
                        uint32_t epoch, int W, int part_kind, int64_t block, int32_t* counts, int32_t* prefix,
                        int32_t* owner_slot, int32_t* uniq, int32_t* pos, hipStream_t s) {
  if (W > DEDUP_MAX_W) return (int)hipErrorInvalidValue;
  const int g = grid_for(n > 0 ? n : 1, 256, 256 * 16);
  if (n > 0) {
    if (!HASHED) hipLaunchKernelGGL(dedup_claim_kernel, dim3(g), dim3(256), 0, s, keys, n, map, epoch);
    const int64_t ga = (n + 256 * DEDUP_ITEMS - 1) / (256 * DEDUP_ITEMS);
    hipLaunchKernelGGL(dedup_assign_kernel<HASHED>, dim3((unsigned)ga), dim3(256), 0, s, keys, hslot, n,
                       (const unsigned long long*)map, W, part_kind, block, counts, owner_slot);
  }
  hipLaunchKernelGGL(dedup_scan_kernel, dim3(1), dim3(64), 0, s, (const int32_t*)counts, W, prefix);
  if (n > 0)
    hipLaunchKernelGGL(dedup_resolve_kernel<HASHED>, dim3(g), dim3(256), 0, s, keys, hslot, n,
                       (const unsigned long long*)map, W, part_kind, block, (const int32_t*)prefix,
                       (const int32_t*)owner_slot, uniq, pos);
  FPS_CHECK_LAUNCH();
  return 0;
}

// counts[W] must be zeroed by the caller; prefix has W+1 entries
// (prefix[W] = number of unique keys); uniq/pos/owner_slot have n entries.
FPS_API int fps_dedup(const int32_t* keys, int64_t n, unsigned long long* map, uint32_t epoch, int W, int part_kind,
                      int64_t block, int32_t* counts, int32_t* prefix, int32_t* owner_slot, int32_t* uniq,
                      int32_t* pos, void* stream) {
  return launch_dedup<false>(keys, nullptr, n, map, epoch, W, part_kind, block, counts, prefix, owner_slot, uniq,
                             pos, (hipStream_t)stream);
}

// Hashed variant for huge id spaces: tab (uint64) and owner_slot (int32) hold
// cap entries (power of two, >= 2n, <= 2^31); hslot has n entries.  Keys >= 0,
// or any int32 with part_kind 2 (sparse ids).
FPS_API int fps_dedup_hashed(const int32_t* keys, int64_t n, unsigned long long* tab, int64_t cap, uint32_t epoch,
                             int W, int part_kind, int64_t block, int32_t* counts, int32_t* prefix, int32_t* hslot,
                             int32_t* owner_slot, int32_t* uniq, int32_t* pos, void* stream) {
  if (cap < 2 * n || (cap & (cap - 1)) != 0 || cap > (1ll << 31)) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  if (n > 0) {
    const int g = grid_for(n, 256, 256 * 16);
    hipLaunchKernelGGL(dedup_hash_insert_kernel, dim3(g), dim3(256), 0, s, keys, n, tab, (uint32_t)(cap - 1), epoch,
                       hslot);
  }
  return launch_dedup<true>(keys, hslot, n, nullptr, epoch, W, part_kind, block, counts, prefix, owner_slot, uniq,
                            pos, s);
}

// Requests grouped by destination shard WITHOUT de-duplication (request plans of
// key spaces far larger than the batch, where repeats are rare and the dedup pass
// costs more than the rows it saves): every request is its own "unique key" --
// the hashed pipeline with an identity slot map (no insert kernel).  pos[b] =
// the request's position in the shard-major uniq[n]; owner_slot has n entries.
FPS_API int fps_route_requests(const int32_t* keys, int64_t n, int W, int part_kind, int64_t block, int32_t* counts,
                               int32_t* prefix, int32_t* owner_slot, int32_t* uniq, int32_t* pos, void* stream) {
  if (n >= (1ll << 31)) return (int)hipErrorInvalidValue;
  return launch_dedup<true>(keys, nullptr, n, nullptr, 0u, W, part_kind, block, counts, prefix, owner_slot, uniq, pos,
                            (hipStream_t)stream);
}

namespace {

// ---- parameter locks (device-mode LockPSLogicA/B, M/server/LockPSLogicA.scala,
// M/server/LockPSLogicB.scala): lock[row] = owner worker or -1.  A request is
// granted when it takes a free lock or already holds it (a worker's duplicate
// requests share its lock, the LockPSLogicB de-duplication).  Launched once
// per source worker segment in rank order, so the lowest rank wins a contended
// row deterministically; denied requests are retried by their worker.
__global__ void lock_acquire_kernel(int32_t* __restrict__ lock, const int32_t* __restrict__ rows, int64_t n,
                                    int32_t src, uint8_t* __restrict__ granted) {
  for (int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; b < n; b += (int64_t)gridDim.x * blockDim.x) {
    const int32_t old = atomicCAS(lock + rows[b], -1, src);
    granted[b] = (old == -1 || old == src) ? 1 : 0;
  }
}

__global__ void lock_release_kernel(int32_t* __restrict__ lock, const int32_t* __restrict__ rows, int64_t n,
                                    const uint8_t* __restrict__ granted) {
  for (int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; b < n; b += (int64_t)gridDim.x * blockDim.x)
    if (granted[b]) lock[rows[b]] = -1;
}

}  // namespace

FPS_API int fps_lock_acquire(int32_t* lock, const int32_t* rows, int64_t n, int32_t src, uint8_t* granted,
                             void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(lock_acquire_kernel, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream, lock, rows, n,
                     src, granted);
  FPS_CHECK_LAUNCH();
  return 0;
}

FPS_API int fps_lock_release(int32_t* lock, const int32_t* rows, int64_t n, const uint8_t* granted, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(lock_release_kernel, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream, lock, rows, n,
                     granted);
  FPS_CHECK_LAUNCH();
  return 0;
}

FPS_API int fps_bucketize(const int32_t* keys, int64_t n, int W, int part_kind, int64_t block, int32_t* shard,
                          int32_t* counts, void* stream) {
  if (n <= 0) return 0;
  const int g = grid_for(n, 256, 256 * 16);
  hipLaunchKernelGGL(bucketize_kernel, dim3(g), dim3(256), 0, (hipStream_t)stream, keys, n, W, part_kind, block, shard,
                     counts);
  FPS_CHECK_LAUNCH();
  return 0;
}

FPS_API int fps_abi_version() { return 1; }

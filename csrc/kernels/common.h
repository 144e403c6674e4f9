// Common device helpers for the gfx950 (MI355X / CDNA4) kernel library.
//
// Wave64 everywhere: a "row group" is TPR consecutive lanes of one wave that
// own one embedding row (TPR = D for D <= 64, one float per lane, so every
// row access is one fully coalesced 4*D-byte transaction and every float
// atomic wave-instruction covers contiguous bytes -- the shape that runs at
// the full ~1.3 TB/s atomic rate, MI355X_MICROARCH.md "Global float atomics").
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#define FPS_API extern "C" __attribute__((visibility("default")))

#define FPS_CHECK_LAUNCH() do { hipError_t e__ = hipGetLastError(); if (e__ != hipSuccess) return (int)e__; } while (0)

namespace fps {

constexpr int kWave = 64;

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// butterfly sum over groups of G lanes (G power of two <= 64)
template <int G>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int G>
__device__ __forceinline__ float group_max(float v) {
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// murmur3 finalizer: counter-based, stateless hash RNG (same function is
// implemented in ops/reference.py for the CPU path / numerics tests).
__device__ __forceinline__ uint32_t fmix32(uint32_t x) {
  x ^= x >> 16; x *= 0x85ebca6bu;
  x ^= x >> 13; x *= 0xc2b2ae35u;
  x ^= x >> 16;
  return x;
}

// uniform in [0,1) from (seed, id, j) -- deterministic per parameter id, so a
// row's init value does not depend on the shard or on the order of first
// touch (RangedRandomFactorInitializer / PseudoRandomFactorInitializer
// semantics, M/matrix/factorization/PseudoRandomFactorInitializer.scala:9-12).
__device__ __forceinline__ float hash_uniform(uint32_t seed, int64_t id, uint32_t j) {
  uint32_t h = fmix32(seed ^ 0x9e3779b9u);
  h = fmix32(h ^ (uint32_t)(id & 0xffffffff));
  h = fmix32(h ^ (uint32_t)((uint64_t)id >> 32) ^ 0x27d4eb2fu);
  h = fmix32(h + j * 0x9e3779b9u);
  return (float)(h >> 8) * (1.0f / 16777216.0f);
}

__device__ __forceinline__ float bf16_to_f32(uint16_t b) {
  return __uint_as_float(((uint32_t)b) << 16);
}

// round-to-nearest-even f32 -> bf16 (NaN kept NaN)
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// no-return float atomic add (global_atomic_add_f32 on gfx950)
__device__ __forceinline__ void atomic_add_noret(float* p, float v) {
  __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// XCD-aware block remap: consecutive logical blocks on one XCD (L2 sharing).
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int nx = 8;
  int q = nwg / nx, r = nwg % nx;
  int x = bid % nx;
  int base = (x < r) ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  return base + bid / nx;
}

inline int grid_for(int64_t work_items, int per_block, int max_blocks = 256 * 16) {
  int64_t g = (work_items + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > max_blocks) g = max_blocks;
  return (int)g;
}

}  // namespace fps

// Passive-Aggressive kernels (gfx950).  K10 (binary), K11 (one-vs-all), K12 (cost-based PB / ML).
//
// A micro-batch of sparse examples in CSR (indptr, per-nnz value, per-nnz
// position ``pos`` into the pulled weight rows of the example's active
// features -- what ``TensorPS.pull`` returns).  One wave per example:
//
//   binary (PassiveAggressiveBinaryAlgorithm.scala:44-65,85-112):
//     m = sum_j x_j w_j ; loss = max(0, 1 - y m) ; tau = PA | PA-I | PA-II
//     delta_j = tau y x_j           -> atomically added to delta[pos_j]
//   one-vs-all (PassiveAggressiveOneVersusAll.scala:40-123), L <= 64 classes
//   on the lanes: d = W^T x ; loss_c = max(0, 1 - d_c y_c) ; tau_c ;
//     delta_{j,c} = x_j tau_c y_c
//   cost-based (PassiveAggressiveCostBased.scala:54-140): q = argmax d (PB) or
//     argmax(d_c - d_y + sqrt(cost[y][c])) (ML); if q != y:
//     tau = (d_q - d_y + sqrt(cost[y][q])) / (2 |x|^2),
//     delta_{j,y} += tau x_j, delta_{j,q} -= tau x_j
//     (each example's deltas independent: the reference's shared builder
//      accumulates across examples).
// Unlabelled examples (label < 0 for multiclass, 0 for binary) only predict.
// wmap (nullable): the delta of pulled row r goes to row wmap[r] of ``delta`` -- at one
// rank the PS push is added straight into the owner's table (the pulled snapshot is
// still what the margins read).
#include "common.h"

using namespace fps;

namespace {

__device__ __forceinline__ float pa_tau(int variant, float loss, float norm_sq, float C) {
  if (variant == 0) return norm_sq > 0.f ? loss / norm_sq : 0.f;                 // PA
  if (variant == 1) return norm_sq > 0.f ? fminf(C, loss / norm_sq) : 0.f;       // PA-I
  return loss / (norm_sq + 1.f / (2.f * C));                                      // PA-II
}

// labels: +1 / -1 train, 0 = predict only.  pred[b] = sign(margin) > 0
__global__ void __launch_bounds__(256) pa_binary_kernel(const int64_t* __restrict__ indptr,
                                                        const float* __restrict__ xval,
                                                        const int32_t* __restrict__ pos,
                                                        const float* __restrict__ w, const int8_t* __restrict__ y,
                                                        int64_t B, int variant, float C, float* __restrict__ delta,
                                                        int8_t* __restrict__ pred, float* __restrict__ loss_out,
                                                        float* __restrict__ flip, const int32_t* __restrict__ wmap) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t b = wave; b < B; b += nw) {
    const int64_t s = indptr[b], e = indptr[b + 1];
    float m = 0.f, n2 = 0.f;
    for (int64_t j = s + lane; j < e; j += 64) {
      const float x = xval[j];
      const float wv = w[pos[j]];
      // in place (flip = the table): a feature's first pull turns its -0.0 "untouched"
      // sentinel into +0.0 (table_ops.hip gather_rows_kernel), no byte-mark pass
      // (a CAS, not a store: another wave may already have added into the fresh row,
      // and a plain +0.0 store would overwrite its update)
      if (flip != nullptr && __float_as_uint(wv) == 0x80000000u)
        atomicCAS(reinterpret_cast<unsigned int*>(flip + pos[j]), 0x80000000u, 0u);
      m = fmaf(x, wv, m);
      n2 = fmaf(x, x, n2);
    }
    m = group_sum<64>(m);
    n2 = group_sum<64>(n2);
    const int label = y[b];
    if (lane == 0 && pred) pred[b] = m > 0.f ? 1 : -1;
    if (label == 0) continue;
    const float loss = fmaxf(0.f, 1.f - (float)label * m);
    if (lane == 0 && loss_out) atomicAdd(loss_out, loss);
    const float mult = pa_tau(variant, loss, n2, C) * (float)label;
    if (mult == 0.f) continue;
    for (int64_t j = s + lane; j < e; j += 64)
      atomic_add_noret(delta + (wmap != nullptr ? wmap[pos[j]] : pos[j]), mult * xval[j]);
  }
}

// mode 0 = OVA (variant PA / PA-I / PA-II), 1 = cost PB, 2 = cost ML.  L <= 64.
// W rows are the pulled [U, L] class-weight vectors of the active features.
__global__ void __launch_bounds__(256) pa_multi_kernel(const int64_t* __restrict__ indptr,
                                                       const float* __restrict__ xval,
                                                       const int32_t* __restrict__ pos, const float* __restrict__ W,
                                                       int L, const int32_t* __restrict__ y, int64_t B, int mode,
                                                       int variant, float C, const float* __restrict__ cost,
                                                       float* __restrict__ delta, int32_t* __restrict__ pred,
                                                       float* __restrict__ loss_out, float* __restrict__ flip,
                                                       const int32_t* __restrict__ wmap) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const bool cl = lane < L;
  for (int64_t b = wave; b < B; b += nw) {
    const int64_t s = indptr[b], e = indptr[b + 1];
    float d = 0.f, n2 = 0.f;
    for (int64_t j = s; j < e; ++j) {  // lanes = classes; row read is L contiguous floats
      const float x = xval[j];
      if (cl) {
        const int64_t o = (int64_t)pos[j] * L + lane;
        const float wv = W[o];
        if (flip != nullptr && __float_as_uint(wv) == 0x80000000u)  // first pull (see binary): CAS, never a store
          atomicCAS(reinterpret_cast<unsigned int*>(flip + o), 0x80000000u, 0u);
        d = fmaf(x, wv, d);
      }
      n2 = fmaf(x, x, n2);
    }
    // argmax over classes (ties -> lowest class, like Breeze argmax)
    float best = cl ? d : -INFINITY;
    int arg = cl ? lane : 0x7fffffff;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ob = __shfl_xor(best, o, 64);
      const int oa = __shfl_xor(arg, o, 64);
      if (ob > best || (ob == best && oa < arg)) { best = ob; arg = oa; }
    }
    if (lane == 0 && pred) pred[b] = arg;
    const int label = y[b];
    if (label < 0) continue;
    if (mode == 0) {
      const float yc = lane == label ? 1.f : -1.f;
      const float loss = cl ? fmaxf(0.f, 1.f - d * yc) : 0.f;
      if (loss_out) { const float ls = group_sum<64>(loss); if (lane == 0) atomicAdd(loss_out, ls); }
      const float mult = cl ? pa_tau(variant, loss, n2, C) * yc : 0.f;
      if (__ballot(mult != 0.f) == 0ull) continue;
      if (cl)
        for (int64_t j = s; j < e; ++j)
          atomic_add_noret(delta + (int64_t)(wmap != nullptr ? wmap[pos[j]] : pos[j]) * L + lane, xval[j] * mult);
    } else {
      const float dy = __shfl(d, label, 64);
      float score = -INFINITY;
      if (cl) score = (mode == 1) ? d : d - dy + sqrtf(cost[label * L + lane]);
      float bs = score;
      int q = cl ? lane : 0x7fffffff;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const float ob = __shfl_xor(bs, o, 64);
        const int oq = __shfl_xor(q, o, 64);
        if (ob > bs || (ob == bs && oq < q)) { bs = ob; q = oq; }
      }
      if (q == label) continue;
      const float dq = __shfl(d, q, 64);
      const float loss = dq - dy + sqrtf(cost[label * L + q]);
      if (lane == 0 && loss_out) atomicAdd(loss_out, loss);
      const float tau = n2 > 0.f ? loss / (2.f * n2) : 0.f;
      for (int64_t j = s + lane; j < e; j += 64) {
        const float v = tau * xval[j];
        const int64_t o = (int64_t)(wmap != nullptr ? wmap[pos[j]] : pos[j]) * L;
        atomic_add_noret(delta + o + label, v);
        atomic_add_noret(delta + o + q, -v);
      }
    }
  }
}

}  // namespace

// flip != nullptr (the in-place path: flip = the table = delta): first pulls turn the
// table's untouched sentinel -0.0 into +0.0 (ShardedTable touch_sentinel).
FPS_API int fps_pa_binary(const int64_t* indptr, const float* xval, const int32_t* pos, const float* w,
                          const int8_t* y, int64_t B, int variant, float C, float* delta, int8_t* pred,
                          float* loss_out, float* flip, const int32_t* wmap, void* stream) {
  if (B <= 0) return 0;
  hipLaunchKernelGGL(pa_binary_kernel, dim3(grid_for(B, 4, 256 * 16)), dim3(256), 0, (hipStream_t)stream, indptr,
                     xval, pos, w, y, B, variant, C, delta, pred, loss_out, flip, wmap);
  FPS_CHECK_LAUNCH();
  return 0;
}

FPS_API int fps_pa_multi(const int64_t* indptr, const float* xval, const int32_t* pos, const float* W, int L,
                         const int32_t* y, int64_t B, int mode, int variant, float C, const float* cost,
                         float* delta, int32_t* pred, float* loss_out, float* flip, const int32_t* wmap,
                         void* stream) {
  if (B <= 0) return 0;
  if (L < 1 || L > 64) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(pa_multi_kernel, dim3(grid_for(B, 4, 256 * 16)), dim3(256), 0, (hipStream_t)stream, indptr,
                     xval, pos, W, L, y, B, mode, variant, C, cost, delta, pred, loss_out, flip, wmap);
  FPS_CHECK_LAUNCH();
  return 0;
}

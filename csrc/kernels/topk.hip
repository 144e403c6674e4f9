// Running top-K merge for the LEMP bucket scan (gfx950).  Kernel K13.
//
// After the MFMA score GEMM of a query batch against one length-sorted item
// bucket (score_gemm.hip), every query row of S[B, n] must be merged into the
// query's running top-k (best_s / best_i, sorted descending).  torch.topk over
// [B, k + n] re-selects from scratch (3.5 ms per 4096 x 65536 bucket,
// profiles/r1_topk_bench.jsonl).  Here one workgroup per query:
//
//   1. tau = current k-th best.  Count the row's scores > tau (after the first
//      bucket nearly none pass: the reference's own pruning argument,
//      M/matrix/factorization/workers/PSTopKGeneratorWorker.scala:35-114).
//   2. If more than max(2k, 128) pass (first bucket), raise the threshold with a
//      radix histogram digit by digit (11 + 11 + 10 bits of the order-preserving
//      float key) to the largest value that still keeps >= k candidates.
//   3. Collect the candidates into LDS, append the running top-k, bitonic-sort
//      (key desc, then item id asc for ties) and keep the first k.
//
// Exact whenever fewer than CAP scores tie with the k-th best (ties beyond that
// are cut at CAP).
#include "common.h"

using namespace fps;

namespace {

constexpr int TK_NT = 256;
constexpr int TK_CAP = 2048;          // collected candidates per query
constexpr int TK_MAXK = 256;          // running top-k capacity
constexpr int TK_SORT = 4096;         // pow2 >= TK_CAP + TK_MAXK
constexpr int TK_BINS = 2048;         // 11-bit radix digits

__device__ __forceinline__ uint32_t fkey(float f) {  // order-preserving float -> uint32
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float kfloat(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

// among hist[0..TK_BINS), find the highest bin b with (#elements in bins >= b) >= need;
// returns b and the count of elements in bins > b via *above.  One wave: lane l
// sums the 32 bins [32*(63-l), 32*(64-l)) (lane 0 the highest), a shuffle scan
// over lanes finds the lane whose range crosses need, and that lane walks its
// 32 bins (the walk of all 2048 bins by one thread took ~85 us per query row)
__device__ int select_bin(const uint32_t* hist, uint32_t need, uint32_t* above, int* bin_out) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const int base = 32 * (63 - lane);
    uint32_t sum = 0;
#pragma unroll 8
    for (int i = 0; i < 32; ++i) sum += hist[base + i];
    uint32_t inc = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(inc, o, 64);
      if (lane >= o) inc += y;
    }
    const uint64_t hit = __ballot(inc >= need);
    const int first = hit ? __ffsll((unsigned long long)hit) - 1 : 63;
    if (lane == first) {
      if (inc >= need) {
        uint32_t run = inc - sum;  // elements in the bins above this lane's range
        int b = base;
        for (int i = 31; i >= 0; --i) {
          if (run + hist[base + i] >= need) { b = base + i; break; }
          run += hist[base + i];
        }
        *bin_out = b;
        *above = run;
      } else {  // fewer than need in total: every bin
        *bin_out = 0;
        *above = inc;
      }
    }
  }
  __syncthreads();
  return *bin_out;
}

// LDS skey/sid[0, nc) hold candidates: append the running top-k (bs, bi), sort
// (key desc, ties: smaller id first) and write back the first k
__device__ void sort_keep_k(uint32_t* skey, int64_t* sid, int nc, float* bs, int64_t* bi, int k) {
  const int tid = threadIdx.x;
  // append the running top-k, pad to a power of two
  int m = nc + k;
  int P = 1;
  while (P < m) P <<= 1;
  for (int i = tid; i < P; i += TK_NT) {
    if (i >= nc && i < m) { skey[i] = fkey(bs[i - nc]); sid[i] = bi[i - nc]; }
    else if (i >= m) { skey[i] = 0u; sid[i] = INT64_MAX; }
  }
  __syncthreads();
  // 4. bitonic sort, descending by key (ties: smaller id first)
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < P; i += TK_NT) {
        const int j = i ^ stride;
        if (j > i) {
          const bool desc = (i & size) == 0;
          const uint32_t ki = skey[i], kj = skey[j];
          const int64_t ii = sid[i], ij = sid[j];
          // "i before j" in the final order: larger key, or equal key and smaller id
          const bool i_first = ki > kj || (ki == kj && ii < ij);
          if (desc != i_first) { skey[i] = kj; skey[j] = ki; sid[i] = ij; sid[j] = ii; }
        }
      }
      __syncthreads();
    }
  }
  for (int i = tid; i < k; i += TK_NT) {
    bs[i] = kfloat(skey[i]);
    bi[i] = skey[i] == 0u ? -1 : sid[i];
  }
}

// REG: the row (n <= TK_NT * TK_REG) is loaded once into registers, every pass below
// reads them -- the streaming passes each waited out 16 dependent global-load round
// trips per thread (the seed segment's 4096 x 4096 merge: 181 us with or without the
// smaller sort)
constexpr int TK_REG = 16;
// the register-row variant sorts at most TK_SORT_R entries (its threshold ends on the
// exact k-th key, so only ties beyond TK_SORT_R - k are cut): 20 KiB of LDS instead of
// 56 KiB, 8 workgroups per CU instead of 2
constexpr int TK_SORT_R = 1024;

template <bool REG>
__global__ void __launch_bounds__(TK_NT) topk_merge_kernel(const float* __restrict__ S, int64_t ldS, int n,
                                                           const int64_t* __restrict__ ids,
                                                           float* __restrict__ best_s, int64_t* __restrict__ best_i,
                                                           int k, const uint8_t* __restrict__ only) {
  if (only != nullptr && only[blockIdx.x] == 0) return;  // fps_topk_select: rows the wave kernel did
  constexpr int SORT = REG ? TK_SORT_R : TK_SORT;
  __shared__ uint32_t hist[TK_BINS];
  __shared__ uint32_t skey[SORT];
  __shared__ int64_t sid[SORT];
  __shared__ uint32_t cnt, above;
  __shared__ int bin_sel;
  const int row = blockIdx.x, tid = threadIdx.x;
  const float* s = S + (int64_t)row * ldS;
  float* bs = best_s + (int64_t)row * k;
  int64_t* bi = best_i + (int64_t)row * k;
  const uint32_t cap = REG ? (uint32_t)(TK_SORT_R - k) : (uint32_t)TK_CAP;  // candidates kept
  uint32_t kr[REG ? TK_REG : 1];
  if constexpr (REG) {
    // all loads in flight at once: unconditional loads of a clamped index, masked after
    // (a guarded load compiled to a branch and a full wait per load: 16 round trips)
    float sv[TK_REG];
#pragma unroll
    for (int q = 0; q < TK_REG; ++q) sv[q] = s[min(tid + q * TK_NT, n - 1)];
#pragma unroll
    for (int q = 0; q < TK_REG; ++q) kr[q] = tid + q * TK_NT < n ? fkey(sv[q]) : 0u;
  }
  // body(j, key) over this thread's entries of the row
  auto for_keys = [&](auto&& body) {
    if constexpr (REG) {
#pragma unroll
      for (int q = 0; q < TK_REG; ++q) {
        const int j = tid + q * TK_NT;
        if (j < n) body(j, kr[q]);
      }
    } else {
      for (int j = tid; j < n; j += TK_NT) body(j, fkey(s[j]));
    }
  };
  const float tau = bs[k - 1];
  const uint32_t ktau = fkey(tau);
  // 1. count candidates strictly above tau (an empty running list: all n pass,
  //    no counting pass needed)
  if (tid == 0) cnt = tau == -INFINITY ? (uint32_t)n : 0u;
  __syncthreads();
  if (tau != -INFINITY) {
    uint32_t c = 0;
    for_keys([&](int, uint32_t kk) { c += kk > ktau; });
    c = (uint32_t)group_sum<64>((float)c);  // exact for counts < 2^24
    if ((tid & 63) == 0) atomicAdd(&cnt, c);
    __syncthreads();
  }
  uint32_t thr = ktau + 1;  // keys >= thr are candidates
  // 2. more candidates than the sort should take (the first bucket / the seed segment:
  //    all n): raise the threshold digit by digit (11 + 11 + 10 bits of the key) until
  //    at most `target` keys pass -- the last digit makes it the exact k-th key, so the
  //    bitonic sort below runs over ~k + k entries instead of up to TK_CAP + k
  const uint32_t target = (uint32_t)max(2 * k, 128);
  if (cnt > target) {
    uint32_t need = (uint32_t)k, above_sum = 0, prefix = 0;
    for (int lvl = 0; lvl < 3; ++lvl) {
      const int sh = lvl == 0 ? 21 : (lvl == 1 ? 10 : 0);  // digit = key bits [sh, sh + 11 or 10)
      const int psh = lvl == 1 ? 21 : 10;                   // the digits above it: key >> psh
      const uint32_t dmask = lvl == 2 ? 1023u : 2047u;
      for (int i = tid; i < TK_BINS; i += TK_NT) hist[i] = 0;
      __syncthreads();
      for_keys([&](int, uint32_t kk) {
        if (kk >= thr && (lvl == 0 || (kk >> psh) == (prefix >> psh))) atomicAdd(&hist[(kk >> sh) & dmask], 1u);
      });
      __syncthreads();
      const int b = select_bin(hist, need, &above, &bin_sel);
      const uint32_t total = above_sum + above + hist[b];
      prefix |= (uint32_t)b << sh;
      thr = prefix > thr ? prefix : thr;
      above_sum += above;
      need = need > above ? need - above : 1u;
      __syncthreads();
      if (total <= target) break;
    }
  }
  // 3. collect candidates (key >= thr), cut at `cap`
  if (tid == 0) cnt = 0;
  __syncthreads();
  for_keys([&](int j, uint32_t kk) {
    if (kk >= thr) {
      const uint32_t slot = atomicAdd(&cnt, 1u);
      if (slot < cap) { skey[slot] = kk; sid[slot] = ids[j]; }
    }
  });
  __syncthreads();
  const int nc = (int)min(cnt, cap);
  sort_keep_k(skey, sid, nc, bs, bi, k);
}

// Candidate lists from the fused scoring (score_gemm.hip: score_filter_kernel):
// query row's cnt[row] candidates are merged into its running top-k.  Two
// kernels split the rows: few candidates (<= TK_NT: every segment after the
// first of a length-sorted scan) merge by rank in a small-LDS kernel, more
// keep the bitonic sort.

// rank merge: each candidate's and each kept entry's final position is the
// number of entries ahead of it (key desc, then id asc; the running list is
// already in that order) -- 4 barriers instead of the sort's ~40, 7 KB of LDS.
// The running entries ahead of a candidate are a prefix of the sorted list
// (binary search, r_c); the candidates ahead of running entry i are those with
// r_c <= i (an LDS histogram of r_c and a wave scan) -- the first version
// walked all k entries per candidate and all candidates per entry (~27 us per
// 4096-row launch, profiles/r2_bf16_topk.md).
// Also flags overflowed rows (cnt > cap: merged incompletely) in ovf.
// NT threads per row (TK_NT / NT candidates and TK_MAXK / NT running entries per
// thread), every load issued before any is used (the guarded loads of the first
// version compiled to a branch and a full wait each: -5 % kernel time on the online
// MF + top-K scan, profiles/r5_merge_rank_nt_ab.txt).  NT = 64 (one wave per row) and
// 128 measured slower or mixed (profiles/r5_merge_rank_wave_ab.txt) -- A/B knob.
#ifndef FPS_MR_NT
#define FPS_MR_NT 256
#endif
template <int NT>
__global__ void __launch_bounds__(NT) topk_merge_rank_kernel(const uint32_t* __restrict__ cand_key,
                                                                const int64_t* __restrict__ cand_id,
                                                                const int32_t* __restrict__ cnt, int cap,
                                                                float* __restrict__ best_s,
                                                                int64_t* __restrict__ best_i, int k,
                                                                int32_t* __restrict__ ovf) {
  static_assert(NT >= 64 && TK_NT % NT == 0 && TK_MAXK % NT == 0, "threads per row");
  constexpr int CPT = TK_NT / NT, EPT = TK_MAXK / NT;
  __shared__ uint32_t ckey[TK_NT];
  __shared__ int64_t cid[TK_NT];
  __shared__ uint32_t bkey[TK_MAXK];
  __shared__ int64_t bid[TK_MAXK];
  __shared__ int32_t hpre[TK_MAXK];
  __shared__ float out_s[TK_MAXK];
  __shared__ int64_t out_i[TK_MAXK];
  const int row = blockIdx.x, tid = threadIdx.x;
  const int c = cnt[row];
  if (ovf != nullptr && c > cap && tid == 0) ovf[0] = 1;
  const int nc = min(min(c, cap), TK_CAP);
  if (nc == 0 || nc > TK_NT) return;  // nothing to merge / the bitonic kernel's row
  float* bs = best_s + (int64_t)row * k;
  int64_t* bi = best_i + (int64_t)row * k;
  uint32_t kq[CPT];
  int64_t iq[CPT];
  float ev[EPT];
  int64_t ei[EPT];
#pragma unroll
  for (int q = 0; q < CPT; ++q) {
    const int64_t j = (int64_t)row * cap + min(tid + NT * q, nc - 1);
    kq[q] = cand_key[j];
    iq[q] = cand_id[j];
  }
#pragma unroll
  for (int q = 0; q < EPT; ++q) {
    const int i = min(tid + NT * q, k - 1);
    ev[q] = bs[i];
    ei[q] = bi[i];
  }
#pragma unroll
  for (int q = 0; q < CPT; ++q)
    if (tid + NT * q < nc) { ckey[tid + NT * q] = kq[q]; cid[tid + NT * q] = iq[q]; }
#pragma unroll
  for (int q = 0; q < EPT; ++q) {
    const int i = tid + NT * q;
    hpre[i] = 0;
    if (i < k) { bkey[i] = fkey(ev[q]); bid[i] = ei[q]; }
  }
  __syncthreads();
  int pos[CPT];
#pragma unroll
  for (int q = 0; q < CPT; ++q) {  // running entries ahead of candidate j (binary search)
    const int j = tid + NT * q;
    int lo = 0, hi = k;
    if (j < nc) {
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        const uint32_t km = bkey[mid];
        if (km > kq[q] || (km == kq[q] && bid[mid] <= iq[q])) lo = mid + 1;
        else hi = mid;
      }
      if (lo < k) atomicAdd(&hpre[lo], 1);  // ahead of running entries lo .. k-1
    }
    pos[q] = lo;
  }
  for (int t = 0; t < nc; ++t) {  // + the candidates ahead of it
    const uint32_t kt = ckey[t];
    const int64_t it = cid[t];
#pragma unroll
    for (int q = 0; q < CPT; ++q)
      pos[q] += kt > kq[q] || (kt == kq[q] && (it < iq[q] || (it == iq[q] && t < tid + NT * q)));
  }
#pragma unroll
  for (int q = 0; q < CPT; ++q)
    if (tid + NT * q < nc && pos[q] < k) { out_s[pos[q]] = kfloat(kq[q]); out_i[pos[q]] = iq[q]; }
  __syncthreads();
  if (tid < 64) {  // inclusive prefix of hpre[0..k): 4 counters per lane + a wave scan
    int32_t c4[4], sum = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = 4 * tid + q;
      c4[q] = i < k ? hpre[i] : 0;
      sum += c4[q];
    }
    int32_t inc = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int32_t y = __shfl_up(inc, o, 64);
      if (tid >= o) inc += y;
    }
    int32_t run = inc - sum;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = 4 * tid + q;
      run += c4[q];
      if (i < k) hpre[i] = run;
    }
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < EPT; ++q) {  // running entry i: its index + the candidates ahead of it
    const int i = tid + NT * q;
    if (i < k) {
      const int p = i + hpre[i];
      if (p < k) { out_s[p] = ev[q]; out_i[p] = ei[q]; }
    }
  }
  __syncthreads();
  for (int i = tid; i < k; i += NT) {
    bs[i] = out_s[i];
    bi[i] = out_i[i];
  }
}

// bitonic merge of the rows with more than TK_NT candidates (<= TK_CAP kept)
// reset (the second of the two kernels, so both read the count first): cnt[row] = 0
// for the next segment's filter -- no fill launch per segment
__global__ void __launch_bounds__(TK_NT) topk_merge_cand_kernel(const uint32_t* __restrict__ cand_key,
                                                                const int64_t* __restrict__ cand_id,
                                                                int32_t* __restrict__ cnt, int cap,
                                                                float* __restrict__ best_s,
                                                                int64_t* __restrict__ best_i, int k, int reset) {
  __shared__ uint32_t skey[TK_SORT];
  __shared__ int64_t sid[TK_SORT];
  const int row = blockIdx.x;
  const int nc = min(min(cnt[row], cap), TK_CAP);
  if (reset) {
    __syncthreads();  // every thread has read cnt[row]
    if (threadIdx.x == 0) cnt[row] = 0;
  }
  if (nc <= TK_NT) return;  // the rank kernel's row
  for (int i = threadIdx.x; i < nc; i += TK_NT) {
    skey[i] = cand_key[(int64_t)row * cap + i];
    sid[i] = cand_id[(int64_t)row * cap + i];
  }
  sort_keep_k(skey, sid, nc, best_s + (int64_t)row * k, best_i + (int64_t)row * k, k);
}


// ---- seen-aware merge of gathered partial top-K lists (CollectTopKFromEachWorker,
// M/matrix/factorization/utils/CollectTopKFromEachWorker.scala:30-59) for the dense
// ring seen store (models/mf/topk_tensor.py SeenStore): one workgroup per batch
// entry.  Entry e of user u is the r-th occurrence of u in the batch; it must not
// recommend the items of u's window as it stands after u's r earlier entries of
// this batch added their rated items (the reference's per-record order).  The
// window is rebuilt in LDS -- the ring row as of the batch start with the r earlier
// items written over its slots (c + j) % M -- so all rounds merge in ONE launch
// (the torch loop over rounds was ~55 small launches per round).  Kept candidates
// (id >= 0, finite score, not in the window) are sorted key desc / id asc (the
// merge kernels' order) and the first K written; rows with fewer than K end in
// -inf / -1.  ring_cur[u] as of the batch start goes to cpre[e] for the update.
__global__ void __launch_bounds__(TK_NT) seen_merge_kernel(
    const float* __restrict__ ss, const int64_t* __restrict__ ii, int m, int K, const int64_t* __restrict__ users,
    const int64_t* __restrict__ items, const int32_t* __restrict__ rnd, const int32_t* __restrict__ first,
    const int64_t* __restrict__ by_user, const int32_t* __restrict__ ring, const int64_t* __restrict__ ring_cur,
    int M, int64_t* __restrict__ cpre, float* __restrict__ best_s, int64_t* __restrict__ best_i) {
  __shared__ int32_t win[TK_MAXK];
  __shared__ uint32_t skey[TK_SORT];
  __shared__ int64_t sid[TK_SORT];
  __shared__ uint32_t cnt;
  const int e = blockIdx.x, tid = threadIdx.x;
  const int64_t u = users[e];
  const int64_t c = ring_cur[u];
  const int r = rnd[e], p0 = first[e];
  if (tid == 0) {
    cnt = 0u;
    cpre[e] = c;
  }
  for (int q = tid; q < M; q += TK_NT) win[q] = ring[u * M + q];
  __syncthreads();
  // the earlier entries' items; only the last M of them survive in the window (distinct slots)
  for (int j = tid; j < r; j += TK_NT)
    if (j >= r - M) win[(int)((c + j) % M)] = (int32_t)items[by_user[p0 + j]];
  __syncthreads();
  if (m <= TK_NT) {
    // one partial list already in the merge order (key desc, then id asc; invalid entries
    // only at its end -- a single shard's sorted top-K): dropping the seen items keeps
    // that order, so a stable compaction replaces the sort (~28 block barriers per row)
    const int t = tid;
    const int64_t id = t < m ? ii[(int64_t)e * m + t] : -1;
    const float sc = t < m ? ss[(int64_t)e * m + t] : -INFINITY;
    const int64_t id1 = t + 1 < m ? ii[(int64_t)e * m + t + 1] : -1;
    const float sc1 = t + 1 < m ? ss[(int64_t)e * m + t + 1] : -INFINITY;
    const bool valid = id >= 0 && isfinite(sc), valid1 = id1 >= 0 && isfinite(sc1);
    const uint32_t k0 = fkey(sc), k1 = fkey(sc1);
    const bool in_order = !valid1 || (valid && (k0 > k1 || (k0 == k1 && id < id1)));
    if (__syncthreads_and(in_order)) {  // uniform
      bool keep = valid;
      if (keep)
        for (int q = 0; q < M; ++q)
          if (win[q] == (int32_t)id) { keep = false; break; }
      __shared__ int32_t wsum[TK_NT / 64];
      const int lane = tid & 63, wv = tid >> 6;
      const uint64_t bal = __ballot(keep);
      if (lane == 0) wsum[wv] = __popcll(bal);
      __syncthreads();
      int pos = __popcll(bal & ((1ull << lane) - 1ull)), total = 0;
#pragma unroll
      for (int w = 0; w < TK_NT / 64; ++w) {
        if (w < wv) pos += wsum[w];
        total += wsum[w];
      }
      if (keep && pos < K) {
        best_s[(int64_t)e * K + pos] = sc;
        best_i[(int64_t)e * K + pos] = id;
      }
      for (int i = total + tid; i < K; i += TK_NT) {
        best_s[(int64_t)e * K + i] = -INFINITY;
        best_i[(int64_t)e * K + i] = -1;
      }
      return;
    }
  }
  for (int t = tid; t < m; t += TK_NT) {
    const int64_t id = ii[(int64_t)e * m + t];
    const float sc = ss[(int64_t)e * m + t];
    bool keep = id >= 0 && isfinite(sc);
    if (keep)
      for (int q = 0; q < M; ++q)
        if (win[q] == (int32_t)id) { keep = false; break; }
    if (keep) {
      const uint32_t slot = atomicAdd(&cnt, 1u);
      skey[slot] = fkey(sc);
      sid[slot] = id;
    }
  }
  __syncthreads();
  const int nc = (int)cnt;
  int P = 1;
  while (P < nc || P < K) P <<= 1;
  for (int i = nc + tid; i < P; i += TK_NT) { skey[i] = 0u; sid[i] = INT64_MAX; }
  __syncthreads();
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < P; i += TK_NT) {
        const int j = i ^ stride;
        if (j > i) {
          const bool desc = (i & size) == 0;
          const uint32_t ki = skey[i], kj = skey[j];
          const int64_t xi = sid[i], xj = sid[j];
          const bool i_first = ki > kj || (ki == kj && xi < xj);
          if (desc != i_first) { skey[i] = kj; skey[j] = ki; sid[i] = xj; sid[j] = xi; }
        }
      }
      __syncthreads();
    }
  }
  for (int i = tid; i < K; i += TK_NT) {
    const uint32_t kk = skey[i];
    best_s[(int64_t)e * K + i] = kk ? kfloat(kk) : -INFINITY;
    best_i[(int64_t)e * K + i] = kk ? sid[i] : -1;
  }
}

// the batch's rated items into the ring, after every merge read it: entry e (round r
// of nu[e] entries of its user) writes slot (c + r) % M if it is among the user's
// last M entries; the user's last entry advances the cursor
__global__ void seen_ring_update_kernel(int B, const int64_t* __restrict__ users, const int64_t* __restrict__ items,
                                        const int32_t* __restrict__ rnd, const int32_t* __restrict__ nu,
                                        const int64_t* __restrict__ cpre, int32_t* __restrict__ ring,
                                        int64_t* __restrict__ ring_cur, int M) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= B) return;
  const int64_t u = users[e];
  const int r = rnd[e], n = nu[e];
  const int64_t c = cpre[e];
  if (r >= n - M) ring[u * M + (int)((c + r) % M)] = (int32_t)items[e];
  if (r == n - 1) ring_cur[u] = c + n;
}


// Occurrence plan of a batch for the one-launch merge: su = users sorted (stable),
// by_user = their entries.  Per entry: its round (0 for a user's first entry in the
// batch ...), the position of its user's first entry in by_user and its user's
// entry count.  One workgroup: each thread takes a contiguous chunk of sorted
// positions; the run start carried into a chunk is an inclusive max-scan of the
// chunks' last run starts, the run end a min-scan from the right.
constexpr int RP_NT = 1024;

__global__ void __launch_bounds__(RP_NT) round_plan_kernel(const int64_t* __restrict__ su,
                                                           const int64_t* __restrict__ by_user, int B,
                                                           int32_t* __restrict__ rnd, int32_t* __restrict__ first,
                                                           int32_t* __restrict__ nu) {
  __shared__ int32_t s_lo[RP_NT], s_hi[RP_NT];
  const int t = threadIdx.x;
  const int C = (B + RP_NT - 1) / RP_NT;
  const int a = min(B, t * C), b = min(B, a + C);
  int32_t last_start = -1, first_end = INT32_MAX;  // in this chunk
  for (int i = a; i < b; ++i)
    if (i == 0 || su[i] != su[i - 1]) last_start = i;
  for (int i = b - 1; i >= a; --i)
    if (i + 1 == B || su[i + 1] != su[i]) first_end = i + 1;  // a run ends after i
  s_lo[t] = last_start;
  s_hi[t] = first_end;
  __syncthreads();
  for (int o = 1; o < RP_NT; o <<= 1) {  // inclusive max-scan (left) and min-scan (right)
    const int32_t lo = t >= o ? s_lo[t - o] : -1;
    const int32_t hi = t + o < RP_NT ? s_hi[t + o] : INT32_MAX;
    __syncthreads();
    s_lo[t] = max(s_lo[t], lo);
    s_hi[t] = min(s_hi[t], hi);
    __syncthreads();
  }
  int32_t start = t > 0 ? s_lo[t - 1] : -1;  // the run start carried into this chunk
  for (int i = a; i < b; ++i) {
    if (i == 0 || su[i] != su[i - 1]) start = i;
    const int64_t e = by_user[i];
    rnd[e] = i - start;
    first[e] = start;
  }
  int32_t end = t + 1 < RP_NT ? s_hi[t + 1] : B;  // the run end carried in from the right
  if (end == INT32_MAX) end = B;
  for (int i = b - 1; i >= a; --i) {
    if (i + 1 == B || su[i + 1] != su[i]) end = i + 1;
    const int64_t e = by_user[i];
    nu[e] = end - first[e];  // first[e] was written by this thread above
  }
}

// ---- fresh top-k of a short row: one wave per query (the seed segment of a scan).
// The block kernel above spent ~100 us on the 4096 x 4096 seed merge (its three radix
// levels and the bitonic sort each cost a dozen block barriers per row).  With an empty
// running list the merge is a plain selection, and a row of <= 4096 scores fits one
// wave's registers: the exact k-th key by three radix levels (11 + 11 + 10 bits) over a
// per-wave LDS histogram, the keys >= it compacted by a wave scan, and a bitonic sort
// of those <= TS_SORT entries (key desc, then id asc -- the block kernel's order).  A row
// whose ties at the k-th key overflow TS_SORT is left to the block kernel (redo[row]).
// waves per SIMD the register allocation must allow: 3 (168 VGPRs, no spills; 197 and
// two waves unconstrained) -- A/B knob
#ifndef FPS_TS_WPE
#define FPS_TS_WPE 3
#endif
constexpr int TS_NPL = 64;    // keys per lane (n <= 64 * TS_NPL = 4096)
constexpr int TS_SORT = 256;  // candidates sorted per row (>= k + ties)

__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(FPS_TS_WPE, 8))) topk_select_wave_kernel(const float* __restrict__ S, int64_t ldS, int n,
                                                              const int64_t* __restrict__ ids,
                                                              float* __restrict__ best_s,
                                                              int64_t* __restrict__ best_i, int k,
                                                              uint8_t* __restrict__ redo) {
  __shared__ __attribute__((aligned(16))) uint32_t hist[TK_BINS];
  __shared__ uint32_t skey[TS_SORT];
  __shared__ int64_t sid[TS_SORT];
  __shared__ uint32_t above;
  __shared__ int bin_sel;
  const int row = blockIdx.x, lane = threadIdx.x;
  const float* s = S + (int64_t)row * ldS;
  uint32_t kr[TS_NPL];
  // all loads in flight (j = lane + 64 q, coalesced): unconditional loads of a clamped
  // index, masked after -- a guarded load compiled to a branch and a full wait per key.
  // The raw bits land in kr itself (a separate float array doubled the live registers)
  const uint32_t* su = reinterpret_cast<const uint32_t*>(s);
#pragma unroll
  for (int q = 0; q < TS_NPL; ++q) kr[q] = su[min(lane + 64 * q, n - 1)];
#pragma unroll
  for (int q = 0; q < TS_NPL; ++q) kr[q] = lane + 64 * q < n ? fkey(__uint_as_float(kr[q])) : 0u;
  // the exact k-th largest key T, digit by digit; need = how many keys == prefix's
  // range are still to take below the digits fixed so far
  uint32_t need = (uint32_t)k, prefix = 0;
  for (int lvl = 0; lvl < 3; ++lvl) {
    const int sh = lvl == 0 ? 21 : (lvl == 1 ? 10 : 0);
    const int psh = lvl == 1 ? 21 : 10;
    const uint32_t dmask = lvl == 2 ? 1023u : 2047u;
    uint4* h4 = reinterpret_cast<uint4*>(hist);
#pragma unroll
    for (int i = lane; i < TK_BINS / 4; i += 64) h4[i] = make_uint4(0, 0, 0, 0);
    __syncthreads();
#pragma unroll
    for (int q = 0; q < TS_NPL; ++q) {
      const uint32_t kk = kr[q];
      if (lvl == 0 || (kk >> psh) == (prefix >> psh)) atomicAdd(&hist[(kk >> sh) & dmask], 1u);
    }
    __syncthreads();
    const int b = select_bin(hist, need, &above, &bin_sel);
    prefix |= (uint32_t)b << sh;
    need -= above;  // keys above bin b (at this level) are in for sure
    __syncthreads();
  }
  const uint32_t T = prefix;  // the k-th largest key; (k - need) keys are > T
  // compact every key >= T (wave scan of the per-lane counts)
  uint32_t c = 0;
#pragma unroll
  for (int q = 0; q < TS_NPL; ++q) c += kr[q] >= T;
  uint32_t inc = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  const uint32_t m = __shfl(inc, 63, 64);
  if (m > (uint32_t)TS_SORT) {  // ties at T beyond the sort: the block kernel redoes this row
    if (lane == 0) redo[row] = 1;
    return;
  }
  uint32_t o = inc - c;
  // positions first (LDS only), the ids after in one coalesced pass: an id load inside
  // the per-key branch serialised ~64 memory round trips per row (93 us per 4096 rows)
  int32_t* spos = reinterpret_cast<int32_t*>(hist);  // the histogram is done
#pragma unroll
  for (int q = 0; q < TS_NPL; ++q) {
    if (kr[q] >= T) {
      skey[o] = kr[q];
      spos[o] = lane + 64 * q;
      ++o;
    }
  }
  int P = 64;
  while (P < (int)m) P <<= 1;
  __syncthreads();
  for (int i = lane; i < P; i += 64) {
    if (i < (int)m) sid[i] = ids[spos[i]];
    else { skey[i] = 0u; sid[i] = INT64_MAX; }
  }
  __syncthreads();
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int p = lane; p < P / 2; p += 64) {  // pair p: (i, i + stride)
        const int i = 2 * stride * (p / stride) + (p % stride), j = i + stride;
        const bool desc = (i & size) == 0;
        const uint32_t ki = skey[i], kj = skey[j];
        const int64_t ii = sid[i], ij = sid[j];
        const bool i_first = ki > kj || (ki == kj && ii < ij);
        if (desc != i_first) { skey[i] = kj; skey[j] = ki; sid[i] = ij; sid[j] = ii; }
      }
      __syncthreads();
    }
  }
  float* bs = best_s + (int64_t)row * k;
  int64_t* bi = best_i + (int64_t)row * k;
  for (int i = lane; i < k; i += 64) {
    bs[i] = kfloat(skey[i]);
    bi[i] = skey[i] == 0u ? -1 : sid[i];
  }
}

}  // namespace

// The top-k of every row of S[B, n] into EMPTY running lists best_s / best_i [B, k]
// (-inf / -1: a fresh scan's first segment): one wave per row (n <= 4096, k <= 128);
// rows whose ties at the k-th key overflow its sort (redo[row] = 1, redo: B zeroed bytes)
// are redone by the block kernel.  Same result as fps_topk_merge on empty lists.
FPS_API int fps_topk_select(const float* S, int64_t ldS, int B, int n, const int64_t* ids, float* best_s,
                            int64_t* best_i, int k, uint8_t* redo, void* stream) {
  if (B <= 0 || n <= 0) return 0;
  if (k <= 0 || k > 128 || n > 64 * TS_NPL || n < k || redo == nullptr) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(topk_select_wave_kernel, dim3(B), dim3(64), 0, st, S, ldS, n, ids, best_s, best_i, k, redo);
  hipLaunchKernelGGL(topk_merge_kernel<true>, dim3(B), dim3(TK_NT), 0, st, S, ldS, n, ids, best_s, best_i, k,
                     (const uint8_t*)redo);
  FPS_CHECK_LAUNCH();
  return 0;
}

// best_s / best_i: [B, k] sorted descending (start: -inf / -1); S: [B, n] with row stride ldS
FPS_API int fps_topk_merge(const float* S, int64_t ldS, int B, int n, const int64_t* ids, float* best_s,
                           int64_t* best_i, int k, void* stream) {
  if (B <= 0 || n <= 0) return 0;
  if (k <= 0 || k > TK_MAXK) return (int)hipErrorInvalidValue;
  if (n <= TK_NT * TK_REG)
    hipLaunchKernelGGL(topk_merge_kernel<true>, dim3(B), dim3(TK_NT), 0, (hipStream_t)stream, S, ldS, n, ids, best_s,
                       best_i, k, (const uint8_t*)nullptr);
  else
    hipLaunchKernelGGL(topk_merge_kernel<false>, dim3(B), dim3(TK_NT), 0, (hipStream_t)stream, S, ldS, n, ids, best_s,
                       best_i, k, (const uint8_t*)nullptr);
  FPS_CHECK_LAUNCH();
  return 0;
}

// candidate lists [B, cap] from fps_score_filter; every cnt[q] must be <= cap (TK_CAP at most)
// ovf (nullable): set to 1 when some cnt[q] > cap (that row's merge is incomplete);
// reset_cnt: cnt[] is zeroed once both kernels read it
FPS_API int fps_topk_merge_cand(const uint32_t* cand_key, const int64_t* cand_id, int32_t* cnt, int cap, int B,
                                float* best_s, int64_t* best_i, int k, int32_t* ovf, int reset_cnt, void* stream) {
  if (B <= 0) return 0;
  if (k <= 0 || k > TK_MAXK || cap <= 0 || cap > TK_CAP) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(topk_merge_rank_kernel<FPS_MR_NT>, dim3(B), dim3(FPS_MR_NT), 0, (hipStream_t)stream, cand_key,
                     cand_id, cnt, cap, best_s, best_i, k, ovf);
  FPS_CHECK_LAUNCH();
  hipLaunchKernelGGL(topk_merge_cand_kernel, dim3(B), dim3(TK_NT), 0, (hipStream_t)stream, cand_key, cand_id, cnt, cap,
                     best_s, best_i, k, reset_cnt);
  FPS_CHECK_LAUNCH();
  return 0;
}

// ss / ii [B, m] gathered partials (m <= TK_CAP), users / items [B] (int64), rnd / first /
// nu [B] int32 (occurrence round, position of the user's first entry in by_user, the
// user's entry count), by_user [B] (entries stably sorted by user), ring [U, M] int32
// (M <= TK_MAXK), ring_cur [U] int64; cpre [B] int64 scratch.  best_s / best_i [B, K].
FPS_API int fps_topk_seen_merge(const float* ss, const int64_t* ii, int B, int m, int K, const int64_t* users,
                                const int64_t* items, const int32_t* rnd, const int32_t* first, const int32_t* nu,
                                const int64_t* by_user, int32_t* ring, int64_t* ring_cur, int M, int64_t* cpre,
                                float* best_s, int64_t* best_i, void* stream) {
  if (B <= 0) return 0;
  if (K <= 0 || K > TK_MAXK || m < 0 || m > TK_CAP || M <= 0 || M > TK_MAXK) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(seen_merge_kernel, dim3(B), dim3(TK_NT), 0, s, ss, ii, m, K, users, items, rnd, first, by_user,
                     (const int32_t*)ring, (const int64_t*)ring_cur, M, cpre, best_s, best_i);
  FPS_CHECK_LAUNCH();
  hipLaunchKernelGGL(seen_ring_update_kernel, dim3((B + 255) / 256), dim3(256), 0, s, B, users, items, rnd, nu,
                     (const int64_t*)cpre, ring, ring_cur, M);
  FPS_CHECK_LAUNCH();
  return 0;
}

// su / by_user [B]: users sorted (stable) and their entries -> rnd / first / nu [B] int32
// (round_plan_kernel); B <= 1M (one workgroup)
FPS_API int fps_round_plan(const int64_t* su, const int64_t* by_user, int B, int32_t* rnd, int32_t* first,
                           int32_t* nu, void* stream) {
  if (B <= 0) return 0;
  if (B > (1 << 20)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(round_plan_kernel, dim3(1), dim3(RP_NT), 0, (hipStream_t)stream, su, by_user, B, rnd, first, nu);
  FPS_CHECK_LAUNCH();
  return 0;
}

// ---- the per-scan set-up of a fused LEMP scan in ONE launch (topk_fast.LempTopK._scan):
// |q| per query row, the bf16 copy of Q the filter reads (RNE), the running lists reset
// (-inf / -1), the candidate counts and the overflow flag zeroed.  Replaces eight small
// launches inside the scan's graph (square / sum / sqrt, bf16 cast, two fills, two zero
// fills: ~40 us of a 0.6 ms LEMP batch, profiles/r6_mf_topk_batch_timeline.md).  One
// wave per query row; the norm's summation order differs from torch's, which the
// bounds allow (they carry a relative slack).
namespace {
__global__ void __launch_bounds__(256) topk_scan_prep_kernel(const float* __restrict__ Q, int B, int D, int k,
                                                             float* __restrict__ qlen, uint16_t* __restrict__ Qb,
                                                             float* __restrict__ best_s, int64_t* __restrict__ best_i,
                                                             int32_t* __restrict__ cnt, int32_t* __restrict__ ovf) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row == 0 && lane == 0 && ovf != nullptr) ovf[0] = 0;
  if (row >= B) return;
  const float* q = Q + (int64_t)row * D;
  float ss = 0.f;
  for (int d = lane; d < D; d += 64) {
    const float v = q[d];
    ss += v * v;
    if (Qb != nullptr) Qb[(int64_t)row * D + d] = f32_to_bf16(v);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
  if (lane == 0) {
    qlen[row] = sqrtf(ss);
    if (cnt != nullptr) cnt[row] = 0;
  }
  for (int i = lane; i < k; i += 64) {
    best_s[(int64_t)row * k + i] = -INFINITY;
    best_i[(int64_t)row * k + i] = -1;
  }
}
}  // namespace

FPS_API int fps_topk_scan_prep(const float* Q, int B, int D, int k, float* qlen, uint16_t* Qb, float* best_s,
                               int64_t* best_i, int32_t* cnt, int32_t* ovf, void* stream) {
  if (B <= 0) return 0;
  if (D <= 0 || k <= 0 || qlen == nullptr || best_s == nullptr || best_i == nullptr) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(topk_scan_prep_kernel, dim3((B + 3) / 4), dim3(256), 0, (hipStream_t)stream, Q, B, D, k, qlen, Qb,
                     best_s, best_i, cnt, ovf);
  FPS_CHECK_LAUNCH();
  return 0;
}

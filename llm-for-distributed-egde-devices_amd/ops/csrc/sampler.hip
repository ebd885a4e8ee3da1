// Fused token sampler — one 1024-thread workgroup per row, one launch per step.
//
// Semantics = HF generate(do_sample=True) processor order used by the reference
// (combine_model_fp_updated.py:95-105): repetition penalty on already-seen ids (divide positive,
// multiply negative scores) -> temperature -> top-k (keep scores >= k-th largest) -> top-p
// (drop the ascending-sorted prefix with cumulative prob <= 1 - p, always keep the best) ->
// sample.  Sampling is Gumbel-max with counter-based noise u(seed, row, step, token) — exact
// sampling from the processed softmax, deterministic and bit-reproducible against
// ops/_ref.py::sample.  HF launches ~10 kernels per token for this; here it is one.
//
// top-k threshold: 4-pass MSB radix select on order-preserving u32 keys with per-wave LDS
// histograms (no global sort).  Candidates (>= threshold, <= CAP) are compacted to LDS,
// bitonic-sorted, softmax-scanned for top-p, then Gumbel-argmaxed.
// The step counter is read from device memory (rng[1]) so the launch can live in a HIP graph.
#include "common.h"

namespace {
constexpr int NT = 1024;
constexpr int NW = NT / 64;
constexpr int CAP = 1024;

__device__ __forceinline__ uint32_t f2key(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

template <bool BF16>
__device__ __forceinline__ float load_logit(const void* lg, size_t i) {
  if constexpr (BF16) return bf2f(reinterpret_cast<const bf16_t*>(lg)[i]);
  else return reinterpret_cast<const float*>(lg)[i];
}

template <bool BF16>
__device__ __forceinline__ float proc(const void* lg, const uint8_t* seen, size_t base, int i, float inv_t, float pen) {
  float s = load_logit<BF16>(lg, base + i);
  if (seen != nullptr && seen[base + i]) s = s < 0.f ? s * pen : s / pen;
  return s * inv_t;
}

// argmax with lowest-index tie break, block-wide (NT threads)
__device__ __forceinline__ void block_argmax(float& v, int& idx, float* rv, int* ri) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(v, o, 64);
    const int oi = __shfl_xor(idx, o, 64);
    if (ov > v || (ov == v && oi < idx)) { v = ov; idx = oi; }
  }
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) { rv[w] = v; ri[w] = idx; }
  __syncthreads();
  if (threadIdx.x < 64) {
    v = threadIdx.x < NW ? rv[threadIdx.x] : -INFINITY;
    idx = threadIdx.x < NW ? ri[threadIdx.x] : 0x7fffffff;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(v, o, 64);
      const int oi = __shfl_xor(idx, o, 64);
      if (ov > v || (ov == v && oi < idx)) { v = ov; idx = oi; }
    }
    if (threadIdx.x == 0) { rv[0] = v; ri[0] = idx; }
  }
  __syncthreads();
  v = rv[0];
  idx = ri[0];
  __syncthreads();
}

// Block-wide reduction of a u32 (OP 0 = min, 1 = max, 2 = sum); `scratch` holds >= NW words.
template <int OP>
__device__ __forceinline__ uint32_t block_reduce_u32(uint32_t v, uint32_t* scratch) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t w = (uint32_t)__shfl_xor((int)v, o, 64);
    v = OP == 0 ? min(v, w) : (OP == 1 ? max(v, w) : v + w);
  }
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) scratch[wv] = v;
  __syncthreads();
  uint32_t r = scratch[0];
#pragma unroll
  for (int i = 1; i < NW; ++i) {
    const uint32_t w = scratch[i];
    r = OP == 0 ? min(r, w) : (OP == 1 ? max(r, w) : r + w);
  }
  return r;
}

__device__ __forceinline__ float gumbel(uint32_t seed, uint32_t row, uint32_t step, uint32_t idx) {
  const float u = uniform_hash(seed, row, step, idx);
  return -logf(-logf(u));
}

// MODE 0: greedy argmax of penalised logits; 1: Gumbel over full vocab; 2: top-k (+ top-p)
template <bool BF16, int MODE>
__global__ void __launch_bounds__(NT) sample_kernel(const void* __restrict__ logits, uint8_t* __restrict__ seen, int V,
                                                    float inv_t, float pen, int top_k, float top_p,
                                                    const int* __restrict__ rng, int64_t* __restrict__ out_tok) {
  __shared__ float rv[NW];
  __shared__ int ri[NW];
  __shared__ uint32_t hist[NW][256];
  __shared__ float cv[CAP];
  __shared__ int ci[CAP];
  __shared__ float pref[CAP];
  __shared__ int ncand, sel_bin, k_rem;

  const int row = blockIdx.x;
  const size_t base = (size_t)row * V;
  const uint32_t seed = (uint32_t)rng[0], step = (uint32_t)rng[1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float bv = -INFINITY;
  int bi = 0x7fffffff;

  if constexpr (MODE == 0 || MODE == 1) {
    for (int i = tid; i < V; i += NT) {
      float s = proc<BF16>(logits, seen, base, i, MODE == 0 ? 1.f : inv_t, pen);
      if constexpr (MODE == 1) s += gumbel(seed, row, step, i);
      if (s > bv || (s == bv && i < bi)) { bv = s; bi = i; }
    }
    block_argmax(bv, bi, rv, ri);
  } else {
    // ---- candidate threshold by bisection on order-preserving u32 keys: find thr with
    // k <= count(key >= thr) <= CAP using block-wide count reductions only (no LDS atomics:
    // logit keys cluster in a few radix bins, which serialised the old histogram select).
    // Keys of up to PT elements per thread stay in registers; larger vocabularies re-read L2.
    constexpr int PT = 48;
    uint32_t kr[PT];
    uint32_t kmin = 0xffffffffu, kmax = 0u;
#pragma unroll
    for (int j = 0; j < PT; ++j) {
      const int i = tid + j * NT;
      kr[j] = (i < V) ? f2key(proc<BF16>(logits, seen, base, i, inv_t, pen)) : 0u;
      if (i < V) { kmin = min(kmin, kr[j]); kmax = max(kmax, kr[j]); }
    }
    for (int i = tid + PT * NT; i < V; i += NT) {
      const uint32_t k = f2key(proc<BF16>(logits, seen, base, i, inv_t, pen));
      kmin = min(kmin, k);
      kmax = max(kmax, k);
    }
    kmin = block_reduce_u32<0>(kmin, &hist[0][0]);
    kmax = block_reduce_u32<1>(kmax, &hist[0][0]);
    uint32_t lo = kmin, hi = kmax;   // invariant: count(>= lo) >= k ; count(>= hi + 1) < k or hi = max
    uint32_t thr = lo;
    for (int it = 0; it < 40 && lo < hi; ++it) {
      const uint32_t mid = lo + (uint32_t)(((uint64_t)hi - lo + 1) >> 1);
      int c = 0;
#pragma unroll
      for (int j = 0; j < PT; ++j) c += (tid + j * NT < V && kr[j] >= mid) ? 1 : 0;
      for (int i = tid + PT * NT; i < V; i += NT) c += f2key(proc<BF16>(logits, seen, base, i, inv_t, pen)) >= mid;
      c = (int)block_reduce_u32<2>((uint32_t)c, &hist[0][0]);
      if (c >= top_k) {
        lo = mid;
        if (c <= CAP) break;
      } else {
        hi = mid - 1;
      }
    }
    thr = lo;
    // ---- compact candidates (key >= thr)
    if (tid == 0) ncand = 0;
    __syncthreads();
    for (int i = tid; i < V; i += NT) {
      const float s = proc<BF16>(logits, seen, base, i, inv_t, pen);
      if (f2key(s) >= thr) {
        const int slot = atomicAdd(&ncand, 1);
        if (slot < CAP) { cv[slot] = s; ci[slot] = i; }
      }
    }
    __syncthreads();
    const int n = min(ncand, CAP);
    int P = 1;
    while (P < n) P <<= 1;
    for (int i = n + tid; i < P; i += NT) { cv[i] = -INFINITY; ci[i] = 0x7fffffff; }
    __syncthreads();
    // ---- bitonic sort, descending by value, ascending index on ties
    for (int k = 2; k <= P; k <<= 1) {
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int i = tid; i < P; i += NT) {
          const int p = i ^ j;
          if (p > i) {
            const bool desc = (i & k) == 0;
            const float a = cv[i], b = cv[p];
            const int ia = ci[i], ib = ci[p];
            const bool a_first = (a > b) || (a == b && ia < ib);
            if (desc ? !a_first : a_first) { cv[i] = b; cv[p] = a; ci[i] = ib; ci[p] = ia; }
          }
        }
        __syncthreads();
      }
    }
    // ---- exact top-k cut: keep every candidate >= the k-th largest value (ties kept, as HF)
    __shared__ int nkeep_s;
    if (tid == 0) {
      int nk = min(top_k, n);
      const float kth = cv[nk - 1];
      while (nk < n && cv[nk] >= kth) ++nk;
      nkeep_s = nk;
    }
    __syncthreads();
    const int nk = nkeep_s;
    // ---- top-p: exclusive prefix of softmax mass in descending order
    const float m = cv[0];
    for (int i = tid; i < P; i += NT) pref[i] = (i < nk) ? __expf(cv[i] - m) : 0.f;
    __syncthreads();
    // Hillis-Steele inclusive scan over P <= 1024 entries
    for (int off = 1; off < P; off <<= 1) {
      float t = 0.f;
      if (tid < P && tid >= off) t = pref[tid - off];
      __syncthreads();
      if (tid < P && tid >= off) pref[tid] += t;
      __syncthreads();
    }
    const float total = pref[nk - 1];
    // ---- Gumbel-argmax over kept candidates
    if (tid < nk) {
      const float excl = (tid == 0) ? 0.f : pref[tid - 1];
      const bool keep = (tid == 0) || (top_p >= 1.f) || (excl / total < top_p);
      if (keep) {
        bv = cv[tid] + gumbel(seed, row, step, ci[tid]);
        bi = ci[tid];
      }
    }
    block_argmax(bv, bi, rv, ri);
  }
  if (tid == 0) {
    out_tok[row] = bi;
    if (seen != nullptr) seen[base + bi] = 1;
  }
}
}  // namespace

// mode: 0 greedy, 1 full-vocab sampling, 2 top-k(+top-p). Returns -5 when the configuration
// needs the host fallback (top-p without top-k, or top-k beyond CAP).
extern "C" int edge_sample(const void* logits, int is_bf16, uint8_t* seen, int B, int V, float temperature,
                           float inv_temperature, float penalty, int top_k, float top_p, int do_sample, const int* rng, int64_t* out_tok,
                           hipStream_t st) {
  if (B == 0) return 0;
  int mode;
  if (!do_sample || temperature <= 0.f) mode = 0;
  else if ((top_k <= 0 || top_k >= V) && top_p >= 1.f) mode = 1;
  else if (top_k > 0 && top_k <= CAP && top_k < V) mode = 2;
  else return -5;
  const float inv_t = (mode == 0) ? 1.f : inv_temperature;  // host computes 1/T in f64 (matches _ref)
#define SL(BF, MD) hipLaunchKernelGGL((sample_kernel<BF, MD>), dim3(B), dim3(NT), 0, st, logits, seen, V, inv_t, penalty, \
                                      top_k, top_p, rng, out_tok)
  if (is_bf16) { if (mode == 0) SL(true, 0); else if (mode == 1) SL(true, 1); else SL(true, 2); }
  else { if (mode == 0) SL(false, 0); else if (mode == 1) SL(false, 1); else SL(false, 2); }
#undef SL
  return (int)hipGetLastError();
}

// Fused token sampler — one workgroup per row, one launch per step.
//
// Semantics = HF generate(do_sample=True) processor order used by the reference
// (combine_model_fp_updated.py:95-105): repetition penalty on already-seen ids (divide positive,
// multiply negative scores) -> temperature -> top-k (keep scores >= k-th largest) -> top-p
// (drop the ascending-sorted prefix with cumulative prob <= 1 - p, always keep the best) ->
// sample.  Sampling is Gumbel-max with counter-based noise u(seed, row, step, token) — exact
// sampling from the processed softmax, deterministic and bit-reproducible against
// ops/_ref.py::sample.  HF launches ~10 kernels per token for this; here it is one.
//
// top-k / top-p (MODE 2, 256 threads): the processed scores' order-preserving u32 keys stay in
// registers; a bisection on the key space with block-wide count reductions (no atomics — logit
// keys cluster in a few radix bins) finds a threshold with k <= count <= TARGET; the candidates
// are compacted to LDS and every thread ranks its candidate against all others (O(n^2) reads of
// broadcast LDS words, no sort stages / barriers), which gives the exact k-th value, the
// descending-order softmax prefix for top-p and the Gumbel-max winner.
// The step counter is read from device memory (rng[1]) so the launch can live in a HIP graph.
#include "common.h"

namespace {
constexpr int CAP = 1024;     // max candidates kept (ties beyond are truncated)
constexpr int TARGET = 128;   // bisection stops once k <= count <= max(TARGET, k)

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

template <int NT>
__device__ __forceinline__ void block_argmax(float& v, int& idx, float* rv, int* ri) {
  constexpr int NW = NT / 64;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(v, o, 64);
    const int oi = __shfl_xor(idx, o, 64);
    if (ov > v || (ov == v && oi < idx)) { v = ov; idx = oi; }
  }
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) { rv[w] = v; ri[w] = idx; }
  __syncthreads();
  v = rv[0];
  idx = ri[0];
#pragma unroll
  for (int i = 1; i < NW; ++i)
    if (rv[i] > v || (rv[i] == v && ri[i] < idx)) { v = rv[i]; idx = ri[i]; }
}

// Block-wide reduction of a u32 (OP 0 = min, 1 = max, 2 = sum); `scratch` holds >= NT/64 words.
template <int NT, int OP>
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
  for (int i = 1; i < NT / 64; ++i) {
    const uint32_t w = scratch[i];
    r = OP == 0 ? min(r, w) : (OP == 1 ? max(r, w) : r + w);
  }
  return r;
}

__device__ __forceinline__ float gumbel(uint32_t seed, uint32_t row, uint32_t step, uint32_t idx) {
  const float u = uniform_hash(seed, row, step, idx);
  return -logf(-logf(u));
}

// ---------------------------------------------------------------- greedy / full-vocab sampling
template <bool BF16, int MODE>
__global__ void __launch_bounds__(1024) sample_argmax_kernel(const void* __restrict__ logits, uint8_t* __restrict__ seen,
                                                             int V, float inv_t, float pen,
                                                             const int* __restrict__ rng, int64_t* __restrict__ out_tok) {
  constexpr int NT = 1024;
  __shared__ float rv[NT / 64];
  __shared__ int ri[NT / 64];
  const int row = blockIdx.x;
  const size_t base = (size_t)row * V;
  const uint32_t seed = (uint32_t)rng[0], step = (uint32_t)rng[1];
  float bv = -INFINITY;
  int bi = 0x7fffffff;
  for (int i = threadIdx.x; i < V; i += NT) {
    float s = proc<BF16>(logits, seen, base, i, MODE == 0 ? 1.f : inv_t, pen);
    if constexpr (MODE == 1) s += gumbel(seed, row, step, i);
    if (s > bv || (s == bv && i < bi)) { bv = s; bi = i; }
  }
  block_argmax<NT>(bv, bi, rv, ri);
  if (threadIdx.x == 0) {
    out_tok[row] = bi;
    if (seen != nullptr) seen[base + bi] = 1;
  }
}

// ---------------------------------------------------------------- top-k (+ top-p)
template <bool BF16, int PT>
__global__ void __launch_bounds__(256) sample_topk_kernel(const void* __restrict__ logits, uint8_t* __restrict__ seen,
                                                          int V, float inv_t, float pen, int top_k, float top_p,
                                                          const int* __restrict__ rng, int64_t* __restrict__ out_tok) {
  constexpr int NT = 256;
  __shared__ uint32_t scratch[NT / 64];
  __shared__ float rv[NT / 64];
  __shared__ int ri[NT / 64];
  __shared__ float cv[CAP];
  __shared__ int ci[CAP];
  __shared__ int ncand;
  __shared__ float kth_s;
  __shared__ float tot_s[NT / 64];
  const int row = blockIdx.x;
  const size_t base = (size_t)row * V;
  const uint32_t seed = (uint32_t)rng[0], step = (uint32_t)rng[1];
  const int tid = threadIdx.x;

  // keys in registers (elements beyond PT*NT are re-read from L2 each pass)
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
  kmin = block_reduce_u32<NT, 0>(kmin, scratch);
  kmax = block_reduce_u32<NT, 1>(kmax, scratch);
  const int target = max(TARGET, top_k);
  // bisection: invariant count(key >= lo) >= top_k
  uint32_t lo = kmin, hi = kmax;
  for (int it = 0; it < 40 && lo < hi; ++it) {
    const uint32_t mid = lo + (uint32_t)(((uint64_t)hi - lo + 1) >> 1);
    int c = 0;
#pragma unroll
    for (int j = 0; j < PT; ++j) c += (tid + j * NT < V && kr[j] >= mid) ? 1 : 0;
    for (int i = tid + PT * NT; i < V; i += NT) c += f2key(proc<BF16>(logits, seen, base, i, inv_t, pen)) >= mid;
    c = (int)block_reduce_u32<NT, 2>((uint32_t)c, scratch);
    if (c >= top_k) {
      lo = mid;
      if (c <= target) break;
    } else {
      hi = mid - 1;
    }
  }
  const uint32_t thr = lo;
  // compact candidates (key >= thr) into LDS
  if (tid == 0) ncand = 0;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < PT; ++j) {
    const int i = tid + j * NT;
    if (i < V && kr[j] >= thr) {
      const int slot = atomicAdd(&ncand, 1);
      if (slot < CAP) { cv[slot] = proc<BF16>(logits, seen, base, i, inv_t, pen); ci[slot] = i; }
    }
  }
  for (int i = tid + PT * NT; i < V; i += NT) {
    const float s = proc<BF16>(logits, seen, base, i, inv_t, pen);
    if (f2key(s) >= thr) {
      const int slot = atomicAdd(&ncand, 1);
      if (slot < CAP) { cv[slot] = s; ci[slot] = i; }
    }
  }
  __syncthreads();
  const int n = min(ncand, CAP);
  // rank every candidate: descending value, ascending token id on ties
  constexpr int PER = (CAP + NT - 1) / NT;
  int rank[PER];
  float myv[PER];
  int myi[PER];
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int c = tid + q * NT;
    rank[q] = 0x7fffffff;
    if (c < n) {
      const float v = cv[c];
      const int id = ci[c];
      int r = 0;
      for (int j = 0; j < n; ++j) {
        const float w = cv[j];
        r += (w > v || (w == v && ci[j] < id)) ? 1 : 0;
      }
      rank[q] = r;
      myv[q] = v;
      myi[q] = id;
    }
  }
  const int kk = min(top_k, n);
#pragma unroll
  for (int q = 0; q < PER; ++q)
    if (rank[q] == kk - 1) kth_s = myv[q];
  if (tid == 0 && n > 0 && kk == 0) kth_s = -INFINITY;
  __syncthreads();
  const float kth = kth_s;
  float vmax = -INFINITY;                               // value of rank 0
  for (int j = 0; j < n; ++j) vmax = fmaxf(vmax, cv[j]);
  // softmax mass of the top-k survivors and each one's exclusive prefix in descending order
  float tot = 0.f;
#pragma unroll
  for (int q = 0; q < PER; ++q)
    if (rank[q] != 0x7fffffff && myv[q] >= kth) tot += __expf(myv[q] - vmax);
  {
    float t = tot;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
    if ((tid & 63) == 0) tot_s[tid >> 6] = t;
    __syncthreads();
    tot = 0.f;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) tot += tot_s[i];
  }
  float bv = -INFINITY;
  int bi = 0x7fffffff;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    if (rank[q] == 0x7fffffff || myv[q] < kth) continue;
    bool keep = rank[q] == 0 || top_p >= 1.f;
    if (!keep) {
      float excl = 0.f;
      const float v = myv[q];
      const int id = myi[q];
      for (int j = 0; j < n; ++j) {
        const float w = cv[j];
        if (w >= kth && (w > v || (w == v && ci[j] < id))) excl += __expf(w - vmax);
      }
      keep = excl / tot < top_p;
    }
    if (keep) {
      const float g = myv[q] + gumbel(seed, row, step, myi[q]);
      if (g > bv || (g == bv && myi[q] < bi)) { bv = g; bi = myi[q]; }
    }
  }
  block_argmax<NT>(bv, bi, rv, ri);
  if (tid == 0) {
    out_tok[row] = bi;
    if (seen != nullptr) seen[base + bi] = 1;
  }
}
}  // namespace

// mode: 0 greedy, 1 full-vocab sampling, 2 top-k(+top-p). Returns -5 when the configuration
// needs the host fallback (top-p without top-k, or top-k beyond CAP).
extern "C" int edge_sample(const void* logits, int is_bf16, uint8_t* seen, int B, int V, float temperature,
                           float inv_temperature, float penalty, int top_k, float top_p, int do_sample, const int* rng,
                           int64_t* out_tok, hipStream_t st) {
  if (B == 0) return 0;
  int mode;
  if (!do_sample || temperature <= 0.f) mode = 0;
  else if ((top_k <= 0 || top_k >= V) && top_p >= 1.f) mode = 1;
  else if (top_k > 0 && top_k <= CAP && top_k < V) mode = 2;
  else return -5;
  const float inv_t = (mode == 0) ? 1.f : inv_temperature;  // host computes 1/T in f64 (matches _ref)
  if (mode == 2) {
#define TK(BF, PTV) hipLaunchKernelGGL((sample_topk_kernel<BF, PTV>), dim3(B), dim3(256), 0, st, logits, seen, V, inv_t, \
                                       penalty, top_k, top_p, rng, out_tok)
    if (is_bf16) { if (V <= 256 * 64) TK(true, 64); else TK(true, 128); }
    else { if (V <= 256 * 64) TK(false, 64); else TK(false, 128); }
#undef TK
  } else {
#define SL(BF, MD) hipLaunchKernelGGL((sample_argmax_kernel<BF, MD>), dim3(B), dim3(1024), 0, st, logits, seen, V, inv_t, \
                                      penalty, rng, out_tok)
    if (is_bf16) { if (mode == 0) SL(true, 0); else SL(true, 1); }
    else { if (mode == 0) SL(false, 0); else SL(false, 1); }
#undef SL
  }
  return (int)hipGetLastError();
}

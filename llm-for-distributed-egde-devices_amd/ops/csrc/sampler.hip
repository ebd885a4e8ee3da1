// Fused token sampler — two short launches per step, whole chip busy.
//
// Semantics = HF generate(do_sample=True) processor order used by the reference
// (combine_model_fp_updated.py:95-105): repetition penalty on already-seen ids (divide positive,
// multiply negative scores) -> temperature -> top-k (keep scores >= k-th largest) -> top-p
// (drop the ascending-sorted prefix with cumulative prob <= 1 - p, always keep the best) ->
// sample.  Sampling is Gumbel-max with counter-based noise u(seed, row, step, token) — exact
// sampling from the processed softmax, deterministic and bit-reproducible against
// ops/_ref.py::sample.  HF launches ~10 kernels per token for this; here it is two.
//
// Split-row design: a decode batch has only B rows (16..64), so one workgroup per row leaves
// >90% of the 256 CUs idle and serialises ~V/256 elements per thread.  Phase 1 cuts every row
// into CH-element chunks (grid C x B, 4 elements per thread in registers):
//   * greedy / full-vocab sampling: per-chunk argmax of the (noised) processed scores;
//   * top-k: the chunk's exact top-k set (all scores >= the chunk's k-th value, ties kept up
//     to CCAP) by bisection on order-preserving u32 keys; counts are wave ballots + one LDS
//     word per wave (parity double-buffered: one barrier per bisection step).
// The union of chunk top-k sets contains the row's top-k, and the row's k-th value is >= the
// largest chunk threshold T0, so phase 2 (one WG per row) keeps only candidates >= T0, bisects
// once more down to <= FCAP, ranks each survivor against the others in LDS (exact k-th cut,
// descending softmax prefix for top-p) and takes the Gumbel-max winner.
// The step counter is read from device memory (rng[1]) so both launches live in a HIP graph.
#include "common.h"

namespace {
constexpr int NT = 256, NW = NT / 64;
constexpr int CH = 1024;      // phase-1 chunk (EPT = 4 scores per thread)
constexpr int EPT = CH / NT;
constexpr int CCAP = 128;     // candidates kept per chunk; the split path needs top_k <= CCAP
constexpr int MCAP = 2048;    // phase-2 candidates >= T0 (ties beyond are truncated)
constexpr int FCAP = 256;     // candidates ranked exactly
constexpr int CAP = 1024;     // single-workgroup fallback for CCAP < top_k <= CAP

__device__ __forceinline__ uint32_t f2key(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

template <bool BF16>
__device__ __forceinline__ float proc(const void* lg, const uint8_t* seen, size_t base, int i, float inv_t, float pen) {
  float s;
  if constexpr (BF16) s = bf2f(reinterpret_cast<const bf16_t*>(lg)[base + i]);
  else s = reinterpret_cast<const float*>(lg)[base + i];
  if (seen != nullptr && seen[base + i]) s = s < 0.f ? s * pen : s / pen;
  return s * inv_t;
}

__device__ __forceinline__ bool better(float v, int i, float bv, int bi) { return v > bv || (v == bv && i < bi); }

__device__ __forceinline__ void wave_argmax(float& v, int& idx) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(v, o, 64);
    const int oi = __shfl_xor(idx, o, 64);
    if (better(ov, oi, v, idx)) { v = ov; idx = oi; }
  }
}

__device__ __forceinline__ void block_argmax(float& v, int& idx, float* rv, int* ri) {
  wave_argmax(v, idx);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) { rv[w] = v; ri[w] = idx; }
  __syncthreads();
  v = rv[0];
  idx = ri[0];
#pragma unroll
  for (int i = 1; i < NW; ++i)
    if (better(rv[i], ri[i], v, idx)) { v = rv[i]; idx = ri[i]; }
}

// OP 0 = min, 1 = max, 2 = sum over the block; `scratch` holds >= NW words.
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

// Block sum of a wave-uniform count with one barrier: `scr` is [2][NW], alternated by `parity`.
__device__ __forceinline__ int block_count(int wave_cnt, int* scr, int& parity) {
  if ((threadIdx.x & 63) == 0) scr[parity * NW + (threadIdx.x >> 6)] = wave_cnt;
  __syncthreads();
  int s = 0;
#pragma unroll
  for (int i = 0; i < NW; ++i) s += scr[parity * NW + i];
  parity ^= 1;
  return s;
}

__device__ __forceinline__ int ballot_count(bool p) { return __popcll(__ballot(p)); }

__device__ __forceinline__ float gumbel(uint32_t seed, uint32_t row, uint32_t step, uint32_t idx) {
  const float u = uniform_hash(seed, row, step, idx);
  return -logf(-logf(u));
}

// Exact top-k (ties at the k-th value kept) -> top-p -> Gumbel-max over n <= PER*NT candidates
// held in LDS.  Every thread ranks its candidates against all others (broadcast LDS reads, no
// sort stages).  Result in (bv, bi) on every thread.
template <int PER>
__device__ __forceinline__ void rank_and_sample(const float* cv, const int* ci, int n, int top_k, float top_p,
                                                uint32_t seed, uint32_t row, uint32_t step, float* kth_s,
                                                float* tot_s, float* rv, int* ri, float& bv, int& bi) {
  const int tid = threadIdx.x;
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
      for (int j = 0; j < n; ++j) r += better(cv[j], ci[j], v, id) ? 1 : 0;
      rank[q] = r;
      myv[q] = v;
      myi[q] = id;
    }
  }
  const int kk = min(top_k, n);
#pragma unroll
  for (int q = 0; q < PER; ++q)
    if (rank[q] == kk - 1) *kth_s = myv[q];
  if (tid == 0 && kk == 0) *kth_s = -INFINITY;
  __syncthreads();
  const float kth = *kth_s;
  float vmax = -INFINITY;
  for (int j = 0; j < n; ++j) vmax = fmaxf(vmax, cv[j]);
  float tot = 0.f;
#pragma unroll
  for (int q = 0; q < PER; ++q)
    if (rank[q] != 0x7fffffff && myv[q] >= kth) tot += __expf(myv[q] - vmax);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o, 64);
  if ((tid & 63) == 0) tot_s[tid >> 6] = tot;
  __syncthreads();
  tot = 0.f;
#pragma unroll
  for (int i = 0; i < NW; ++i) tot += tot_s[i];
  bv = -INFINITY;
  bi = 0x7fffffff;
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
        if (w >= kth && better(w, ci[j], v, id)) excl += __expf(w - vmax);
      }
      keep = excl / tot < top_p;
    }
    if (keep) {
      const float g = myv[q] + gumbel(seed, row, step, myi[q]);
      if (better(g, myi[q], bv, bi)) { bv = g; bi = myi[q]; }
    }
  }
  block_argmax(bv, bi, rv, ri);
}

// ---------------------------------------------------------------- phase 1
// Per-chunk argmax of the processed (MODE 1: + Gumbel noise) scores -> pv/pi[row*C + c].
template <bool BF16, int MODE>
__global__ void __launch_bounds__(NT) argmax_chunk_kernel(const void* __restrict__ logits,
                                                          const uint8_t* __restrict__ seen, int V, int C, float inv_t,
                                                          float pen, const int* __restrict__ rng,
                                                          float* __restrict__ pv, int* __restrict__ pi) {
  __shared__ float rv[NW];
  __shared__ int ri[NW];
  const int c = blockIdx.x, row = blockIdx.y;
  const size_t base = (size_t)row * V;
  const uint32_t seed = (uint32_t)rng[0], step = (uint32_t)rng[1];
  float bv = -INFINITY;
  int bi = 0x7fffffff;
#pragma unroll
  for (int j = 0; j < EPT; ++j) {
    const int i = c * CH + j * NT + threadIdx.x;
    if (i < V) {
      float s = proc<BF16>(logits, seen, base, i, inv_t, pen);
      if constexpr (MODE == 1) s += gumbel(seed, row, step, i);
      if (better(s, i, bv, bi)) { bv = s; bi = i; }
    }
  }
  block_argmax(bv, bi, rv, ri);
  if (threadIdx.x == 0) {
    pv[(size_t)row * C + c] = bv;
    pi[(size_t)row * C + c] = bi;
  }
}

// Per-chunk exact top-k set -> pv/pi[(row*C + c)*CCAP + s], pn = kept count, pthr = key threshold.
template <bool BF16>
__global__ void __launch_bounds__(NT) topk_chunk_kernel(const void* __restrict__ logits,
                                                        const uint8_t* __restrict__ seen, int V, int C, float inv_t,
                                                        float pen, int top_k, float* __restrict__ pv,
                                                        int* __restrict__ pi, uint32_t* __restrict__ pthr,
                                                        int* __restrict__ pn) {
  __shared__ uint32_t red[NW];
  __shared__ int scr[2 * NW];
  __shared__ int cnt;
  const int c = blockIdx.x, row = blockIdx.y, tid = threadIdx.x;
  const size_t base = (size_t)row * V;
  const int c0 = c * CH;
  const int nvalid = min(CH, V - c0);
  float sv[EPT];
  uint32_t kr[EPT];
  uint32_t kmin = 0xffffffffu, kmax = 0u;
#pragma unroll
  for (int j = 0; j < EPT; ++j) {
    const int o = j * NT + tid;
    sv[j] = o < nvalid ? proc<BF16>(logits, seen, base, c0 + o, inv_t, pen) : -INFINITY;
    kr[j] = o < nvalid ? f2key(sv[j]) : 0u;
    if (o < nvalid) { kmin = min(kmin, kr[j]); kmax = max(kmax, kr[j]); }
  }
  uint32_t thr = 0u;                       // chunk no larger than k: keep everything
  if (nvalid > top_k) {
    kmin = block_reduce_u32<0>(kmin, red);
    kmax = block_reduce_u32<1>(kmax, red);
    // invariant: count(key >= lo) >= top_k
    uint32_t lo = kmin, hi = kmax;
    int parity = 0;
    for (int it = 0; it < 34 && lo < hi; ++it) {
      const uint32_t mid = lo + (uint32_t)(((uint64_t)hi - lo + 1) >> 1);
      int wc = 0;
#pragma unroll
      for (int j = 0; j < EPT; ++j) wc += ballot_count(j * NT + tid < nvalid && kr[j] >= mid);
      const int n = block_count(wc, scr, parity);
      if (n >= top_k) {
        lo = mid;
        if (n <= CCAP) break;
      } else {
        hi = mid - 1;
      }
    }
    thr = lo;
  }
  if (tid == 0) cnt = 0;
  __syncthreads();
  const size_t slot0 = ((size_t)row * C + c) * CCAP;
#pragma unroll
  for (int j = 0; j < EPT; ++j) {
    const int o = j * NT + tid;
    if (o < nvalid && kr[j] >= thr) {
      const int s = atomicAdd(&cnt, 1);
      if (s < CCAP) { pv[slot0 + s] = sv[j]; pi[slot0 + s] = c0 + o; }
    }
  }
  __syncthreads();
  if (tid == 0) {
    pn[(size_t)row * C + c] = min(cnt, CCAP);
    pthr[(size_t)row * C + c] = thr;
  }
}

// ---------------------------------------------------------------- phase 2
__global__ void __launch_bounds__(64) argmax_merge_kernel(const float* __restrict__ pv, const int* __restrict__ pi,
                                                          int C, int V, uint8_t* __restrict__ seen,
                                                          int64_t* __restrict__ out_tok) {
  const int row = blockIdx.x;
  float bv = -INFINITY;
  int bi = 0x7fffffff;
  for (int c = threadIdx.x; c < C; c += 64) {
    const float v = pv[(size_t)row * C + c];
    const int i = pi[(size_t)row * C + c];
    if (better(v, i, bv, bi)) { bv = v; bi = i; }
  }
  wave_argmax(bv, bi);
  if (threadIdx.x == 0) {
    out_tok[row] = bi;
    if (seen != nullptr) seen[(size_t)row * V + bi] = 1;
  }
}

__global__ void __launch_bounds__(NT) topk_merge_kernel(const float* __restrict__ pv, const int* __restrict__ pi,
                                                        const uint32_t* __restrict__ pthr, const int* __restrict__ pn,
                                                        int C, int V, int top_k, float top_p,
                                                        const int* __restrict__ rng, uint8_t* __restrict__ seen,
                                                        int64_t* __restrict__ out_tok) {
  __shared__ float cv[MCAP];
  __shared__ int ci[MCAP];
  __shared__ float fv[FCAP];
  __shared__ int fi[FCAP];
  __shared__ uint32_t red[NW];
  __shared__ int scr[2 * NW];
  __shared__ int ncand, nfin;
  __shared__ float kth_s, tot_s[NW], rv[NW];
  __shared__ int ri[NW];
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t seed = (uint32_t)rng[0], step = (uint32_t)rng[1];
  uint32_t t0 = 0u;
  for (int c = tid; c < C; c += NT) t0 = max(t0, pthr[(size_t)row * C + c]);
  t0 = block_reduce_u32<1>(t0, red);
  if (tid == 0) { ncand = 0; nfin = 0; }
  __syncthreads();
  for (int c = w; c < C; c += NW) {                     // one wave per chunk, lanes over its slots
    const int nc = pn[(size_t)row * C + c];
    const size_t s0 = ((size_t)row * C + c) * CCAP;
    for (int s = lane; s < nc; s += 64) {
      const float v = pv[s0 + s];
      if (f2key(v) >= t0) {
        const int slot = atomicAdd(&ncand, 1);
        if (slot < MCAP) { cv[slot] = v; ci[slot] = pi[s0 + s]; }
      }
    }
  }
  __syncthreads();
  const int n = min(ncand, MCAP);
  constexpr int PM = MCAP / NT;
  uint32_t thr = 0u;
  if (n > FCAP) {                                        // bisect the survivors down to <= CCAP
    uint32_t kmin = 0xffffffffu, kmax = 0u;
#pragma unroll
    for (int q = 0; q < PM; ++q) {
      const int j = tid + q * NT;
      if (j < n) { const uint32_t k = f2key(cv[j]); kmin = min(kmin, k); kmax = max(kmax, k); }
    }
    kmin = block_reduce_u32<0>(kmin, red);
    kmax = block_reduce_u32<1>(kmax, red);
    uint32_t lo = kmin, hi = kmax;
    int parity = 0;
    for (int it = 0; it < 34 && lo < hi; ++it) {
      const uint32_t mid = lo + (uint32_t)(((uint64_t)hi - lo + 1) >> 1);
      int wc = 0;
#pragma unroll
      for (int q = 0; q < PM; ++q) {
        const int j = tid + q * NT;
        wc += ballot_count(j < n && f2key(cv[j]) >= mid);
      }
      const int cn = block_count(wc, scr, parity);
      if (cn >= top_k) {
        lo = mid;
        if (cn <= CCAP) break;
      } else {
        hi = mid - 1;
      }
    }
    thr = lo;
  }
#pragma unroll
  for (int q = 0; q < PM; ++q) {
    const int j = tid + q * NT;
    if (j < n && f2key(cv[j]) >= thr) {
      const int slot = atomicAdd(&nfin, 1);
      if (slot < FCAP) { fv[slot] = cv[j]; fi[slot] = ci[j]; }
    }
  }
  __syncthreads();
  float bv;
  int bi;
  rank_and_sample<FCAP / NT>(fv, fi, min(nfin, FCAP), top_k, top_p, seed, row, step, &kth_s, tot_s, rv, ri, bv, bi);
  if (tid == 0) {
    out_tok[row] = bi;
    if (seen != nullptr) seen[(size_t)row * V + bi] = 1;
  }
}

// ---------------------------------------------------------------- single-WG fallback (large k)
template <bool BF16>
__global__ void __launch_bounds__(NT) topk_row_kernel(const void* __restrict__ logits, uint8_t* __restrict__ seen,
                                                      int V, float inv_t, float pen, int top_k, float top_p,
                                                      const int* __restrict__ rng, int64_t* __restrict__ out_tok) {
  __shared__ uint32_t red[NW];
  __shared__ float cv[CAP];
  __shared__ int ci[CAP];
  __shared__ int ncand;
  __shared__ float kth_s, tot_s[NW], rv[NW];
  __shared__ int ri[NW];
  const int row = blockIdx.x, tid = threadIdx.x;
  const size_t base = (size_t)row * V;
  const uint32_t seed = (uint32_t)rng[0], step = (uint32_t)rng[1];
  uint32_t kmin = 0xffffffffu, kmax = 0u;
  for (int i = tid; i < V; i += NT) {
    const uint32_t k = f2key(proc<BF16>(logits, seen, base, i, inv_t, pen));
    kmin = min(kmin, k);
    kmax = max(kmax, k);
  }
  kmin = block_reduce_u32<0>(kmin, red);
  kmax = block_reduce_u32<1>(kmax, red);
  uint32_t lo = kmin, hi = kmax;
  for (int it = 0; it < 34 && lo < hi; ++it) {
    const uint32_t mid = lo + (uint32_t)(((uint64_t)hi - lo + 1) >> 1);
    uint32_t c = 0;
    for (int i = tid; i < V; i += NT) c += f2key(proc<BF16>(logits, seen, base, i, inv_t, pen)) >= mid;
    c = block_reduce_u32<2>(c, red);
    if ((int)c >= top_k) {
      lo = mid;
      if ((int)c <= CAP) break;
    } else {
      hi = mid - 1;
    }
  }
  if (tid == 0) ncand = 0;
  __syncthreads();
  for (int i = tid; i < V; i += NT) {
    const float s = proc<BF16>(logits, seen, base, i, inv_t, pen);
    if (f2key(s) >= lo) {
      const int slot = atomicAdd(&ncand, 1);
      if (slot < CAP) { cv[slot] = s; ci[slot] = i; }
    }
  }
  __syncthreads();
  float bv;
  int bi;
  rank_and_sample<CAP / NT>(cv, ci, min(ncand, CAP), top_k, top_p, seed, row, step, &kth_s, tot_s, rv, ri, bv, bi);
  if (tid == 0) {
    out_tok[row] = bi;
    if (seen != nullptr) seen[base + bi] = 1;
  }
}
}  // namespace

// Device workspace (bytes) the split sampler needs for B rows of V scores.
extern "C" size_t edge_sample_workspace(int B, int V) {
  const size_t C = (size_t)(V + CH - 1) / CH;
  return (size_t)B * C * (CCAP * (sizeof(float) + sizeof(int)) + sizeof(uint32_t) + sizeof(int));
}

// mode: 0 greedy, 1 full-vocab sampling, 2 top-k(+top-p). Returns -5 when the configuration
// needs the host fallback (top-p without top-k, or top-k beyond CAP).
extern "C" int edge_sample(const void* logits, int is_bf16, uint8_t* seen, int B, int V, float temperature,
                           float inv_temperature, float penalty, int top_k, float top_p, int do_sample, const int* rng,
                           int64_t* out_tok, void* workspace, hipStream_t st) {
  if (B == 0) return 0;
  int mode;
  if (!do_sample || temperature <= 0.f) mode = 0;
  else if ((top_k <= 0 || top_k >= V) && top_p >= 1.f) mode = 1;
  else if (top_k > 0 && top_k <= CAP && top_k < V) mode = 2;
  else return -5;
  const float inv_t = (mode == 0) ? 1.f : inv_temperature;  // host computes 1/T in f64 (matches _ref)
  const int C = (V + CH - 1) / CH;
  const size_t nslot = (size_t)B * C * CCAP;
  float* pv = reinterpret_cast<float*>(workspace);
  int* pi = reinterpret_cast<int*>(pv + nslot);
  uint32_t* pthr = reinterpret_cast<uint32_t*>(pi + nslot);
  int* pn = reinterpret_cast<int*>(pthr + (size_t)B * C);
  const dim3 g1(C, B);
  if (mode == 2 && top_k > CCAP) {
    if (is_bf16) hipLaunchKernelGGL(topk_row_kernel<true>, dim3(B), dim3(NT), 0, st, logits, seen, V, inv_t, penalty,
                                    top_k, top_p, rng, out_tok);
    else hipLaunchKernelGGL(topk_row_kernel<false>, dim3(B), dim3(NT), 0, st, logits, seen, V, inv_t, penalty, top_k,
                            top_p, rng, out_tok);
  } else if (mode == 2) {
    if (is_bf16) hipLaunchKernelGGL(topk_chunk_kernel<true>, g1, dim3(NT), 0, st, logits, seen, V, C, inv_t, penalty,
                                    top_k, pv, pi, pthr, pn);
    else hipLaunchKernelGGL(topk_chunk_kernel<false>, g1, dim3(NT), 0, st, logits, seen, V, C, inv_t, penalty, top_k,
                            pv, pi, pthr, pn);
    hipLaunchKernelGGL(topk_merge_kernel, dim3(B), dim3(NT), 0, st, pv, pi, pthr, pn, C, V, top_k, top_p, rng, seen,
                       out_tok);
  } else {
#define AC(BF, MD) hipLaunchKernelGGL((argmax_chunk_kernel<BF, MD>), g1, dim3(NT), 0, st, logits, seen, V, C, inv_t, \
                                      penalty, rng, pv, pi)
    if (is_bf16) { if (mode == 0) AC(true, 0); else AC(true, 1); }
    else { if (mode == 0) AC(false, 0); else AC(false, 1); }
#undef AC
    hipLaunchKernelGGL(argmax_merge_kernel, dim3(B), dim3(64), 0, st, pv, pi, C, V, seen, out_tok);
  }
  return (int)hipGetLastError();
}

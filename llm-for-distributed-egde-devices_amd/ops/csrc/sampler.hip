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
// into 2048/4096-score chunks (grid C x B, 8/16 scores per thread in registers):
//   * greedy / full-vocab sampling: per-chunk argmax of the (noised) processed scores;
//   * top-k: a superset of the chunk's top-k (every score >= a threshold t_c with
//     k <= count <= CCAP).  Thresholds are searched on order-preserving u32 keys, probing at the
//     VALUE midpoint first (logit-like distributions land in the [k, CCAP] window in 2-4 probes)
//     and at the key midpoint once that stalls, so the search always terminates.  Counts are
//     wave ballots + one LDS word per wave (parity double-buffered: one barrier per probe).
// Candidates travel as one 64-bit composite (key<<32 | ~index: orders by value, then lower index;
// unused slots 0), so the merge pays a single cross-XCD memory round trip.  The row's k-th value
// is >= T0 = max_c t_c, so phase 2 (one WG per row) gathers only the candidates >= T0 (if they
// would overflow LDS it first searches the chunk lists in global memory), narrows them to
// <= FCAP, and ranks every survivor against the others with one 64-bit LDS read per comparison —
// giving the exact k-th cut, the descending softmax prefix for top-p, and the Gumbel-max winner.
// The step counter is read from device memory (rng[1]) so both launches live in a HIP graph.
#include "common.h"

namespace {
constexpr int NT = 256, NW = NT / 64;
// Phase-1 chunk = NT * EPT scores (EPT 8 for V <= 64K, else 16).  Chunk candidate sets are
// ~k/chunk of the row; bigger chunks keep the phase-2 survivor count (~k * V / chunk) in MCAP.
__host__ __device__ constexpr int chunk_ept(int V) { return V <= 65536 ? 8 : 16; }
constexpr int CCAP = 128;     // candidates kept per chunk; the split path needs top_k <= CCAP
constexpr int CCAP_LOG2 = 7;
constexpr int MCAP = 2048;    // phase-2 candidates >= T0
constexpr int FCAP = 256;     // candidates ranked exactly (ties beyond the caps are truncated)
constexpr int CAP = 1024;     // single-workgroup fallback for CCAP < top_k <= CAP

// Phase timestamps of row 0's merge workgroup (wall_clock64 ticks), recorded when g_ts_on.
__device__ unsigned long long g_ts[16];
__device__ int g_ts_on;
#define TS(i) do { if (g_ts_on && blockIdx.x == 0 && threadIdx.x == 0) g_ts[i] = wall_clock64(); } while (0)
#define TS1(i) do { if (g_ts_on && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) g_ts[i] = wall_clock64(); } while (0)

__device__ __forceinline__ uint32_t f2key(float f) {
  const uint32_t u = __float_as_uint(f + 0.0f);       // -0 -> +0 so equal scores tie
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key2f(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}
// Composite rank key: larger = better (higher score, then lower token id).
__device__ __forceinline__ uint64_t ckey(float v, int i) { return ((uint64_t)f2key(v) << 32) | (uint32_t)(~i); }
__device__ __forceinline__ float cval(uint64_t c) { return key2f((uint32_t)(c >> 32)); }
__device__ __forceinline__ int cidx(uint64_t c) { return (int)(~(uint32_t)c); }

// Decode-step bookkeeping fused into the sampler's last launch (Adv.tok != nullptr): the workgroup
// that samples a row also does that row's part of decode_advance_kernel (tok = nxt, out[:, step] =
// nxt, pos / seq_lens += 1), and the last row to finish (an agent-scope arrival counter; row 0 itself
// at B = 1) advances step and rng[1].  Every workgroup has read step and rng[1] before it arrives,
// so none sees the advanced values.  At batch 1 this removes a launch (~4 us of a 1.9 ms step).
// The final kernels that take an Adv read rng through a plain (not __restrict__) pointer: adv.rng
// writes the same words, so the compiler must not treat the rng load as invariant.
struct Adv {
  int64_t* tok;
  int64_t* out;
  int64_t out_sb;
  int ncols;
  int64_t* step;
  int* pos;
  int* lens;
  int* ctr;                                 // arrival counter, zero between launches (B > 1 only)
  int* rng;
};

__device__ __forceinline__ void finish_row(const Adv& a, int row, int B, int tok) {
  if (a.tok == nullptr) return;
  const int64_t s = a.step[0];
  a.tok[row] = tok;
  if (s >= 0 && s < a.ncols) a.out[row * a.out_sb + s] = tok;
  a.pos[row] += 1;
  a.lens[row] += 1;
  bool last = B == 1;
  if (!last) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");    // this row's reads of step / rng have returned
    last = __hip_atomic_fetch_add(a.ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == B - 1;
    if (last) __hip_atomic_store(a.ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (last) {
    a.step[0] = s + 1;
    a.rng[1] += 1;
  }
}

// Next probe in (lo, hi]: the value midpoint while it is finite and strictly inside, else the
// key midpoint.
__device__ __forceinline__ uint32_t probe(uint32_t lo, uint32_t hi, int it) {
  if (it < 12) {
    const float a = key2f(lo), b = key2f(hi);
    if (isfinite(a) && isfinite(b)) {
      const uint32_t m = f2key(0.5f * a + 0.5f * b);
      if (m > lo && m <= hi) return m;
    }
  }
  return lo + (uint32_t)(((uint64_t)hi - lo + 1) >> 1);
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

template <int NTT = NT>
__device__ __forceinline__ void block_argmax(float& v, int& idx, float* rv, int* ri) {
  wave_argmax(v, idx);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) { rv[w] = v; ri[w] = idx; }
  __syncthreads();
  v = rv[0];
  idx = ri[0];
#pragma unroll
  for (int i = 1; i < NTT / 64; ++i)
    if (better(rv[i], ri[i], v, idx)) { v = rv[i]; idx = ri[i]; }
}

// Block-wide (min, max) of u32 keys; `scratch` holds >= 2*(NTT/64) words.
template <int NTT = NT>
__device__ __forceinline__ void block_minmax_u32(uint32_t& mn, uint32_t& mx, uint32_t* scratch) {
  constexpr int W = NTT / 64;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    mn = min(mn, (uint32_t)__shfl_xor((int)mn, o, 64));
    mx = max(mx, (uint32_t)__shfl_xor((int)mx, o, 64));
  }
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) { scratch[w] = mn; scratch[W + w] = mx; }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < W; ++i) { mn = min(mn, scratch[i]); mx = max(mx, scratch[W + i]); }
}

__device__ __forceinline__ uint32_t block_max_u32(uint32_t v, uint32_t* scratch) {
  uint32_t dummy = 0xffffffffu;
  block_minmax_u32(dummy, v, scratch);
  return v;
}

__device__ __forceinline__ uint32_t block_sum_u32(uint32_t v, uint32_t* scratch) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) scratch[threadIdx.x >> 6] = v;
  __syncthreads();
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < NW; ++i) r += scratch[i];
  return r;
}

// Block sum of a wave-uniform count with one barrier: `scr` is [2][NTT/64], alternated by `parity`.
template <int NTT = NT>
__device__ __forceinline__ int block_count(int wave_cnt, int* scr, int& parity) {
  constexpr int W = NTT / 64;
  if ((threadIdx.x & 63) == 0) scr[parity * W + (threadIdx.x >> 6)] = wave_cnt;
  __syncthreads();
  int s = 0;
#pragma unroll
  for (int i = 0; i < W; ++i) s += scr[parity * W + i];
  parity ^= 1;
  return s;
}

__device__ __forceinline__ int ballot_count(bool p) { return __popcll(__ballot(p)); }

__device__ __forceinline__ float gumbel(uint32_t seed, uint32_t row, uint32_t step, uint32_t idx) {
  const float u = uniform_hash(seed, row, step, idx);
  return -logf(-logf(u));
}

// Wave-aggregated slot allocation: one LDS atomic per wave instead of one per lane (all lanes of
// a wave hitting one counter serialise).  Returns this lane's slot; meaningful only if `pred`.
__device__ __forceinline__ int wave_alloc(bool pred, int* counter) {
  const uint64_t m = __ballot(pred);
  if (m == 0) return -1;
  const int leader = __ffsll((unsigned long long)m) - 1;
  int base = 0;
  if ((int)(threadIdx.x & 63) == leader) base = atomicAdd(counter, __popcll(m));
  base = __shfl(base, leader, 64);
  return base + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Exact top-k (ties at the k-th value kept) -> top-p -> Gumbel-max over the n <= PER*NT
// composite keys in `fc` (LDS, zero-padded to a multiple of 8).  `fe` is LDS scratch of the same
// length.  One pass gives each candidate its rank and the softmax mass of the strictly better
// candidates (those all sit at or above the k-th value, so no k-th cut is needed in the pass);
// the reads are unrolled x8 so the broadcast LDS loads overlap.  Result on every thread.
template <int PER, int NTT = NT>
__device__ __forceinline__ void rank_and_sample(const uint64_t* fc, float* fe, int n, int top_k, float top_p,
                                                uint32_t seed, uint32_t row, uint32_t step, float* sh,
                                                uint32_t* red, float* rv, int* ri, float& bv, int& bi) {
  // sh: [0] k-th value, [1..1+NTT/64) partial sums
  const int tid = threadIdx.x;
  uint64_t my[PER];
  uint32_t kmax = 0u, kmin_unused = 0xffffffffu;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int c = tid + q * NTT;
    my[q] = c < n ? fc[c] : 0ull;
    kmax = max(kmax, (uint32_t)(my[q] >> 32));
  }
  block_minmax_u32<NTT>(kmin_unused, kmax, red);
  const float vmax = key2f(kmax);
  float e[PER];
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int c = tid + q * NTT;
    e[q] = c < n ? __expf(cval(my[q]) - vmax) : 0.f;
    if (c < ((n + 7) & ~7)) fe[c] = e[q];
  }
  __syncthreads();
  int rank[PER];
  float excl[PER];
#pragma unroll
  for (int q = 0; q < PER; ++q) { rank[q] = 0; excl[q] = 0.f; }
  for (int j = 0; j < n; j += 8) {
    uint64_t f[8];
    float g[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) { f[u] = fc[j + u]; g[u] = fe[j + u]; }
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int q = 0; q < PER; ++q)
        if (f[u] > my[q]) { rank[q] += 1; excl[q] += g[u]; }
  }
  const int kk = min(top_k, n);
#pragma unroll
  for (int q = 0; q < PER; ++q)
    if (tid + q * NTT < n && rank[q] == kk - 1) sh[0] = cval(my[q]);
  __syncthreads();
  const float kth = sh[0];
  float tot = 0.f;
#pragma unroll
  for (int q = 0; q < PER; ++q)
    if (tid + q * NTT < n && cval(my[q]) >= kth) tot += e[q];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o, 64);
  if ((tid & 63) == 0) sh[1 + (tid >> 6)] = tot;
  __syncthreads();
  tot = 0.f;
#pragma unroll
  for (int i = 0; i < NTT / 64; ++i) tot += sh[1 + i];
  bv = -INFINITY;
  bi = 0x7fffffff;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const float v = cval(my[q]);
    if (tid + q * NTT >= n || v < kth) continue;
    if (rank[q] == 0 || top_p >= 1.f || excl[q] / tot < top_p) {
      const int id = cidx(my[q]);
      const float g = v + gumbel(seed, row, step, id);
      if (better(g, id, bv, bi)) { bv = g; bi = id; }
    }
  }
  block_argmax<NTT>(bv, bi, rv, ri);
}

// Zero-pad fc[n .. round_up(n, 8)) (0 ranks below every real candidate).
__device__ __forceinline__ void pad8(uint64_t* fc, int n) {
  const int t = n + (int)threadIdx.x;
  if (t < ((n + 7) & ~7)) fc[t] = 0ull;
}

// A thread's EPT processed scores of a chunk, element o = o0 + j * ostr (``run_map``): with `vec`
// (V % 8 == 0, aligned rows) a run of EPT consecutive elements (ostr = 1) read by 16-byte logits
// loads and 8-byte `seen` loads; without it one element at a time in the coalesced strided map
// (o0 = tid, ostr = NT: lane l reads element j NT + l), as also for a partial run.
// Invalid elements are -inf.  (Which thread holds which element never changes a result: the
// argmax breaks ties by id and the top-k merge ranks its candidate set exactly.)
__device__ __forceinline__ void run_map(bool vec, int tid, int ept, int& o0, int& ostr) {
  o0 = vec ? tid * ept : tid;
  ostr = vec ? 1 : NT;
}

template <bool BF16, int EPT>
__device__ __forceinline__ void load_run(const void* lg, const uint8_t* seen, size_t base, int c0, int o0, int ostr,
                                         int nvalid, bool vec, float inv_t, float pen, float (&sv)[EPT]) {
  static_assert(EPT % 8 == 0, "runs of whole 8-element groups");
  if (vec && o0 + EPT <= nvalid) {
    const size_t e0 = base + c0 + o0;
#pragma unroll
    for (int q = 0; q < EPT / 8; ++q) {
      float v[8];
      if constexpr (BF16) {
        unpack8(*reinterpret_cast<const uint4*>(reinterpret_cast<const bf16_t*>(lg) + e0 + 8 * q), v);
      } else {
        const float4 a = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(lg) + e0 + 8 * q);
        const float4 b = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(lg) + e0 + 8 * q + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
      }
      const uint64_t sn = seen != nullptr ? *reinterpret_cast<const uint64_t*>(seen + e0 + 8 * q) : 0ull;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        float x = v[u];
        if ((sn >> (8 * u)) & 0xffu) x = x < 0.f ? x * pen : x / pen;
        sv[8 * q + u] = x * inv_t;
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < EPT; ++j)
      sv[j] = o0 + j * ostr < nvalid ? proc<BF16>(lg, seen, base, c0 + o0 + j * ostr, inv_t, pen) : -INFINITY;
  }
}

// ---------------------------------------------------------------- phase 1
// Per-chunk best composite (value, then lower id) of the processed (MODE 1: + Gumbel noise)
// scores -> pc[row*C + c].  v0: global token id of column 0 (a vocab shard of the LM head: the
// noise and the composite carry global ids, so shard results merge exactly).
template <bool BF16, int MODE, int EPT>
__global__ void __launch_bounds__(NT) argmax_chunk_kernel(const void* __restrict__ logits,
                                                          const uint8_t* __restrict__ seen, int V, int C, float inv_t,
                                                          float pen, const int* __restrict__ rng,
                                                          uint64_t* __restrict__ pc, int vec, int v0) {
  __shared__ float rv[NW];
  __shared__ int ri[NW];
  const int c = blockIdx.x, row = blockIdx.y;
  const size_t base = (size_t)row * V;
  const uint32_t seed = (uint32_t)rng[0], step = (uint32_t)rng[1];
  const int c0 = c * (NT * EPT), nvalid = min(NT * EPT, V - c0);
  int o0, ostr;
  run_map(vec != 0, (int)threadIdx.x, EPT, o0, ostr);
  float sv[EPT];
  load_run<BF16, EPT>(logits, seen, base, c0, o0, ostr, nvalid, vec != 0, inv_t, pen, sv);
  float bv = -INFINITY;
  int bi = 0x7fffffff;
#pragma unroll
  for (int j = 0; j < EPT; ++j) {
    const int i = v0 + c0 + o0 + j * ostr;
    if (o0 + j * ostr < nvalid) {
      float s = sv[j];
      if constexpr (MODE == 1) s += gumbel(seed, row, step, i);
      if (better(s, i, bv, bi)) { bv = s; bi = i; }
    }
  }
  block_argmax(bv, bi, rv, ri);
  if (threadIdx.x == 0) pc[(size_t)row * C + c] = ckey(bv, bi);
}

// Per-chunk candidate superset -> pc[(row*C + c)*CCAP + s] as composite keys (unused slots 0),
// pthr[row*C + c] = threshold key.  Thread t holds EPT elements of the chunk in ``run_map``'s layout:
// [t * EPT, (t + 1) * EPT) with `vec`, else t + j * NT (strided by the block size).
// v0: global id of column 0 (vocab shard).
template <bool BF16, int EPT>
__global__ void __launch_bounds__(NT) topk_chunk_kernel(const void* __restrict__ logits,
                                                        const uint8_t* __restrict__ seen, int V, int C, float inv_t,
                                                        float pen, int top_k, uint64_t* __restrict__ pc,
                                                        uint32_t* __restrict__ pthr, int vec, int v0) {
  __shared__ uint32_t red[2 * NW];
  __shared__ int scr[2 * NW];
  __shared__ int cnt;
  const int c = blockIdx.x, row = blockIdx.y, tid = threadIdx.x;
  const size_t base = (size_t)row * V;
  const int c0 = c * (NT * EPT);
  const int nvalid = min(NT * EPT, V - c0);
  TS1(10);
  float sv[EPT];
  uint32_t kr[EPT];
  uint32_t kmin = 0xffffffffu, kmax = 0u;
  int o0, ostr;
  run_map(vec != 0, tid, EPT, o0, ostr);
  load_run<BF16, EPT>(logits, seen, base, c0, o0, ostr, nvalid, vec != 0, inv_t, pen, sv);
#pragma unroll
  for (int j = 0; j < EPT; ++j) {
    const int o = o0 + j * ostr;
    kr[j] = o < nvalid ? f2key(sv[j]) : 0u;
    if (o < nvalid) { kmin = min(kmin, kr[j]); kmax = max(kmax, kr[j]); }
  }
  if (tid == 0) cnt = 0;
  uint32_t thr = 1u;                       // chunk no larger than k: keep every valid score
  if (nvalid > top_k) {
    block_minmax_u32(kmin, kmax, red);
    TS1(11);
    uint32_t lo = kmin, hi = kmax;         // invariant: count(key >= lo) >= top_k
    int parity = 0;
    int it = 0;
    for (; it < 48 && lo < hi; ++it) {
      const uint32_t mid = probe(lo, hi, it);
      int wc = 0;
#pragma unroll
      for (int j = 0; j < EPT; ++j) wc += ballot_count(kr[j] >= mid);   // invalid keys are 0 < mid
      const int n = block_count(wc, scr, parity);
      if (n >= top_k) {
        lo = mid;
        if (n <= CCAP) break;
      } else {
        hi = mid - 1;
      }
    }
    thr = max(lo, 1u);
    if (g_ts_on && blockIdx.x == 0 && blockIdx.y == 0 && tid == 0) g_ts[14] = it;
  }
  TS1(12);
  __syncthreads();
  const size_t slot0 = ((size_t)row * C + c) * CCAP;
#pragma unroll
  for (int j = 0; j < EPT; ++j) {
    const int o = o0 + j * ostr;
    const bool ok = o < nvalid && kr[j] >= thr;
    const int s = wave_alloc(ok, &cnt);
    if (ok && s < CCAP) pc[slot0 + s] = ckey(sv[j], v0 + c0 + o);
  }
  __syncthreads();
  for (int s = min(cnt, CCAP) + tid; s < CCAP; s += NT) pc[slot0 + s] = 0ull;
  if (tid == 0) pthr[(size_t)row * C + c] = thr;
  TS1(13);
}

// ---------------------------------------------------------------- phase 2
__global__ void __launch_bounds__(64) argmax_merge_kernel(const uint64_t* __restrict__ pc, int C, int V,
                                                          uint8_t* __restrict__ seen, int64_t* __restrict__ out_tok,
                                                          Adv adv) {
  const int row = blockIdx.x;
  uint64_t best = 0ull;
  for (int c = threadIdx.x; c < C; c += 64) best = max(best, pc[(size_t)row * C + c]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t other = ((uint64_t)(uint32_t)__shfl_xor((int)(best >> 32), o, 64) << 32) |
                           (uint32_t)__shfl_xor((int)(uint32_t)best, o, 64);
    best = max(best, other);
  }
  if (threadIdx.x == 0) {
    const int bi = cidx(best);
    out_tok[row] = bi;
    if (seen != nullptr) seen[(size_t)row * V + bi] = 1;
    finish_row(adv, row, gridDim.x, bi);
  }
}

constexpr int G = 16;                      // candidate slots per thread per gather round

// Append the composites of one gather round with key >= thr to cv (LDS); count in *ncand.
__device__ __forceinline__ void collect(const uint64_t (&v)[G], uint32_t thr, uint64_t* cv, int* ncand) {
#pragma unroll
  for (int u = 0; u < G; ++u) {
    const bool ok = (uint32_t)(v[u] >> 32) >= thr;
    const int slot = wave_alloc(ok, ncand);
    if (ok && slot < MCAP) cv[slot] = v[u];
  }
}

__device__ __forceinline__ void load_round(const uint64_t* pc, size_t s0, int nslots, int r0, uint64_t (&v)[G]) {
#pragma unroll
  for (int u = 0; u < G; ++u) {
    const int sidx = r0 + u * NT + (int)threadIdx.x;
    v[u] = sidx < nslots ? pc[s0 + sidx] : 0ull;
  }
}

__global__ void __launch_bounds__(NT) topk_merge_kernel(const uint64_t* __restrict__ pc,
                                                        const uint32_t* __restrict__ pthr, int C, int V, int top_k,
                                                        float top_p, const int* rng,
                                                        uint8_t* __restrict__ seen, int64_t* __restrict__ out_tok,
                                                        Adv adv) {
  __shared__ uint64_t cv[MCAP];
  __shared__ uint64_t fc[FCAP];
  __shared__ float fe[FCAP];
  __shared__ uint32_t red[2 * NW];
  __shared__ int scr[2 * NW];
  __shared__ int ncand, nfin;
  __shared__ float sh[1 + NW], rv[NW];
  __shared__ int ri[NW];
  const int row = blockIdx.x, tid = threadIdx.x;
  TS(0);
  const uint32_t seed = (uint32_t)rng[0], step = (uint32_t)rng[1];
  const int nslots = C * CCAP;
  const size_t s0 = (size_t)row * nslots;
  // The lists were written by other XCDs, so every load misses L2: issue the thresholds and the
  // first round of candidates together (one memory round trip), then filter.
  uint32_t t0 = 0u;
  for (int c = tid; c < C; c += NT) t0 = max(t0, pthr[(size_t)row * C + c]);
  uint64_t v[G];
  load_round(pc, s0, nslots, 0, v);
  if (tid == 0) { ncand = 0; nfin = 0; }
  t0 = block_max_u32(t0, red);
  TS(1);
  collect(v, t0, cv, &ncand);
  for (int r0 = G * NT; r0 < nslots; r0 += G * NT) {
    load_round(pc, s0, nslots, r0, v);
    collect(v, t0, cv, &ncand);
  }
  __syncthreads();
  int total = ncand;
  TS(2);
  if (g_ts_on && blockIdx.x == 0 && tid == 0) g_ts[8] = total;
  if (total > MCAP) {
    // Rare: too many survivors for LDS.  Search the chunk lists in global memory for a
    // threshold leaving top_k..MCAP candidates, then gather again.
    uint32_t lo = t0, hi = 0xffffffffu;
    for (int it = 0; it < 48 && lo < hi; ++it) {
      const uint32_t mid = probe(lo, hi, it);
      uint32_t cntm = 0;
      for (int sidx = tid; sidx < nslots; sidx += NT) cntm += (uint32_t)(pc[s0 + sidx] >> 32) >= mid ? 1u : 0u;
      cntm = block_sum_u32(cntm, red);
      if ((int)cntm >= top_k) {
        lo = mid;
        if ((int)cntm <= MCAP) break;
      } else {
        hi = mid - 1;
      }
    }
    __syncthreads();
    if (tid == 0) ncand = 0;
    __syncthreads();
    for (int r0 = 0; r0 < nslots; r0 += G * NT) {
      load_round(pc, s0, nslots, r0, v);
      collect(v, lo, cv, &ncand);
    }
    __syncthreads();
    total = ncand;
  }
  const int n = min(total, MCAP);
  constexpr int PM = MCAP / NT;
  uint32_t thr = 0u;
  if (n > FCAP) {                                        // narrow the survivors to <= FCAP
    uint32_t kmin = 0xffffffffu, kmax = 0u;
    uint32_t kr[PM];
#pragma unroll
    for (int q = 0; q < PM; ++q) {
      const int j = tid + q * NT;
      kr[q] = j < n ? (uint32_t)(cv[j] >> 32) : 0u;
      if (j < n) { kmin = min(kmin, kr[q]); kmax = max(kmax, kr[q]); }
    }
    block_minmax_u32(kmin, kmax, red);
    uint32_t lo = kmin, hi = kmax;
    int parity = 0;
    for (int it = 0; it < 48 && lo < hi; ++it) {
      const uint32_t mid = probe(lo, hi, it);
      int wc = 0;
#pragma unroll
      for (int q = 0; q < PM; ++q) wc += ballot_count(kr[q] >= mid);
      const int cn = block_count(wc, scr, parity);
      if (cn >= top_k) {
        lo = mid;
        if (cn <= FCAP) break;
      } else {
        hi = mid - 1;
      }
    }
    thr = lo;
  }
  TS(3);
#pragma unroll
  for (int q = 0; q < PM; ++q) {
    const int j = tid + q * NT;
    const uint64_t x = j < n ? cv[j] : 0ull;
    const bool ok = j < n && (uint32_t)(x >> 32) >= thr;
    const int slot = wave_alloc(ok, &nfin);
    if (ok && slot < FCAP) fc[slot] = x;
  }
  __syncthreads();
  const int nf = min(nfin, FCAP);
  pad8(fc, nf);
  TS(4);
  if (g_ts_on && blockIdx.x == 0 && tid == 0) g_ts[9] = nfin;
  float bv;
  int bi;
  rank_and_sample<FCAP / NT>(fc, fe, nf, top_k, top_p, seed, row, step, sh, red, rv, ri, bv, bi);
  TS(5);
  if (tid == 0) {
    out_tok[row] = bi;
    if (seen != nullptr) seen[(size_t)row * V + bi] = 1;
    finish_row(adv, row, gridDim.x, bi);
  }
}

// ---------------------------------------------------------------- single-WG fallback (large k)
template <bool BF16>
__global__ void __launch_bounds__(NT) topk_row_kernel(const void* __restrict__ logits, uint8_t* __restrict__ seen,
                                                      int V, float inv_t, float pen, int top_k, float top_p,
                                                      const int* rng, int64_t* __restrict__ out_tok,
                                                      Adv adv) {
  __shared__ uint32_t red[2 * NW];
  __shared__ uint64_t fc[CAP];
  __shared__ float fe[CAP];
  __shared__ int ncand;
  __shared__ float sh[1 + NW], rv[NW];
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
  if (tid == 0) ncand = 0;
  block_minmax_u32(kmin, kmax, red);
  uint32_t lo = kmin, hi = kmax;
  for (int it = 0; it < 48 && lo < hi; ++it) {
    const uint32_t mid = probe(lo, hi, it);
    uint32_t c = 0;
    for (int i = tid; i < V; i += NT) c += f2key(proc<BF16>(logits, seen, base, i, inv_t, pen)) >= mid;
    c = block_sum_u32(c, red);
    if ((int)c >= top_k) {
      lo = mid;
      if ((int)c <= CAP) break;
    } else {
      hi = mid - 1;
    }
  }
  for (int i = tid; i < V; i += NT) {
    const float s = proc<BF16>(logits, seen, base, i, inv_t, pen);
    const bool ok = f2key(s) >= lo;
    const int slot = wave_alloc(ok, &ncand);          // divergent tail: inactive lanes are not in the ballot
    if (ok && slot < CAP) fc[slot] = ckey(s, i);
  }
  __syncthreads();
  const int nf = min(ncand, CAP);
  pad8(fc, nf);
  float bv;
  int bi;
  rank_and_sample<CAP / NT>(fc, fe, nf, top_k, top_p, seed, row, step, sh, red, rv, ri, bv, bi);
  if (tid == 0) {
    out_tok[row] = bi;
    if (seen != nullptr) seen[base + bi] = 1;
    finish_row(adv, row, gridDim.x, bi);
  }
}

// ---------------------------------------------------------------- whole-row form (large batches)
// One 1024-thread workgroup per row, ONE launch: at B >= ~128 rows the split form's two launches,
// its 1 KiB zero-padded candidate list per 2K chunk and the merge's cross-XCD reload cost more than
// they spread.  Each thread holds NS x 8 consecutive scores as u32 keys in registers (one 16-byte
// logits load + one 8-byte `seen` load per 8), the threshold search runs on the whole row
// (count(key >= t) in [top_k, RCAP]), the survivors go straight to LDS and rank_and_sample runs
// on them — same processor order, same Gumbel noise, same ties as the split form and _ref.sample.
constexpr int NTR = 1024, NWR = NTR / 64;
constexpr int RCAP = 256;                  // candidates ranked exactly (== FCAP)

template <bool BF16, int NS>
__global__ void __launch_bounds__(NTR) topk_rowwide_kernel(const void* __restrict__ logits,
                                                           uint8_t* __restrict__ seen, int V, float inv_t, float pen,
                                                           int top_k, float top_p, const int* rng,
                                                           int64_t* __restrict__ out_tok, Adv adv) {
  __shared__ uint32_t red[2 * NWR];
  __shared__ int scr[2 * NWR];
  __shared__ uint64_t fc[RCAP];
  __shared__ float fe[RCAP];
  __shared__ int ncand;
  __shared__ float sh[1 + NWR], rv[NWR];
  __shared__ int ri[NWR];
  const int row = blockIdx.x, tid = threadIdx.x;
  const size_t base = (size_t)row * V;
  const uint32_t seed = (uint32_t)rng[0], step = (uint32_t)rng[1];
  uint32_t kr[NS][8];
  uint32_t kmin = 0xffffffffu, kmax = 0u;
#pragma unroll
  for (int q = 0; q < NS; ++q) {
    const int e0 = (q * NTR + tid) * 8;
    if (e0 < V) {
      float v[8];
      if constexpr (BF16) {
        const uint4 raw = *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16_t*>(logits) + base + e0);
        const uint32_t w[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          v[2 * u] = __uint_as_float(w[u] << 16);
          v[2 * u + 1] = __uint_as_float(w[u] & 0xffff0000u);
        }
      } else {
        const float4 a = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(logits) + base + e0);
        const float4 b = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(logits) + base + e0 + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
      }
      uint64_t sn = 0;
      if (seen != nullptr) sn = *reinterpret_cast<const uint64_t*>(seen + base + e0);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        float x = v[u];
        if ((sn >> (8 * u)) & 0xffu) x = x < 0.f ? x * pen : x / pen;
        kr[q][u] = f2key(x * inv_t);
        kmin = min(kmin, kr[q][u]);
        kmax = max(kmax, kr[q][u]);
      }
    } else {
#pragma unroll
      for (int u = 0; u < 8; ++u) kr[q][u] = 0u;
    }
  }
  if (tid == 0) ncand = 0;
  uint32_t thr = 1u;
  if (V > top_k) {
    block_minmax_u32<NTR>(kmin, kmax, red);
    uint32_t lo = kmin, hi = kmax;         // invariant: count(key >= lo) >= top_k
    int parity = 0;
    for (int it = 0; it < 48 && lo < hi; ++it) {
      const uint32_t mid = probe(lo, hi, it);
      int wc = 0;
#pragma unroll
      for (int q = 0; q < NS; ++q)
#pragma unroll
        for (int u = 0; u < 8; ++u) wc += ballot_count(kr[q][u] >= mid);   // invalid keys are 0 < mid
      const int n = block_count<NTR>(wc, scr, parity);
      if (n >= top_k) {
        lo = mid;
        if (n <= RCAP) break;
      } else {
        hi = mid - 1;
      }
    }
    thr = max(lo, 1u);
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < NS; ++q)
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const bool ok = kr[q][u] >= thr;
      const int slot = wave_alloc(ok, &ncand);
      if (ok && slot < RCAP) fc[slot] = ((uint64_t)kr[q][u] << 32) | (uint32_t)(~((q * NTR + tid) * 8 + u));
    }
  __syncthreads();
  const int nf = min(ncand, RCAP);
  pad8(fc, nf);
  __syncthreads();
  float bv;
  int bi;
  rank_and_sample<1, NTR>(fc, fe, nf, top_k, top_p, seed, row, step, sh, red, rv, ri, bv, bi);
  if (tid == 0) {
    out_tok[row] = bi;
    if (seen != nullptr) seen[base + bi] = 1;
    finish_row(adv, row, gridDim.x, bi);
  }
}

// Decode-step bookkeeping after the sampler, one launch for what were five element-wise ops (each
// a kernel boundary in the captured step: ~4.5 us apiece at batch 1): tok = nxt, out[:, step] =
// nxt, pos += inc, seq_lens += inc (inc = 1, or the per-row active flags of a slot decoder), rng[1] += 1,
// step += 1.  One workgroup: every thread reads step before the barrier, thread 0 advances it after.
__global__ void __launch_bounds__(256) decode_advance_kernel(const int64_t* __restrict__ nxt, int64_t* __restrict__ tok,
                                                             int64_t* __restrict__ out, int64_t out_sb, int ncols,
                                                             int64_t* __restrict__ step, int* __restrict__ pos,
                                                             int* __restrict__ lens, int* __restrict__ rng,
                                                             const int* __restrict__ inc, int B) {
  const int64_t s = step[0];
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    const int64_t t = nxt[b];
    tok[b] = t;
    if (s >= 0 && s < ncols) out[b * out_sb + s] = t;
    const int d = inc != nullptr ? inc[b] : 1;
    pos[b] += d;
    lens[b] += d;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    step[0] = s + 1;
    rng[1] += 1;
  }
}
}  // namespace

extern "C" int edge_decode_advance(const int64_t* nxt, int64_t* tok, int64_t* out, int64_t out_sb, int ncols,
                                   int64_t* step, int* pos, int* lens, int* rng, const int* inc, int B,
                                   hipStream_t st) {
  if (B <= 0) return 0;
  hipLaunchKernelGGL(decode_advance_kernel, dim3(1), dim3(256), 0, st, nxt, tok, out, out_sb, ncols, step, pos, lens,
                     rng, inc, B);
  return (int)hipGetLastError();
}

// Rows at or above which the whole-row sampler form runs (V % 8 == 0, V <= 32K: 32 keys per
// thread stay in registers, 64 spill; top_k <= 128);
// tune key "sample_rowwide" (0 = never).
static int g_sample_rowwide_min = 128;
extern "C" void edge_sample_rowwide_min(int v) { g_sample_rowwide_min = v; }
// Split forms: 16-byte score loads in the chunk kernels (tune key "sample_vec"; 0 = per element).
static int g_sample_vec = 1;
extern "C" void edge_sample_vec(int v) { g_sample_vec = v; }

// Debug: enable/read the merge-phase timestamps (ticks of the 100 MHz wall clock).
extern "C" int edge_sample_timestamps(int enable, unsigned long long* host_out16) {
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_ts_on), &enable, sizeof(int)) != hipSuccess) return -1;
  if (host_out16 != nullptr && hipMemcpyFromSymbol(host_out16, HIP_SYMBOL(g_ts), 16 * sizeof(unsigned long long)) != hipSuccess)
    return -1;
  return 0;
}

// Device workspace (bytes) the split sampler needs for B rows of V scores.
extern "C" size_t edge_sample_workspace(int B, int V) {
  const int ch = NT * chunk_ept(V);
  const size_t C = (size_t)(V + ch - 1) / ch;
  return (size_t)B * C * (CCAP * sizeof(uint64_t) + sizeof(uint32_t));
}

// mode: 0 greedy, 1 full-vocab sampling, 2 top-k(+top-p). Returns -5 when the configuration
// needs the host fallback (top-p without top-k, or top-k beyond CAP).
static int sample_launch(const void* logits, int is_bf16, uint8_t* seen, int B, int V, float temperature,
                         float inv_temperature, float penalty, int top_k, float top_p, int do_sample, const int* rng,
                         int64_t* out_tok, void* workspace, const Adv& adv, hipStream_t st) {
  if (B == 0) return 0;
  int mode;
  if (!do_sample || temperature <= 0.f) mode = 0;
  else if ((top_k <= 0 || top_k >= V) && top_p >= 1.f) mode = 1;
  else if (top_k > 0 && top_k <= CAP && top_k < V) mode = 2;
  else return -5;
  const float inv_t = (mode == 0) ? 1.f : inv_temperature;  // host computes 1/T in f64 (matches _ref)
  const int ept = chunk_ept(V);
  const int C = (V + NT * ept - 1) / (NT * ept);
  uint64_t* pc = reinterpret_cast<uint64_t*>(workspace);
  uint32_t* pthr = reinterpret_cast<uint32_t*>(pc + (size_t)B * C * CCAP);
  const dim3 g1(C, B);
  // phase-1 chunk kernels: 16-byte score loads (whole aligned runs)
  const int vec = g_sample_vec && V % 8 == 0 && reinterpret_cast<uintptr_t>(logits) % 16 == 0 &&
                  (seen == nullptr || reinterpret_cast<uintptr_t>(seen) % 8 == 0);
  if (mode == 2 && top_k > CCAP) {
    if (is_bf16) hipLaunchKernelGGL(topk_row_kernel<true>, dim3(B), dim3(NT), 0, st, logits, seen, V, inv_t, penalty,
                                    top_k, top_p, rng, out_tok, adv);
    else hipLaunchKernelGGL(topk_row_kernel<false>, dim3(B), dim3(NT), 0, st, logits, seen, V, inv_t, penalty, top_k,
                            top_p, rng, out_tok, adv);
  } else if (mode == 2 && g_sample_rowwide_min > 0 && B >= g_sample_rowwide_min && V % 8 == 0 && V <= 32768) {
    const int ns = (V + NTR * 8 - 1) / (NTR * 8);
#define RW(BF, N) hipLaunchKernelGGL((topk_rowwide_kernel<BF, N>), dim3(B), dim3(NTR), 0, st, logits, seen, V, inv_t, \
                                     penalty, top_k, top_p, rng, out_tok, adv)
    if (is_bf16) { if (ns <= 2) RW(true, 2); else RW(true, 4); }
    else { if (ns <= 2) RW(false, 2); else RW(false, 4); }
#undef RW
  } else if (mode == 2) {
#define TC(BF, E) hipLaunchKernelGGL((topk_chunk_kernel<BF, E>), g1, dim3(NT), 0, st, logits, seen, V, C, inv_t, \
                                     penalty, top_k, pc, pthr, vec, 0)
    if (is_bf16) { if (ept == 8) TC(true, 8); else TC(true, 16); }
    else { if (ept == 8) TC(false, 8); else TC(false, 16); }
#undef TC
    hipLaunchKernelGGL(topk_merge_kernel, dim3(B), dim3(NT), 0, st, pc, pthr, C, V, top_k, top_p, rng, seen,
                       out_tok, adv);
  } else {
#define AC(BF, MD) do { if (ept == 8) hipLaunchKernelGGL((argmax_chunk_kernel<BF, MD, 8>), g1, dim3(NT), 0, st, logits, \
                                                        seen, V, C, inv_t, penalty, rng, pc, vec, 0); \
                           else hipLaunchKernelGGL((argmax_chunk_kernel<BF, MD, 16>), g1, dim3(NT), 0, st, logits, seen, \
                                                   V, C, inv_t, penalty, rng, pc, vec, 0); } while (0)
    if (is_bf16) { if (mode == 0) AC(true, 0); else AC(true, 1); }
    else { if (mode == 0) AC(false, 0); else AC(false, 1); }
#undef AC
    hipLaunchKernelGGL(argmax_merge_kernel, dim3(B), dim3(64), 0, st, pc, C, V, seen, out_tok, adv);
  }
  return (int)hipGetLastError();
}

extern "C" int edge_sample(const void* logits, int is_bf16, uint8_t* seen, int B, int V, float temperature,
                           float inv_temperature, float penalty, int top_k, float top_p, int do_sample, const int* rng,
                           int64_t* out_tok, void* workspace, hipStream_t st) {
  const Adv none{};
  return sample_launch(logits, is_bf16, seen, B, V, temperature, inv_temperature, penalty, top_k, top_p, do_sample,
                       rng, out_tok, workspace, none, st);
}

// edge_sample + edge_decode_advance (inc = 1) in the sampler's last launch: out_tok = nxt as well.
// ctr: an int32 that is zero before the first call (each call leaves it zero); unused at B = 1.
// rng is advanced, so it is not const here.
extern "C" int edge_sample_advance(const void* logits, int is_bf16, uint8_t* seen, int B, int V, float temperature,
                                   float inv_temperature, float penalty, int top_k, float top_p, int do_sample,
                                   int* rng, int64_t* out_tok, void* workspace, int64_t* tok, int64_t* out,
                                   int64_t out_sb, int ncols, int64_t* step, int* pos, int* lens, int* ctr,
                                   hipStream_t st) {
  if (tok == nullptr || out == nullptr || step == nullptr || pos == nullptr || lens == nullptr ||
      (B > 1 && ctr == nullptr))
    return -2;
  const Adv adv{tok, out, out_sb, ncols, step, pos, lens, ctr, rng};
  return sample_launch(logits, is_bf16, seen, B, V, temperature, inv_temperature, penalty, top_k, top_p, do_sample,
                       rng, out_tok, workspace, adv, st);
}

// ---------------------------------------------------------------- vocab-sharded LM head
// A pipeline whose LM head is split by vocabulary over its ranks (parallel/vocab_head.py): every
// rank runs phase 1 on its shard [v0, v0 + Vs) (global ids in the composites and the noise), the
// candidate lists travel to one rank, and phase 2 merges the concatenated lists [B][C_total] —
// the same two kernels as one unsplit row, so the token is the one the unsplit sampler draws.
// mode: 0 greedy, 1 full-vocab sampling, 2 top-k (<= CCAP) (+ top-p); -5: not shardable.
static int shard_mode(int do_sample, float temperature, int top_k, float top_p, int V) {
  if (!do_sample || temperature <= 0.f) return 0;
  if ((top_k <= 0 || top_k >= V) && top_p >= 1.f) return 1;
  if (top_k > 0 && top_k <= CCAP && top_k < V) return 2;
  return -5;
}

extern "C" int edge_sample_shard_mode(int do_sample, float temperature, int top_k, float top_p, int V) {
  return shard_mode(do_sample, temperature, top_k, top_p, V);
}

// Chunks of a shard of Vs scores (phase-1 chunk width for a V-wide row).
extern "C" int edge_sample_shard_chunks(int Vs, int V) {
  const int ch = NT * chunk_ept(V);
  return (Vs + ch - 1) / ch;
}

// Phase 1 over one shard: pc [B][C][CCAP] + pthr [B][C] (mode 2) or pc [B][C] (modes 0 / 1).
extern "C" int edge_sample_shard(const void* logits, int is_bf16, const uint8_t* seen, int B, int Vs, int v0, int V,
                                 float temperature, float inv_temperature, float penalty, int top_k, float top_p,
                                 int do_sample, const int* rng, uint64_t* pc, uint32_t* pthr, hipStream_t st) {
  const int mode = shard_mode(do_sample, temperature, top_k, top_p, V);
  if (mode < 0) return mode;
  if (B == 0) return 0;
  const float inv_t = mode == 0 ? 1.f : inv_temperature;
  const int ept = chunk_ept(V);
  const int C = (Vs + NT * ept - 1) / (NT * ept);
  const dim3 g1(C, B);
  const int vec = g_sample_vec && Vs % 8 == 0 && reinterpret_cast<uintptr_t>(logits) % 16 == 0 &&
                  (seen == nullptr || reinterpret_cast<uintptr_t>(seen) % 8 == 0);
  if (mode == 2) {
#define TC(BF, E) hipLaunchKernelGGL((topk_chunk_kernel<BF, E>), g1, dim3(NT), 0, st, logits, seen, Vs, C, inv_t, \
                                     penalty, top_k, pc, pthr, vec, v0)
    if (is_bf16) { if (ept == 8) TC(true, 8); else TC(true, 16); }
    else { if (ept == 8) TC(false, 8); else TC(false, 16); }
#undef TC
  } else {
#define AC(BF, MD) do { if (ept == 8) hipLaunchKernelGGL((argmax_chunk_kernel<BF, MD, 8>), g1, dim3(NT), 0, st, logits, \
                                                        seen, Vs, C, inv_t, penalty, rng, pc, vec, v0); \
                           else hipLaunchKernelGGL((argmax_chunk_kernel<BF, MD, 16>), g1, dim3(NT), 0, st, logits, seen, \
                                                   Vs, C, inv_t, penalty, rng, pc, vec, v0); } while (0)
    if (is_bf16) { if (mode == 0) AC(true, 0); else AC(true, 1); }
    else { if (mode == 0) AC(false, 0); else AC(false, 1); }
#undef AC
  }
  return (int)hipGetLastError();
}

// Phase 2 over the concatenated shard lists (C chunks per row in total) -> out_tok [B].  No `seen`
// update here: each rank marks the sampled ids of its own shard.
extern "C" int edge_sample_merge(const uint64_t* pc, const uint32_t* pthr, int B, int C, int V, float temperature,
                                 int top_k, float top_p, int do_sample, const int* rng, int64_t* out_tok,
                                 hipStream_t st) {
  const int mode = shard_mode(do_sample, temperature, top_k, top_p, V);
  if (mode < 0) return mode;
  if (B == 0) return 0;
  const Adv none{};
  if (mode == 2)
    hipLaunchKernelGGL(topk_merge_kernel, dim3(B), dim3(NT), 0, st, pc, pthr, C, V, top_k, top_p, rng, nullptr,
                       out_tok, none);
  else
    hipLaunchKernelGGL(argmax_merge_kernel, dim3(B), dim3(64), 0, st, pc, C, V, nullptr, out_tok, none);
  return (int)hipGetLastError();
}

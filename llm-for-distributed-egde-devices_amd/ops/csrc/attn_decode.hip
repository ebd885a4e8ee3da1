// Split-K flash-decoding over a head-major KV cache.
//
// q [B, Hq, D] (one new token per sequence), caches [B, Hkv, S, D] with row stride D, valid
// positions [0, seq_lens[b]).  Decode attention is HBM-bound on the K/V read, so the kernel is
// shaped for streaming rather than MFMA: one workgroup = (split, kv-head, batch); its G = Hq/Hkv
// query heads share every K/V row it loads (GQA reuse), and LPK lanes cooperate on one key row
// (LPK*16 B contiguous per key, 1 KiB per wave-instruction at D=128 -> fully coalesced).
// One pass over the split: every wave runs an online softmax (running max m, sum l, acc) over
// its key slice with K and V rows of a chunk loaded together and the next chunk prefetched, then
// the 4 waves are merged in LDS.  At decode contexts of a few hundred keys the kernel is bound by
// the serial load-latency chain, so fusing the old scores / softmax / P.V phases (each a round
// of dependent loads) is what matters.
// With nsplit > 1 each split writes (acc, m, l) and a combine kernel merges them; with one
// split the normalised output is written directly.
//
// FUSED variant (decode step of the model): q comes straight from the QKV projection row and is
// rotated in-kernel (HF rotate_half on the first `rot` dims, cos/sin from the host table, rounded
// to bf16 exactly like ops.rope_kv_write), and the split that owns the new position appends the
// rotated k and the v row to the head-major cache before reading it — the separate RoPE/KV-write
// launch disappears.  QOUT additionally emits the output as int8 with one scale per (token, 64
// columns) (layout [cols/64][Mpad]) for the W8A8 o-projection, replacing the per-token quant launch.
#include "common.h"

namespace {
constexpr int NT = 256;
constexpr int NW = NT / 64;
constexpr int UNROLL_DEF = 4;   // key groups per wave per chunk (tune "decode_attn_unroll": 8 at MHA D = 128)

struct Fuse {
  const int* pos;       // [B] cache position of the new token (seq_lens - 1)
  const float* cs;      // rope table [max_pos, rot/2] float2 (cos, sin) or null
  int rot;              // rotary dims (0: no rotation)
  int64_t qkv_sb;       // row stride of the QKV input (elements)
  int8_t* out_q;        // QOUT: [B, Hq*D] int8
  float* out_s;         // QOUT: [(Hq*D)/64][Mpad] scales
  int Mpad;
  int gs;               // query heads of one KV head split over gs workgroups (G = 1 in the kernel)
  int early;            // OCC > 0: issue the first K/V chunk at kernel entry (A/B knob decode_attn_early)
};

// Rotate the 8 values at head offset e0 (HF rotate_half convention), x/partner read from `head`.
template <bool HF>
__device__ __forceinline__ void rope8(const bf16_t* __restrict__ head, int e0, int rot, const float2* csp,
                                      float (&v)[8]) {
  const int half = rot / 2;
  const bool lo = e0 < half;
  const int pe = lo ? e0 + half : e0 - half;
  const int fi = lo ? e0 : e0 - half;
  float p[8];
  unpack8e<HF>(*reinterpret_cast<const uint4*>(head + pe), p);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float2 r = csp[fi + j];
    v[j] = lo ? (v[j] * r.x - p[j] * r.y) : (v[j] * r.x + p[j] * r.y);
  }
}

// Quantise one 64-column group held one value per lane (a full wave) and store it.
__device__ __forceinline__ void quant_group_store(float v, int8_t* q, float* s_slot, int lane) {
  const float amax = fmaxf(wave_max(fabsf(v)), 1e-8f);
  *q = quant_i8(v, 127.f / amax);
  if (lane == 0) *s_slot = amax / 127.f;
}

template <int D> struct Lanes { static constexpr int v = (D / 8 <= 8) ? 8 : ((D / 8 <= 16) ? 16 : 32); };

// OCC > 0: single-buffered key loop, nontemporal K/V loads and at least OCC waves per SIMD
// (occupancy instead of a second register buffer), and FUSED keeps the new key in registers (no
// append barrier); OCC = 0: two register buffers, no occupancy target.  NWV: waves per workgroup.
// HF: q / K / V / out are IEEE fp16 instead of bf16 (the reference's fp16 agents); fp32 softmax.
template <int D, int G, bool DIRECT, bool FUSED, bool QOUT, int OCC, bool HF, int NWV = NW, int UNROLL = UNROLL_DEF>
__global__ void __launch_bounds__(NWV * 64, OCC > 0 ? OCC : 1) decode_attn_kernel(
    const bf16_t* __restrict__ q, int64_t q_sb, bf16_t* __restrict__ kc, bf16_t* __restrict__ vc,
    int64_t c_sb, int64_t c_sh, const int* __restrict__ seq_lens, float scale_log2, int CH, int nsplit,
    bf16_t* __restrict__ out, int64_t o_sb, float* __restrict__ part_acc, float* __restrict__ part_ml, Fuse fz) {
  constexpr int LPK = Lanes<D>::v;        // lanes per key row
  constexpr int KPW = 64 / LPK;           // keys per wave-instruction
  constexpr int KPB = KPW * NWV;           // keys per workgroup step
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* red = smem;                      // [NWV][G][D] per-wave rescaled accumulators
  float* wm = red + NWV * G * D;           // [NWV][G] per-wave running max
  float* wl = wm + NWV * G;                // [NWV][G] per-wave rescaled sums
  float* mstat = wl + NWV * G;             // [G]
  float* lstat = mstat + G;               // [G]

  // head split (fz.gs > 1, G = 1): workgroup y serves query head y of KV head y / gs; every
  // such workgroup rebuilds the new key / value in registers, only the first one stores it
  const int split = blockIdx.x, kvh = blockIdx.y / fz.gs, qh0 = blockIdx.y * G, b = blockIdx.z;
  const int Hq = gridDim.y * G;
  const int len = seq_lens[b];
  const int start = split * CH;
  const int end = min(start + CH, len);
  const int n = end - start;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int dl = lane % LPK, kl = lane / LPK;
  const int d0 = dl * 8;
  const bool dvalid = d0 < D;

  if (n <= 0) {  // empty split (seq shorter than the grid's hint): publish an empty partial
    if (!DIRECT) {
      for (int i = threadIdx.x; i < G * D; i += (NWV * 64)) {
        const int h = i / D, d = i - h * D;
        part_acc[(((size_t)b * Hq + qh0 + h) * nsplit + split) * D + d] = 0.f;
      }
      if (threadIdx.x < G) {
        float* ml = part_ml + (((size_t)b * Hq + qh0 + threadIdx.x) * nsplit + split) * 2;
        ml[0] = -INFINITY; ml[1] = 0.f;
      }
    }
    return;
  }

  const bf16_t* kb = kc + b * c_sb + kvh * c_sh + (size_t)start * D;
  const bf16_t* vb = vc + b * c_sb + kvh * c_sh + (size_t)start * D;

  // K / V loads of UNROLL key groups from `base`: rows at or past `bound` load row 0 (unconditional
  // 16-byte loads; consume() masks every key past nl)
  constexpr int STEP = KPB * UNROLL;      // keys per workgroup per chunk
  const int dc = dvalid ? d0 : 0;
  auto load_b = [&](int base, int bound, uint4 (&kr)[UNROLL], uint4 (&vr)[UNROLL]) {
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int k = base + kl + u * KPB;
      const size_t off = (size_t)(k < bound ? k : 0) * D + dc;
      if (UNROLL > UNROLL_DEF && base + u * KPB >= bound) {   // wave-uniform: a whole group past the end
        kr[u] = uint4{0, 0, 0, 0};                              // (masked in consume; zero, never NaN)
        vr[u] = uint4{0, 0, 0, 0};
        continue;
      }
      if constexpr (OCC > 0) {                   // read once per step: nontemporal
        kr[u] = __builtin_bit_cast(uint4, __builtin_nontemporal_load(reinterpret_cast<const v4i*>(kb + off)));
        vr[u] = __builtin_bit_cast(uint4, __builtin_nontemporal_load(reinterpret_cast<const v4i*>(vb + off)));
      } else {
        kr[u] = *reinterpret_cast<const uint4*>(kb + off);
        vr[u] = *reinterpret_cast<const uint4*>(vb + off);
      }
    }
  };
  // OCC > 0: the wave's first chunk goes out now, before the q / RoPE / append work below (it
  // needs only the split's start and length), so one memory round trip of each workgroup's
  // critical path overlaps the q loads.  Bound n, not nl: in the split that owns the new position
  // that row may load stale, and consume() masks it (key nl) like every key past nl.
  const int base0 = wave * KPW;
  uint4 ka[UNROLL], va[UNROLL];
  if constexpr (OCC > 0) {
    if (fz.early && base0 < n) load_b(base0, n, ka, va);
  }

  // q first: its loads (and the RoPE partner loads) overlap the KV append below
  float qf[G][8];
#pragma unroll
  for (int h = 0; h < G; ++h) {
    if (dvalid) {
      const bf16_t* qh = q + b * q_sb + (size_t)(qh0 + h) * D;
      unpack8e<HF>(*reinterpret_cast<const uint4*>(qh + d0), qf[h]);
      if constexpr (FUSED) {
        if (d0 < fz.rot) {
          rope8<HF>(qh, d0, fz.rot, reinterpret_cast<const float2*>(fz.cs) + (size_t)fz.pos[b] * (fz.rot / 2), qf[h]);
#pragma unroll
          for (int j = 0; j < 8; ++j) qf[h][j] = e2f<HF>(f2e<HF>(qf[h][j]));   // q is 16-bit in the unfused path
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[h][j] *= scale_log2;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[h][j] = 0.f;
    }
  }

  // OCC > 0 keeps the new token's rotated k and v in wave 0's registers (lanes kl = 0 / 1 hold
  // dims d0..d0+7) and adds that key to the softmax directly, so no barrier orders the append
  // before the cache reads and the K/V loads start at once; the cache loop skips the new key.
  float knew[8], vnew[8];
  bool own = false;
  if constexpr (FUSED) {
    // append the new token's rotated k and its v (only the split that owns the position)
    const int pos = fz.pos[b];
    own = pos >= start && pos < end;
    const int Hkv = gridDim.y / fz.gs;
    const bf16_t* row = q + b * fz.qkv_sb;
    const float2* csp = reinterpret_cast<const float2*>(fz.cs) + (size_t)pos * (fz.rot / 2);
    if constexpr (OCC > 0) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { knew[j] = 0.f; vnew[j] = 0.f; }
      if (own && wave == 0 && kl < 2 && dvalid) {
        const bool is_v = kl == 1;
        const bf16_t* head = row + (size_t)((is_v ? Hq + Hkv : Hq) + kvh) * D;
        float v[8];
        unpack8e<HF>(*reinterpret_cast<const uint4*>(head + d0), v);
        if (!is_v && d0 < fz.rot) rope8<HF>(head, d0, fz.rot, csp, v);
        if (blockIdx.y % fz.gs == 0)
          *reinterpret_cast<uint4*>((is_v ? vc : kc) + b * c_sb + kvh * c_sh + (size_t)pos * D + d0) = pack8e<HF>(v);
#pragma unroll
        for (int j = 0; j < 8; ++j) {                // the cached 16-bit value
          const float r = e2f<HF>(f2e<HF>(v[j]));
          knew[j] = is_v ? 0.f : r;
          vnew[j] = is_v ? r : 0.f;
        }
      }
    } else {
      if (own) {
        for (int c = threadIdx.x; c < 2 * (D / 8); c += (NWV * 64)) {
          const bool is_v = c >= D / 8;
          const int e0 = (is_v ? c - D / 8 : c) * 8;
          const bf16_t* head = row + (size_t)((is_v ? Hq + Hkv : Hq) + kvh) * D;
          float v[8];
          unpack8e<HF>(*reinterpret_cast<const uint4*>(head + e0), v);
          if (!is_v && e0 < fz.rot) rope8<HF>(head, e0, fz.rot, csp, v);
          *reinterpret_cast<uint4*>((is_v ? vc : kc) + b * c_sb + kvh * c_sh + (size_t)pos * D + e0) = pack8e<HF>(v);
        }
      }
      // Only this workgroup reads the new row, so the barrier's workgroup-scope release/acquire is
      // enough (an agent-scope __threadfence would write back L2 in every workgroup: 3x slower).
      __syncthreads();
    }
  }
  const int nl = (OCC > 0 && FUSED && own) ? n - 1 : n;   // keys read from the cache

  // ---- one pass: each wave keeps an online softmax (m, l, acc) over its key slice; K and V rows
  // are loaded together and the next chunk is in flight while the current one is consumed
  // (two register buffers, alternated by a 2x unrolled loop: copying a buffer that still has
  // loads outstanding would force a full wait).  Out-of-range keys load a clamped row and are
  // masked in the score (unconditional 16-byte loads; a conditional one compiles to branches).
  float m[G], l[G], acc[G][8];
#pragma unroll
  for (int h = 0; h < G; ++h) {
    m[h] = -INFINITY;
    l[h] = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[h][j] = 0.f;
  }
  auto load = [&](int base, uint4 (&kr)[UNROLL], uint4 (&vr)[UNROLL]) { load_b(base, nl, kr, vr); };
  auto consume = [&](int base, const uint4 (&kr)[UNROLL], const uint4 (&vr)[UNROLL]) {
    float s[UNROLL][G];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      float kf[8];
      unpack8e<HF>(kr[u], kf);
#pragma unroll
      for (int h = 0; h < G; ++h) {
        float a = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) a += qf[h][j] * kf[j];
        s[u][h] = a;
      }
    }
#pragma unroll
    for (int o = LPK / 2; o > 0; o >>= 1)
#pragma unroll
      for (int u = 0; u < UNROLL; ++u)
#pragma unroll
        for (int h = 0; h < G; ++h) s[u][h] += __shfl_xor(s[u][h], o, 64);
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
      if (base + kl + u * KPB >= nl) {
#pragma unroll
        for (int h = 0; h < G; ++h) s[u][h] = -INFINITY;
      }
#pragma unroll
    for (int h = 0; h < G; ++h) {
      float cm = s[0][h];
#pragma unroll
      for (int u = 1; u < UNROLL; ++u) cm = fmaxf(cm, s[u][h]);
#pragma unroll
      for (int o = LPK; o < 64; o <<= 1) cm = fmaxf(cm, __shfl_xor(cm, o, 64));
      // cm is finite: key `base` (kl = 0, u = 0) is in range whenever a chunk is consumed
      const float mn = fmaxf(m[h], cm);
      const float alpha = __builtin_amdgcn_exp2f(m[h] - mn);        // 0 on the first chunk (m = -inf)
      m[h] = mn;
      l[h] *= alpha;
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[h][j] *= alpha;
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      float vf[8];
      unpack8e<HF>(vr[u], vf);
#pragma unroll
      for (int h = 0; h < G; ++h) {
        const float p = __builtin_amdgcn_exp2f(s[u][h] - m[h]);    // masked keys: exp2(-inf) = 0
        l[h] += p;
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[h][j] += p * vf[j];
      }
    }
  };
  if constexpr (OCC > 0 && FUSED) {
    if (own && wave == 0) {                          // the new key first: m = its score, l = 1
#pragma unroll
      for (int h = 0; h < G; ++h) {
        float sp = 0.f;
        if (kl == 0) {
#pragma unroll
          for (int j = 0; j < 8; ++j) sp += qf[h][j] * knew[j];
        }
#pragma unroll
        for (int o = LPK / 2; o > 0; o >>= 1) sp += __shfl_xor(sp, o, 64);
        m[h] = __shfl(sp, dl, 64);                   // lane dl holds the kl = 0 group's sum
        if (kl == 1) {
          l[h] = 1.f;
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[h][j] = vnew[j];
        }
      }
    }
  }
  if constexpr (OCC > 0) {
    for (int base = base0; base < nl; base += STEP) {  // wave-uniform trip count (shuffles inside)
      if (base != base0 || !fz.early) load(base, ka, va);   // (early: the first chunk went out at entry)
      consume(base, ka, va);
    }
  } else {
    uint4 kb2[UNROLL], vb2[UNROLL];
    int base = wave * KPW;                           // wave-uniform trip count (shuffles inside)
    if (base < nl) load(base, ka, va);
    while (base < nl) {
      const int nb = base + STEP;
      if (nb < nl) load(nb, kb2, vb2);
      consume(base, ka, va);
      if (nb >= nl) break;
      const int nb2 = nb + STEP;
      if (nb2 < nl) load(nb2, ka, va);
      consume(nb, kb2, vb2);
      base = nb2;
    }
  }
  // reduce over the KPW key groups of this wave (lanes sharing dl)
#pragma unroll
  for (int o = LPK; o < 64; o <<= 1)
#pragma unroll
    for (int h = 0; h < G; ++h) {
      l[h] += __shfl_xor(l[h], o, 64);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[h][j] += __shfl_xor(acc[h][j], o, 64);
    }
  // merge the waves: rescale each to the workgroup max
  if (lane == 0) {
#pragma unroll
    for (int h = 0; h < G; ++h) wm[wave * G + h] = m[h];
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < G; ++h) {
    float M = wm[h];
#pragma unroll
    for (int w = 1; w < NWV; ++w) M = fmaxf(M, wm[w * G + h]);
    const float sc_w = m[h] == -INFINITY ? 0.f : exp2f(m[h] - M);   // wave without keys: 0
    if (kl == 0 && dvalid) {
#pragma unroll
      for (int j = 0; j < 8; ++j) red[(wave * G + h) * D + d0 + j] = acc[h][j] * sc_w;
    }
    if (lane == 0) wl[wave * G + h] = l[h] * sc_w;
    if (wave == 0 && lane == 0) mstat[h] = M;
  }
  __syncthreads();
  if (threadIdx.x < G) {
    float L = 0.f;
#pragma unroll
    for (int w = 0; w < NWV; ++w) L += wl[w * G + threadIdx.x];
    lstat[threadIdx.x] = L;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < G * D; i += (NWV * 64)) {
    const int h = i / D, d = i - h * D;
    float a = 0.f;
#pragma unroll
    for (int w = 0; w < NWV; ++w) a += red[(w * G + h) * D + d];
    const int hq = qh0 + h;
    if (DIRECT) {
      if constexpr (QOUT) {     // D % 64 == 0: each 64-column group is one wave of this loop
        const float vq = e2f<HF>(f2e<HF>(a / lstat[h]));
        const int col = hq * D + d;
        quant_group_store(vq, fz.out_q + (size_t)b * Hq * D + col, fz.out_s + (size_t)(col >> 6) * fz.Mpad + b,
                          threadIdx.x & 63);
      } else {
        out[b * o_sb + (size_t)hq * D + d] = f2e<HF>(a / lstat[h]);
      }
    } else {
      part_acc[(((size_t)b * Hq + hq) * nsplit + split) * D + d] = a;
    }
  }
  if (!DIRECT && threadIdx.x < G) {
    float* ml = part_ml + (((size_t)b * Hq + qh0 + threadIdx.x) * nsplit + split) * 2;
    ml[0] = mstat[threadIdx.x];
    ml[1] = lstat[threadIdx.x];
  }
}

template <bool QOUT, bool HF>
__global__ void __launch_bounds__(256) decode_combine_kernel(const float* __restrict__ part_acc,
                                                             const float* __restrict__ part_ml, int nsplit, int D,
                                                             bf16_t* __restrict__ out, int64_t o_sb, Fuse fz) {
  const int hq = blockIdx.x, b = blockIdx.y, Hq = gridDim.x;
  const float* ml = part_ml + ((size_t)b * Hq + hq) * nsplit * 2;
  float M = -INFINITY;
  for (int s = 0; s < nsplit; ++s) M = fmaxf(M, ml[2 * s]);
  float L = 0.f;
  for (int s = 0; s < nsplit; ++s)
    if (ml[2 * s] != -INFINITY) L += exp2f(ml[2 * s] - M) * ml[2 * s + 1];
  const float invL = 1.f / L;
  const float* pa = part_acc + ((size_t)b * Hq + hq) * nsplit * D;
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    float a = 0.f;
    for (int s = 0; s < nsplit; ++s)
      if (ml[2 * s] != -INFINITY) a += exp2f(ml[2 * s] - M) * pa[(size_t)s * D + d];
    if constexpr (QOUT) {
      const int col = hq * D + d;
      quant_group_store(e2f<HF>(f2e<HF>(a * invL)), fz.out_q + (size_t)b * Hq * D + col,
                        fz.out_s + (size_t)(col >> 6) * fz.Mpad + b, threadIdx.x & 63);
    } else {
      out[b * o_sb + (size_t)hq * D + d] = f2e<HF>(a * invL);
    }
  }
}
}  // namespace

// Workspace sizes (floats) for a given launch; the binding allocates them.
static int g_target_wg = 512;   // >= 2 workgroups per CU before splitting K
// fused kernels: 4 (default) / 5 = single-buffered, barrier-free, >= 4 / 5 waves per SIMD; 0 = the
// double-buffered form with the append barrier (168 VGPRs, 3 waves per SIMD).  Measured at 128
// sequences x 32 heads, context 160 (tools/bench_ops.py attn_fused): 57.7 / 60.4 / 66.6 us.
static int g_attn_occ = 4;
// query-head split for small grids (tune "decode_attn_gsplit"): 0 automatic, 1 off, 2 always (GQA)
static int g_attn_gsplit = 0, g_attn_early = 1;
// key groups per wave per chunk of the barrier-free MHA D = 128 form (4 / 8; tune "decode_attn_unroll")
static int g_attn_unroll = 4;
extern "C" void edge_decode_attn_unroll(int v) { g_attn_unroll = v == 8 ? 8 : 4; }
// MHA grids below this many workgroups (batch 1: 32 on Llama-2-7B) take the double-buffered form:
// each workgroup walks its keys in several chunks, and there the next chunk in flight beats the
// single-buffered form's extra occupancy (tools/recipes/r4occ_b1.sh: 1 x 200 keys 8.71 -> 7.95 us,
// batch-1 Llama-2-7B 1.960 -> 1.919 ms; 16 x 200 is slower, 16.6 vs 14.6 us).  Tune "decode_attn_small".
static int g_attn_small_wg = 64;
extern "C" void edge_decode_attn_small(int v) { g_attn_small_wg = v; }
extern "C" void edge_decode_attn_gsplit(int v) { g_attn_gsplit = v; }
extern "C" void edge_decode_attn_early(int v) { g_attn_early = v; }
extern "C" void edge_decode_attn_config(int target_wg) { g_target_wg = target_wg > 0 ? target_wg : 512; }
extern "C" void edge_decode_attn_occ(int occ) { g_attn_occ = occ == 0 || occ == 5 ? occ : 4; }

namespace {
template <int D, int G, bool DI, bool FU, bool QO, bool HF>
void launch_attn(dim3 grid, size_t lds, hipStream_t st, const void* q, int64_t q_sb, void* k_cache, void* v_cache,
                 int64_t c_sb, int64_t c_sh, const int* seq_lens, float sl2, int ch, int nsplit, void* out,
                 int64_t o_sb, float* part_acc, float* part_ml, const Fuse& fz, bool small_grid) {
#define ATTN_ARGS grid, dim3(NT), lds, st, (const bf16_t*)q, q_sb, (bf16_t*)k_cache, (bf16_t*)v_cache, c_sb, c_sh, \
                  seq_lens, sl2, ch, nsplit, (bf16_t*)out, o_sb, part_acc, part_ml, fz
  if constexpr (FU) {                           // the model's decode step: barrier-free form selectable
    // occupancy target per GQA group size: the per-head q / accumulator registers grow with G, and
    // a 4-waves-per-SIMD bound spills 250-900 B/lane at G >= 4 (ISA resource report)
    constexpr int OCC4 = G <= 2 ? 4 : (G == 4 ? 2 : 1), OCC5 = G <= 2 ? 5 : OCC4;
    // (8- and 16-wave workgroups for batch-1 grids measured slower: Llama-3.2-1B decode step
    // 1.08 -> 1.19 ms with 8 waves)
    if constexpr (D == 128 && G == 1) {
      if (g_attn_occ == 4 && !small_grid && g_attn_unroll == 8) {
        hipLaunchKernelGGL((decode_attn_kernel<D, G, DI, FU, QO, OCC4, HF, NW, 8>), ATTN_ARGS);
        return;
      }
    }
    if (g_attn_occ == 4 && !small_grid) { hipLaunchKernelGGL((decode_attn_kernel<D, G, DI, FU, QO, OCC4, HF>), ATTN_ARGS); return; }
    if (g_attn_occ == 5) { hipLaunchKernelGGL((decode_attn_kernel<D, G, DI, FU, QO, OCC5, HF>), ATTN_ARGS); return; }
  }
  hipLaunchKernelGGL((decode_attn_kernel<D, G, DI, FU, QO, 0, HF>), ATTN_ARGS);
#undef ATTN_ARGS
}
}  // namespace

extern "C" int edge_decode_attn_plan(int B, int Hkv, int max_len, int D, int* ch_out, int* nsplit_out) {
  const int target_wg = g_target_wg;
  int per = B * Hkv;
  int nsplit = (target_wg + per - 1) / per;
  int ch = (max_len + nsplit - 1) / nsplit;
  ch = ((ch + 63) / 64) * 64;
  // at least 256 keys per split: below that the combine launch and the partial round trip cost
  // more than the split saves (batch 1, Llama-3.2-1B, context <= 256: 15.7 + 4.8 us per layer with
  // 4 splits of 64 keys; Llama-2-7B W8A8 batch 1 at context ~200: 2.16 ms/token direct against
  // 2.33-2.42 ms with 2 splits of 128 keys + combine)
  const int ch_min = 256;
  if (ch < ch_min) ch = ch_min;
  if (ch > 1024) ch = 1024;
  nsplit = (max_len + ch - 1) / ch;
  if (nsplit < 1) nsplit = 1;
  *ch_out = ch;
  *nsplit_out = nsplit;
  return 0;
}

namespace {
template <bool HF>
int run_attn(const void* q, int64_t q_sb, void* k_cache, void* v_cache, int64_t c_sb, int64_t c_sh,
             const int* seq_lens, int B, int Hq, int Hkv, int D, float scale, int ch, int nsplit, void* out,
             int64_t o_sb, float* part_acc, float* part_ml, const int* pos, const float* cs, int rot, void* out_q,
             float* out_s, int Mpad, hipStream_t st) {
  const int G0 = Hq / Hkv;
  const bool fused = pos != nullptr, qout = out_q != nullptr;
  // grids of a few dozen workgroups (batch 1-4 on a GQA model: 8 KV heads) are bound by each
  // workgroup's serial chain over its keys x G query heads: give every query head its own
  // workgroup instead (K/V rows re-read G times, from L2).  Needs the barrier-free fused form
  // (the new key in registers) or the plain kernel: no workgroup reads a row another one appends.
  const bool gs_ok = G0 > 1 && (!fused || g_attn_occ != 0);
  const int gs = gs_ok && (g_attn_gsplit == 2 || (g_attn_gsplit == 0 && B * Hkv * nsplit < 128)) ? G0 : 1;
  const int G = G0 / gs;
  const Fuse fz{pos, cs, fused ? rot : 0, q_sb, (int8_t*)out_q, out_s, Mpad, gs, g_attn_early};
  const float sl2 = scale * 1.4426950408889634f;
  const size_t lds = (size_t)(NW * G * D + 2 * NW * G + 2 * G) * sizeof(float);
  const dim3 grid(nsplit, Hkv * gs, B);
  const bool direct = nsplit == 1;
  const bool small_grid = G0 == 1 && direct && fused && B * Hkv < g_attn_small_wg;
  // fp16 rows (HF) have no int8-output form: the fp16 agents' o-projection is fp16
#define DK(DD, GG, DI, FU, QO)                                                                                     \
  launch_attn<DD, GG, DI, FU, QO, HF>(grid, lds, st, q, q_sb, k_cache, v_cache, c_sb, c_sh, seq_lens, sl2, ch, nsplit, \
                                      out, o_sb, part_acc, part_ml, fz, small_grid)
#define DLAUNCH(DD, GG)                                                     \
  do {                                                                      \
    if (direct) {                                                           \
      if constexpr (!HF) {                                                  \
        if (qout) { if (fused) DK(DD, GG, true, true, true); else DK(DD, GG, true, false, true); break; } \
      }                                                                     \
      if (fused) DK(DD, GG, true, true, false); else DK(DD, GG, true, false, false);             \
    } else {                                                                \
      if (fused) DK(DD, GG, false, true, false); else DK(DD, GG, false, false, false);           \
    }                                                                       \
  } while (0)
#define GSW(DD)                                   \
  switch (G) {                                    \
    case 1: DLAUNCH(DD, 1); break;                \
    case 2: DLAUNCH(DD, 2); break;                \
    case 4: DLAUNCH(DD, 4); break;                \
    case 8: DLAUNCH(DD, 8); break;                \
    default: return -3;                           \
  }
  switch (D) {
    case 64: GSW(64); break;
    case 80: GSW(80); break;
    case 128: GSW(128); break;
    case 256: GSW(256); break;
    default: return -4;
  }
#undef GSW
#undef DLAUNCH
#undef DK
  if (!direct) {
    const dim3 cg(Hq, B), cb(D <= 128 ? 128 : 256);
    if constexpr (!HF) {
      if (qout) {
        hipLaunchKernelGGL((decode_combine_kernel<true, false>), cg, cb, 0, st, part_acc, part_ml, nsplit, D,
                           (bf16_t*)out, o_sb, fz);
        return (int)hipGetLastError();
      }
    }
    hipLaunchKernelGGL((decode_combine_kernel<false, HF>), cg, cb, 0, st, part_acc, part_ml, nsplit, D, (bf16_t*)out,
                       o_sb, fz);
  }
  return (int)hipGetLastError();
}
}  // namespace

// q: [B, *] rows with the Hq query heads at offset 0 (q_sb elements apart).  FUSED (pos != null):
// q points at the QKV projection output, rows hold [q heads | k heads | v heads], the new token's
// k/v are appended to the caches at pos[b] and q is rotated in-kernel.  QOUT (out_q != null,
// D % 64 == 0, bf16 only): int8 output + [Hq*D/64][Mpad] scales instead of `out`.  h16: q, caches
// and out are fp16.
extern "C" int edge_decode_attn(const void* q, int64_t q_sb, void* k_cache, void* v_cache, int64_t c_sb,
                                int64_t c_sh, const int* seq_lens, int B, int Hq, int Hkv, int D, float scale,
                                int ch, int nsplit, void* out, int64_t o_sb, float* part_acc, float* part_ml,
                                const int* pos, const float* cs, int rot, void* out_q, float* out_s, int Mpad,
                                int h16, hipStream_t st) {
  if (B == 0) return 0;
  const int G0 = Hq / Hkv;
  if (G0 * Hkv != Hq) return -2;
  const bool fused = pos != nullptr, qout = out_q != nullptr;
  if (qout && (D % 64 != 0 || Mpad < B || h16)) return -2;
  if (fused && rot > 0 && (cs == nullptr || rot % 16 != 0 || rot > D)) return -2;
  return h16 ? run_attn<true>(q, q_sb, k_cache, v_cache, c_sb, c_sh, seq_lens, B, Hq, Hkv, D, scale, ch, nsplit, out,
                              o_sb, part_acc, part_ml, pos, cs, rot, out_q, out_s, Mpad, st)
             : run_attn<false>(q, q_sb, k_cache, v_cache, c_sb, c_sh, seq_lens, B, Hq, Hkv, D, scale, ch, nsplit, out,
                               o_sb, part_acc, part_ml, pos, cs, rot, out_q, out_s, Mpad, st);
}

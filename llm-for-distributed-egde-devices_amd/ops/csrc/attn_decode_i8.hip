// Decode attention over an INT8 KV cache (per-(token, head) scales), fused with RoPE and the
// quantising append of the new token (VERDICT r1 "fewer bytes" lever).
//
// Cache layout: k, v int8 [B, Hkv, S, D] (head-major, row stride D) and fp32 scales ks, vs
// [B, Hkv, S]: x = q * scale, q = rint(x * 127 / amax(|x|)) over the D values of one (token,
// head) row.  A key costs D + 4 bytes per tensor instead of 2 D: at D = 128, 264 B of K+V per
// token-head instead of 512, so the HBM-bound decode attention reads 1.94x fewer bytes.
//
// Shape of the kernel (the bf16 kernel's barrier-free fused form, attn_decode.hip, re-tiled for
// 1-byte elements): one workgroup = (split, kv-head, batch), 4 waves; LPK = D / 16 lanes cover
// one key row with one 16-byte load each (1 KiB per wave-instruction at every D), so every lane
// holds 16 consecutive dims of q, k, v and of its accumulators.  Scores: 16 int8 x fp32 q FMAs
// per lane, an LPK-lane shuffle sum, times the key's scale; the value scale folds into the
// softmax weight (acc += (p * vs) * v).  The new token: wave 0's lane groups kl = 0 (k) and 1 (v)
// rotate / quantise / store it and keep its DEQUANTISED values in registers, so the score and
// output use exactly what a later step will read back, and no barrier orders the append before
// the cache reads.  QOUT and split-K partials are identical to the bf16 kernel's.
//
// Also here: the quantising append for prefill (kv_quant_append_kernel): bf16 rows [B, Hkv, *, D]
// (the rotated k / v the prefill attention reads) at positions [start_pos[b], +T) -> int8 cache.
#include "common.h"

namespace {
constexpr int NT = 256;
constexpr int NW = NT / 64;

struct Fuse8 {
  const int* pos;       // [B] cache position of the new token
  const float* cs;      // rope table [max_pos, rot/2] float2 or null
  int rot;
  int64_t qkv_sb;       // row stride of the QKV input (elements)
  int8_t* out_q;        // QOUT: [B, Hq*D] int8
  float* out_s;         // QOUT: [(Hq*D)/64][Mpad]
  int Mpad;
  int S;                // cache capacity (positions): loads below it are in bounds before seq_lens is known
};

__device__ __forceinline__ void rope8i(const bf16_t* __restrict__ head, int e0, int rot, const float2* csp,
                                       float (&v)[8]) {
  const int half = rot / 2;
  const bool lo = e0 < half;
  const int pe = lo ? e0 + half : e0 - half;
  const int fi = lo ? e0 : e0 - half;
  float p[8];
  unpack8(*reinterpret_cast<const uint4*>(head + pe), p);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float2 r = csp[fi + j];
    v[j] = lo ? (v[j] * r.x - p[j] * r.y) : (v[j] * r.x + p[j] * r.y);
  }
}

// 16 int8 (one uint4) -> 16 floats
__device__ __forceinline__ void unpack16i(const uint4& u, float* f) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) f[4 * i + j] = (float)(int8_t)((w[i] >> (8 * j)) & 0xff);
  }
}

// 16 int8 as OFFSET bytes: u = q + 128 in [1, 255], one v_cvt_f32_ubyteN per element (the XOR flips
// the sign bit of all 4 bytes of a dword in one op); the caller subtracts 128 * sum(weights).
__device__ __forceinline__ void unpack16u(const uint4& u, float* f) {
  const uint32_t w[4] = {u.x ^ 0x80808080u, u.y ^ 0x80808080u, u.z ^ 0x80808080u, u.w ^ 0x80808080u};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) f[4 * i + j] = (float)((w[i] >> (8 * j)) & 0xffu);
  }
}

// Sum / max over the LPK lanes of a key group (aligned groups of LPK lanes).
template <int LPK>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = LPK / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
template <int LPK>
__device__ __forceinline__ float group_max(float v) {
#pragma unroll
  for (int o = LPK / 2; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Quantise 16 values per lane of an LPK-lane row group: returns the packed int8 and the scale,
// and overwrites v with the dequantised values (what the cache will hold).
template <int LPK>
__device__ __forceinline__ uint4 quant_row16(float (&v)[16], float& scale) {
  float a = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) a = fmaxf(a, fabsf(v[j]));
  a = fmaxf(group_max<LPK>(a), 1e-8f);
  const float inv = 127.f / a;
  scale = a / 127.f;
  uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int8_t q = quant_i8(v[j], inv);
    w[j >> 2] |= ((uint32_t)(uint8_t)q) << (8 * (j & 3));
    v[j] = (float)q * scale;
  }
  return uint4{w[0], w[1], w[2], w[3]};
}

__device__ __forceinline__ void quant_group_store8(float v, int8_t* q, float* s_slot, int lane) {
  const float amax = fmaxf(wave_max(fabsf(v)), 1e-8f);
  *q = quant_i8(v, 127.f / amax);
  if (lane == 0) *s_slot = amax / 127.f;
}

// OCC: minimum waves per SIMD (register budget).
template <int D, int G, bool DIRECT, bool QOUT, int OCC>
__global__ void __launch_bounds__(NT, OCC) decode_attn_i8_kernel(
    const bf16_t* __restrict__ qkv, int8_t* __restrict__ kc, int8_t* __restrict__ vc, float* __restrict__ ksc,
    float* __restrict__ vsc, int64_t c_sb, int64_t c_sh, int64_t s_sb, int64_t s_sh, const int* __restrict__ seq_lens,
    float scale_log2, int CH, int nsplit, bf16_t* __restrict__ out, int64_t o_sb, float* __restrict__ part_acc,
    float* __restrict__ part_ml, Fuse8 fz) {
  constexpr int LPK = D / 16;             // lanes per key row (16 int8 each)
  constexpr int KPW = 64 / LPK;           // keys per wave-instruction
  constexpr int KPB = KPW * NW;           // keys per workgroup step
  constexpr int UNROLL = G >= 4 ? 2 : 4;  // key rows per lane per chunk (q / acc grow with G)
  static_assert(D % 64 == 0 && LPK >= 4 && LPK <= 16, "D in {64, 128, 256}");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* red = smem;                      // [NW][G][D]
  float* wm = red + NW * G * D;           // [NW][G]
  float* wl = wm + NW * G;                // [NW][G]
  float* mstat = wl + NW * G;             // [G]
  float* lstat = mstat + G;               // [G]

  const int split = blockIdx.x, kvh = blockIdx.y, b = blockIdx.z;
  const int Hkv = gridDim.y, Hq = Hkv * G;
  const int len = seq_lens[b];
  const int start = split * CH;
  const int end = min(start + CH, len);
  const int n = end - start;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int dl = lane % LPK, kl = lane / LPK;
  const int d0 = dl * 16;

  if (n <= 0) {
    if (!DIRECT) {
      for (int i = threadIdx.x; i < G * D; i += NT) {
        const int h = i / D, d = i - h * D;
        part_acc[(((size_t)b * Hq + kvh * G + h) * nsplit + split) * D + d] = 0.f;
      }
      if (threadIdx.x < G) {
        float* ml = part_ml + (((size_t)b * Hq + kvh * G + threadIdx.x) * nsplit + split) * 2;
        ml[0] = -INFINITY; ml[1] = 0.f;
      }
    }
    return;
  }

  const int8_t* kb = kc + b * c_sb + kvh * c_sh + (size_t)start * D;
  const int8_t* vb = vc + b * c_sb + kvh * c_sh + (size_t)start * D;
  const float* ksb = ksc + b * s_sb + kvh * s_sh + start;
  const float* vsb = vsc + b * s_sb + kvh * s_sh + start;
  // The first chunk's K/V rows are requested before anything else (they depend only on the grid
  // position, clamped to the cache capacity, not on seq_lens): at decode contexts of a few
  // hundred keys that is the whole split, so the kernel pays one HBM round trip, overlapped with
  // the q / RoPE / append work, instead of one after it.
  constexpr int STEP = KPB * UNROLL;
  const int lim = min(CH, fz.S - start) - 1;              // last in-bounds key of this split
  uint4 kr[UNROLL], vr[UNROLL];
  float ks[UNROLL], vs[UNROLL];
  auto load = [&](int base, int bound) {
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int k = base + kl + u * KPB;
      const int kk = k <= bound ? k : 0;
      kr[u] = __builtin_bit_cast(uint4, __builtin_nontemporal_load(reinterpret_cast<const v4i*>(kb + (size_t)kk * D + d0)));
      vr[u] = __builtin_bit_cast(uint4, __builtin_nontemporal_load(reinterpret_cast<const v4i*>(vb + (size_t)kk * D + d0)));
      ks[u] = ksb[kk];
      vs[u] = vsb[kk];
    }
  };
  load(wave * KPW, lim);

  // q (rotated, rounded to bf16 as the unfused path would store it, pre-scaled by log2e/sqrt(D))
  const bf16_t* row = qkv + b * fz.qkv_sb;
  const int pos = fz.pos[b];
  const float2* csp = reinterpret_cast<const float2*>(fz.cs) + (size_t)pos * (fz.rot / 2);
  float qf[G][16];
#pragma unroll
  for (int h = 0; h < G; ++h) {
    const bf16_t* qh = row + (size_t)(kvh * G + h) * D;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      float v[8];
      unpack8(*reinterpret_cast<const uint4*>(qh + d0 + 8 * c), v);
      if (d0 + 8 * c < fz.rot) {
        rope8i(qh, d0 + 8 * c, fz.rot, csp, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = bf2f(f2bf(v[j]));
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[h][8 * c + j] = v[j] * scale_log2;
    }
  }
  float qsum[G];                                           // offset-byte keys: score -= 128 * qsum
#pragma unroll
  for (int h = 0; h < G; ++h) {
    qsum[h] = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) qsum[h] += qf[h][j];
  }

  // append: lane groups kl = 0 (k) / 1 (v) of wave 0 in the owning split
  const bool own = pos >= start && pos < end;
  float xnew[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) xnew[j] = 0.f;
  if (own && wave == 0 && kl < 2) {                 // whole LPK-lane groups: shuffles stay inside
    const bool is_v = kl == 1;
    const bf16_t* head = row + (size_t)((is_v ? Hq + Hkv : Hq) + kvh) * D;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      float v[8];
      unpack8(*reinterpret_cast<const uint4*>(head + d0 + 8 * c), v);
      if (!is_v && d0 + 8 * c < fz.rot) rope8i(head, d0 + 8 * c, fz.rot, csp, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) xnew[8 * c + j] = bf2f(f2bf(v[j]));   // the bf16 value, as the bf16 cache holds
    }
    float sc;
    const uint4 qv = quant_row16<LPK>(xnew, sc);
    const size_t roff = (size_t)pos * D + d0;
    *reinterpret_cast<uint4*>((is_v ? vc : kc) + b * c_sb + kvh * c_sh + roff) = qv;
    if (dl == 0) (is_v ? vsc : ksc)[b * s_sb + kvh * s_sh + pos] = sc;
  }
  const int nl = own ? n - 1 : n;                  // keys read from the cache (the new one is last)

  float m[G], l[G], acc[G][16], vbias[G];
#pragma unroll
  for (int h = 0; h < G; ++h) {
    m[h] = -INFINITY;
    l[h] = 0.f;
    vbias[h] = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[h][j] = 0.f;
  }
  if (own && wave == 0) {                          // the new key first: m = its score, l = 1
#pragma unroll
    for (int h = 0; h < G; ++h) {
      float sp = 0.f;
      if (kl == 0) {
#pragma unroll
        for (int j = 0; j < 16; ++j) sp += qf[h][j] * xnew[j];
      }
      sp = group_sum<LPK>(sp);
      m[h] = __shfl(sp, dl, 64);                   // lane dl (group kl = 0) holds the sum
      if (kl == 1) {
        l[h] = 1.f;
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[h][j] = xnew[j];
      }
    }
  }

  for (int base = wave * KPW; base < nl; base += STEP) {     // wave-uniform trip count
    if (base != wave * KPW) load(base, lim);                   // later chunks (long contexts)
    float s[UNROLL][G];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      float kf[16];
      unpack16u(kr[u], kf);
#pragma unroll
      for (int h = 0; h < G; ++h) {
        float a = -128.f * qsum[h];
#pragma unroll
        for (int j = 0; j < 16; ++j) a += qf[h][j] * kf[j];
        s[u][h] = a;
      }
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
#pragma unroll
      for (int h = 0; h < G; ++h) s[u][h] = group_sum<LPK>(s[u][h]) * ks[u];
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
      const float mn = fmaxf(m[h], cm);            // finite: key `base` is in range
      const float alpha = __builtin_amdgcn_exp2f(m[h] - mn);
      m[h] = mn;
      l[h] *= alpha;
      vbias[h] *= alpha;
#pragma unroll
      for (int j = 0; j < 16; ++j) acc[h][j] *= alpha;
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      float vf[16];
      unpack16u(vr[u], vf);
#pragma unroll
      for (int h = 0; h < G; ++h) {
        const float p = __builtin_amdgcn_exp2f(s[u][h] - m[h]);
        l[h] += p;
        const float pv = p * vs[u];
        vbias[h] += pv;
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[h][j] += pv * vf[j];
      }
    }
  }
#pragma unroll
  for (int h = 0; h < G; ++h)
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[h][j] -= 128.f * vbias[h];
  // reduce over the KPW key groups of this wave: the group totals of l; acc per dim lane
#pragma unroll
  for (int o = LPK; o < 64; o <<= 1)
#pragma unroll
    for (int h = 0; h < G; ++h) {
      l[h] += __shfl_xor(l[h], o, 64);
#pragma unroll
      for (int j = 0; j < 16; ++j) acc[h][j] += __shfl_xor(acc[h][j], o, 64);
    }
  // l was accumulated per lane group (every lane of a group holds the same l): no dim reduction
  if (lane == 0) {
#pragma unroll
    for (int h = 0; h < G; ++h) wm[wave * G + h] = m[h];
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < G; ++h) {
    float M = wm[h];
#pragma unroll
    for (int w = 1; w < NW; ++w) M = fmaxf(M, wm[w * G + h]);
    const float sc_w = m[h] == -INFINITY ? 0.f : exp2f(m[h] - M);
    if (kl == 0) {
#pragma unroll
      for (int j = 0; j < 16; ++j) red[(wave * G + h) * D + d0 + j] = acc[h][j] * sc_w;
    }
    if (lane == 0) wl[wave * G + h] = l[h] * sc_w;
    if (wave == 0 && lane == 0) mstat[h] = M;
  }
  __syncthreads();
  if (threadIdx.x < G) {
    float L = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) L += wl[w * G + threadIdx.x];
    lstat[threadIdx.x] = L;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < G * D; i += NT) {
    const int h = i / D, d = i - h * D;
    float a = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) a += red[(w * G + h) * D + d];
    const int hq = kvh * G + h;
    if (DIRECT) {
      if constexpr (QOUT) {
        const float vq = bf2f(f2bf(a / lstat[h]));
        const int col = hq * D + d;
        quant_group_store8(vq, fz.out_q + (size_t)b * Hq * D + col, fz.out_s + (size_t)(col >> 6) * fz.Mpad + b,
                           threadIdx.x & 63);
      } else {
        out[b * o_sb + (size_t)hq * D + d] = f2bf(a / lstat[h]);
      }
    } else {
      part_acc[(((size_t)b * Hq + hq) * nsplit + split) * D + d] = a;
    }
  }
  if (!DIRECT && threadIdx.x < G) {
    float* ml = part_ml + (((size_t)b * Hq + kvh * G + threadIdx.x) * nsplit + split) * 2;
    ml[0] = mstat[threadIdx.x];
    ml[1] = lstat[threadIdx.x];
  }
}

// Wave-per-(sequence, head) form for MHA at large batch and short contexts (the Llama-2-7B decode
// step at 128 rows x 32 heads x ~160 keys): the workgroup-per-head kernel above runs its 4096
// workgroups in 4 rounds per CU, each paying the whole dependent-load chain (sequence length ->
// q / RoPE -> K/V chunks -> LDS merge behind 3 barriers), and is latency-bound at ~2.6 TB/s.  Here
// every wave owns one (b, h) pair and walks all its keys itself — 4 pairs per 256-thread
// workgroup, so all B*H waves are resident in ONE round (16 per CU at 4 waves/SIMD), the online
// softmax never leaves the wave (no LDS, no barrier) and the next chunk's K/V rows are in flight
// while the current chunk is consumed (two register buffers).  Offset-byte conversion
// (unpack16u) halves the int8 -> float cost; the -128 bias is folded into one FMA per key
// (scores) and one running sum (values).
template <int D, bool QOUT>
__global__ void __launch_bounds__(NT, 4) decode_attn_i8_wave_kernel(
    const bf16_t* __restrict__ qkv, int8_t* __restrict__ kc, int8_t* __restrict__ vc, float* __restrict__ ksc,
    float* __restrict__ vsc, int64_t c_sb, int64_t c_sh, int64_t s_sb, int64_t s_sh, const int* __restrict__ seq_lens,
    float scale_log2, int Hkv, int npairs, bf16_t* __restrict__ out, int64_t o_sb, Fuse8 fz) {
  constexpr int LPK = D / 16, KPW = 64 / LPK, U = 2;     // U key rows per lane per buffer
  constexpr int CHUNK = KPW * U;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int pair = blockIdx.x * NW + wave;
  if (pair >= npairs) return;                           // whole wave exits (no barriers below)
  const int b = pair / Hkv, h = pair - b * Hkv;
  const int Hq = Hkv;
  const int dl = lane % LPK, kl = lane / LPK, d0 = dl * 16;
  const int8_t* kb = kc + b * c_sb + h * c_sh;
  const int8_t* vb = vc + b * c_sb + h * c_sh;
  const float* ksb = ksc + b * s_sb + h * s_sh;
  const float* vsb = vsc + b * s_sb + h * s_sh;
  const int lim = fz.S - 1;                             // loads clamp to the cache, masks use nl

  uint4 kr[2][U], vr[2][U];
  float ks[2][U], vs[2][U];
  auto load = [&](int buf, int base) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = base + kl + u * KPW;
      const int kk = k <= lim ? k : 0;
      kr[buf][u] = __builtin_bit_cast(uint4, __builtin_nontemporal_load(reinterpret_cast<const v4i*>(kb + (size_t)kk * D + d0)));
      vr[buf][u] = __builtin_bit_cast(uint4, __builtin_nontemporal_load(reinterpret_cast<const v4i*>(vb + (size_t)kk * D + d0)));
      ks[buf][u] = ksb[kk];
      vs[buf][u] = vsb[kk];
    }
  };
  load(0, 0);                                           // first chunk in flight before seq_lens is read
  const int len = seq_lens[b];
  const int pos = fz.pos[b];
  const int nl = len - 1;                               // cached keys [0, pos); the new one is at pos

  const bf16_t* row = qkv + b * fz.qkv_sb;
  const float2* csp = reinterpret_cast<const float2*>(fz.cs) + (size_t)pos * (fz.rot / 2);
  float qf[16], qsum = 0.f;
  {
    const bf16_t* qh = row + (size_t)h * D;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      float v[8];
      unpack8(*reinterpret_cast<const uint4*>(qh + d0 + 8 * c), v);
      if (d0 + 8 * c < fz.rot) {
        rope8i(qh, d0 + 8 * c, fz.rot, csp, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = bf2f(f2bf(v[j]));
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) { qf[8 * c + j] = v[j] * scale_log2; qsum += qf[8 * c + j]; }
    }
  }
  // the new token: key groups kl = 0 (k) and 1 (v) rotate / quantise / store it
  float xnew[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) xnew[j] = 0.f;
  if (kl < 2) {
    const bool is_v = kl == 1;
    const bf16_t* head = row + (size_t)((is_v ? Hq + Hkv : Hq) + h) * D;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      float v[8];
      unpack8(*reinterpret_cast<const uint4*>(head + d0 + 8 * c), v);
      if (!is_v && d0 + 8 * c < fz.rot) rope8i(head, d0 + 8 * c, fz.rot, csp, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) xnew[8 * c + j] = bf2f(f2bf(v[j]));
    }
    float sc;
    const uint4 qv = quant_row16<LPK>(xnew, sc);
    *reinterpret_cast<uint4*>((is_v ? vc : kc) + b * c_sb + h * c_sh + (size_t)pos * D + d0) = qv;
    if (dl == 0) (is_v ? vsc : ksc)[b * s_sb + h * s_sh + pos] = sc;
  }
  // online softmax state, uniform across the wave; the new key seeds it (m = its score, l = 1)
  float sp = 0.f;
  if (kl == 0) {
#pragma unroll
    for (int j = 0; j < 16; ++j) sp += qf[j] * xnew[j];
  }
  sp = group_sum<LPK>(sp);
  float m = __shfl(sp, dl, 64), l = kl == 1 ? 1.f : 0.f, vbias = 0.f;
  float acc[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) acc[j] = kl == 1 ? xnew[j] : 0.f;
  // acc holds sum p * vs * u (offset bytes) + the new value; vbias = sum p * vs (for the -128 term)

  int buf = 0;
  for (int base = 0; base < nl; base += CHUNK) {        // wave-uniform
    if (base + CHUNK < nl) load(buf ^ 1, base + CHUNK);
    float s[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float kf[16];
      unpack16u(kr[buf][u], kf);
      float a = -128.f * qsum;
#pragma unroll
      for (int j = 0; j < 16; ++j) a += qf[j] * kf[j];
      s[u] = group_sum<LPK>(a) * ks[buf][u];
      if (base + kl + u * KPW >= nl) s[u] = -INFINITY;
    }
    float cm = s[0];
#pragma unroll
    for (int u = 1; u < U; ++u) cm = fmaxf(cm, s[u]);
#pragma unroll
    for (int o = LPK; o < 64; o <<= 1) cm = fmaxf(cm, __shfl_xor(cm, o, 64));
    const float mn = fmaxf(m, cm);
    const float alpha = __builtin_amdgcn_exp2f(m - mn);
    m = mn;
    l *= alpha;
    vbias *= alpha;
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] *= alpha;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float vf[16];
      unpack16u(vr[buf][u], vf);
      const float p = __builtin_amdgcn_exp2f(s[u] - m);
      l += p;
      const float pv = p * vs[buf][u];
      vbias += pv;
#pragma unroll
      for (int j = 0; j < 16; ++j) acc[j] += pv * vf[j];
    }
    buf ^= 1;
  }
#pragma unroll
  for (int j = 0; j < 16; ++j) acc[j] -= 128.f * vbias;
#pragma unroll
  for (int o = LPK; o < 64; o <<= 1) {
    l += __shfl_xor(l, o, 64);
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] += __shfl_xor(acc[j], o, 64);
  }
  const float inv = 1.f / l;
  float o[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) o[j] = bf2f(f2bf(acc[j] * inv));
  if constexpr (QOUT) {
    // per (token, 64 columns): 4 lanes x 16 dims; every key group holds the same values
    float a = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) a = fmaxf(a, fabsf(o[j]));
    a = fmaxf(group_max<4>(a), 1e-8f);
    const float iv = 127.f / a;
    uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j >> 2] |= ((uint32_t)(uint8_t)quant_i8(o[j], iv)) << (8 * (j & 3));
    const int col = h * D + d0;
    if (kl == 0) {
      *reinterpret_cast<uint4*>(fz.out_q + (size_t)b * Hq * D + col) = uint4{w[0], w[1], w[2], w[3]};
      if ((dl & 3) == 0) fz.out_s[(size_t)(col >> 6) * fz.Mpad + b] = a / 127.f;
    }
  } else {
    if (kl == 0) {
      bf16_t* op = out + b * o_sb + (size_t)h * D + d0;
      *reinterpret_cast<uint4*>(op) = pack8(o);
      *reinterpret_cast<uint4*>(op + 8) = pack8(o + 8);
    }
  }
}

template <bool QOUT>
__global__ void __launch_bounds__(256) decode_combine_i8_kernel(const float* __restrict__ part_acc,
                                                                const float* __restrict__ part_ml, int nsplit, int D,
                                                                bf16_t* __restrict__ out, int64_t o_sb, Fuse8 fz) {
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
      quant_group_store8(bf2f(f2bf(a * invL)), fz.out_q + (size_t)b * Hq * D + col,
                         fz.out_s + (size_t)(col >> 6) * fz.Mpad + b, threadIdx.x & 63);
    } else {
      out[b * o_sb + (size_t)hq * D + d] = f2bf(a * invL);
    }
  }
}

// Prefill append: quantise bf16 rows src[b, h, start_pos[b] + t, :] (t < T) into the int8 cache.
// One wave per (b, h, t) row group of 4 rows: LPK = D / 16 lanes per row.
template <int D>
__global__ void __launch_bounds__(256) kv_quant_append_kernel(const bf16_t* __restrict__ src, int64_t x_sb,
                                                              int64_t x_sh, const int* __restrict__ start_pos,
                                                              int8_t* __restrict__ dst, int64_t c_sb, int64_t c_sh,
                                                              float* __restrict__ sc, int64_t s_sb, int64_t s_sh,
                                                              int Hkv, int T, int S, int nrows) {
  constexpr int LPK = D / 16, RPW = 64 / LPK;                 // rows per wave
  const int lane = threadIdx.x & 63;
  const int r = ((blockIdx.x * 256 + threadIdx.x) >> 6) * RPW + lane / LPK;   // (b, h, t) row index
  const int dl = lane % LPK;
  const bool valid = r < nrows;
  const int rr = valid ? r : 0;
  const int t = rr % T, bh = rr / T, h = bh % Hkv, b = bh / Hkv;
  const int pos = start_pos[b] + t;
  const bf16_t* x = src + b * x_sb + h * x_sh + (size_t)pos * D + dl * 16;
  float v[16];
  unpack8(*reinterpret_cast<const uint4*>(x), v);
  unpack8(*reinterpret_cast<const uint4*>(x + 8), v + 8);
  float s;
  const uint4 q = quant_row16<LPK>(v, s);                     // whole groups: shuffles stay inside
  if (valid && pos < S) {
    *reinterpret_cast<uint4*>(dst + b * c_sb + h * c_sh + (size_t)pos * D + dl * 16) = q;
    if (dl == 0) sc[b * s_sb + h * s_sh + pos] = s;
  }
}

// Prefill history: dequantise int8 cache rows [b, h, t < T] (+ their per-(token, head) scales)
// straight into a bf16 [B, Hkv, *, D] scratch (one 16-B int8 chunk -> 32 B of bf16 per lane) — the
// rows chunked prefill attends to beside the new tokens, without fp32 temporaries.
template <int D>
__global__ void __launch_bounds__(256) kv_dequant_kernel(const int8_t* __restrict__ src, int64_t c_sb, int64_t c_sh,
                                                         const float* __restrict__ sc, int64_t s_sb, int64_t s_sh,
                                                         bf16_t* __restrict__ dst, int64_t d_sb, int64_t d_sh, int Hkv,
                                                         int T, int nrows) {
  constexpr int LPK = D / 16, RPW = 64 / LPK;
  const int lane = threadIdx.x & 63;
  const int r = ((blockIdx.x * 256 + threadIdx.x) >> 6) * RPW + lane / LPK;
  if (r >= nrows) return;
  const int dl = lane % LPK;
  const int t = r % T, bh = r / T, h = bh % Hkv, b = bh / Hkv;
  const uint4 q = *reinterpret_cast<const uint4*>(src + b * c_sb + h * c_sh + (size_t)t * D + dl * 16);
  const float s = sc[b * s_sb + h * s_sh + t];
  const int8_t* qb = reinterpret_cast<const int8_t*>(&q);
  float v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = (float)qb[i] * s;
  bf16_t* o = dst + b * d_sb + h * d_sh + (size_t)t * D + dl * 16;
  *reinterpret_cast<uint4*>(o) = pack8(v);
  *reinterpret_cast<uint4*>(o + 8) = pack8(v + 8);
}
}  // namespace

extern "C" int edge_kv_dequant(const void* src, int64_t c_sb, int64_t c_sh, const float* sc, int64_t s_sb,
                               int64_t s_sh, void* dst, int64_t d_sb, int64_t d_sh, int B, int Hkv, int T, int D,
                               hipStream_t st) {
  const int nrows = B * Hkv * T;
  if (nrows == 0) return 0;
  const int rpw = 64 / (D / 16), waves = (nrows + rpw - 1) / rpw, blocks = (waves + 3) / 4;
#define DQ(DD) hipLaunchKernelGGL(kv_dequant_kernel<DD>, dim3(blocks), dim3(256), 0, st, (const int8_t*)src, c_sb, c_sh, \
                                  sc, s_sb, s_sh, (bf16_t*)dst, d_sb, d_sh, Hkv, T, nrows)
  switch (D) {
    case 64: DQ(64); break;
    case 128: DQ(128); break;
    case 256: DQ(256); break;
    default: return -4;
  }
#undef DQ
  return (int)hipGetLastError();
}

static int g_attn8_target_wg = 512;

extern "C" int edge_decode_attn_i8(const void* qkv, int64_t qkv_sb, void* kc, void* vc, float* ks, float* vs,
                                   int64_t c_sb, int64_t c_sh, int64_t s_sb, int64_t s_sh, const int* seq_lens,
                                   int B, int Hq, int Hkv, int D, float scale, int ch, int nsplit, void* out,
                                   int64_t o_sb, float* part_acc, float* part_ml, const int* pos, const float* cs,
                                   int rot, void* out_q, float* out_s, int Mpad, int S, hipStream_t st) {
  if (B == 0) return 0;
  const int G = Hq / Hkv;
  if (G * Hkv != Hq) return -2;
  const bool qout = out_q != nullptr;
  if (qout && (D % 64 != 0 || Mpad < B)) return -2;
  if (rot > 0 && (cs == nullptr || rot % 16 != 0 || rot > D)) return -2;
  // S = the cache's positions per head (not c_sh / D: a head pitch may exceed S * D, e.g. HeadInfer's
  // staging buffers interleave each head's K and V blocks)
  const Fuse8 fz{pos, cs, rot, qkv_sb, (int8_t*)out_q, out_s, Mpad, S};
  const float sl2 = scale * 1.4426950408889634f;
  if (G == 1 && ch < 0) {                 // wave-per-(sequence, head) form (edge_decode_attn_i8_plan)
    const int npairs = B * Hkv, blocks = (npairs + NW - 1) / NW;
#define WV(DD, QO) hipLaunchKernelGGL((decode_attn_i8_wave_kernel<DD, QO>), dim3(blocks), dim3(NT), 0, st,       \
                                      (const bf16_t*)qkv, (int8_t*)kc, (int8_t*)vc, ks, vs, c_sb, c_sh, s_sb, s_sh, \
                                      seq_lens, sl2, Hkv, npairs, (bf16_t*)out, o_sb, fz)
#define WVQ(DD) do { if (qout) WV(DD, true); else WV(DD, false); } while (0)
    switch (D) {
      case 64: WVQ(64); break;
      case 128: WVQ(128); break;
      case 256: WVQ(256); break;
      default: return -4;
    }
#undef WVQ
#undef WV
    return (int)hipGetLastError();
  }
  const size_t lds = (size_t)(NW * G * D + 2 * NW * G + 2 * G) * sizeof(float);
  const dim3 grid(nsplit, Hkv, B);
  const bool direct = nsplit == 1;
#define I8ARGS grid, dim3(NT), lds, st, (const bf16_t*)qkv, (int8_t*)kc, (int8_t*)vc, ks, vs, c_sb, c_sh, s_sb, s_sh, \
               seq_lens, sl2, ch, nsplit, (bf16_t*)out, o_sb, part_acc, part_ml, fz
#define I8K(DD, GG, DI, QO) hipLaunchKernelGGL((decode_attn_i8_kernel<DD, GG, DI, QO, (GG == 1 ? 4 : (GG == 2 ? 2 : 1))>), I8ARGS)
#define I8L(DD, GG)                                                            \
  do {                                                                         \
    if (direct) { if (qout) I8K(DD, GG, true, true); else I8K(DD, GG, true, false); } \
    else I8K(DD, GG, false, false);                                            \
  } while (0)
#define I8G(DD)                                  \
  switch (G) {                                   \
    case 1: I8L(DD, 1); break;                   \
    case 2: I8L(DD, 2); break;                   \
    case 4: I8L(DD, 4); break;                   \
    case 8: I8L(DD, 8); break;                   \
    default: return -3;                          \
  }
  switch (D) {
    case 64: I8G(64); break;
    case 128: I8G(128); break;
    case 256: I8G(256); break;
    default: return -4;
  }
#undef I8G
#undef I8L
#undef I8K
#undef I8ARGS
  if (!direct) {
    const dim3 cg(Hq, B), cb(D <= 128 ? 128 : 256);
    if (qout) hipLaunchKernelGGL(decode_combine_i8_kernel<true>, cg, cb, 0, st, part_acc, part_ml, nsplit, D,
                                 (bf16_t*)out, o_sb, fz);
    else hipLaunchKernelGGL(decode_combine_i8_kernel<false>, cg, cb, 0, st, part_acc, part_ml, nsplit, D,
                            (bf16_t*)out, o_sb, fz);
  }
  return (int)hipGetLastError();
}

// Split plan for the int8 cache: the bf16 plan's rule on bytes (>= 64 KiB of K+V per split).
// ch = -1 selects the wave-per-(sequence, head) kernel: MHA with enough pairs to put every CU to
// work with one round of resident waves (B * Hkv >= 2048) and contexts a single wave walks in a
// few chunks (<= g_attn8_wave_max keys).
static int g_attn8_wave_max = 0;     // wave form off by default (measured slower at 128 x 160; tune "attn8_wave_max")
extern "C" void edge_decode_attn_i8_wave_max(int v) { g_attn8_wave_max = v; }
extern "C" int edge_decode_attn_i8_plan(int B, int Hkv, int max_len, int D, int* ch_out, int* nsplit_out,
                                        int G) {
  const int per = B * Hkv;
  if (G == 1 && per >= 2048 && max_len <= g_attn8_wave_max) {
    *ch_out = -1;
    *nsplit_out = 1;
    return 0;
  }
  int nsplit = (g_attn8_target_wg + per - 1) / per;
  int ch = (max_len + nsplit - 1) / nsplit;
  ch = ((ch + 63) / 64) * 64;
  const int ch_min = D > 0 ? ((32768 / D + 63) / 64) * 64 : 64;
  if (ch < ch_min) ch = ch_min;
  if (ch > 2048) ch = 2048;
  nsplit = (max_len + ch - 1) / ch;
  if (nsplit < 1) nsplit = 1;
  *ch_out = ch;
  *nsplit_out = nsplit;
  return 0;
}

extern "C" int edge_kv_quant_append(const void* src, int64_t x_sb, int64_t x_sh, const int* start_pos, void* dst,
                                    int64_t c_sb, int64_t c_sh, float* sc, int64_t s_sb, int64_t s_sh, int B, int Hkv,
                                    int T, int D, int S, hipStream_t st) {
  const int nrows = B * Hkv * T;
  if (nrows == 0) return 0;
  const int rpw = 64 / (D / 16), waves = (nrows + rpw - 1) / rpw, blocks = (waves + 3) / 4;
#define QA(DD) hipLaunchKernelGGL(kv_quant_append_kernel<DD>, dim3(blocks), dim3(256), 0, st, (const bf16_t*)src, x_sb, \
                                  x_sh, start_pos, (int8_t*)dst, c_sb, c_sh, sc, s_sb, s_sh, Hkv, T, S, nrows)
  switch (D) {
    case 64: QA(64); break;
    case 128: QA(128); break;
    case 256: QA(256); break;
    default: return -4;
  }
#undef QA
  return (int)hipGetLastError();
}

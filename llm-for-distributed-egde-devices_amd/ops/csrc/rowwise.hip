// Row-wise memory-bound kernels (one 256-thread workgroup per row, 16-byte vector I/O).
//   * RMSNorm / LayerNorm with fused residual add            
//   * the same with a fused per-token symmetric INT8 quant   (W8A8 activation quant)
//   * SiLU*mul (SwiGLU) and GELU (tanh / erf), optional quant (K7)
//   * per-token INT8 quant of a bf16 row
//   * embedding gather (K1), max-softmax-probability "confidence" reduction (K13)
// Every row is held in registers between its reduction and its write: one HBM read and one
// write per element (Guideline 13: bf16 always moved as 8-element uint4).
#include "common.h"

namespace {

constexpr int NT = 256;

template <int NCH>
struct Row {
  float v[NCH][8];
};

// Load a bf16 row (optionally + residual) into registers. Elements >= H read as 0.
template <int NCH, bool HF = false>
__device__ __forceinline__ void load_row(const bf16_t* __restrict__ x, int H, float (&v)[NCH][8]) {
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int e = (c * NT + threadIdx.x) * 8;
    if (e < H) {
      uint4 u = *reinterpret_cast<const uint4*>(x + e);
      unpack8e<HF>(u, v[c]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[c][j] = 0.f;
    }
  }
}

template <int NCH, bool HF = false>
__device__ __forceinline__ void store_row(bf16_t* __restrict__ y, int H, const float (&v)[NCH][8]) {
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int e = (c * NT + threadIdx.x) * 8;
    if (e < H) *reinterpret_cast<uint4*>(y + e) = pack8e<HF>(v[c]);
  }
}

// Quantise registers to int8 with a per-row scale (block-reduced absmax).  pkt > 0: row `row` goes
// to the FRAGMENT-PACKED int8 layout of the 256-row decode GEMM (gemm_i8.hip w8a8_r256_kernel):
// piece (row / 16, k / 64) = 1 KiB at (row / 16 * pkt + k / 64) * 1024, byte (row & 15 +
// 16 ((k & 63) >> 4)) * 16 + (k & 15); pkt = H / 64 k-tiles.  A thread's 8 consecutive k stay 8
// contiguous bytes.  Otherwise q is the row (row-major).
template <int NCH>
__device__ __forceinline__ void quant_store(float (&v)[NCH][8], int H, int8_t* __restrict__ q,
                                            float* __restrict__ scale_out, float* red, int pkt = 0,
                                            size_t row = 0) {
  float amax = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(v[c][j]));
  amax = block_max<NT>(amax, red);
  amax = fmaxf(amax, 1e-8f);
  const float scale = amax / 127.f;
  const float inv = 127.f / amax;
  if (threadIdx.x == 0) *scale_out = scale;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int e = (c * NT + threadIdx.x) * 8;
    if (e < H) {
      uint32_t lo = 0, hi = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) lo |= ((uint32_t)(uint8_t)quant_i8(v[c][j], inv)) << (8 * j);
#pragma unroll
      for (int j = 0; j < 4; ++j) hi |= ((uint32_t)(uint8_t)quant_i8(v[c][4 + j], inv)) << (8 * j);
      int8_t* dst = pkt > 0 ? q + ((row >> 4) * (size_t)pkt + (e >> 6)) * 1024 +
                                  ((row & 15) + 16 * ((e & 63) >> 4)) * 16 + (e & 15)
                            : q + e;
      *reinterpret_cast<uint2*>(dst) = make_uint2(lo, hi);
    }
  }
}

// ----------------------------------------------------------------------------- norms
// PART: x arrives as S fp32 split-K partial slices [S][rows][H] of a W8A8 projection
// (gemm_i8.hip EPI_PART); they are summed in slice order and rounded to bf16 — the value the
// unsplit GEMV would have written — and that bf16 row is always written to res_out.
template <int NCH, bool RMS, bool HAS_RES, bool QUANT, bool PART, bool HF = false>
__global__ void __launch_bounds__(NT) norm_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ res, const bf16_t* __restrict__ w,
    const bf16_t* __restrict__ b, bf16_t* __restrict__ y, int8_t* __restrict__ yq,
    float* __restrict__ ys, bf16_t* __restrict__ res_out, int H, float eps, const float* __restrict__ xpart,
    int S, int pkt) {
  __shared__ float red[NT / 64];
  const size_t row = blockIdx.x;
  // gamma (and beta) chunks are loaded up front with the row, so no global load sits between
  // the reductions and the output (one memory round trip per kernel)
  uint4 wv[NCH], bv[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int e = min((c * NT + (int)threadIdx.x) * 8, H - 8);
    wv[c] = *reinterpret_cast<const uint4*>(w + e);
    if constexpr (!RMS) bv[c] = b != nullptr ? *reinterpret_cast<const uint4*>(b + e) : make_uint4(0, 0, 0, 0);
  }
  // the residual row too: its loads are in flight with the input's (partial slices'), so the
  // kernel pays one memory round trip, not two (decode at 1-128 rows is latency-bound here)
  uint4 rv[NCH];
  if constexpr (HAS_RES) {
#pragma unroll
    for (int c = 0; c < NCH; ++c)
      rv[c] = *reinterpret_cast<const uint4*>(res + row * H + min((c * NT + (int)threadIdx.x) * 8, H - 8));
  }
  float v[NCH][8];
  if constexpr (PART) {
    // every slice's loads are issued before the first add (S <= 8: one memory round trip, not S)
    const size_t slice = (size_t)gridDim.x * H;
    float4 pv[NCH][8][2];
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int e = min((c * NT + (int)threadIdx.x) * 8, H - 8);
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (k < S) {
          const float4* p = reinterpret_cast<const float4*>(xpart + k * slice + row * H + e);
          pv[c][k][0] = p[0];
          pv[c][k][1] = p[1];
        }
    }
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int e = (c * NT + threadIdx.x) * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[c][j] = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (k < S) {
          const float4 p0 = pv[c][k][0], p1 = pv[c][k][1];
          v[c][0] += p0.x; v[c][1] += p0.y; v[c][2] += p0.z; v[c][3] += p0.w;
          v[c][4] += p1.x; v[c][5] += p1.y; v[c][6] += p1.z; v[c][7] += p1.w;
        }
      if (e < H) {
        unpack8e<HF>(pack8e<HF>(v[c]), v[c]);                        // the GEMV output is bf16
        if constexpr (!HAS_RES) *reinterpret_cast<uint4*>(res_out + row * H + e) = pack8e<HF>(v[c]);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] = 0.f;
      }
    }
  } else {
    load_row<NCH, HF>(x + row * H, H, v);
  }
  if constexpr (HAS_RES) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      if ((c * NT + (int)threadIdx.x) * 8 >= H) continue;    // clamped load: not this row's data
      float r[8];
      unpack8e<HF>(rv[c], r);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[c][j] += r[j];
    }
    // the residual stream is kept in bf16 (as HF does); normalise the rounded value
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int e = (c * NT + threadIdx.x) * 8;
      if (e < H) {
        uint4 u = pack8e<HF>(v[c]);
        *reinterpret_cast<uint4*>(res_out + row * H + e) = u;
        unpack8e<HF>(u, v[c]);
      }
    }
  }
  float mean = 0.f;
  if constexpr (!RMS) {
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[c][j];
    mean = block_sum<NT>(s, red) / (float)H;
  }
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int e = (c * NT + threadIdx.x) * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float d = (e < H) ? v[c][j] - mean : 0.f;
      ss += d * d;
    }
  }
  const float rstd = rsqrtf(block_sum<NT>(ss, red) / (float)H + eps);
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int e = (c * NT + threadIdx.x) * 8;
    if (e < H) {
      float wf[8], bfv[8];
      unpack8e<HF>(wv[c], wf);
      if constexpr (!RMS) unpack8e<HF>(bv[c], bfv);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float t = (v[c][j] - mean) * rstd * wf[j];
        if constexpr (!RMS) t += bfv[j];
        v[c][j] = t;
      }
    }
  }
  if constexpr (QUANT) {
    if (pkt > 0) quant_store<NCH>(v, H, yq, ys + row, red, pkt, row);
    else quant_store<NCH>(v, H, yq + row * H, ys + row, red);
  } else {
    store_row<NCH, HF>(y + row * H, H, v);
  }
}

// ----------------------------------------------------------------------------- activations
// MODE 0: silu(gate)*up with input [gate | up] of width 2F; 1: gelu tanh; 2: gelu erf;
// 3: silu GLU over the 16-blocked [gate(16) | up(16)] layout (F % 16 == 0)
template <int NCH, int MODE, bool QUANT, bool HF = false>
__global__ void __launch_bounds__(NT) act_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                 int8_t* __restrict__ yq, float* __restrict__ ys, int F) {
  __shared__ float red[NT / 64];
  const size_t row = blockIdx.x;
  float v[NCH][8];
  if constexpr (MODE == 0) {
    const bf16_t* xr = x + row * (size_t)(2 * F);
    float u[NCH][8];
    load_row<NCH, HF>(xr, F, v);
    load_row<NCH, HF>(xr + F, F, u);
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float g = v[c][j];
        v[c][j] = g / (1.f + __expf(-g)) * u[c][j];
      }
  } else if constexpr (MODE == 3) {
    // 16-blocked GLU layout (gate_up weights packed for the fused decode epilogue): feature e's
    // gate sits at (e/16)*32 + e%16 and its up 16 columns later
    const bf16_t* xr = x + row * (size_t)(2 * F);
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int e = (c * NT + threadIdx.x) * 8;
      if (e < F) {
        const bf16_t* g = xr + (e >> 4) * 32 + (e & 15);
        float u[8];
        unpack8e<HF>(*reinterpret_cast<const uint4*>(g), v[c]);
        unpack8e<HF>(*reinterpret_cast<const uint4*>(g + 16), u);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] = v[c][j] / (1.f + __expf(-v[c][j])) * u[j];
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] = 0.f;
      }
    }
  } else {
    load_row<NCH, HF>(x + row * (size_t)F, F, v);
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float a = v[c][j];
        if constexpr (MODE == 1) {
          const float k0 = 0.7978845608028654f, k1 = 0.044715f;
          v[c][j] = 0.5f * a * (1.f + tanhf(k0 * (a + k1 * a * a * a)));
        } else {
          v[c][j] = 0.5f * a * (1.f + erff(a * 0.7071067811865476f));
        }
      }
  }
  if constexpr (QUANT) quant_store<NCH>(v, F, yq + row * (size_t)F, ys + row, red);
  else store_row<NCH, HF>(y + row * (size_t)F, F, v);
}

template <int NCH, bool HF = false>
__global__ void __launch_bounds__(NT) quant_kernel(const bf16_t* __restrict__ x, int8_t* __restrict__ q,
                                                   float* __restrict__ s, int H) {
  __shared__ float red[NT / 64];
  const size_t row = blockIdx.x;
  float v[NCH][8];
  load_row<NCH, HF>(x + row * (size_t)H, H, v);
  quant_store<NCH>(v, H, q + row * (size_t)H, s + row, red);
}

// ----------------------------------------------------------------------------- embedding
template <bool F32, bool HF = false>
__global__ void __launch_bounds__(NT) embed_kernel(const int64_t* __restrict__ ids, const bf16_t* __restrict__ table,
                                                   void* __restrict__ out, int H, int V) {
  const size_t row = blockIdx.x;
  int64_t id = ids[row];
  id = id < 0 ? 0 : (id >= V ? V - 1 : id);
  const uint4* src = reinterpret_cast<const uint4*>(table + (size_t)id * H);
  if constexpr (F32) {                                  // fp32 rows: the bf16 values widened (exact)
    float4* dst = reinterpret_cast<float4*>(reinterpret_cast<float*>(out) + row * H);
    for (int e = threadIdx.x; e < H / 8; e += NT) {
      float v[8];
      unpack8e<HF>(src[e], v);
      dst[2 * e] = make_float4(v[0], v[1], v[2], v[3]);
      dst[2 * e + 1] = make_float4(v[4], v[5], v[6], v[7]);
    }
  } else {
    uint4* dst = reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(out) + row * H);
    for (int e = threadIdx.x; e < H / 8; e += NT) dst[e] = src[e];
  }
}

// ----------------------------------------------------------------------------- confidence
// out[row] = max_v softmax(l)[v] = 1 / sum_v exp(l_v - max)   (online, one pass)
template <bool BF16, bool HF = false>
__global__ void __launch_bounds__(NT) max_prob_kernel(const void* __restrict__ logits, float* __restrict__ out, int V) {
  __shared__ float red[NT / 64];
  const size_t row = blockIdx.x;
  float m = -INFINITY, s = 0.f;
  for (int i = threadIdx.x; i < V; i += NT) {
    float l;
    if constexpr (BF16) l = e2f<HF>(reinterpret_cast<const bf16_t*>(logits)[row * V + i]);   // 16-bit logits
    else l = reinterpret_cast<const float*>(logits)[row * V + i];
    if (l > m) { s = s * __expf(m - l) + 1.f; m = l; }
    else s += __expf(l - m);
  }
  const float gm = block_max<NT>(m, red);
  s = (m == -INFINITY) ? 0.f : s * __expf(m - gm);
  s = block_sum<NT>(s, red);
  if (threadIdx.x == 0) out[row] = 1.f / s;
}

}  // namespace

// ============================================================================= launchers
#define NCH_DISPATCH(H, ...)                                        \
  do {                                                              \
    const int need = ((H) + NT * 8 - 1) / (NT * 8);                 \
    if (need <= 1) { constexpr int NCH = 1; __VA_ARGS__; }          \
    else if (need <= 2) { constexpr int NCH = 2; __VA_ARGS__; }     \
    else if (need <= 4) { constexpr int NCH = 4; __VA_ARGS__; }     \
    else if (need <= 8) { constexpr int NCH = 8; __VA_ARGS__; }     \
    else return -1;                                                 \
  } while (0)

extern "C" int edge_norm(const void* x, const void* res, const void* w, const void* b, void* y, void* yq,
                         float* ys, void* res_out, int rows, int H, float eps, int rms, int quant,
                         const float* xpart, int S, int h16, hipStream_t st) {
  // quant 2: int8 output fragment-packed for the 256-row decode GEMM (H % 64 == 0, <= 256 rows)
  if (H % 8 || (quant == 2 && (H % 64 != 0 || rows > 256))) return -2;
  // h16: fp16 rows (the fp16 agents' bf16-free path): no int8 output
  if (h16 && quant) return -2;
  const int pkt = quant == 2 ? H / 64 : 0;
  if (xpart != nullptr && (!rms || res_out == nullptr || S < 1)) return -2;
  if (rows == 0) return 0;
  const bf16_t *X = (const bf16_t*)x, *R = (const bf16_t*)res, *W = (const bf16_t*)w, *Bb = (const bf16_t*)b;
  bf16_t *Y = (bf16_t*)y, *RO = (bf16_t*)res_out;
  int8_t* Q = (int8_t*)yq;
#define LAUNCH_NORM(RMS, HR, QU) \
  hipLaunchKernelGGL((norm_kernel<NCH, RMS, HR, QU, false>), dim3(rows), dim3(NT), 0, st, X, R, W, Bb, Y, Q, ys, RO, H, \
                     eps, nullptr, 0, pkt)
#define LAUNCH_NORMP(HR, QU) \
  hipLaunchKernelGGL((norm_kernel<NCH, true, HR, QU, true>), dim3(rows), dim3(NT), 0, st, X, R, W, Bb, Y, Q, ys, RO, H, \
                     eps, xpart, S, pkt)
  if (xpart != nullptr && (S < 1 || S > 8 || H % 8 != 0)) return -2;   // partial slices: 1..8
#define LAUNCH_NORMH(RMS, HR) \
  hipLaunchKernelGGL((norm_kernel<NCH, RMS, HR, false, false, true>), dim3(rows), dim3(NT), 0, st, X, R, W, Bb, Y, Q, ys, \
                     RO, H, eps, nullptr, 0, 0)
#define LAUNCH_NORMPH(HR) \
  hipLaunchKernelGGL((norm_kernel<NCH, true, HR, false, true, true>), dim3(rows), dim3(NT), 0, st, X, R, W, Bb, Y, Q, ys, \
                     RO, H, eps, xpart, S, 0)
  NCH_DISPATCH(H, {
    if (h16 && xpart != nullptr) {
      if (res) LAUNCH_NORMPH(true); else LAUNCH_NORMPH(false);
    } else if (h16) {
      if (rms) { if (res) LAUNCH_NORMH(true, true); else LAUNCH_NORMH(true, false); }
      else { if (res) LAUNCH_NORMH(false, true); else LAUNCH_NORMH(false, false); }
    } else if (xpart != nullptr) {
      if (res) { if (quant) LAUNCH_NORMP(true, true); else LAUNCH_NORMP(true, false); }
      else { if (quant) LAUNCH_NORMP(false, true); else LAUNCH_NORMP(false, false); }
    } else if (rms) {
      if (res) { if (quant) LAUNCH_NORM(true, true, true); else LAUNCH_NORM(true, true, false); }
      else { if (quant) LAUNCH_NORM(true, false, true); else LAUNCH_NORM(true, false, false); }
    } else {
      if (res) { if (quant) LAUNCH_NORM(false, true, true); else LAUNCH_NORM(false, true, false); }
      else { if (quant) LAUNCH_NORM(false, false, true); else LAUNCH_NORM(false, false, false); }
    }
  });
#undef LAUNCH_NORM
#undef LAUNCH_NORMP
#undef LAUNCH_NORMH
#undef LAUNCH_NORMPH
  return (int)hipGetLastError();
}

extern "C" int edge_act(const void* x, void* y, void* yq, float* ys, int rows, int F, int mode, int quant,
                        int h16, hipStream_t st) {
  if (F % 8 || (h16 && quant)) return -2;
  if (rows == 0) return 0;
  const bf16_t* X = (const bf16_t*)x;
  bf16_t* Y = (bf16_t*)y;
  int8_t* Q = (int8_t*)yq;
#define LAUNCH_ACT(M, QU) hipLaunchKernelGGL((act_kernel<NCH, M, QU>), dim3(rows), dim3(NT), 0, st, X, Y, Q, ys, F)
#define LAUNCH_ACTH(M) hipLaunchKernelGGL((act_kernel<NCH, M, false, true>), dim3(rows), dim3(NT), 0, st, X, Y, Q, ys, F)
  NCH_DISPATCH(F, {
    if (h16) {
      if (mode == 0) LAUNCH_ACTH(0); else if (mode == 1) LAUNCH_ACTH(1); else if (mode == 3) LAUNCH_ACTH(3);
      else LAUNCH_ACTH(2);
    } else if (mode == 0) { if (quant) LAUNCH_ACT(0, true); else LAUNCH_ACT(0, false); }
    else if (mode == 1) { if (quant) LAUNCH_ACT(1, true); else LAUNCH_ACT(1, false); }
    else if (mode == 3) { if (quant) LAUNCH_ACT(3, true); else LAUNCH_ACT(3, false); }
    else { if (quant) LAUNCH_ACT(2, true); else LAUNCH_ACT(2, false); }
  });
#undef LAUNCH_ACT
#undef LAUNCH_ACTH
  return (int)hipGetLastError();
}

// Per-(row, 64-column) int8 quantisation (decode GEMV input layout: scales [K/64][Mpad]).  One
// wave covers 512 columns of a row, 8 per lane; a group's 8 lanes reduce its absmax with three
// xor-shuffles.  Used between the fused SwiGLU GEMV and the down projection.
template <bool HF = false>
__global__ void __launch_bounds__(NT) group_quant_kernel(const bf16_t* __restrict__ x, int8_t* __restrict__ q,
                                                         float* __restrict__ s, int M, int K, int Mpad) {
  const int gw = blockIdx.x * (NT / 64) + (threadIdx.x >> 6);
  const int wpr = (K + 511) / 512;
  const int row = gw / wpr, wr = gw - row * wpr;
  if (row >= M) return;
  const int lane = threadIdx.x & 63;
  const int e = wr * 512 + lane * 8;
  const bool ok = e < K;                       // K % 64 == 0: a group's 8 lanes agree
  float v[8];
  if (ok) unpack8e<HF>(*reinterpret_cast<const uint4*>(x + (size_t)row * K + e), v);
  else {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = 0.f;
  }
  float m = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(v[j]));
#pragma unroll
  for (int o = 1; o < 8; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  m = fmaxf(m, 1e-8f);
  if (!ok) return;
  const float inv = 127.f / m;
  uint32_t lo = 0, hi = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) lo |= ((uint32_t)(uint8_t)quant_i8(v[j], inv)) << (8 * j);
#pragma unroll
  for (int j = 0; j < 4; ++j) hi |= ((uint32_t)(uint8_t)quant_i8(v[4 + j], inv)) << (8 * j);
  *reinterpret_cast<uint2*>(q + (size_t)row * K + e) = make_uint2(lo, hi);
  if ((lane & 7) == 0) s[(size_t)(e >> 6) * Mpad + row] = m / 127.f;
}

extern "C" int edge_group_quant(const void* x, void* q, float* s, int M, int K, int Mpad, hipStream_t st) {
  if (K % 64 || Mpad < M) return -2;
  if (M == 0) return 0;
  const int waves = M * ((K + 511) / 512);
  hipLaunchKernelGGL(group_quant_kernel<false>, dim3((waves + 3) / 4), dim3(NT), 0, st, (const bf16_t*)x, (int8_t*)q, s, M, K,
                     Mpad);
  return (int)hipGetLastError();
}

extern "C" int edge_quant(const void* x, void* q, float* s, int rows, int H, hipStream_t st) {
  if (H % 8) return -2;
  if (rows == 0) return 0;
  NCH_DISPATCH(H, {
    hipLaunchKernelGGL((quant_kernel<NCH>), dim3(rows), dim3(NT), 0, st, (const bf16_t*)x, (int8_t*)q, s, H);
  });
  return (int)hipGetLastError();
}

extern "C" int edge_embedding(const int64_t* ids, const void* table, void* out, int rows, int H, int V, int out_f32,
                              int h16, hipStream_t st) {
  if (H % 8) return -2;
  if (rows == 0) return 0;
  if (out_f32 && h16) hipLaunchKernelGGL((embed_kernel<true, true>), dim3(rows), dim3(NT), 0, st, ids, (const bf16_t*)table, out, H, V);
  else if (out_f32) hipLaunchKernelGGL(embed_kernel<true>, dim3(rows), dim3(NT), 0, st, ids, (const bf16_t*)table, out, H, V);
  else hipLaunchKernelGGL(embed_kernel<false>, dim3(rows), dim3(NT), 0, st, ids, (const bf16_t*)table, out, H, V);
  return (int)hipGetLastError();
}

// dt: 0 fp32 logits, 1 bf16, 2 fp16
extern "C" int edge_max_prob(const void* logits, float* out, int rows, int V, int dt, hipStream_t st) {
  if (rows == 0) return 0;
  if (dt == 2) hipLaunchKernelGGL((max_prob_kernel<true, true>), dim3(rows), dim3(NT), 0, st, logits, out, V);
  else if (dt == 1) hipLaunchKernelGGL((max_prob_kernel<true>), dim3(rows), dim3(NT), 0, st, logits, out, V);
  else hipLaunchKernelGGL((max_prob_kernel<false>), dim3(rows), dim3(NT), 0, st, logits, out, V);
  return (int)hipGetLastError();
}

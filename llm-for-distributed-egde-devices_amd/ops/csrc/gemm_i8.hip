// W8A8 INT8 GEMM on CDNA4 MFMA (v_mfma_i32_16x16x64_i8) with fused dequant epilogues.
//   out[m][n] = (sum_k A[m][k] * W[n][k]) * a_scale * w_scale[n] (+ bias[n])   -> bf16
// the kernel behind both the SmoothQuant W8A8 mode and the LLM.int8 inlier GEMM.
//
// Weight layout ("MFMA-packed"): the [N, K] int8 matrix is stored as 1 KiB tiles of
// 16 output channels x 64 k; tile (nt, kt) sits at byte ((nt * KT) + kt) * 1024 and lane l's
// 16 bytes are W[nt*16 + (l & 15)][kt*64 + 16*(l >> 4) .. +16] — exactly the B fragment of
// the i8 16x16x64 MFMA, so a wave fetches one fragment with one fully-coalesced 1 KiB load
// and a workgroup streams a column panel as one contiguous byte range.  A (activations) is
// row-major [M, K]; its fragment is lane l <- A[m0 + (l & 15)][k0 + 16*(l >> 4) .. +16].
// Both operands use the same (lane, byte) -> k map, so the MFMA sums the right products.
//
// Decode kernels (the prefill GEMMs are in gemm_i8_prefill.hip, the shared layout and helpers in
// gemm_i8.h):
//   gemv:  M <= 64.  HBM-bound on W: a workgroup owns NTW 16-column tiles of one 16-row block,
//          its NW waves split K (k-tile kt -> wave kt % NW) and keep UNROLL fragments per tile in
//          flight (no LDS staging: the weights are read exactly once, nontemporal), partial sums
//          reduced through LDS.  Activation modes:
//            A_TOKEN  int8 A, one scale per token (from the fused norm+quant kernel)
//            A_GROUP  int8 A, one scale per (token, 64 columns) [KT][Mpad] (fused attention)
//          With per-group scales each k-tile's MFMA starts from zero and is folded into a float
//          accumulator with its scale (4 cvt + 4 fma per 16x16 tile).
//          Epilogues: EPI_OUT bf16 (+bias).  The GLU epilogues read gate_up rows packed
//          16-blocked ([gate f0..f0+15 | up f0..f0+15] per 32 rows), so tile pair (2p, 2p+1) of a
//          workgroup is (gate, up) of 16 features: EPI_GLU writes silu(g) * up as bf16 h [M, N/2]
//          (2 or 4 tiles per workgroup; rowwise.hip::group_quant_kernel quantises it for the down
//          projection); EPI_GLUQ (8 tiles = 64 features) also quantises h per (token, 64 features)
//          in the epilogue and writes int8 h + scales [N/128][Mpad] directly.
//   ring2: 65-256 rows (and the bf16 decode projections at 17-256 rows): both operands by
//          LDS-DMA into rings of decoupled depth, dedicated weight / activation loader waves.
//   r256:  129-256 rows on fragment-packed activations (qkv).
#include "gemm_i8.h"
#include <type_traits>

namespace {
// int8 A fragment of k-tile k for this lane's row (ragged K: byte-wise, zero padded)
__device__ __forceinline__ v4i load_a_i8(const int8_t* __restrict__ arow_p, bool aval, int k, int kend, int akc,
                                         int K, bool k16) {
  const int kk = k * 64 + akc;
  if (aval && k < kend && kk + 16 <= K && k16) return *reinterpret_cast<const v4i*>(arow_p + kk);
  if (aval && k < kend && kk < K) {
    int8_t t[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) t[j] = (kk + j < K) ? arow_p[kk + j] : 0;
    return *reinterpret_cast<v4i*>(t);
  }
  return v4i{0, 0, 0, 0};
}

// ------------------------------------------------------------------------------------ gemv
// Weight-stationary over the rows: one workgroup owns NTW 16-column tiles for ALL M <= 16*MB
// rows, so every weight fragment is fetched once and feeds MB MFMAs.  NW = TG x KW waves: wave
// (tg, kw) holds tiles [tg*TPW, (tg+1)*TPW) and k-tiles kt = kw (mod KW); per step it keeps
// U x TPW nontemporal 1 KiB weight fragments in flight.  Sizing rule (tools/membw.hip on
// MI355X, cache-cold): 16 waves per CU-resident workgroup and >= 172 workgroups stream a
// 50-90 MB panel at 5.6-6.2 TB/s, while 4-wave workgroups or < 256 groups of few waves stall at
// 2-4 TB/s — so the launcher always runs 16 waves and sizes NTW for ~256 workgroups.
// Partial tiles are reduced across the KW k-waves through LDS (KW x NTW x MB KiB).  Everything
// the epilogue reads from global memory (weight scales, bias, per-token scales) is loaded at
// kernel start, so the tail of the kernel never waits on an HBM round trip.

#ifndef GEMV_UNROLL_FIXED
#define GEMV_UNROLL_FIXED 1
#endif

// Epilogue operands preloaded per owned fragment (EPI_OUT) or gate/up pair (GLU).
template <int OWN>
struct EpiPre {
  float s0[OWN], s1[OWN];    // sw[col] (EPI_OUT) | sw[gate col], sw[up col]
  float b0[OWN], b1[OWN];    // bias likewise (0 when absent)
};

template <int MB, int NTW, int NW, int EPI>
constexpr int epi_units() {
  return (EPI == EPI_OUT || EPI == EPI_PART || EPI == EPI_GELUQT || EPI == EPI_GELUQE) ? NTW * MB : NTW / 2 * MB;
}

template <int MB, int NTW, int NW, int EPI>
__device__ __forceinline__ EpiPre<(epi_units<MB, NTW, NW, EPI>() + NW - 1) / NW> epi_preload(
    const float* __restrict__ sw, const bf16_t* __restrict__ bias, int nt0, int NTt, int wave, int lane) {
  constexpr int UNITS = epi_units<MB, NTW, NW, EPI>(), OWN = (UNITS + NW - 1) / NW;
  EpiPre<OWN> p;
#pragma unroll
  for (int o = 0; o < OWN; ++o) {
    const int u = wave + o * NW;
    constexpr bool PAIR = EPI == EPI_GLU || EPI == EPI_GLUQ;
    const int t = PAIR ? 2 * (u / MB) : u / MB;                      // (gate) tile
    const bool ok = u < UNITS && nt0 + t + (PAIR ? 1 : 0) < NTt;
    (void)ok;                                   // out-of-range units are never stored: clamp, no branch
    const int N = NTt * 16;
    const int c0 = min((nt0 + t) * 16 + (lane & 15), N - 1), c1 = min(c0 + 16, N - 1);
    p.s0[o] = sw[c0];
    p.s1[o] = PAIR ? sw[c1] : 0.f;
    const bf16_t* bp = bias != nullptr ? bias : g_zero_bf16;   // absent bias: read a zero word
    p.b0[o] = bf2f(bp[bias != nullptr ? c0 : 0]);
    p.b1[o] = PAIR ? bf2f(bp[bias != nullptr ? c1 : 0]) : 0.f;
  }
  return p;
}

// Reduce the KW partial fragments in `red` ([KW][NTW*MB][64] v4i) and write the outputs.
// sa: per-token scales (A_TOKEN; may point to LDS), unused when SCALED.  EPI_GLUQ needs every
// wave to arrive (it holds a workgroup barrier).
template <int MB, int NTW, int NW, int KW, bool SCALED, int EPI, int OWN>
__device__ __forceinline__ void gemv_epilogue(const v4i* __restrict__ red, const float* sa, const EpiPre<OWN>& pre,
                                              void* __restrict__ outv, float* __restrict__ os, float (*gmax)[4][16],
                                              int M, int N, int NTt, int Mpad, int nt0, int wave, int lane, int ks = 0) {
  constexpr int F = NTW * MB;
  auto total = [&](int f) -> v4i {
    if constexpr (SCALED) {
      v4f s = __builtin_bit_cast(v4f, red[f * 64 + lane]);
#pragma unroll
      for (int w = 1; w < KW; ++w) s += __builtin_bit_cast(v4f, red[(w * F + f) * 64 + lane]);
      return __builtin_bit_cast(v4i, s);
    } else {
      v4i s = red[f * 64 + lane];
#pragma unroll
      for (int w = 1; w < KW; ++w) s += red[(w * F + f) * 64 + lane];
      return s;
    }
  };
  if constexpr (EPI == EPI_PART) {
    float* part = reinterpret_cast<float*>(outv) + (size_t)ks * M * N;
#pragma unroll
    for (int o = 0; o < OWN; ++o) {
      const int f = wave + o * NW;
      const int t = f / MB, i = f % MB;
      if (f >= F || nt0 + t >= NTt) continue;
      const v4i tot = total(f);
      const int col = (nt0 + t) * 16 + (lane & 15);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = i * 16 + 4 * (lane >> 4) + q;
        if (row < M && col < N) {
          const float v = SCALED ? __builtin_bit_cast(v4f, tot)[q] : (float)tot[q] * sa[row];
          part[(size_t)row * N + col] = v * pre.s0[o] + (ks == 0 ? pre.b0[o] : 0.f);
        }
      }
    }
  } else if constexpr (EPI == EPI_OUT) {
    bf16_t* out = reinterpret_cast<bf16_t*>(outv);
    // os, unused by this epilogue, may carry a bf16 addend [M, N] (the other branch of a parallel-
    // residual block): out = bf16(bf16(y) + addend), the unfused bf16 add's value
    const bf16_t* add = reinterpret_cast<const bf16_t*>(os);
#pragma unroll
    for (int o = 0; o < OWN; ++o) {
      const int f = wave + o * NW;
      const int t = f / MB, i = f % MB;
      if (f >= F || nt0 + t >= NTt) continue;
      const v4i tot = total(f);
      const int col = (nt0 + t) * 16 + (lane & 15);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = i * 16 + 4 * (lane >> 4) + q;
        if (row < M && col < N) {
          float v = SCALED ? __builtin_bit_cast(v4f, tot)[q] : (float)tot[q] * sa[row];
          v = v * pre.s0[o] + pre.b0[o];
          if (add != nullptr) v = bf2f(f2bf(v)) + bf2f(add[(size_t)row * N + col]);
          out[(size_t)row * N + col] = f2bf(v);
        }
      }
    }
  } else if constexpr (EPI == EPI_GELUQT || EPI == EPI_GELUQE) {
    // unit (tile t, row block i): gelu of the bf16-rounded output (the unfused GEMM's), row maxima
    // over the tile's 16 columns to LDS, one barrier, then each row's scale over the workgroup's
    // 4 tiles (= one 64-column group; N % 64 == 0) and the int8 store
    float h[OWN][4];
    bool owner[OWN];
    int tt[OWN], ii[OWN];
#pragma unroll
    for (int o = 0; o < OWN; ++o) {
      const int f = wave + o * NW;
      const bool live = f < F;
      const int t = live ? f / MB : 0, i = live ? f % MB : 0;
      tt[o] = t;
      ii[o] = i;
      owner[o] = live && nt0 + t < NTt;
#pragma unroll
      for (int q = 0; q < 4; ++q) h[o][q] = 0.f;
      if (owner[o]) {
        const v4i tot = total(f);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int row = i * 16 + 4 * (lane >> 4) + q;
          const float v = (float)tot[q] * (row < M ? sa[row] : 0.f) * pre.s0[o] + pre.b0[o];
          const float a = bf2f(f2bf(v));
          float g;
          if constexpr (EPI == EPI_GELUQT) g = 0.5f * a * (1.f + tanhf(0.7978845608028654f * (a + 0.044715f * a * a * a)));
          else g = 0.5f * a * (1.f + erff(a * 0.7071067811865476f));
          h[o][q] = bf2f(f2bf(g));            // the unfused activation output is bf16
          float m = fabsf(h[o][q]);
#pragma unroll
          for (int d = 1; d < 16; d <<= 1) m = fmaxf(m, __shfl_xor(m, d, 64));
          if ((lane & 15) == 0) gmax[i][t][4 * (lane >> 4) + q] = m;
        }
      }
    }
    __syncthreads();
    int8_t* hq = reinterpret_cast<int8_t*>(outv);
    const int grp = nt0 / 4;
#pragma unroll
    for (int o = 0; o < OWN; ++o) {
      if (!owner[o]) continue;
      const int t = tt[o], i = ii[o];
      const int col = (nt0 + t) * 16 + (lane & 15);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int rr = 4 * (lane >> 4) + q, row = i * 16 + rr;
        const float amax = fmaxf(fmaxf(fmaxf(gmax[i][0][rr], gmax[i][1][rr]), fmaxf(gmax[i][2][rr], gmax[i][3][rr])), 1e-8f);
        if (row < M) hq[(size_t)row * N + col] = quant_i8(h[o][q], 127.f / amax);
        if (t == 0 && (lane & 15) == 0 && row < Mpad) os[(size_t)grp * Mpad + row] = row < M ? amax / 127.f : 0.f;
      }
    }
  } else {
    // pair p = (gate tile 2p, up tile 2p+1) -> feature (nt0/2 + p) * 16 + (lane & 15); a wave owns
    // pairs wave, wave + NW, ...  EPI_GLUQ: every owned pair's row maxima reach LDS before the
    // single barrier, then each 64-feature group (4 pairs) is quantised with one scale per row
    const int Fo = N / 2;
    constexpr int NP = NTW / 2 * MB;
    float h[OWN][4];
    bool owner[OWN];
    int pp[OWN], ii[OWN];
#pragma unroll
    for (int o = 0; o < OWN; ++o) {
      const int pf = wave + o * NW;
      const bool live = pf < NP;
      const int p = live ? pf / MB : 0, i = live ? pf % MB : 0;
      pp[o] = p;
      ii[o] = i;
      owner[o] = live && nt0 + 2 * p + 1 < NTt;
      const int feat = (nt0 / 2 + p) * 16 + (lane & 15);
#pragma unroll
      for (int q = 0; q < 4; ++q) h[o][q] = 0.f;
      if (owner[o]) {
        const v4i g4 = total((2 * p) * MB + i), u4 = total((2 * p + 1) * MB + i);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int row = i * 16 + 4 * (lane >> 4) + q;
          const float s_a = row < M ? sa[row] : 0.f;
          float g = (float)g4[q] * s_a * pre.s0[o] + pre.b0[o];
          float u = (float)u4[q] * s_a * pre.s1[o] + pre.b1[o];
          g = bf2f(f2bf(g));                // the unfused GEMM output is bf16
          u = bf2f(f2bf(u));
          h[o][q] = g / (1.f + __expf(-g)) * u;
          if constexpr (EPI == EPI_GLU)
            if (row < M) reinterpret_cast<bf16_t*>(outv)[(size_t)row * Fo + feat] = f2bf(h[o][q]);
        }
        if constexpr (EPI == EPI_GLUQ) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            float m = fabsf(h[o][q]);
#pragma unroll
            for (int d = 1; d < 16; d <<= 1) m = fmaxf(m, __shfl_xor(m, d, 64));
            if ((lane & 15) == 0) gmax[i][p][4 * (lane >> 4) + q] = m;
          }
        }
      }
    }
    if constexpr (EPI == EPI_GLUQ) {
      __syncthreads();
      int8_t* hq = reinterpret_cast<int8_t*>(outv);
      const int grp = nt0 / 8;
#pragma unroll
      for (int o = 0; o < OWN; ++o) {
        if (!owner[o]) continue;
        const int p = pp[o], i = ii[o];
        const int feat = (nt0 / 2 + p) * 16 + (lane & 15);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int rr = 4 * (lane >> 4) + q, row = i * 16 + rr;
          const float amax = fmaxf(fmaxf(fmaxf(gmax[i][0][rr], gmax[i][1][rr]), fmaxf(gmax[i][2][rr], gmax[i][3][rr])), 1e-8f);
          if (row < M) hq[(size_t)row * Fo + feat] = quant_i8(h[o][q], 127.f / amax);
          if (p == 0 && (lane & 15) == 0 && row < Mpad) os[(size_t)grp * Mpad + row] = row < M ? amax / 127.f : 0.f;
        }
      }
    }
  }
}

// Decode RMSNorm prologue (NRM > 0, M <= 4 rows): the activation rows are not an input but the
// RMSNorm of the previous split-K projection's fp32 partial slices plus the residual, quantised
// per token (rowwise.hip norm_kernel<PART, HAS_RES, QUANT> moved into the consumer: one launch
// fewer per norm, and the first weight steps are in flight while the rows are normalised).  The
// 1024 threads form four 256-thread groups, one row each; a group runs the norm kernel's
// exact element layout and reduction order (NCH chunks of 8 per thread), so the int8 rows and
// their scales are bit-identical.  Workgroup 0 writes the new residual rows.
struct NormIn {
  const float* part;      // [S][M][K] fp32 slices
  const bf16_t* res;      // [M][K] residual in
  const bf16_t* gamma;    // [K]
  bf16_t* res_out;        // [M][K] residual out (must not alias res: other workgroups still read it)
  float eps;
  int S;
  const bf16_t* x = nullptr;      // LN (NRM >= 64): [M][K] bf16 input rows, LayerNorm of x + res
  const bf16_t* beta = nullptr;   // LN: [K] (may be null)
  float thr = 0.f;                // LLM.int8 (NRM >= 128): outlier threshold on |x|
  const int8_t* wt = nullptr;     // LLM.int8: int8 W^T [K][N] (an outlier column is one row)
  const float* scb = nullptr;     // LLM.int8: per-row weight absmax SCB [N]
  bf16_t* y_out = nullptr;        // LLM.int8 of a normed row: the normalised row too (may be null)
};
constexpr int NRM_ROWS = 4;
constexpr int L8_CMAX = 256;      // LLM.int8 outlier columns per row held in LDS (llmint8.hip's cap)

// The prologue's global loads (slices, residual, gamma) are issued by norm_load BEFORE the
// weight stream and consumed by norm_prologue after it is issued: a wave's loads retire in issue
// order, so prologue loads queued behind the weights would wait for the whole stream and leave
// the norm, the MFMAs and the epilogue as a tail after the last weight byte.
template <int NCH, int SMAX>
struct NormRegs {
  uint4 rv[NCH];
  float4 pv[NCH][SMAX][2];                                // S <= SMAX slices (register budget)
  uint4 gv[NCH];
};

template <int NCH, int SMAX>
__device__ __forceinline__ void norm_load_now(const NormIn& na, int H, int M, NormRegs<NCH, SMAX>& r) {
  const int t = threadIdx.x & 255, row = threadIdx.x >> 8;
  if (row < M) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int e = min((c * 256 + t) * 8, H - 8);
      r.rv[c] = na.res != nullptr ? *reinterpret_cast<const uint4*>(na.res + (size_t)row * H + e)
                                  : uint4{0u, 0u, 0u, 0u};                 // no residual (a stage's first norm)
#pragma unroll
      for (int k = 0; k < SMAX; ++k)
        if (k < na.S) {
          const float4* p = reinterpret_cast<const float4*>(na.part + ((size_t)k * M + row) * H + e);
          r.pv[c][k][0] = p[0];
          r.pv[c][k][1] = p[1];
        }
      if constexpr (NCH * SMAX <= 4) r.gv[c] = *reinterpret_cast<const uint4*>(na.gamma + e);
    }
  }
}

// hoisted while NCH x SMAX <= 4 (K = 4096 with up to 2 slices, K = 2048 with up to 4); K = 4096
// with 3-4 slices would spill, so those load in the prologue
template <int NCH, int SMAX>
__device__ __forceinline__ void norm_load(const NormIn& na, int H, int M, NormRegs<NCH, SMAX>& r) {
  if constexpr (NCH * SMAX <= 4) {
    norm_load_now(na, H, M, r);
    asm volatile("" ::: "memory");                        // these loads issue before the weights
  }
}

template <int NCH, int SMAX>
__device__ __forceinline__ void norm_prologue(const NormIn& na, int H, int M, int8_t* aq, float* nsa, float* nred,
                                              const NormRegs<NCH, SMAX>& held) {
  const int t = threadIdx.x & 255, g = threadIdx.x >> 8, w = t >> 6;
  {                                                       // one pass: M <= NRM_ROWS = 4
    const int row = g;
    const bool act = row < M;
    float v[NCH][8];
    float ss = 0.f, amax = 0.f;
    if (act) {
      NormRegs<NCH, SMAX> late;                           // 3-4 slices: loaded here, as late as possible
      if constexpr (NCH * SMAX > 4) norm_load_now(na, H, M, late);
      const NormRegs<NCH, SMAX>& regs = NCH * SMAX > 4 ? late : held;
      const uint4* rv = regs.rv;
      const auto& pv = regs.pv;
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const int e = (c * 256 + t) * 8;
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] = 0.f;
#pragma unroll
        for (int k = 0; k < SMAX; ++k)
          if (k < na.S) {
            const float4 p0 = pv[c][k][0], p1 = pv[c][k][1];
            v[c][0] += p0.x; v[c][1] += p0.y; v[c][2] += p0.z; v[c][3] += p0.w;
            v[c][4] += p1.x; v[c][5] += p1.y; v[c][6] += p1.z; v[c][7] += p1.w;
          }
        if (e < H) {
          unpack8(pack8(v[c]), v[c]);                       // the projection's bf16 output
          float r[8];
          unpack8(rv[c], r);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[c][j] += r[j];
          const uint4 u = pack8(v[c]);                      // residual stream in bf16
          if (blockIdx.x == 0) *reinterpret_cast<uint4*>(na.res_out + (size_t)row * H + e) = u;
          unpack8(u, v[c]);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[c][j] = 0.f;
        }
      }
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const int e = (c * 256 + t) * 8;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = (e < H) ? v[c][j] - 0.f : 0.f;
          ss += d * d;
        }
      }
      ss = wave_sum(ss);
      if ((t & 63) == 0) nred[4 * g + w] = ss;
    }
    __syncthreads();
    const float* gr = nred + 4 * g;
    const float rstd = rsqrtf((((0.f + gr[0]) + gr[1]) + gr[2] + gr[3]) / (float)H + na.eps);
    __syncthreads();
    if (act) {
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const int e = (c * 256 + t) * 8;
        if (e < H) {
          float wf[8];
          unpack8(NCH * SMAX <= 4 ? held.gv[c] : *reinterpret_cast<const uint4*>(na.gamma + min(e, H - 8)), wf);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[c][j] = (v[c][j] - 0.f) * rstd * wf[j];
        }
      }
#pragma unroll
      for (int c = 0; c < NCH; ++c)
#pragma unroll
        for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(v[c][j]));
      amax = wave_max(amax);
      if ((t & 63) == 0) nred[4 * g + w] = amax;
    }
    __syncthreads();
    float gm = -INFINITY;
#pragma unroll
    for (int i = 0; i < 4; ++i) gm = fmaxf(gm, gr[i]);
    gm = fmaxf(gm, 1e-8f);
    const float inv = 127.f / gm;
    if (act && t == 0) nsa[row] = gm / 127.f;
    if (act) {
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const int e = (c * 256 + t) * 8;
        if (e < H) {
          uint32_t lo = 0, hi = 0;
#pragma unroll
          for (int j = 0; j < 4; ++j) lo |= ((uint32_t)(uint8_t)quant_i8(v[c][j], inv)) << (8 * j);
#pragma unroll
          for (int j = 0; j < 4; ++j) hi |= ((uint32_t)(uint8_t)quant_i8(v[c][4 + j], inv)) << (8 * j);
          *reinterpret_cast<uint2*>(aq + (size_t)row * H + e) = make_uint2(lo, hi);
        }
      }
    }
    __syncthreads();                                      // aq complete
  }
}

// LayerNorm prologue (NRM >= 64: the parallel-residual decoders, GPT-NeoX / Phi): the LayerNorm of
// the bf16 rows x + residual, int8 per token, with norm_kernel<NCH, !RMS, HAS_RES, QUANT, !PART>'s
// element layout, reduction order and roundings (bit-identical rows and scales).  Its loads issue
// before the weight stream (ln_load), like the RMS form's.
template <int NCH>
struct LnRegs {
  uint4 xv[NCH], rv[NCH], gv[NCH], bv[NCH];
};

template <int NCH>
__device__ __forceinline__ void ln_load(const NormIn& na, int H, int M, LnRegs<NCH>& r) {
  const int t = threadIdx.x & 255, row = threadIdx.x >> 8;
  if (row < M) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int e = min((c * 256 + t) * 8, H - 8);
      r.xv[c] = *reinterpret_cast<const uint4*>(na.x + (size_t)row * H + e);
      r.rv[c] = na.res != nullptr ? *reinterpret_cast<const uint4*>(na.res + (size_t)row * H + e) : uint4{0u, 0u, 0u, 0u};
      r.gv[c] = *reinterpret_cast<const uint4*>(na.gamma + e);
      r.bv[c] = na.beta != nullptr ? *reinterpret_cast<const uint4*>(na.beta + e) : uint4{0u, 0u, 0u, 0u};
    }
  }
  asm volatile("" ::: "memory");                          // these loads issue before the weights
}

template <int NCH>
__device__ __forceinline__ void ln_prologue(const NormIn& na, int H, int M, int8_t* aq, float* nsa, float* nred,
                                            const LnRegs<NCH>& r) {
  const int t = threadIdx.x & 255, row = threadIdx.x >> 8, w = t >> 6;
  const bool act = row < M;
  float v[NCH][8];
  float sm = 0.f;
  if (act) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int e = (c * 256 + t) * 8;
      if (e < H) {
        unpack8(r.xv[c], v[c]);
        float rr[8];
        unpack8(r.rv[c], rr);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] += rr[j];
        const uint4 u = pack8(v[c]);                          // residual stream in bf16
        if (blockIdx.x == 0) *reinterpret_cast<uint4*>(na.res_out + (size_t)row * H + e) = u;
        unpack8(u, v[c]);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] = 0.f;
      }
    }
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int j = 0; j < 8; ++j) sm += v[c][j];
    sm = wave_sum(sm);
    if ((t & 63) == 0) nred[4 * row + w] = sm;
  }
  __syncthreads();
  const float* gr = nred + 4 * (row < NRM_ROWS ? row : 0);
  const float mean = ((((0.f + gr[0]) + gr[1]) + gr[2]) + gr[3]) / (float)H;
  float ss = 0.f;
  if (act) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int e = (c * 256 + t) * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = (e < H) ? v[c][j] - mean : 0.f;
        ss += d * d;
      }
    }
    ss = wave_sum(ss);
  }
  __syncthreads();
  if (act && (t & 63) == 0) nred[4 * row + w] = ss;
  __syncthreads();
  const float rstd = rsqrtf(((((0.f + gr[0]) + gr[1]) + gr[2]) + gr[3]) / (float)H + na.eps);
  __syncthreads();
  float amax = 0.f;
  if (act) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int e = (c * 256 + t) * 8;
      if (e < H) {
        float wf[8], bf[8];
        unpack8(r.gv[c], wf);
        unpack8(r.bv[c], bf);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] = (v[c][j] - mean) * rstd * wf[j] + bf[j];
      }
    }
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(v[c][j]));
    amax = wave_max(amax);
    if ((t & 63) == 0) nred[4 * row + w] = amax;
  }
  __syncthreads();
  float gm = -INFINITY;
#pragma unroll
  for (int i = 0; i < 4; ++i) gm = fmaxf(gm, gr[i]);
  gm = fmaxf(gm, 1e-8f);
  const float inv = 127.f / gm;
  if (act && t == 0) nsa[row] = gm / 127.f;
  if (act) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int e = (c * 256 + t) * 8;
      if (e < H) {
        uint32_t lo = 0, hi = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) lo |= ((uint32_t)(uint8_t)quant_i8(v[c][j], inv)) << (8 * j);
#pragma unroll
        for (int j = 0; j < 4; ++j) hi |= ((uint32_t)(uint8_t)quant_i8(v[c][4 + j], inv)) << (8 * j);
        *reinterpret_cast<uint2*>(aq + (size_t)row * H + e) = make_uint2(lo, hi);
      }
    }
  }
  __syncthreads();                                        // aq complete
}

// LLM.int8 prologue (NRM >= 128, one row): llmint8.hip's decode preparation inside the GEMV, so a
// batch-1 LLM.int8 projection is one launch instead of three (prep, GEMV, outlier add).  Threads
// 0-255 hold the row in norm_prologue's layout (column (c 256 + t) 8 + j); columns with |x| > thr
// are ranked in column order by a block prefix sum per chunk, the first L8_CMAX go to LDS (index,
// value); the per-token absmax over the other columns, then int8 x with the taken columns zeroed.
// The epilogue adds sum_j x[c_j] W^T[c_j][n] SCB[n] / 127 to the rounded output, in llmint8.hip's
// order and roundings: the output bits equal prep + GEMV + outlier kernel.
// SRC 1 / 2 (NRM = 192 + 8 NCH + SRC): the row is first the RMSNorm / LayerNorm of x + residual
// (norm_kernel's HAS_RES path, rounded to bf16 as its output), so an LLM.int8 layer's norm is no
// launch of its own either; workgroup 0 writes the new residual row and, when y_out is set, the
// normalised row (for a second consumer).
template <int NCH, int SRC>
struct L8Regs {
  uint4 xv[NCH];
  uint4 rv[SRC ? NCH : 1], gv[SRC ? NCH : 1], bv[SRC == 2 ? NCH : 1];
};

template <int NCH, int SRC>
__device__ __forceinline__ void l8_load(const NormIn& na, int H, L8Regs<NCH, SRC>& r) {
  const int t = threadIdx.x;
  if (t < 256) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int e = min((c * 256 + t) * 8, H - 8);
      r.xv[c] = *reinterpret_cast<const uint4*>(na.x + e);
      if constexpr (SRC > 0) {
        r.rv[c] = na.res != nullptr ? *reinterpret_cast<const uint4*>(na.res + e) : uint4{0u, 0u, 0u, 0u};
        r.gv[c] = *reinterpret_cast<const uint4*>(na.gamma + e);
      }
      if constexpr (SRC == 2)
        r.bv[c] = na.beta != nullptr ? *reinterpret_cast<const uint4*>(na.beta + e) : uint4{0u, 0u, 0u, 0u};
    }
  }
  asm volatile("" ::: "memory");                          // these loads issue before the weights
}

template <int NCH, int SRC>
__device__ __forceinline__ void l8_prologue(const NormIn& na, int H, int8_t* aq, float* nsa, float* nred, int* cols,
                                            float* xo, int* scr, const L8Regs<NCH, SRC>& r, bf16_t* y_out) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const bool act = t < 256;
  float v[NCH][8];
  if (act) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) unpack8(r.xv[c], v[c]);
  }
  if constexpr (SRC > 0) {
    float sm = 0.f;
    if (act) {
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const int e = (c * 256 + t) * 8;
        if (e < H) {
          float rr[8];
          unpack8(r.rv[c], rr);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[c][j] += rr[j];
          const uint4 u = pack8(v[c]);                      // residual stream in bf16
          if (blockIdx.x == 0) *reinterpret_cast<uint4*>(na.res_out + e) = u;
          unpack8(u, v[c]);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[c][j] = 0.f;
        }
      }
      if constexpr (SRC == 2) {
#pragma unroll
        for (int c = 0; c < NCH; ++c)
#pragma unroll
          for (int j = 0; j < 8; ++j) sm += v[c][j];
        sm = wave_sum(sm);
        if (lane == 0) nred[w] = sm;
      }
    }
    float mean = 0.f;
    if constexpr (SRC == 2) {
      __syncthreads();
      mean = ((((0.f + nred[0]) + nred[1]) + nred[2]) + nred[3]) / (float)H;
      __syncthreads();
    }
    float ss = 0.f;
    if (act) {
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const int e = (c * 256 + t) * 8;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = (e < H) ? v[c][j] - mean : 0.f;
          ss += d * d;
        }
      }
      ss = wave_sum(ss);
      if (lane == 0) nred[w] = ss;
    }
    __syncthreads();
    const float rstd = rsqrtf(((((0.f + nred[0]) + nred[1]) + nred[2]) + nred[3]) / (float)H + na.eps);
    __syncthreads();                                      // nred is reused below
    if (act) {
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const int e = (c * 256 + t) * 8;
        if (e < H) {
          float wf[8], bf[8];
          unpack8(r.gv[c], wf);
          if constexpr (SRC == 2) unpack8(r.bv[c], bf);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float tv = (v[c][j] - mean) * rstd * wf[j];
            if constexpr (SRC == 2) tv += bf[j];
            v[c][j] = tv;
          }
          const uint4 u = pack8(v[c]);                      // the norm's bf16 output row
          if (y_out != nullptr && blockIdx.x == 0) *reinterpret_cast<uint4*>(y_out + e) = u;
          unpack8(u, v[c]);
        }
      }
    }
  }
  uint32_t take[NCH];
  int base = 0;                                           // outliers in the chunks before c
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int e = (c * 256 + (act ? t : 0)) * 8;
    uint32_t bits = 0;
    if (act) {
      if (e < H) {
#pragma unroll
        for (int j = 0; j < 8; ++j) bits |= (fabsf(v[c][j]) > na.thr ? 1u : 0u) << j;
      }
    }
    const int pc = __popc(bits);
    int incl = pc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int tt = __shfl_up(incl, o, 64);
      if (lane >= o) incl += tt;
    }
    if (act && lane == 63) scr[w] = incl;                 // wave totals of this chunk
    __syncthreads();
    int wb = base;
    if (act) {
      for (int i = 0; i < w; ++i) wb += scr[i];
    }
    const int tot = scr[0] + scr[1] + scr[2] + scr[3];
    __syncthreads();                                      // scr reused by the next chunk
    uint32_t tk = 0;
    if (act) {
      int slot = wb + incl - pc;
#pragma unroll
      for (int j = 0; j < 8; ++j) {                       // (static indices: v stays in registers)
        if ((bits >> j) & 1u) {
          if (slot < L8_CMAX) {
            cols[slot] = e + j;
            xo[slot] = v[c][j];
            tk |= 1u << j;
          }
          ++slot;
        }
      }
    }
    take[c] = tk;
    base += tot;
  }
  if (t == 0) scr[8] = min(base, L8_CMAX);
  float am = 0.f;
  if (act) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int e = (c * 256 + t) * 8;
      if (e < H) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (!((take[c] >> j) & 1u)) am = fmaxf(am, fabsf(v[c][j]));
      }
    }
    am = wave_max(am);
    if (lane == 0) nred[w] = am;
  }
  __syncthreads();
  const float rm = fmaxf(fmaxf(fmaxf(fmaxf(0.f, nred[0]), nred[1]), nred[2]), nred[3]);
  const float gm = fmaxf(rm, 1e-8f);
  if (t == 0) nsa[0] = gm / 127.f;
  const float inv = 127.f / gm;
  if (act) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int e = (c * 256 + t) * 8;
      if (e < H) {
        uint32_t lo = 0, hi = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          lo |= ((uint32_t)(uint8_t)((take[c] >> j) & 1u ? 0 : quant_i8(v[c][j], inv))) << (8 * j);
#pragma unroll
        for (int j = 0; j < 4; ++j)
          hi |= ((uint32_t)(uint8_t)((take[c] >> (4 + j)) & 1u ? 0 : quant_i8(v[c][4 + j], inv))) << (8 * j);
        *reinterpret_cast<uint2*>(aq + e) = make_uint2(lo, hi);
      }
    }
  }
  __syncthreads();                                        // aq, cols, xo, the count complete
}

template <int MB, int NTW, int TG, int KW, int U, int AMODE, int EPI, int NRM = 0>
__global__ void __launch_bounds__(TG * KW * 64) w8a8_gemv_kernel(const int8_t* __restrict__ A, const float* __restrict__ sa,
                                                                 const int8_t* __restrict__ Wp, const float* __restrict__ sw,
                                                                 const bf16_t* __restrict__ bias, void* __restrict__ outv,
                                                                 float* __restrict__ os, int M, int N, int K, int KT,
                                                                 int NTt, int Mpad, int S, NormIn na) {
  constexpr int NW = TG * KW, TPW = NTW / TG;
  static_assert(NTW % TG == 0, "tiles split evenly over tile groups");
  static_assert(NRM == 0 || (MB == 1 && AMODE == A_TOKEN && EPI != EPI_PART && NW == 16), "norm prologue: batch 1");
  // NRM: the int8 activation row lives in LDS (norm_prologue), its per-token scale in nsa[0]
  // NRM = 8 * NCH + SMAX (norm_prologue<NCH, SMAX>)
  constexpr bool L8_N = NRM >= 128;                          // LLM.int8 preparation (+ 128) ...
  constexpr int L8SRC_N = NRM >= 192 ? NRM % 8 : 0;          // ... of a normed row (+ 192 + 1 RMS / 2 LN
  constexpr int L8S_N = L8SRC_N & 3;                         //     (+ 4: SwiGLU of [gate | up] tiles)
  constexpr bool L8G_N = (L8SRC_N & 4) != 0;
  constexpr int L8ACT_N = NRM >= 256 ? (NRM - 256) / 64 + 1 : 0;   // + 256 (+ 64): gelu tanh (erf) epilogue
  constexpr bool LN_N = NRM >= 64 && !L8_N;                  // LayerNorm of bf16 rows (+ 64)
  constexpr int NCH_N = (NRM % 64) / 8, SMAX_N = LN_N || L8_N ? 1 : NRM % 8;
  static_assert(!L8_N || (EPI == EPI_OUT && MB == 1), "LLM.int8 prologue: one row, plain output");
  __shared__ int l8_cols[L8_N ? L8_CMAX : 1];
  __shared__ float l8_xo[L8_N ? L8_CMAX : 1];
  __shared__ int l8_scr[16];
  __shared__ int8_t aq_l[NRM > 0 ? NRM_ROWS * NCH_N * 2048 : 16];
  __shared__ float nsa[16], nred[16];
  constexpr bool GELUQ = EPI == EPI_GELUQT || EPI == EPI_GELUQE;
  static_assert(EPI == EPI_OUT || EPI == EPI_PART || (AMODE == A_TOKEN && (GELUQ || TPW % 2 == 0)),
                "GLU: gate/up pairs per wave, per-token A");
  static_assert(EPI != EPI_GLUQ || NTW == 8, "quantising GLU: 64 features per workgroup");
  static_assert(!GELUQ || NTW == 4, "quantising GELU: 64 columns per workgroup");
  // LDS reduction buffer: one partial set per k-wave, or per pair of k-waves when that would
  // exceed 128 KiB (the upper half adds into the lower half first)
  constexpr int KR = KW * NTW * MB * 1024 <= 131072 ? KW : KW / 2;
  static_assert(KR * NTW * MB * 1024 <= 131072 && KW % KR == 0 && KW / KR <= 2, "LDS reduction budget");
  constexpr bool SCALED = AMODE == A_GROUP;
  __shared__ v4i red[KR][NTW * MB][64];
  __shared__ float gmax[MB][4][16];
  // EPI_PART (split-K): workgroup (group, s) reduces k-tiles [KT*s/S, KT*(s+1)/S) of its tiles and
  // writes fp32 partial sums part[s][M][N]; the consumer (norm kernel) adds the S slices in order
  const int grp = EPI == EPI_PART ? (int)blockIdx.x / S : (int)blockIdx.x;
  const int ks = EPI == EPI_PART ? (int)blockIdx.x % S : 0;
  const int kbeg = EPI == EPI_PART ? (int)((int64_t)KT * ks / S) : 0;
  const int kend = EPI == EPI_PART ? (int)((int64_t)KT * (ks + 1) / S) : KT;
  // L8G (SwiGLU, natural [gate | up] rows): the workgroup's 2 tiles are gate tile grp and up tile grp + NTt / 2
  const int nt0 = L8G_N ? grp : grp * NTW;
  static_assert(!L8G_N || (NTW == 2 && TG == 1), "LLM.int8 SwiGLU: one gate + one up tile per workgroup");
  // wave index in an SGPR: every k-loop guard below is then a scalar branch (an MFMA must never
  // sit under an EXEC-masked branch — it ignores EXEC and would add a clamped duplicate k-tile)
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tg = wave / KW, kw = wave % KW, t0 = tg * TPW;
  const int akc = 16 * (lane >> 4);

  const v4i* wp[TPW];
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    const int nt = L8G_N ? (j == 0 ? nt0 : nt0 + NTt / 2) : min(nt0 + t0 + j, NTt - 1);
    wp[j] = reinterpret_cast<const v4i*>(Wp + ((size_t)nt * KT) * 1024) + lane;
  }
  const int8_t* ap[MB];
#pragma unroll
  for (int i = 0; i < MB; ++i)
    ap[i] = (NRM > 0 ? aq_l : A) + (size_t)min(i * 16 + (lane & 15), M - 1) * K;
  const bool kfull = NRM > 0 || (K & 63) == 0;
  const auto pre = epi_preload<MB, NTW, NW, EPI>(sw, bias, nt0, NTt, wave, lane);
  v4i acc[TPW][MB];
  v4f accf[TPW][MB];
#pragma unroll
  for (int j = 0; j < TPW; ++j)
#pragma unroll
    for (int i = 0; i < MB; ++i) { acc[j][i] = v4i{0, 0, 0, 0}; accf[j][i] = v4f{0.f, 0.f, 0.f, 0.f}; }

  struct Step {
    v4i b[U][TPW];
    v4i a[U][MB];
    v4f sg[U][MB];
  };
  // one step = U k-tiles: weight fragments (nontemporal), activation fragments and (SCALED)
  // per-group scales; clamped addresses, no branches
  auto issue_w = [&](Step& st, int kbase) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < TPW; ++j)
        st.b[u][j] = __builtin_nontemporal_load(wp[j] + (size_t)min(kbase + u * KW, kend - 1) * 64);
  };
  auto issue_a = [&](Step& st, int kbase) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = min(kbase + u * KW, kend - 1);
#pragma unroll
      for (int i = 0; i < MB; ++i) {
        if (kfull) st.a[u][i] = *reinterpret_cast<const v4i*>(ap[i] + k * 64 + akc);
        else st.a[u][i] = load_a_i8(ap[i], true, k, KT, akc, K, (K & 15) == 0);
        if constexpr (SCALED)
          st.sg[u][i] = *reinterpret_cast<const v4f*>(sa + (size_t)k * Mpad + min(i * 16, Mpad - 16) + 4 * (lane >> 4));
      }
    }
  };
  auto issue = [&](Step& st, int kbase) {
    issue_w(st, kbase);
    issue_a(st, kbase);
  };
  // NRM: the first step's weight loads go out before the norm prologue; its activations after
  NormRegs<(NRM > 0 && !LN_N && !L8_N ? NCH_N : 1), (NRM > 0 && !LN_N && !L8_N ? SMAX_N : 1)> nr;
  LnRegs<(LN_N ? NCH_N : 1)> lr;
  L8Regs<(L8_N ? NCH_N : 1), L8S_N> l8r;
  auto nload = [&]() {
    if constexpr (L8_N) l8_load(na, K, l8r);
    else if constexpr (LN_N) ln_load(na, K, M, lr);
    else norm_load(na, K, M, nr);
  };
  auto nprologue = [&]() {
    if constexpr (L8_N) l8_prologue(na, K, aq_l, nsa, nred, l8_cols, l8_xo, l8_scr, l8r, na.y_out);
    else if constexpr (LN_N) ln_prologue(na, K, M, aq_l, nsa, nred, lr);
    else norm_prologue(na, K, M, aq_l, nsa, nred, nr);
  };
  auto first = [&](Step& st, int kbase) {
    if constexpr (NRM > 0) {
      nload();
      issue_w(st, kbase);
      nprologue();
      issue_a(st, kbase);
    } else {
      issue(st, kbase);
    }
  };
  auto compute = [&](const Step& st, int kbase) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (kbase + u * KW < kend) {                       // wave-uniform tail guard
#pragma unroll
        for (int j = 0; j < TPW; ++j)
#pragma unroll
          for (int i = 0; i < MB; ++i) {
            if constexpr (SCALED) fold(accf[j][i], mfma_i8(st.a[u][i], st.b[u][j], v4i{0, 0, 0, 0}), st.sg[u][i]);
            else acc[j][i] = mfma_i8(st.a[u][i], st.b[u][j], acc[j][i]);
          }
      }
    }
  };
  // one step of U k-tiles per iteration: all its loads in flight, then its MFMAs.  The k range
  // lengths of the decode shapes (64, 32, 16 k-tiles) get a compile-time trip count, fully
  // unrolled, so the scheduler can hoist the next steps' loads above this step's MFMAs (a wave's
  // time is otherwise about one memory latency per step); other lengths take the runtime loop.
  auto fixed = [&](auto nk) {
    constexpr int NK = decltype(nk)::value, STEPS = (NK + KW * U - 1) / (KW * U);
    Step st[STEPS];
    if constexpr (NRM > 0 && STEPS <= 2 && NCH_N * SMAX_N <= 4 && (!L8_N || NCH_N <= (L8SRC_N ? 1 : 2))) {
      // batch-1 norm prologue: every step's weights (at most 2) in flight across it (K = 4096 with
      // 4 slices keeps one step: its prologue registers would spill)
      nload();
#pragma unroll
      for (int i = 0; i < STEPS; ++i) issue_w(st[i], kbeg + kw + i * KW * U);
      nprologue();
#pragma unroll
      for (int i = 0; i < STEPS; ++i) {
        issue_a(st[i], kbeg + kw + i * KW * U);
        compute(st[i], kbeg + kw + i * KW * U);
      }
      return;
    }
    first(st[0], kbeg + kw);
#pragma unroll
    for (int i = 0; i < STEPS; ++i) {                   // one step of lookahead, no register copies
      if (i + 1 < STEPS) issue(st[i + 1], kbeg + kw + (i + 1) * KW * U);
      compute(st[i], kbeg + kw + i * KW * U);
    }
  };
  // only where two steps plus the accumulators fit the register budget (measured: larger forms spill)
  constexpr int REG_EST = 2 * U * (TPW * 4 + MB * 4 * (SCALED ? 2 : 1)) + TPW * MB * 4;
  constexpr bool FIXED_OK = GEMV_UNROLL_FIXED && REG_EST <= (NW >= 16 ? 80 : 180) && (!SCALED || MB == 1);
  const int nk = kend - kbeg;
  if (FIXED_OK && nk == 64 && KW * U <= 64) fixed(std::integral_constant<int, 64>{});
  else if (FIXED_OK && nk == 32 && KW * U <= 32) fixed(std::integral_constant<int, 32>{});
  else if (FIXED_OK && nk == 16 && KW * U <= 16) fixed(std::integral_constant<int, 16>{});
  else if constexpr (NRM > 0) {
    // next step's weights in flight during this step's MFMAs (the loop below leaves that to the
    // scheduler; here the first step's weights are already loaded across the prologue)
    Step st;
    first(st, kbeg + kw);
    for (int kt = kbeg + kw; kt < kend; kt += KW * U) {
      Step nx;
      if (kt + KW * U < kend) issue_w(nx, kt + KW * U);
      compute(st, kt);
      if (kt + KW * U < kend) {
        issue_a(nx, kt + KW * U);
        st = nx;
      }
    }
  } else if constexpr (SCALED && MB <= 4 && 2 * REG_EST <= (NW >= 16 ? 160 : 360)) {
    // other k-range lengths (the down projection's 86 k-tiles per slice): one step of lookahead
    // in two named register sets, the loop run twice per iteration (no copies of a set with
    // loads outstanding).  Batch-1 down 11.6 us had three full memory round trips per wave here.
    // Grouped-scale inputs only (the model's o / down): cache-cold down at 64 rows 39.4 -> 34.3 us,
    // 1-32 rows unchanged; per-token inputs measured mixed (16 rows 14.5 -> 15.4 us), so they keep
    // the plain loop (profiles/gemv_lookahead_rows_r6.jsonl).
    Step s0, s1;
    int kt = kbeg + kw;
    if (kt < kend) issue(s0, kt);
    while (kt < kend) {
      const int k1 = kt + KW * U;
      if (k1 < kend) issue(s1, k1);
      compute(s0, kt);
      if (k1 >= kend) break;
      const int k2 = k1 + KW * U;
      if (k2 < kend) issue(s0, k2);
      compute(s1, k1);
      kt = k2;
    }
  } else {
    for (int kt = kbeg + kw; kt < kend; kt += KW * U) {
      Step st;
      issue(st, kt);
      compute(st, kt);
    }
  }
  if (KR == KW || kw >= KR) {
#pragma unroll
    for (int j = 0; j < TPW; ++j)
#pragma unroll
      for (int i = 0; i < MB; ++i)
        red[kw - (KW - KR)][(t0 + j) * MB + i][lane] = SCALED ? __builtin_bit_cast(v4i, accf[j][i]) : acc[j][i];
  }
  __syncthreads();
  if constexpr (KR != KW) {
    if (kw < KR) {
#pragma unroll
      for (int j = 0; j < TPW; ++j)
#pragma unroll
        for (int i = 0; i < MB; ++i) {
          v4i& r = red[kw][(t0 + j) * MB + i][lane];
          if constexpr (SCALED) r = __builtin_bit_cast(v4i, __builtin_bit_cast(v4f, r) + accf[j][i]);
          else r += acc[j][i];
        }
    }
    __syncthreads();
  }
  if constexpr (L8G_N) {
    // wave 0, lanes 0-15: gate and up columns of feature nt0 * 16 + lane, each as the plain L8
    // epilogue below computes it (bf16), then silu(g) * u as rowwise.hip act_kernel MODE 0 does
    if (wave == 0 && lane < 16) {
      const v4i* rb = &red[0][0][0];
      float gu[2];
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        int tot = rb[jj * 64 + lane][0];
#pragma unroll
        for (int w = 1; w < KR; ++w) tot += rb[(w * NTW + jj) * 64 + lane][0];
        const int col = (jj == 0 ? nt0 : nt0 + NTt / 2) * 16 + lane;
        float y = (float)tot * nsa[0];
        y = y * sw[col] + (bias != nullptr ? bf2f(bias[col]) : 0.f);
        const int nt = l8_scr[8];
        if (nt > 0) {
          float a = 0.f;
          for (int j = 0; j < nt; ++j) a += l8_xo[j] * (float)na.wt[(size_t)l8_cols[j] * N + col];
          const float s = na.scb[col] / 127.f;
          y = bf2f(f2bf(y)) + a * s;
        }
        gu[jj] = bf2f(f2bf(y));
      }
      const float g = gu[0], u = gu[1];
      reinterpret_cast<bf16_t*>(outv)[nt0 * 16 + lane] = f2bf(g / (1.f + __expf(-g)) * u);
    }
  } else if constexpr (L8_N) {
    // row 0 of each tile (lanes 0-15, q = 0): the int8 part as the EPI_OUT epilogue rounds it, then
    // the outlier columns' 16-bit part (llmint8.hip llmint8_outlier_kernel's sum order and rounding)
    if (wave < NTW && lane < 16 && nt0 + wave < NTt) {
      const v4i* rb = &red[0][0][0];
      int tot = rb[wave * 64 + lane][0];
#pragma unroll
      for (int w = 1; w < KR; ++w) tot += rb[(w * NTW + wave) * 64 + lane][0];
      const int col = (nt0 + wave) * 16 + lane;
      if (col < N) {
        float y = (float)tot * nsa[0];
        y = y * pre.s0[0] + pre.b0[0];
        const int nt = l8_scr[8];
        if (nt > 0) {
          float a = 0.f;
          for (int j = 0; j < nt; ++j) a += l8_xo[j] * (float)na.wt[(size_t)l8_cols[j] * N + col];
          const float s = na.scb[col] / 127.f;
          y = bf2f(f2bf(y)) + a * s;
        }
        if constexpr (L8ACT_N > 0) {                    // rowwise.hip act_kernel MODE 1 / 2 of the bf16 output
          const float a = bf2f(f2bf(y));
          if constexpr (L8ACT_N == 1) y = 0.5f * a * (1.f + tanhf(0.7978845608028654f * (a + 0.044715f * a * a * a)));
          else y = 0.5f * a * (1.f + erff(a * 0.7071067811865476f));
        }
        reinterpret_cast<bf16_t*>(outv)[col] = f2bf(y);
      }
    }
  } else {
    gemv_epilogue<MB, NTW, NW, KR, SCALED, EPI>(&red[0][0][0], NRM > 0 ? nsa : sa, pre, outv, os, gmax, M, N, NTt,
                                                Mpad, nt0, wave, lane, ks);
  }
}

// ------------------------------------------------------------------------------------ ring2
// 65-128 decode rows with DECOUPLED prefetch depths for the two operands.  Streaming weights from
// HBM at full rate needs ~2.5-4 us of loaded latency covered, while the activation re-reads are
// L2 hits.  In the one-ring kernel above most of the ~110 KiB in flight per CU is activation
// pieces, so only ~30 KiB of weights are in flight.  vmcnt retires a wave's loads in issue order,
// so one wave cannot keep a deep weight queue behind a shallow activation queue — separate waves
// can:
//   * NWL loader waves issue only weight tiles, DW = RW - 1 stages ahead (RW slots);
//   * 4 compute waves issue only activation pieces (whole 128-B lines: 8 rows x 128 B per piece),
//     DA = RA - 1 stages ahead, and own 2 row blocks x NTW tiles of accumulators each.
// A stage is two k-tiles.  One bare barrier per stage: every wave first waits (counted vmcnt) for
// its own DMA of stage s, then the barrier makes slot s visible to all and frees slot s - 1,
// which the next issue reuses.  Stages past the end re-load the last one (never read).
// Epilogues as the ring kernel (EPI_OUT bf16, EPI_GLUQ SwiGLU + per-64 int8, EPI_PART fp32 split-K
// slices); K % 128 == 0.  SC (per-(token, 64) activation scales, the o / down inputs): the loader
// waves also DMA each stage's scales (one 1 KiB piece: 2 k-tiles x Mpad rows, lanes split over the
// loader waves) into a third ring, and every k-tile's int32 MFMA result is folded in fp32.
// EPI_PART: blockIdx = group * S + slice; slice ks reduces stages [NS ks / S, NS (ks + 1) / S).
// Weights stream with the nontemporal cache policy (each byte is read once per step).
// ROT: the k order is rotated per workgroup (65-128-row split-K, where the ~256 workgroups would
// otherwise request the same activation lines at the same moment).
// MS == 2 (129-256 rows, one 256-row decode micro-batch): the rows are cut into two halves of at
// most 128 and each logical workgroup runs once per half.  The two halves of one weight panel are
// blocks b and b + 8: under the observed round-robin dispatch they share an XCD, and the second
// reader of a weight line finds it in that XCD's L2 (speed only: each half is a complete,
// independent computation).  Launch 16 * ceil(G / 8) blocks for G logical workgroups; surplus
// blocks exit.
// NAL > 0: NAL dedicated activation-loader waves issue every activation piece (DA stages ahead) and
// the compute waves only read LDS and run MFMAs.  With NAL == 0 the compute waves issue their own
// activation DMA, and at 128 rows x 6 tiles that DMA issue (the CU's texture path is busy with
// 28 KiB per stage) serialised with their MFMAs: ~1400 cycles per stage against ~470 of DMA and ~400
// of MFMA (tools/bench_ops.py --only rows256, qkv 22 us at M = 256).
// NCW == 8: eight compute waves (two per SIMD) as 4 (rows) x 2 (tiles), each with 2 row blocks x
// NTW / 2 tiles: the per-k-tile fold of the grouped scales (8 VALU per MFMA) then issues from two
// waves per SIMD beside the other wave's MFMAs instead of serialising behind one wave's own.
// (A restaged 16-B store epilogue — qkv's 12 x 8-B stores per lane as 6 x 16-B, gate_up's 8 x 4-B as
// 2 x 16-B — measured neutral at 256 rows, 22.74 vs 22.77 us / 34.65 vs 34.69: the tail is not
// store-issue bound here, so the direct per-fragment stores stay.)
template <int NTW, int NWL, int RW, int RA, int EPI, bool ROT = false, bool SC = false, int MS = 1, int NAL = 0,
          int NCW = 4, int DT = 0>
__global__ void __launch_bounds__((NCW + NWL + NAL) * 64, 1) w8a8_gemv_ring2_kernel(
    const int8_t* __restrict__ A, const float* __restrict__ sa, const int8_t* __restrict__ Wp,
    const float* __restrict__ sw, const bf16_t* __restrict__ bias, void* __restrict__ outv, float* __restrict__ os,
    int M, int N, int K, int NTt, int Mpad, int S = 1, int G = 0) {
  constexpr int MB = 8, WST = 2 * NTW, WPW = WST / NWL, DW = RW - 1, DA = RA - 1, APW = 16 / NCW;
  constexpr int NTH = NCW == 8 ? NTW / 2 : NTW;       // tiles per compute wave
  // GLUQ: a compute wave's tiles must be whole 64-feature quant groups (4 gate/up pairs): NTH == 8
  static_assert(NCW == 4 || (NCW == 8 && NTW % 2 == 0 && (EPI != EPI_GLUQ || NTW == 16)), "compute waves");
  constexpr int LPW = WPW + (SC ? 1 : 0);             // loader pieces per stage (+ the scale piece)
  static_assert(WST % NWL == 0, "weight pieces split evenly over the loader waves");
  static_assert(DW * LPW <= 63 && DA * APW <= 63 && DA >= 1, "vmcnt range");
  static_assert(EPI == EPI_OUT || EPI == EPI_PART || (EPI == EPI_GLUQ && NTH == 8 && !SC && DT == 0) ||
                (EPI == EPI_GLU && NTH % 2 == 0 && DT == 1), "epilogues");
  static_assert(DT != 1 || !SC, "bf16 operands carry no activation scales");
  static_assert(DT != 2 || SC, "the magic-number fold is a grouped-scale (SC) form");
  static_assert(MS == 1 || MS == 2, "row split");
  static_assert(NAL == 0 || (16 % NAL == 0 && DA * (16 / NAL) <= 63), "activation loaders");
  // + EPK KiB: the workgroup's weight scales and bias (fp32, EPC columns each), staged once for the epilogue
  constexpr int EPC = NTW * 16 <= 128 ? 128 : 256, EPK = EPC / 128;
  constexpr int LDS_KB = RW * WST + RA * 16 + (SC ? RW : 0) + EPK;
  static_assert(LDS_KB * 1024 <= 160 * 1024, "LDS budget");
  static_assert(NTW * 16 <= 256, "epilogue operand area");
  __shared__ __attribute__((aligned(1024))) int8_t lds[LDS_KB * 1024];
  int8_t* const wring = lds;
  int8_t* const aring = lds + RW * WST * 1024;
  int8_t* const sring = aring + RA * 16 * 1024;       // SC only
  float* const epi_sw = reinterpret_cast<float*>(lds + (LDS_KB - EPK) * 1024);
  float* const epi_b = epi_sw + EPC;
  int lbid = (int)blockIdx.x, row0 = 0;
  if constexpr (MS == 2) {
    // XCD-contiguous logical order: blocks b = 8 j + x (x = b & 7 labels the blocks that share an
    // XCD under round-robin dispatch) take logical workgroup x * ceil(G / 8) + (j >> 1), half j & 1,
    // so both halves of a panel AND neighbouring column groups (whose output rows meet inside one
    // 128-B line) share an XCD's L2 — partial lines merge there instead of in HBM (speed only)
    // EPI_PART keeps the round-robin order: an XCD then holds a fixed subset of the K slices, and
    // the activation bytes of those slices stay in its L2 (measured: o 14.9 vs 17.0 us, down 31.3
    // vs 34.9 at M = 256 against the contiguous order)
    const int x = (int)blockIdx.x & 7, j = (int)blockIdx.x >> 3, gx = (G + 7) >> 3;
    row0 = (j & 1) * 128;
    lbid = EPI == EPI_PART ? x | ((j >> 1) << 3) : x * gx + (j >> 1);
    if ((j >> 1) >= gx || lbid >= G) return;          // whole workgroup: no barrier is left waiting
  }
  const int Ml = min(128, M - row0);                  // rows of this half (>= 1: MS == 2 only for M > 128)
  const int KT = K / 64, NSA = KT / 2;
  const int grp = EPI == EPI_PART ? lbid / S : lbid;
  const int ks = EPI == EPI_PART ? lbid % S : 0;
  const int sbeg = EPI == EPI_PART ? (int)((int64_t)NSA * ks / S) : 0;
  const int NS = EPI == EPI_PART ? (int)((int64_t)NSA * (ks + 1) / S) - sbeg : NSA;
  const int nt0 = grp * NTW;
  // physical weight tile of the workgroup's logical tile t.  EPI_GLU (bf16): W = [gate | up] in
  // natural order (F = N / 2 rows each); logical tiles (2p, 2p + 1) = (gate, up) of feature tile
  // nt0 / 2 + p, so the GLU epilogue pairs them as the blocked int8 layout does
  auto phys_tile = [&](int t) -> int {
    if constexpr (EPI == EPI_GLU) {
      const int F16 = NTt >> 1, ft = min(nt0 / 2 + (t >> 1), F16 - 1);
      return (t & 1) ? F16 + ft : ft;
    } else {
      return min(nt0 + t, NTt - 1);
    }
  };
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int mw = NCW == 8 ? (wave & 3) : wave, tb = NCW == 8 ? (wave >> 2) * NTH : 0;   // compute waves
  // k order rotated per workgroup (int32 sums: exact in any order; SC: a fixed per-workgroup fp32
  // order): the ~256 workgroups do not all request the same activation lines at the same moment
  const int rot = ROT ? (int)((grp * 5u) % (unsigned)NS) : 0;
  auto phys = [&](int st) { const int k = min(st, NS - 1) + rot; return sbeg + (k >= NS ? k - NS : k); };

  const int8_t* const Ah = A + (size_t)row0 * K;
  if constexpr (NAL > 0) {
    if (wave >= NCW + NWL) {                          // ---- activation loader: line pieces al * APL ..
      constexpr int APL = 16 / NAL;
      const int al = wave - NCW - NWL;
      uint32_t aoff[APL];
#pragma unroll
      for (int i = 0; i < APL; ++i)
        aoff[i] = (uint32_t)min((al * APL + i) * 8 + (lane >> 3), Ml - 1) * (uint32_t)K + 16 * ((lane & 7) ^ (lane >> 3));
      auto issue = [&](int st) {
        const int8_t* ab = Ah + (size_t)phys(st) * 128;
#pragma unroll
        for (int i = 0; i < APL; ++i)
          glds16(ab + aoff[i], aring + ((st % RA) * 16 + al * APL + i) * 1024);
      };
      for (int st = 0; st < DA; ++st) issue(st);
      for (int s = 0; s < NS; ++s) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"((DA - 1) * APL) : "memory");   // own pieces of stage s
        __builtin_amdgcn_s_barrier();
        issue(s + DA);                                  // into the slot of stage s - 1
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      return;
    }
  }
  if (wave >= NCW) {                                  // ---- weight loader: pieces (k-tile c, tile t)
    const int lw = wave - NCW;
    uint32_t woff[WPW];
#pragma unroll
    for (int i = 0; i < WPW; ++i) {
      const int q = lw * WPW + i, c = q / NTW, t = q % NTW;
      woff[i] = ((uint32_t)phys_tile(t) * (uint32_t)KT + c) * 1024u + lane * 16;
    }
    // scale piece: lanes 0-31 the rows of k-tile 2 p, lanes 32-63 of 2 p + 1 (4 rows per lane)
    const uint32_t soff = (uint32_t)((lane >> 5) * Mpad + row0 + min(4 * (lane & 31), Mpad - row0 - 4));
    const bool smine = (lane % NWL) == lw;
    auto issue = [&](int st) {
      const int p = phys(st);
      const int8_t* wb = Wp + (size_t)p * 2048;
#pragma unroll
      for (int i = 0; i < WPW; ++i) glds16_nt(wb + woff[i], wring + ((st % RW) * WST + lw * WPW + i) * 1024);
      if constexpr (SC) {
        if (smine) glds16(sa + (size_t)(2 * p) * Mpad + soff, sring + (st % RW) * 1024);
      }
    };
    for (int st = 0; st < DW; ++st) issue(st);
    for (int s = 0; s < NS; ++s) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((DW - 1) * LPW) : "memory");   // own pieces of stage s
      __builtin_amdgcn_s_barrier();
      issue(s + DW);                                  // into the slot of stage s - 1
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA into LDS outlives the workgroup
    return;
  }

  // ---- compute waves: activation line pieces 4 wave .. 4 wave + 3 (rows 8p .. 8p + 7, 128 B)
  uint32_t aoff[APW];
#pragma unroll
  for (int i = 0; i < APW; ++i)
    aoff[i] = (uint32_t)min((APW * wave + i) * 8 + (lane >> 3), Ml - 1) * (uint32_t)K + 16 * ((lane & 7) ^ (lane >> 3));
  auto issue = [&](int st) {
    if constexpr (NAL == 0) {
      const int8_t* ab = Ah + (size_t)phys(st) * 128;
#pragma unroll
      for (int i = 0; i < APW; ++i)
        glds16(ab + aoff[i], aring + ((st % RA) * 16 + APW * wave + i) * 1024);
    }
  };
  // The MFMA operands are swapped (weight tile = A operand, activations = B): a lane's accumulator
  // holds 4 CONSECUTIVE output columns (4 (lane >> 4) + q of tile t) of ONE row ((lane & 15) of row
  // block j), so the epilogue stores 8 B (bf16) / 16 B (fp32) per lane instead of 2 / 4 B, and a
  // row's activation scale is one value per lane.  The workgroup's weight scales and bias go to
  // LDS once now (ordered for the epilogue by the stage barriers); the tail never waits on memory.
  {
    const int c = threadIdx.x;                        // compute waves: >= 256 threads, <= 256 columns
    if (c < NTW * 16) {
      const int col = min(phys_tile(c >> 4) * 16 + (c & 15), N - 1);
      epi_sw[c] = sw != nullptr ? sw[col] : 1.f;
      epi_b[c] = bias != nullptr ? bf2f(bias[col]) : 0.f;
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  }
  float sa_r[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) sa_r[j] = SC || DT ? 1.f : sa[row0 + min((2 * mw + j) * 16 + (lane & 15), Ml - 1)];
  v4i acc[2][NTH];
  v4f accf[2][NTH];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int t = 0; t < NTH; ++t) { acc[j][t] = v4i{0, 0, 0, 0}; accf[j][t] = v4f{0.f, 0.f, 0.f, 0.f}; }

  for (int st = 0; st < DA; ++st) issue(st);
  // row block rb = 2 wave + j lives in line pieces 2 rb, 2 rb + 1; k-tile c's chunk is 4 c + (lane >> 4)
  const uint32_t a0 = lds_off(aring) + (4 * mw + ((lane & 15) >> 3)) * 1024 + (lane & 7) * 128;
  const uint32_t ax[2] = {(uint32_t)(((lane >> 4) ^ (lane & 7)) << 4), (uint32_t)(((4 + (lane >> 4)) ^ (lane & 7)) << 4)};
  const uint32_t w0 = lds_off(wring) + lane * 16 + tb * 1024;
  const uint32_t s0 = lds_off(sring) + ((2 * mw) * 16 + (lane & 15)) * 4;
  // one k-tile's fragments: [2 row blocks | NTW tiles | SC: 2 row blocks' scales (lane's row, in
  // element 0)], double-buffered by k-tile, so the MFMAs of one k-tile run while the next one's LDS
  // reads are in flight (across the stage barrier too)
  constexpr int NF = 2 + NTH + (SC ? 2 : 0);
  auto read_kt = [&](int st, int c, v4i (&f)[NF]) {
    const uint32_t ab = a0 + (st % RA) * 16 * 1024, wb = w0 + (st % RW) * WST * 1024;
#pragma unroll
    for (int j = 0; j < 2; ++j) f[j] = lds_read16(ab + j * 2048 + ax[c]);
    v4i b[NTH];
    lds_read_row<NTH>(wb + c * NTW * 1024, b);
#pragma unroll
    for (int t = 0; t < NTH; ++t) f[2 + t] = b[t];
    if constexpr (SC) {
#pragma unroll
      for (int j = 0; j < 2; ++j) f[2 + NTH + j][0] = lds_read4(s0 + (st % RW) * 1024 + c * 512 + j * 64);
    }
  };
  // DT == 2, the one-VALU fold: each k-tile's MFMA starts from the bit pattern of 1.5 * 2^23
  // (0x4B400000) instead of 0, so the int32 sum (|sum| <= 64 * 127^2 < 2^22) lands in the low
  // mantissa bits and the result, read as a float, is exactly 12582912 + sum: one v_fmac per
  // element replaces cvt + fma.  The 12582912 * scale terms are taken out every 8 k-tiles from a
  // per-row running scale sum (ssum), which keeps the accumulator's magnitude, and so its
  // rounding, within 8 such terms.
  // (hipcc, ROCm 7.2: with the MFMA's i32 result reinterpreted as float element by element and no
  // pin on it, the generated code read only element 0 of the result for all four accumulator
  // elements; the opaque C operand and the pinned result below give the correct per-element form)
  constexpr float MAGIC_F = 12582912.f;
  v4i MAGIC_I = v4i{0x4B400000, 0x4B400000, 0x4B400000, 0x4B400000};
  asm volatile("" : "+v"(MAGIC_I));
  float ssum[2] = {0.f, 0.f};
  auto unbias = [&]() {
    if constexpr (DT == 2) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const float c = -MAGIC_F * ssum[j];
#pragma unroll
        for (int t = 0; t < NTH; ++t)
#pragma unroll
          for (int q = 0; q < 4; ++q) accf[j][t][q] += c;
        ssum[j] = 0.f;
      }
    }
  };
  auto mma = [&](v4i (&f)[NF]) {
#pragma unroll
    for (int i = 0; i < NF; ++i) asm volatile("" : "+v"(f[i]));
    if constexpr (SC && DT == 2) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const float sg = __builtin_bit_cast(float, f[2 + NTH + j][0]);
#pragma unroll
        for (int t = 0; t < NTH; ++t) {
          v4i r = mfma_i8(f[2 + t], f[j], MAGIC_I);
          asm volatile("" : "+v"(r));                 // (see MAGIC_F: keeps the four elements apart)
          const v4f rf = __builtin_bit_cast(v4f, r);
#pragma unroll
          for (int q = 0; q < 4; ++q) accf[j][t][q] = __builtin_fmaf(rf[q], sg, accf[j][t][q]);
        }
        ssum[j] += sg;
      }
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int t = 0; t < NTH; ++t) asm volatile("" : "+v"(accf[j][t]));
    } else if constexpr (SC) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const float sg = __builtin_bit_cast(float, f[2 + NTH + j][0]);
#pragma unroll
        for (int t = 0; t < NTH; ++t) fold1(accf[j][t], mfma_i8(f[2 + t], f[j], v4i{0, 0, 0, 0}), sg);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int t = 0; t < NTH; ++t) asm volatile("" : "+v"(accf[j][t]));
    } else if constexpr (DT == 1) {                   // bf16 x bf16 -> fp32, 32 k per 64 B
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int t = 0; t < NTH; ++t)
          accf[j][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(v8s, f[2 + t]),
                                                              __builtin_bit_cast(v8s, f[j]), accf[j][t], 0, 0, 0);
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int t = 0; t < NTH; ++t) asm volatile("" : "+v"(accf[j][t]));
    } else {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int t = 0; t < NTH; ++t) acc[j][t] = mfma_i8(f[2 + t], f[j], acc[j][t]);
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int t = 0; t < NTH; ++t) asm volatile("" : "+v"(acc[j][t]));
    }
  };
  // barrier k certifies stage k (both operands) and frees the slots of stage k - 1
  auto sync_stage = [&](int st) {
    if constexpr (NAL == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((DA - 1) * APW) : "memory");    // own pieces of stage st
    __builtin_amdgcn_s_barrier();
    issue(st + DA);
  };
  v4i x[NF], y[NF];
  sync_stage(0);
  read_kt(0, 0, x);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  for (int s = 0; s < NS; ++s) {                     // x holds k-tile (s, 0)
    read_kt(s, 1, y);
    mma(x);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (s + 1 < NS) {                                 // wave-uniform
      sync_stage(s + 1);
      read_kt(s + 1, 0, x);
    }
    mma(y);
    if constexpr (DT == 2) {
      if ((s & 3) == 3 || s + 1 == NS) unbias();     // wave-uniform; the last stage always
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // epilogue: lane holds row (2 wave + j) * 16 + (lane & 15), columns 4 (lane >> 4) .. + 3 of tile t
  const int g4 = 4 * (lane >> 4);
  if constexpr (EPI == EPI_OUT || EPI == EPI_PART) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int lrow = (2 * mw + j) * 16 + (lane & 15);
      if (lrow >= Ml) continue;
      const int row = row0 + lrow;
#pragma unroll
      for (int t = 0; t < NTH; ++t) {
        const int cl = (tb + t) * 16 + g4, col = nt0 * 16 + cl;
        if (col >= N) continue;
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float a = SC || DT ? accf[j][t][q] : (float)acc[j][t][q] * sa_r[j];
          v[q] = a * epi_sw[cl + q] + ((EPI == EPI_OUT || ks == 0) ? epi_b[cl + q] : 0.f);
        }
        if constexpr (EPI == EPI_PART) {
          float* o = reinterpret_cast<float*>(outv) + ((size_t)ks * M + row) * N + col;
          if (col + 3 < N && (N & 3) == 0) *reinterpret_cast<v4f*>(o) = v4f{v[0], v[1], v[2], v[3]};
          else for (int q = 0; q < 4 && col + q < N; ++q) o[q] = v[q];
        } else {
          bf16_t* o = reinterpret_cast<bf16_t*>(outv) + (size_t)row * N + col;
          if (col + 3 < N && (N & 3) == 0) *reinterpret_cast<uint2*>(o) = uint2{pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3])};
          else for (int q = 0; q < 4 && col + q < N; ++q) o[q] = f2bf(v[q]);
        }
      }
    }
  } else if constexpr (EPI == EPI_GLU) {             // bf16: h = silu(gate) * up -> bf16 [M, N / 2]
    const int Fo = N / 2, F16 = NTt >> 1;
    bf16_t* h = reinterpret_cast<bf16_t*>(outv);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int lrow = (2 * mw + j) * 16 + (lane & 15);
      if (lrow >= Ml) continue;
      const int row = row0 + lrow;
#pragma unroll
      for (int p = 0; p < NTH / 2; ++p) {
        const int ft = (nt0 + tb) / 2 + p;
        if (ft >= F16) continue;
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int cg = (tb + 2 * p) * 16 + g4 + q, cu = cg + 16;
          const float g = bf2f(f2bf(accf[j][2 * p][q] * epi_sw[cg] + epi_b[cg]));     // the unfused GEMM output is bf16
          const float u = bf2f(f2bf(accf[j][2 * p + 1][q] * epi_sw[cu] + epi_b[cu]));
          v[q] = g / (1.f + __expf(-g)) * u;
        }
        *reinterpret_cast<uint2*>(h + (size_t)row * Fo + ft * 16 + g4) = uint2{pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3])};
      }
    }
  } else {                                            // EPI_GLUQ: tiles (2p, 2p + 1) = (gate, up) of 16 features
    // the wave's 8 tiles [tb, tb + 8) are one 64-feature quant group (NCW == 8: two per workgroup)
    const int Fo = N / 2, grp64 = (nt0 + tb) / 8;
    int8_t* hq = reinterpret_cast<int8_t*>(outv);
    const bool live = nt0 + tb + 7 < NTt;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int lrow = (2 * mw + j) * 16 + (lane & 15);
      const int row = row0 + lrow;
      float h[4][4], amax = 0.f;
#pragma unroll
      for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int cg = (tb + 2 * p) * 16 + g4 + q, cu = cg + 16;
          const float g = bf2f(f2bf((float)acc[j][2 * p][q] * sa_r[j] * epi_sw[cg] + epi_b[cg]));     // the unfused GEMM output is bf16
          const float u = bf2f(f2bf((float)acc[j][2 * p + 1][q] * sa_r[j] * epi_sw[cu] + epi_b[cu]));
          h[p][q] = g / (1.f + __expf(-g)) * u;
          amax = fmaxf(amax, fabsf(h[p][q]));
        }
      amax = fmaxf(amax, __shfl_xor(amax, 16, 64));   // the row's 64 features sit in lanes l, l ^ 16, l ^ 32, l ^ 48
      amax = fmaxf(amax, __shfl_xor(amax, 32, 64));
      amax = fmaxf(amax, 1e-8f);
      const float inv = 127.f / amax;
      if (live && lrow < Ml) {
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          uint32_t w = 0;
#pragma unroll
          for (int q = 0; q < 4; ++q) w |= (uint32_t)(uint8_t)quant_i8(h[p][q], inv) << (8 * q);
          *reinterpret_cast<uint32_t*>(hq + (size_t)row * Fo + ((nt0 + tb) / 2 + p) * 16 + g4) = w;   // Fo % 64 == 0
        }
      }
      if (live && lane < 16 && row < Mpad) os[(size_t)grp64 * Mpad + row] = lrow < Ml ? amax / 127.f : 0.f;
    }
  }
}

// ------------------------------------------------------------------------------------ r256
// 129-256 decode rows (one 256-row decode micro-batch), activations FRAGMENT-PACKED: piece (rb, kt)
// = 1 KiB at (rb * KT + kt) * 1024, lane l's 16 B = A[16 rb + (l & 15)][64 kt + 16 (l >> 4) ..]
// (pack_a_kernel's layout; the decode producers — RMSNorm + quant, attention's int8 output, the
// quantising SwiGLU epilogue — write it directly, `Mpad` rows).
// Why: in ring2 above a compute wave's activation rows are private to it, so staging the activation
// half through LDS buys nothing but a layout change and costs 16 KiB of LDS-DMA writes + 16 KiB of
// LDS reads per 2-k-tile stage beside the weight ring's traffic.  Here every compute wave loads
// its own A fragments global -> VGPR, DA stages ahead (one coalesced 1 KiB load per fragment, L2
// hits), and only the weight panel — shared by all compute waves — goes through the LDS-DMA ring
// (NWL loader waves, RW slots, one bare barrier per stage as in ring2).  Measured against ring2 with
// tools/r256_lab.hip (Llama-2-7B shapes, 256 rows, HBM-cold weights): qkv 22.0-23.6 -> 20.6 us,
// plain gate_up 45 -> 38.5, plain o 15.3 -> 11.3.
// Geometry: RG x TG compute waves; wave (rg, tg) owns row blocks [rg RBW, (rg + 1) RBW) of the
// workgroup's rows (RBW = rows / 16 / RG) and tiles [tg NTH, (tg + 1) NTH) (NTH = NTW / TG).
// MS = 2: 128-row halves, blocks b and b + 8 share a weight panel (ring2's mapping); MS = 1: all 256
// rows in one workgroup (every weight byte read by one CU).  NSL stages (2 k-tiles each) per
// workgroup, fully unrolled so every activation register set has a name and the compiler waits on
// them with counted vmcnt; EPI_PART: S split-K slices of NSL stages (K = 128 S NSL).
// SC: per-(token, 64) activation scales [KT][Mpad] (the o / down inputs), loaded beside the
// fragments, every k-tile's int32 MFMA sum folded into fp32 with ring2's one-VALU magic-number fold.
// Epilogues: EPI_OUT bf16 (+ bias), EPI_PART fp32 slices, EPI_GLUQ SwiGLU + int8 per 64 features
// (NTH == 8: a wave's tiles are one quant group), optionally written fragment-packed (PKO) for the
// next 256-row GEMM.
template <int NTW, int RG, int TG, int NWL, int RW, int DA, int MS, int NSL, int EPI, bool SC, bool PKO = false>
__global__ void __launch_bounds__((RG * TG + NWL) * 64, 1) w8a8_r256_kernel(
    const int8_t* __restrict__ Ap, const float* __restrict__ sa, const int8_t* __restrict__ Wp,
    const float* __restrict__ sw, const bf16_t* __restrict__ bias, void* __restrict__ outv, float* __restrict__ os,
    int M, int N, int NTt, int Mpad, int KT, int S, int G) {
  constexpr int NCW = RG * TG, NTH = NTW / TG, ROWS = 256 / MS, RBW = ROWS / 16 / RG;
  constexpr int WST = 2 * NTW, WPW = WST / NWL, DW = RW - 1, APS = RBW * 2;   // A loads per stage
  static_assert(NTW % TG == 0 && (ROWS / 16) % RG == 0 && WST % NWL == 0, "geometry");
  static_assert(DW * WPW <= 63 && DA * APS * (SC ? 2 : 1) <= 63 && DA >= 1, "vmcnt range");
  static_assert(EPI == EPI_OUT || EPI == EPI_PART || (EPI == EPI_GLUQ && NTH == 8 && !SC), "epilogues");
  static_assert(!PKO || EPI == EPI_GLUQ, "packed output: the quantising SwiGLU epilogue");
  constexpr int EPC = NTW * 16 <= 128 ? 128 : 256;
  constexpr int LDS_B = RW * WST * 1024 + 2 * EPC * 4;
  static_assert(LDS_B <= 160 * 1024, "LDS budget");
  __shared__ __attribute__((aligned(1024))) int8_t lds[LDS_B];
  int8_t* const wring = lds;
  float* const epi_sw = reinterpret_cast<float*>(lds + RW * WST * 1024);
  float* const epi_b = epi_sw + EPC;
  int lbid = (int)blockIdx.x, row0 = 0;
  if constexpr (MS == 2) {
    // ring2's mapping: both halves of a panel (and neighbouring column groups) on one XCD under
    // round-robin dispatch; EPI_PART keeps the round-robin order (an XCD holds a fixed subset of
    // the K slices, whose activation bytes then stay in its L2).  Speed only.
    const int x = (int)blockIdx.x & 7, j = (int)blockIdx.x >> 3, gx = (G + 7) >> 3;
    row0 = (j & 1) * 128;
    lbid = EPI == EPI_PART ? x | ((j >> 1) << 3) : x * gx + (j >> 1);
    if ((j >> 1) >= gx || lbid >= G) return;        // whole workgroup: no barrier is left waiting
  } else {
    if (lbid >= G) return;
  }
  const int Ml = min(ROWS, M - row0);
  const int grp = EPI == EPI_PART ? lbid / S : lbid;
  const int ks = EPI == EPI_PART ? lbid % S : 0;
  const int sbeg = ks * NSL;                          // first stage of this workgroup
  // stages of this workgroup: NSL, fewer in the last split-K slice of a K that S does not divide
  // (stages past nloc re-load its last stage and are skipped: the barrier count stays NSL)
  const int nloc = min(NSL, KT / 2 - sbeg);
  const int nt0 = grp * NTW;
  auto phys_tile = [&](int t) -> int { return min(nt0 + t, NTt - 1); };
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);

  if (wave >= NCW) {                                  // ---- weight loaders: pieces (k-tile c, tile t)
    const int lw = wave - NCW;
    uint32_t woff[WPW];
#pragma unroll
    for (int i = 0; i < WPW; ++i) {
      const int q = lw * WPW + i, c = q / NTW, t = q % NTW;
      woff[i] = ((uint32_t)phys_tile(t) * (uint32_t)KT + c) * 1024u + lane * 16;
    }
    auto issue = [&](int st) {                        // stages past the end re-load the last one
      const int8_t* wb = Wp + (size_t)(sbeg + min(st, nloc - 1)) * 2048;
#pragma unroll
      for (int i = 0; i < WPW; ++i) glds16_nt(wb + woff[i], wring + ((st % RW) * WST + lw * WPW + i) * 1024);
    };
    for (int st = 0; st < DW; ++st) issue(st);
    for (int s = 0; s < NSL; ++s) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((DW - 1) * WPW) : "memory");   // own pieces of stage s
      __builtin_amdgcn_s_barrier();
      issue(s + DW);                                  // into the slot of stage s - 1
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA into LDS outlives the workgroup
    return;
  }

  // ---- compute wave (rg, tg)
  const int rg = wave % RG, tg = wave / RG, tb = tg * NTH;
  {
    const int c = threadIdx.x;                        // >= 128 compute threads; EPC columns
    for (int cc = c; cc < NTW * 16; cc += NCW * 64) {
      const int col = min(phys_tile(cc >> 4) * 16 + (cc & 15), N - 1);
      epi_sw[cc] = sw != nullptr ? sw[col] : 1.f;
      epi_b[cc] = bias != nullptr ? bf2f(bias[col]) : 0.f;
    }
  }
  float sa_r[RBW];
#pragma unroll
  for (int j = 0; j < RBW; ++j) sa_r[j] = SC ? 1.f : sa[row0 + min((rg * RBW + j) * 16 + (lane & 15), Ml - 1)];
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  const int8_t* ap = Ap + ((size_t)(row0 / 16 + rg * RBW) * KT + (size_t)sbeg * 2) * 1024 + lane * 16;
  const float* sp = sa + (size_t)sbeg * 2 * Mpad + row0 + rg * RBW * 16 + (lane & 15);   // SC
  v4i af[DA][RBW][2];
  float sf[DA][RBW][2];
  auto load_a = [&](int st, v4i (&f)[RBW][2], float (&g)[RBW][2]) {
    const int p = min(st, nloc - 1);                  // past the end: re-load the last stage (unused)
#pragma unroll
    for (int j = 0; j < RBW; ++j)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        f[j][c] = *reinterpret_cast<const v4i*>(ap + ((size_t)j * KT + 2 * p + c) * 1024);
        if constexpr (SC) g[j][c] = sp[(size_t)(2 * p + c) * Mpad + j * 16];
      }
  };
  v4i acc[RBW][NTH];
  v4f accf[RBW][NTH];
#pragma unroll
  for (int j = 0; j < RBW; ++j)
#pragma unroll
    for (int t = 0; t < NTH; ++t) { acc[j][t] = v4i{0, 0, 0, 0}; accf[j][t] = v4f{0.f, 0.f, 0.f, 0.f}; }
  // the one-VALU grouped-scale fold (ring2 DT = 2): each k-tile's MFMA starts from the bits of
  // 1.5 * 2^23, so the int32 sum read as a float is 12582912 + sum; the offsets come out every 4
  // stages from a per-row running scale sum
  constexpr float MAGIC_F = 12582912.f;
  v4i MAGIC_I = v4i{0x4B400000, 0x4B400000, 0x4B400000, 0x4B400000};
  asm volatile("" : "+v"(MAGIC_I));
  float ssum[RBW];
#pragma unroll
  for (int j = 0; j < RBW; ++j) ssum[j] = 0.f;
  auto unbias = [&]() {
#pragma unroll
    for (int j = 0; j < RBW; ++j) {
      const float cb = -MAGIC_F * ssum[j];
#pragma unroll
      for (int t = 0; t < NTH; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) accf[j][t][q] += cb;
      ssum[j] = 0.f;
    }
  };
  const uint32_t w0 = lds_off(wring) + lane * 16 + tb * 1024;
  auto read_w = [&](int st, int c, v4i (&f)[NTH]) { lds_read_row<NTH>(w0 + ((st % RW) * WST + c * NTW) * 1024, f); };
  auto mma = [&](const v4i (&a)[RBW][2], const float (&g)[RBW][2], int c, v4i (&f)[NTH]) {
#pragma unroll
    for (int i = 0; i < NTH; ++i) asm volatile("" : "+v"(f[i]));
    if constexpr (SC) {
#pragma unroll
      for (int j = 0; j < RBW; ++j) {
#pragma unroll
        for (int t = 0; t < NTH; ++t) {
          v4i r = mfma_i8(f[t], a[j][c], MAGIC_I);
          asm volatile("" : "+v"(r));                 // (ring2: keeps the four elements apart)
          const v4f rf = __builtin_bit_cast(v4f, r);
#pragma unroll
          for (int q = 0; q < 4; ++q) accf[j][t][q] = __builtin_fmaf(rf[q], g[j][c], accf[j][t][q]);
        }
        ssum[j] += g[j][c];
      }
#pragma unroll
      for (int j = 0; j < RBW; ++j)
#pragma unroll
        for (int t = 0; t < NTH; ++t) asm volatile("" : "+v"(accf[j][t]));
    } else {
#pragma unroll
      for (int j = 0; j < RBW; ++j)
#pragma unroll
        for (int t = 0; t < NTH; ++t) acc[j][t] = mfma_i8(f[t], a[j][c], acc[j][t]);
#pragma unroll
      for (int j = 0; j < RBW; ++j)
#pragma unroll
        for (int t = 0; t < NTH; ++t) asm volatile("" : "+v"(acc[j][t]));
    }
  };
#pragma unroll
  for (int u = 0; u < DA; ++u) load_a(u, af[u], sf[u]);
  v4i xw[NTH], yw[NTH];
  __builtin_amdgcn_s_barrier();                      // weight stage 0 visible
  read_w(0, 0, xw);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int s = 0; s < NSL; ++s) {
    const bool live = s < nloc;                       // wave-uniform
    read_w(s, 1, yw);
    if (live) mma(af[s % DA], sf[s % DA], 0, xw);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (s + 1 < NSL) {
      __builtin_amdgcn_s_barrier();                  // stage s + 1's weights; frees stage s - 1's slot
      read_w(s + 1, 0, xw);
    }
    if (live) mma(af[s % DA], sf[s % DA], 1, yw);
    if constexpr (SC) {
      if ((s & 3) == 3 || s + 1 == NSL) unbias();
    }
    load_a(s + DA, af[s % DA], sf[s % DA]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // epilogue: lane holds row (rg RBW + j) * 16 + (lane & 15), columns 4 (lane >> 4) .. + 3 of tile t
  const int g4 = 4 * (lane >> 4);
  if constexpr (EPI == EPI_OUT || EPI == EPI_PART) {
#pragma unroll
    for (int j = 0; j < RBW; ++j) {
      const int lrow = (rg * RBW + j) * 16 + (lane & 15);
      if (lrow >= Ml) continue;
      const int row = row0 + lrow;
#pragma unroll
      for (int t = 0; t < NTH; ++t) {
        const int cl = (tb + t) * 16 + g4, col = nt0 * 16 + cl;
        if (col >= N) continue;
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float a = SC ? accf[j][t][q] : (float)acc[j][t][q] * sa_r[j];
          v[q] = a * epi_sw[cl + q] + ((EPI == EPI_OUT || ks == 0) ? epi_b[cl + q] : 0.f);
        }
        if constexpr (EPI == EPI_PART) {
          float* o = reinterpret_cast<float*>(outv) + ((size_t)ks * M + row) * N + col;
          if (col + 3 < N && (N & 3) == 0) *reinterpret_cast<v4f*>(o) = v4f{v[0], v[1], v[2], v[3]};
          else for (int q = 0; q < 4 && col + q < N; ++q) o[q] = v[q];
        } else {
          bf16_t* o = reinterpret_cast<bf16_t*>(outv) + (size_t)row * N + col;
          if (col + 3 < N && (N & 3) == 0) *reinterpret_cast<uint2*>(o) = uint2{pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3])};
          else for (int q = 0; q < 4 && col + q < N; ++q) o[q] = f2bf(v[q]);
        }
      }
    }
  } else {                                            // EPI_GLUQ: tiles (2p, 2p + 1) = (gate, up) of 16 features
    const int Fo = N / 2, grp64 = (nt0 + tb) / 8;
    int8_t* hq = reinterpret_cast<int8_t*>(outv);
    const bool live = nt0 + tb + 7 < NTt;
    const int FT = Fo / 64;                           // k-tiles of the packed output (the down input)
#pragma unroll
    for (int j = 0; j < RBW; ++j) {
      const int lrow = (rg * RBW + j) * 16 + (lane & 15);
      const int row = row0 + lrow;
      float h[4][4], amax = 0.f;
#pragma unroll
      for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int cg = (tb + 2 * p) * 16 + g4 + q, cu = cg + 16;
          const float g = bf2f(f2bf((float)acc[j][2 * p][q] * sa_r[j] * epi_sw[cg] + epi_b[cg]));   // the unfused GEMM output is bf16
          const float u = bf2f(f2bf((float)acc[j][2 * p + 1][q] * sa_r[j] * epi_sw[cu] + epi_b[cu]));
          h[p][q] = g / (1.f + __expf(-g)) * u;
          amax = fmaxf(amax, fabsf(h[p][q]));
        }
      amax = fmaxf(amax, __shfl_xor(amax, 16, 64));   // the row's 64 features sit in lanes l, l ^ 16, l ^ 32, l ^ 48
      amax = fmaxf(amax, __shfl_xor(amax, 32, 64));
      amax = fmaxf(amax, 1e-8f);
      const float inv = 127.f / amax;
      if (live && (PKO ? row < Mpad : lrow < Ml)) {
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          uint32_t w = 0;
#pragma unroll
          for (int q = 0; q < 4; ++q) w |= (uint32_t)(uint8_t)quant_i8(h[p][q], inv) << (8 * q);
          const int f = ((nt0 + tb) / 2 + p) * 16 + g4;          // output feature (4 consecutive)
          if constexpr (PKO) {
            // packed piece (row / 16, f / 64), lane slot (row & 15) + 16 ((f & 63) >> 4), byte f & 15
            const size_t off = ((size_t)(row >> 4) * FT + (f >> 6)) * 1024 + ((row & 15) + 16 * ((f & 63) >> 4)) * 16 + (f & 15);
            *reinterpret_cast<uint32_t*>(hq + off) = lrow < Ml ? w : 0u;
          } else {
            *reinterpret_cast<uint32_t*>(hq + (size_t)row * Fo + f) = w;   // Fo % 64 == 0
          }
        }
      }
      if (live && lane < 16 && row < Mpad) os[(size_t)grp64 * Mpad + row] = lrow < Ml ? amax / 127.f : 0.f;
    }
  }
}

// One r256 configuration: -1 when it does not take the shape (K % 128, or S slices of NSL stages
// not covering K / 128 with every slice non-empty).
template <int NTW, int RG, int TG, int NWL, int RW, int DA, int MS, int NSL, int EPI, bool SC, bool PKO = false>
int launch_r256x(const void* Ap, const float* sa, const void* Wp, const float* sw, const void* bias, void* out,
                 float* os, int M, int N, int K, int Mpad, int S, hipStream_t st) {
  const int NTt = (N + 15) / 16, KT = K / 64, NS = KT / 2;
  if (K % 128 != 0 || M > 256 || Mpad < 256 || S < 1 || (EPI != EPI_PART && S != 1) || NSL * S < NS ||
      NSL * (S - 1) >= NS)
    return -1;
  const int G = (NTt + NTW - 1) / NTW * S;
  const int blocks = MS == 2 ? (G + 7) / 8 * 16 : G;
  hipLaunchKernelGGL((w8a8_r256_kernel<NTW, RG, TG, NWL, RW, DA, MS, NSL, EPI, SC, PKO>), dim3(blocks),
                     dim3((RG * TG + NWL) * 64), 0, st, (const int8_t*)Ap, sa, (const int8_t*)Wp, sw,
                     (const bf16_t*)bias, out, os, M, N, NTt, Mpad, KT, S, G);
  return (int)hipGetLastError();
}
}  // namespace

static int g_gemv_kw = 0, g_gemv_unroll = 0, g_gemv_ntw = 0, g_gemv_ring = 2;
extern "C" int edge_w8a8_prefill(const void* A, const float* sa, const void* Wp, const float* sw, const void* bias,
                                 void* out, int M, int N, int K, int KT, hipStream_t st);
// tuning hooks (microbenchmarks): 0 = automatic choice
extern "C" void edge_w8a8_gemv_config(int kw, int unroll) { g_gemv_kw = kw; g_gemv_unroll = unroll; }
extern "C" void edge_w8a8_gemv_ntw(int ntw) { g_gemv_ntw = ntw; }
extern "C" void edge_w8a8_gemv_ring(int on) { g_gemv_ring = on; }

namespace {
template <int MB, int NTW, int TG, int KW, int U, int AM, int EP>
int launch_one(const void* A, const float* sa, const void* Wp, const float* sw, const void* bias, void* out, float* os,
               int M, int N, int K, int KT, int Mpad, hipStream_t st, int S = 1) {
  const int NTt = (N + 15) / 16;
  hipLaunchKernelGGL((w8a8_gemv_kernel<MB, NTW, TG, KW, U, AM, EP>), dim3((NTt + NTW - 1) / NTW * S), dim3(TG * KW * 64),
                     0, st, (const int8_t*)A, sa, (const int8_t*)Wp, sw, (const bf16_t*)bias, out, os, M, N, K, KT, NTt,
                     Mpad, S, NormIn{});
  return (int)hipGetLastError();
}

template <int NTW, int TG, int KW, int EP, int NRM>
int launch_norm(const NormIn& na, const void* Wp, const float* sw, const void* bias, void* out, float* os, int M,
                int N, int K, hipStream_t st) {
  const int NTt = (N + 15) / 16;
  hipLaunchKernelGGL((w8a8_gemv_kernel<1, NTW, TG, KW, 2, A_TOKEN, EP, NRM>), dim3((NTt + NTW - 1) / NTW),
                     dim3(TG * KW * 64), 0, st, (const int8_t*)nullptr, (const float*)nullptr, (const int8_t*)Wp, sw,
                     (const bf16_t*)bias, out, os, M, N, K, K / 64, NTt, 16, 1, na);   // Mpad 16: scales [N/128][16]
  return (int)hipGetLastError();
}

// 65-128 decode rows (two 64-row micro-batches, or one 128-row one) on the ring2 kernel (geometries
// measured with tools/bench_ops.py --only ring):
//  * split-K (o / down): 8 compute waves (two per SIMD: the grouped-scale per-k-tile fold issues
//    beside the partner's MFMAs), 2 weight + 2 activation loader waves, >= 4 stages per slice
//    (down, K = 11008: 22.4 -> 20.1 us against the earlier one-ring kernel);
//  * qkv-like EPI_OUT (3 tiles) and the quantising GLU (8 tiles = one 64-feature group) with
//    dedicated weight loaders (the 2-lane bench 32.0k against 28.3k tok/s in round 2).
// K % 128 == 0 (split-K: >= 4 stages per slice; rows128_ok).  The quantising GLU takes it from 33
// rows (gate_up at 64 rows: 26.6 us here against 33.9 for the weight-stationary GEMV; the ring's
// surplus rows are clamped reads, never stored).  -1: no kernel for this call.
template <int EP>
int launch_ring_rows128(const void* A, const float* sa, const void* Wp, const float* sw, const void* bias, void* out,
                        float* os, int M, int N, int K, int Mpad, bool scaled, hipStream_t st, int S) {
  if (!g_gemv_ring || M <= (EP == EPI_GLUQ ? 32 : 64) || M > 128 || K % 128 != 0 || (EP == EPI_PART) != (S > 1))
    return -1;
  if (scaled && (Mpad < 16 || Mpad % 16 != 0)) return -1;
  const int NTt = (N + 15) / 16;
#define RING2(NTWV, NWLV, RWV, RAV, EPV, SCV, NALV, NCWV, NW)                                                      \
  hipLaunchKernelGGL((w8a8_gemv_ring2_kernel<NTWV, NWLV, RWV, RAV, EPV, EPV == EPI_PART, SCV, 1, NALV, NCWV>),  \
                     dim3((NTt + NTWV - 1) / NTWV * S), dim3((NW) * 64), 0, st, (const int8_t*)A, sa,             \
                     (const int8_t*)Wp, sw, (const bf16_t*)bias, out, os, M, N, K, NTt, Mpad, S);               \
  return (int)hipGetLastError()
  if constexpr (EP == EPI_PART) {
    if (K / 128 < 4 * S) return -1;
    if (scaled) { RING2(4, 2, 8, 4, EPI_PART, true, 2, 8, 12); }
    RING2(4, 2, 8, 4, EPI_PART, false, 2, 8, 12);
  } else if constexpr (EP == EPI_GLUQ) {
    if (scaled || N % 128 != 0) return -1;
    RING2(8, 4, 5, 4, EPI_GLUQ, false, 0, 4, 8);
  } else if constexpr (EP == EPI_OUT) {
    if (scaled) { RING2(3, 3, 12, 4, EPI_OUT, true, 0, 4, 7); }   // (the scale ring: 2 weight stages fewer)
    RING2(3, 3, 14, 4, EPI_OUT, false, 0, 4, 7);
  }
#undef RING2
  return -1;
}

// 129-256 rows (one 256-row decode micro-batch): ring2 with the rows cut in two halves that stream
// the same weight panel on one XCD (MS = 2), so a decode step reads every weight from HBM once for
// all 256 sequences instead of once per 128-row lane, and with dedicated activation-loader waves.
// Tiles per workgroup are chosen for ~256 launched workgroups (the logical grid doubles); weights
// stream nontemporal (1-4 % ahead of normal allocation at M = 256).  -1: no kernel for this call.
// Geometries measured with tools/bench_ops.py --only rows256 (profiles/bench_ops_r3_rows256*.json):
//  * split-K (o / down, >= 4 stages per slice): 8 compute waves (two per SIMD: the grouped-scale
//    fold issues beside the partner's MFMAs: o 17.4 -> 14.9 us, down 34.8 -> 28.9), 2 + 2 loaders,
//    4 tiles for o-like N (128 logical at 2 slices), 8 for down (N 4096, 4 slices); grouped scales
//    fold with one VALU per element (DT = 2, magic-number bias);
//  * quantising gate_up: one round of 16-tile workgroups, 8 compute waves each owning one
//    64-feature group (43.7 -> 34.7 us against two rounds of 8-tile ones);
//  * qkv-like EPI_OUT: 3 tiles for N <= 8192, 6 for qkv-sized N, 8 beyond.
template <int NTWV, int NWLV, int RWV, int RAV, int NALV, int EPV, bool SCV, int NCWV = 4, int DTV = 0>
int launch_r256(const void* A, const float* sa, const void* Wp, const float* sw, const void* bias, void* out, float* os,
                int M, int N, int K, int Mpad, hipStream_t st, int S) {
  const int NTt = (N + 15) / 16, G = (NTt + NTWV - 1) / NTWV * S;
  hipLaunchKernelGGL((w8a8_gemv_ring2_kernel<NTWV, NWLV, RWV, RAV, EPV, false, SCV, 2, NALV, NCWV, DTV>),
                     dim3((G + 7) / 8 * 16), dim3((NCWV + NWLV + NALV) * 64), 0, st, (const int8_t*)A, sa,
                     (const int8_t*)Wp, sw, (const bf16_t*)bias, out, os, M, N, K, NTt, Mpad, S, G);
  return (int)hipGetLastError();
}

}  // namespace
// the weights-in-VGPR form (gemm_i8_wreg.hip); g_wreg: 0 off, 4 / 6 = stages in flight
extern "C" int edge_w8a8_wreg(const void* A, const float* sa, const void* Wp, const float* sw, const void* bias,
                              void* out, float* os, int M, int N, int K, int Mpad, int epi, int da, hipStream_t st);
static int g_wreg = 0;
extern "C" void edge_w8a8_wreg_cfg(int v) { g_wreg = v; }
namespace {

template <int EP>
int launch_rows256(const void* A, const float* sa, const void* Wp, const float* sw, const void* bias, void* out,
                   float* os, int M, int N, int K, int Mpad, bool scaled, hipStream_t st, int S) {
  if (M <= 128 || M > 256 || K % 128 != 0 || (EP == EPI_PART) != (S > 1) || (scaled && EP != EPI_PART)) return -1;
  if constexpr (EP == EPI_GLUQ || EP == EPI_OUT) {
    if (g_wreg && !scaled && S == 1) {
      const int r = edge_w8a8_wreg(A, sa, Wp, sw, bias, out, os, M, N, K, Mpad, EP, g_wreg, st);
      if (r != -2) return r;
    }
  }
  const int NTt = (N + 15) / 16;
  if constexpr (EP == EPI_PART) {
    if (K / 128 < 4 * S || (scaled && (Mpad < M || Mpad % 16 != 0))) return -1;
    const bool narrow = (NTt + 3) / 4 * S <= 160;     // o (N 4096, 2 slices): 128 logical at 4 tiles
    if (narrow)
      return scaled ? launch_r256<4, 2, 8, 4, 2, EP, true, 8, 2>(A, sa, Wp, sw, bias, out, os, M, N, K, Mpad, st, S)
                    : launch_r256<4, 2, 8, 4, 2, EP, false, 8>(A, sa, Wp, sw, bias, out, os, M, N, K, Mpad, st, S);
    return scaled ? launch_r256<8, 2, 5, 4, 2, EP, true, 8, 2>(A, sa, Wp, sw, bias, out, os, M, N, K, Mpad, st, S)
                  : launch_r256<8, 2, 5, 4, 2, EP, false, 8>(A, sa, Wp, sw, bias, out, os, M, N, K, Mpad, st, S);
  } else if constexpr (EP == EPI_GLUQ) {
    if (N % 128 != 0 || scaled) return -1;
    if (NTt % 16 == 0) return launch_r256<16, 2, 3, 3, 2, EP, false, 8>(A, sa, Wp, sw, bias, out, os, M, N, K, Mpad, st, S);
    return launch_r256<8, 2, 5, 4, 2, EP, false>(A, sa, Wp, sw, bias, out, os, M, N, K, Mpad, st, S);
  } else {
    if (scaled || S != 1) return -1;
    if (NTt <= 512) return launch_r256<3, 2, 14, 4, 2, EP, false>(A, sa, Wp, sw, bias, out, os, M, N, K, Mpad, st, S);
    if (NTt <= 1024) return launch_r256<6, 2, 7, 4, 2, EP, false>(A, sa, Wp, sw, bias, out, os, M, N, K, Mpad, st, S);
    return launch_r256<8, 2, 5, 4, 2, EP, false>(A, sa, Wp, sw, bias, out, os, M, N, K, Mpad, st, S);
  }
  return -1;
}

}  // namespace

// 129-256 decode rows on FRAGMENT-PACKED activations (w8a8_r256_kernel; the producers write the
// packed layout: rowwise.hip norm quant = 2).  Ap: a [256, K] packed buffer; sa: per-token scales
// [>= M]; epi 0: bf16 out [M, N] (+ bias).  Geometries from tools/r256_lab.hip (Llama-2-7B, 256
// rows, HBM-cold weights): 6 tiles (96 columns) per 128-row half for qkv-sized N, 2 tiles for
// N <= 8192 (o-sized: 11.3 us against ring2's 15.3).  -2: no packed kernel for this shape (the
// caller then feeds row-major activations to edge_w8a8_gemm).
static int g_r256_packed = 1;
extern "C" void edge_w8a8_r256_cfg(int on) { g_r256_packed = on; }
extern "C" int edge_w8a8_r256_ok(int M, int N, int K, int epi) {
  return g_r256_packed && M > 128 && M <= 256 && epi == EPI_OUT && (K == 2048 || K == 4096) && N % 4 == 0;
}
extern "C" int edge_w8a8_r256(const void* Ap, const float* sa, const void* Wp, const float* sw, const void* bias,
                              void* out, int M, int N, int K, int epi, hipStream_t st) {
  if (!edge_w8a8_r256_ok(M, N, K, epi)) return -2;
  const int NTt = (N + 15) / 16;
  const bool wide = NTt > 512;
#define R256(NTW, RW, NSL) return launch_r256x<NTW, 4, 1, 2, RW, 3, 2, NSL, EPI_OUT, false>(Ap, sa, Wp, sw, bias, out, \
                                                                                    nullptr, M, N, K, 256, 1, st)
  if (K == 4096) { if (wide) R256(6, 7, 32); R256(2, 14, 32); }
  if (wide) R256(6, 7, 16);
  R256(2, 14, 16);
#undef R256
}

// split-K slices the 129-256-row kernels use for a K (0: none): 2 for o-like K, 4 for down-like K
// (fewer slices also cut the fp32 partial bytes the next RMSNorm reads;
// profiles/bench_r3_down_splits_ab.jsonl, bench_r3_i8_o_splits_ab.jsonl)
extern "C" int edge_w8a8_rows256_splits(int K) { return K % 128 != 0 ? 0 : (K / 128 >= 64 ? 4 : 2); }
// whether the 129-256-row decode kernels take this K (whole K; split-K at rows256_splits(K))
extern "C" int edge_w8a8_rows256_ok(int K) { return K % 128 == 0 && K / 128 >= 8; }

// whether the 65-128-row decode kernels (launch_ring_rows128) take this K: the whole K (S = 1) or S
// split-K slices of >= 4 stages of 128 k
extern "C" int edge_w8a8_rows128_ok(int K, int S) {
  return K > 0 && S >= 1 && K % 128 == 0 && (S == 1 || K / 128 >= 4 * S);
}

namespace {
// EPI_OUT: 16 waves; KW = 16 while the LDS reduction fits (KW x NTW x MB KiB <= 128 KiB), else 8
template <int MB, int AM>
int launch_out(int ntw, int un, int kw, const void* A, const float* sa, const void* Wp, const float* sw,
               const void* bias, void* out, int M, int N, int K, int KT, int Mpad, hipStream_t st, float* add) {
#define L(NTWV, KWV, UV) return launch_one<MB, NTWV, 1, KWV, UV, AM, EPI_OUT>(A, sa, Wp, sw, bias, out, add, M, N, K, \
                                                                          KT, Mpad, st)
#define BY_KW(NTWV, UV)                                                   \
  do {                                                                    \
    if constexpr ((AM == A_GROUP && (NTWV >= 4 || (MB > 1 && NTWV > 2) || MB > 2)) || (MB > 2 && NTWV >= 3)) L(NTWV, 8, UV); \
    else { if (kw <= 8) L(NTWV, 8, UV); else L(NTWV, 16, UV); }           \
  } while (0)
  // four row blocks, A_TOKEN: 16 waves with one k-tile in flight each (U = 1) fit the 128-VGPR
  // budget where U = 2 needs 8 waves; un == 2 selects the 8-wave form (A/B)
  if constexpr (MB == 4 && AM == A_TOKEN) {
    if (un != 2 && ntw == 3) L(3, 16, 1);
  }
  if (ntw <= 1) {
    if constexpr (MB == 1) { if (un >= 4) BY_KW(1, 4); }
    BY_KW(1, 2);
  }
  if (ntw == 2) BY_KW(2, 2);
  if (ntw == 3) BY_KW(3, 2);
  BY_KW(4, 2);
#undef BY_KW
#undef L
}
}  // namespace

// Split-K GEMV (M <= 64, K % 64 == 0): S workgroups per 4-tile group, each reducing KT/S k-tiles
// into fp32 partial slices part[S][M][N].  Cuts each workgroup's activation reads S-fold — at
// decode shapes every CU re-reads the whole activation matrix from L2, and those bytes share the
// CU's load path with the weight stream (tools/membw.hip "a" mode: +1 L2 byte per weight byte
// costs +13 % time at 50 MB).  The consumer adds the slices (rowwise.hip norm_kernel<PART>).
extern "C" int edge_w8a8_gemm_splitk(const void* A, const float* sa, const void* Wp, const float* sw, const void* bias,
                                     float* part, int M, int N, int K, int KT, int a_mode, int Mpad, int S,
                                     hipStream_t st) {
  if (M <= 0 || M > 256 || K % 64 != 0 || K / 64 != KT || S < 1 || S > KT) return -2;
  const int mblocks = (M + 15) / 16;
  if (a_mode == A_GROUP && Mpad < mblocks * 16) return -2;
  if (M > 128) {
    const int r = launch_rows256<EPI_PART>(A, sa, Wp, sw, bias, part, nullptr, M, N, K, Mpad, a_mode == A_GROUP, st, S);
    return r == -1 ? -2 : r;
  }
  if (M > 64) {
    const int r = launch_ring_rows128<EPI_PART>(A, sa, Wp, sw, bias, part, nullptr, M, N, K, Mpad, a_mode == A_GROUP, st, S);
    return r == -1 ? -2 : r;
  }
  // 2 tiles per workgroup for one row block, 4 for more (the binding sizes S for ~256 workgroups;
  // measured on Llama-2-7B o/down: S = 2 best at 16 rows, S = 4 at 32)
#define SK(MBV, KWV, AMV)                                                                                          \
  return mblocks > 1 ? launch_one<MBV, 4, 1, KWV, 2, AMV, EPI_PART>(A, sa, Wp, sw, bias, part, nullptr, M, N, K, KT, Mpad, \
                                                              st, S)                                               \
                : launch_one<MBV, 2, 1, KWV, 2, AMV, EPI_PART>(A, sa, Wp, sw, bias, part, nullptr, M, N, K, KT, Mpad, \
                                                              st, S)
  if (a_mode == A_GROUP) {
    if (mblocks <= 1) SK(1, 16, A_GROUP);
    if (mblocks <= 2) SK(2, 8, A_GROUP);
    SK(4, 8, A_GROUP);
  }
  if (mblocks <= 1) SK(1, 16, A_TOKEN);
  if (mblocks <= 2) SK(2, 16, A_TOKEN);
  SK(4, 8, A_TOKEN);
#undef SK
}

// Decode GEMV (M <= 4 rows) whose activation rows are RMSNorm(sum of S fp32 partial slices +
// residual), int8 per token, computed in the kernel's prologue (NormIn above).  epi 0 (EPI_OUT:
// bf16 [M, N]) or 2 (EPI_GLUQ: 16-blocked gate_up -> SwiGLU -> int8 per 64 features, `os` scales
// [N/128][16]).
// K in {2048, 4096} (256 threads x NCH chunks of 8, NCH <= 2), 1 <= S <= 4; res may be null (no
// residual: a stage's first norm over the embedding); res_out written by workgroup 0 and must not
// alias res.  -2: not taken.
static int g_gemv_norm = 1;      // 0: the norm stays a kernel of its own (A/B knob "gemv_norm")
extern "C" void edge_w8a8_gemv_norm_cfg(int on) { g_gemv_norm = on; }
extern "C" int edge_w8a8_gemv_norm_on() { return g_gemv_norm; }
extern "C" int edge_w8a8_gemv_norm(const float* part, int S, const void* res, const void* gamma, float eps,
                                   void* res_out, const void* Wp, const float* sw, const void* bias, void* out,
                                   float* os, int M, int N, int K, int epi, hipStream_t st) {
  if (M < 1 || M > NRM_ROWS || S < 1 || S > 4 || (K != 2048 && K != 4096) || N % 16 != 0 || res_out == nullptr ||
      res == res_out)
    return -2;
  const NormIn na{part, (const bf16_t*)res, (const bf16_t*)gamma, (bf16_t*)res_out, eps, S};
  // template NRM = 8 * (K / 2048) + (S <= 2 ? 2 : 4): two-slice sums keep 32 VGPRs free, which
  // lets the qkv form hold both of its weight steps across the prologue without spilling
#define NRM_L(NTW, TG, KW, EP, OS)                                                                       \
  return K == 4096 ? (S <= 2 ? launch_norm<NTW, TG, KW, EP, 18>(na, Wp, sw, bias, out, OS, M, N, K, st)     \
                             : launch_norm<NTW, TG, KW, EP, 20>(na, Wp, sw, bias, out, OS, M, N, K, st))    \
                   : (S <= 2 ? launch_norm<NTW, TG, KW, EP, 10>(na, Wp, sw, bias, out, OS, M, N, K, st)     \
                             : launch_norm<NTW, TG, KW, EP, 12>(na, Wp, sw, bias, out, OS, M, N, K, st))
  if (epi == EPI_OUT) NRM_L(3, 1, 16, EPI_OUT, nullptr);
  if (epi == EPI_GLUQ) {
    if (N % 128 != 0 || os == nullptr) return -2;
    NRM_L(8, 2, 8, EPI_GLUQ, os);
  }
#undef NRM_L
  return -2;
}

// Decode GEMV (M <= 4 rows) whose activation rows are LayerNorm(x + res) of bf16 rows x, int8 per
// token, computed in the kernel's prologue (ln_prologue; the parallel-residual decoders).  epi 0
// (EPI_OUT: bf16 [M, N]) or EPI_GELUQT / EPI_GELUQE (gelu of the bf16 output, int8 per (token, 64
// columns), `os` scales [N/64][16]).  K % 64 == 0, K <= 4096; res may be null; res_out written by
// workgroup 0.  -2: not taken.
extern "C" int edge_w8a8_gemv_ln(const void* x, const void* res, const void* gamma, const void* beta, float eps,
                                 void* res_out, const void* Wp, const float* sw, const void* bias, void* out,
                                 float* os, int M, int N, int K, int epi, hipStream_t st) {
  if (!g_gemv_norm || M < 1 || M > NRM_ROWS || K % 64 != 0 || K > 4096 || N % 16 != 0 || res_out == nullptr ||
      res == res_out || x == res_out || x == nullptr)
    return -2;
  NormIn na{nullptr, (const bf16_t*)res, (const bf16_t*)gamma, (bf16_t*)res_out, eps, 0};
  na.x = (const bf16_t*)x;
  na.beta = (const bf16_t*)beta;
#define LN_L(NTW, TG, KW, EP, OS)                                                                   \
  return K <= 2048 ? launch_norm<NTW, TG, KW, EP, 64 + 8>(na, Wp, sw, bias, out, OS, M, N, K, st)  \
                   : launch_norm<NTW, TG, KW, EP, 64 + 16>(na, Wp, sw, bias, out, OS, M, N, K, st)
  if (epi == EPI_OUT) LN_L(3, 1, 16, EPI_OUT, nullptr);
  if (epi == EPI_GELUQT || epi == EPI_GELUQE) {
    if (N % 64 != 0 || os == nullptr) return -2;
    if (epi == EPI_GELUQT) LN_L(4, 1, 16, EPI_GELUQT, os);
    LN_L(4, 1, 16, EPI_GELUQE, os);
  }
#undef LN_L
  return -2;
}

// LLM.int8 projection of one bf16 row in one launch (l8_prologue): out bf16 [1, N] = int8 GEMV of x
// with its outlier columns (|x| > thr, the first 256 in column order) zeroed, per-token scale, sw =
// SCB / 127 (+ bias), plus the outlier columns' part from wt = int8 W^T [K, N].  K % 64 == 0,
// K <= 12288.  -2: not taken.
extern "C" int edge_llmint8_gemv(const void* x, float thr, const void* Wp, const float* sw, const void* bias,
                                 const void* wt, const float* scb, void* out, int N, int K, hipStream_t st, int act) {
  if (K % 64 != 0 || K > 12288 || K < 64 || N % 16 != 0) return -2;
  NormIn na{nullptr, nullptr, nullptr, nullptr, 0.f, 0};
  na.x = (const bf16_t*)x;
  na.thr = thr;
  na.wt = (const int8_t*)wt;
  na.scb = scb;
  if (act == 1 || act == 2) {                            // + gelu (tanh / erf) of the output, K <= 4096
    if (K > 4096) return -2;
    if (act == 1) return K <= 2048 ? launch_norm<3, 1, 16, EPI_OUT, 256 + 8>(na, Wp, sw, bias, out, nullptr, 1, N, K, st)
                                   : launch_norm<3, 1, 16, EPI_OUT, 256 + 16>(na, Wp, sw, bias, out, nullptr, 1, N, K, st);
    return K <= 2048 ? launch_norm<3, 1, 16, EPI_OUT, 320 + 8>(na, Wp, sw, bias, out, nullptr, 1, N, K, st)
                     : launch_norm<3, 1, 16, EPI_OUT, 320 + 16>(na, Wp, sw, bias, out, nullptr, 1, N, K, st);
  }
  switch ((K + 2047) / 2048) {                            // row chunks of 2048 per 256 threads
    case 1: return launch_norm<3, 1, 16, EPI_OUT, 128 + 8>(na, Wp, sw, bias, out, nullptr, 1, N, K, st);
    case 2: return launch_norm<3, 1, 16, EPI_OUT, 128 + 16>(na, Wp, sw, bias, out, nullptr, 1, N, K, st);
    case 3: return launch_norm<3, 1, 16, EPI_OUT, 128 + 24>(na, Wp, sw, bias, out, nullptr, 1, N, K, st);
    case 4: return launch_norm<3, 1, 16, EPI_OUT, 128 + 32>(na, Wp, sw, bias, out, nullptr, 1, N, K, st);
    case 5: return launch_norm<3, 1, 16, EPI_OUT, 128 + 40>(na, Wp, sw, bias, out, nullptr, 1, N, K, st);
    default: return launch_norm<3, 1, 16, EPI_OUT, 128 + 48>(na, Wp, sw, bias, out, nullptr, 1, N, K, st);
  }
}

// The same over the RMSNorm (ln 0) / LayerNorm (ln 1) of x + res (res may be null): res_out gets
// x + res, y_out (may be null) the normalised row.  K <= 4096, K % 64 == 0.  -2: not taken.
extern "C" int edge_llmint8_gemv_norm(const void* x, const void* res, const void* gamma, const void* beta, float eps,
                                      int ln, void* res_out, void* y_out, float thr, const void* Wp, const float* sw,
                                      const void* bias, const void* wt, const float* scb, void* out, int N, int K,
                                      hipStream_t st, int glu, int act) {
  if (!g_gemv_norm || K % 64 != 0 || K > 4096 || N % 16 != 0 || res_out == nullptr || res == res_out ||
      x == res_out || (y_out != nullptr && (y_out == x || y_out == res_out)) || (glu && (ln || N % 32 != 0)))
    return -2;
  NormIn na{nullptr, (const bf16_t*)res, (const bf16_t*)gamma, (bf16_t*)res_out, eps, 0};
  na.x = (const bf16_t*)x;
  na.beta = (const bf16_t*)beta;
  na.thr = thr;
  na.wt = (const int8_t*)wt;
  na.scb = scb;
  na.y_out = (bf16_t*)y_out;
  if (act == 1 || act == 2) {              // + gelu (tanh / erf) of the output
    if (glu) return -2;
    if (act == 1) {
      if (K <= 2048) return ln ? launch_norm<3, 1, 16, EPI_OUT, 256 + 8 + 2>(na, Wp, sw, bias, out, nullptr, 1, N, K, st)
                               : launch_norm<3, 1, 16, EPI_OUT, 256 + 8 + 1>(na, Wp, sw, bias, out, nullptr, 1, N, K, st);
      return ln ? launch_norm<3, 1, 16, EPI_OUT, 256 + 16 + 2>(na, Wp, sw, bias, out, nullptr, 1, N, K, st)
                : launch_norm<3, 1, 16, EPI_OUT, 256 + 16 + 1>(na, Wp, sw, bias, out, nullptr, 1, N, K, st);
    }
    if (K <= 2048) return ln ? launch_norm<3, 1, 16, EPI_OUT, 320 + 8 + 2>(na, Wp, sw, bias, out, nullptr, 1, N, K, st)
                             : launch_norm<3, 1, 16, EPI_OUT, 320 + 8 + 1>(na, Wp, sw, bias, out, nullptr, 1, N, K, st);
    return ln ? launch_norm<3, 1, 16, EPI_OUT, 320 + 16 + 2>(na, Wp, sw, bias, out, nullptr, 1, N, K, st)
              : launch_norm<3, 1, 16, EPI_OUT, 320 + 16 + 1>(na, Wp, sw, bias, out, nullptr, 1, N, K, st);
  }
  if (glu)                                  // SwiGLU of [gate | up] (N = 2F): out [1, N / 2]
    return K <= 2048 ? launch_norm<2, 1, 16, EPI_OUT, 192 + 8 + 5>(na, Wp, sw, bias, out, nullptr, 1, N, K, st)
                     : launch_norm<2, 1, 16, EPI_OUT, 192 + 16 + 5>(na, Wp, sw, bias, out, nullptr, 1, N, K, st);
  if (K <= 2048)
    return ln ? launch_norm<3, 1, 16, EPI_OUT, 192 + 8 + 2>(na, Wp, sw, bias, out, nullptr, 1, N, K, st)
              : launch_norm<3, 1, 16, EPI_OUT, 192 + 8 + 1>(na, Wp, sw, bias, out, nullptr, 1, N, K, st);
  return ln ? launch_norm<3, 1, 16, EPI_OUT, 192 + 16 + 2>(na, Wp, sw, bias, out, nullptr, 1, N, K, st)
            : launch_norm<3, 1, 16, EPI_OUT, 192 + 16 + 1>(na, Wp, sw, bias, out, nullptr, 1, N, K, st);
}

// sa: per-token [M] (a_mode 0) or per-group [KT][Mpad] (a_mode 1, M <= 64).
// epi 0: `os`, when not null, is a bf16 addend [M, N] added to the output (M <= 64 only; larger M
//        must pass null).
// epi 1: fused SwiGLU on 16-blocked gate/up rows, `out` is bf16 [M, N/2] (a_mode 0, M <= 64).
// epi 2: as epi 1, then per-(token, 64 features) int8 quantisation: `out` int8 [M, N/2],
//        `os` scales [N/128][Mpad] (N % 128 == 0).
extern "C" int edge_w8a8_gemm(const void* A, const float* sa, const void* Wp, const float* sw, const void* bias,
                              void* out, float* os, int M, int N, int K, int KT, int a_mode, int Mpad, int epi,
                              hipStream_t st) {
  if (M == 0 || N == 0) return 0;
  const int NTt = (N + 15) / 16;
  const int mblocks = (M + 15) / 16;
  if (a_mode == A_GROUP && Mpad < mblocks * 16) return -2;
  if (M > 64 && M <= 128 && epi == EPI_OUT && g_gemv_unroll != 1) {
    const int r = launch_ring_rows128<EPI_OUT>(A, sa, Wp, sw, bias, out, nullptr, M, N, K, Mpad, a_mode == A_GROUP, st, 1);
    if (r != -1) return r;
  }
  if (M > 128 && M <= 256 && (epi == EPI_OUT || epi == EPI_GLUQ) && a_mode == A_TOKEN && g_gemv_ring) {
    const int r = epi == EPI_OUT
                      ? launch_rows256<EPI_OUT>(A, sa, Wp, sw, bias, out, nullptr, M, N, K, Mpad, false, st, 1)
                      : (os == nullptr || Mpad < mblocks * 16
                             ? -1
                             : launch_rows256<EPI_GLUQ>(A, sa, Wp, sw, bias, out, os, M, N, K, Mpad, false, st, 1));
    if (r != -1) return r;
  }
  if (a_mode != A_TOKEN && M > 64) return -2;
  if (epi == EPI_GELUQT || epi == EPI_GELUQE) {
    // 4 tiles = one 64-column quant group per workgroup, 16 waves splitting K
    if (a_mode != A_TOKEN || M > 64 || N % 64 != 0 || os == nullptr || Mpad < mblocks * 16) return -2;
#define GQ(MBV, KWV)                                                                                              \
  return epi == EPI_GELUQT                                                                                        \
             ? launch_one<MBV, 4, 1, KWV, 2, A_TOKEN, EPI_GELUQT>(A, sa, Wp, sw, bias, out, os, M, N, K, KT, Mpad, st) \
             : launch_one<MBV, 4, 1, KWV, 2, A_TOKEN, EPI_GELUQE>(A, sa, Wp, sw, bias, out, os, M, N, K, KT, Mpad, st)
    if (mblocks <= 1) GQ(1, 16);
    if (mblocks <= 2) GQ(2, 16);
    GQ(4, 8);
#undef GQ
  }
  if (epi == EPI_GLU || epi == EPI_GLUQ) {
    if (a_mode != A_TOKEN || M > (epi == EPI_GLUQ ? 128 : 64) || N % (epi == EPI_GLUQ ? 128 : 32) != 0)
      return -2;
    if (epi == EPI_GLUQ) {
      if (os == nullptr || Mpad < mblocks * 16) return -2;
      // 8 tiles = 64 features; 16 waves as (TG tile groups) x (KW k-waves) within the LDS budget
      // one tile group (TG = 1): every wave holds all 8 tiles, so each activation fragment is
      // fetched once per workgroup (TG > 1 re-fetched it per group: 1 MB of L2 reads per CU at 64 rows)
      if (mblocks <= 1) {
        // 16 waves as 2 tile groups x 8 k-waves (batch 1, Llama-2-7B gate_up: 19.1 us against 21.1 us
        // for 8 waves holding all 8 tiles; the re-fetched activation row is 4 KiB); kw = 8 selects the latter
        if (g_gemv_kw == 8) return launch_one<1, 8, 1, 8, 2, A_TOKEN, EPI_GLUQ>(A, sa, Wp, sw, bias, out, os, M, N, K, KT, Mpad, st);
        return launch_one<1, 8, 2, 8, 2, A_TOKEN, EPI_GLUQ>(A, sa, Wp, sw, bias, out, os, M, N, K, KT, Mpad, st);
      }
      if (mblocks <= 2) return launch_one<2, 8, 1, 8, 2, A_TOKEN, EPI_GLUQ>(A, sa, Wp, sw, bias, out, os, M, N, K, KT, Mpad, st);
      {
        const int r = launch_ring_rows128<EPI_GLUQ>(A, sa, Wp, sw, bias, out, os, M, N, K, Mpad, false, st, 1);
        if (r != -1) return r;
        if (mblocks > 4) return -2;
      }
      // (4 waves with U = 2 / 4 and AGPR accumulators measured 45.6 / 41.4 us against 34.3 us here)
      return launch_one<4, 8, 1, 8, 1, A_TOKEN, EPI_GLUQ>(A, sa, Wp, sw, bias, out, os, M, N, K, KT, Mpad, st);
    }
    if (mblocks <= 1) return launch_one<1, 4, 2, 8, 2, A_TOKEN, EPI_GLU>(A, sa, Wp, sw, bias, out, nullptr, M, N, K, KT, Mpad, st);
    if (mblocks <= 2) return launch_one<2, 4, 2, 8, 2, A_TOKEN, EPI_GLU>(A, sa, Wp, sw, bias, out, nullptr, M, N, K, KT, Mpad, st);
    return launch_one<4, 4, 2, 4, 2, A_TOKEN, EPI_GLU>(A, sa, Wp, sw, bias, out, nullptr, M, N, K, KT, Mpad, st);
  }
  if (M > 64 && K % 64 == 0 && K / 64 == KT && N % 8 == 0)       // prefill (gemm_i8_prefill.hip)
    return edge_w8a8_prefill(A, sa, Wp, sw, bias, out, M, N, K, KT, st);
  if (M > 64) {
    // ragged-K prefill (tiny models): 64-row slabs through the GEMV
    for (int m0 = 0; m0 < M; m0 += 64) {
      const int rc = edge_w8a8_gemm((const int8_t*)A + (size_t)m0 * K, sa + m0, Wp, sw, bias,
                                    (bf16_t*)out + (size_t)m0 * N, nullptr, min(64, M - m0), N, K, KT, a_mode, 0, 0, st);
      if (rc) return rc;
    }
    return 0;
  }
  // NTW tiles per workgroup so that the grid is ~256 workgroups (one 16-wave group per CU)
  int ntw = g_gemv_ntw > 0 ? g_gemv_ntw : (NTt >= 512 ? min(4, (NTt + 128) / 256) : 1);
  const int un = g_gemv_unroll > 0 ? g_gemv_unroll : (ntw == 1 && KT >= 128 ? 4 : (mblocks > 2 ? 1 : 2));
  const int kw = g_gemv_kw > 0 ? g_gemv_kw : 16;
#define OUT(MBV, AMV) return launch_out<MBV, AMV>(ntw, un, kw, A, sa, Wp, sw, bias, out, M, N, K, KT, Mpad, st, \
                                                  epi == EPI_OUT ? os : nullptr)
  if (a_mode == A_GROUP) {
    if (mblocks <= 1) OUT(1, A_GROUP);
    if (mblocks <= 2) OUT(2, A_GROUP);
    OUT(4, A_GROUP);
  }
  if (mblocks <= 1) OUT(1, A_TOKEN);
  if (mblocks <= 2) OUT(2, A_TOKEN);
  OUT(4, A_TOKEN);
#undef OUT
}

// ------------------------------------------------------------------------------ bf16 ring2
// bf16 decode projections at 17-256 rows on the ring2 kernel (DT = 1).  The bf16 fragment-packed
// weight (ops.pack_bf16_weight: 1 KiB tiles of 16 rows x 32 k) and a row-major bf16 activation
// have, BYTE for byte, the layout of the int8 operands (a 64-B k-tile = 32 bf16, lane l's 16 B =
// k 8 (l >> 4) .. + 8 of row l & 15), so the kernel streams them unchanged with K counted in bytes
// and swaps the MFMA for v_mfma_f32_16x16x32_bf16 (same 16 cycles per 64 B of k as the i8 form).
// Rows 129-256 run as two 128-row halves that share each weight panel through one XCD's L2
// (MS = 2), so a 256-row decode step reads the bf16 weights from HBM once.
// Row floor 65: at 17-64 rows the ring kernel still computes 128-row tiles and re-reads the
// (clamped) activation lines, and hipBLASLt is ahead on qkv / gate_up.
extern "C" int edge_bf16_ring_min_rows() { return 65; }

namespace {
template <int NTWV, int NWLV, int RWV, int RAV, int NALV, int NCWV, int EPV, int MSV>
int launch_bfr(const void* A, const void* W, const void* bias, void* out, int M, int N, int K, int S, hipStream_t st) {
  const int NTt = N / 16, G = (NTt + NTWV - 1) / NTWV * S;
  const dim3 grid(MSV == 2 ? (G + 7) / 8 * 16 : G);
  hipLaunchKernelGGL((w8a8_gemv_ring2_kernel<NTWV, NWLV, RWV, RAV, EPV, false, false, MSV, NALV, NCWV, 1>), grid,
                     dim3((NCWV + NWLV + NALV) * 64), 0, st, (const int8_t*)A, nullptr, (const int8_t*)W, nullptr,
                     (const bf16_t*)bias, out, nullptr, M, N, 2 * K, NTt, 0, S, G);
  return (int)hipGetLastError();
}

template <int MSV>
int bfr_dispatch(const void* A, const void* W, const void* bias, void* out, int M, int N, int K, int epi, int S,
                 hipStream_t st) {
  const int NTt = N / 16;
  // logical workgroups wanted: ~256 launched blocks (MS = 2 launches each logical workgroup twice)
  const int want = MSV == 2 ? 128 : 256;
#define BFR(NTWV, NWLV, RWV, RAV, NALV, NCWV, EPV) \
  return launch_bfr<NTWV, NWLV, RWV, RAV, NALV, NCWV, EPV, MSV>(A, W, bias, out, M, N, K, S, st)
  if (epi == EPI_GLU) {                               // gate_up: NTW / 2 feature tiles per workgroup
    // one round of fat workgroups beats two rounds of thin ones (tools/bench_ops.py --only
    // bf16ring, Llama-2-7B gate_up at 256 rows: 16 tiles / 172 blocks 64.4 us, 8 tiles / 344
    // blocks 80.6 us)
    const int ft = NTt / 2;
    if (MSV == 2 && ft >= 8 * 64) BFR(16, 2, 3, 3, 2, 8, EPI_GLU);
    if (ft >= 4 * 128) BFR(8, 2, 5, 4, 2, 4, EPI_GLU);
    BFR(4, 2, 10, 4, 2, 4, EPI_GLU);
  }
  if (epi == EPI_PART) {                              // split-K slices (o / down before the norm)
    const int per = NTt * S / want;
    if (per >= 6) BFR(8, 2, 5, 4, 2, 4, EPI_PART);
    if (per >= 3) BFR(4, 2, 10, 4, 2, 4, EPI_PART);
    if (per >= 2) BFR(2, 2, 14, 4, 2, 4, EPI_PART);
    BFR(1, 2, 16, 4, 2, 4, EPI_PART);
  }
  const int per = (NTt + want / 2) / want;            // EPI_OUT
  if (per >= 12) BFR(16, 2, 3, 3, 2, 8, EPI_OUT);     // LM heads: one round (32000 x 4096 at 256 rows)
  if (per >= 7) BFR(8, 2, 5, 4, 2, 4, EPI_OUT);
  if (per >= 5) BFR(6, 2, 7, 4, 2, 4, EPI_OUT);
  if (per >= 4) BFR(4, 2, 10, 4, 2, 4, EPI_OUT);
  if (per >= 3) BFR(3, 2, 14, 4, 2, 4, EPI_OUT);
  if (per >= 2) BFR(2, 2, 14, 4, 2, 4, EPI_OUT);
  BFR(1, 2, 16, 4, 2, 4, EPI_OUT);
#undef BFR
}
}  // namespace

// Split-K slices S for the bf16 ring path's EPI_PART at this (N, K): >= 4 stages of 64 k per slice
extern "C" int edge_bf16_ring_splits(int N, int K) {
  const int stages = K / 64;                           // 128-B stages of bf16 k
  // fewer slices halve each workgroup's activation re-reads; narrow N takes more to fill the chip.
  // N = 4096 measured S=4 over S=2 (o 14.4 vs 15.2 us at 128 rows, down 37.5 vs 42.8 us at 256 rows;
  // +1.6 % / +3.1 % bench tok/s at 1x256 / 2x128, profiles/bench_ops_r3_bf16splits.json)
  const int NTt = N / 16;
  int S = NTt >= 384 ? 2 : (NTt >= 64 ? 4 : 8);
  while (S > 1 && stages < 4 * S) --S;
  return S;
}

// y = x . W^T (+ bias) for bf16 x [M, K] and fragment-packed bf16 W (17 <= M <= 256, K % 64 == 0,
// N % 16 == 0; GLU: N % 32 == 0).  epi 0: bf16 [M, N]; 1: silu(gate) * up bf16 [M, N / 2] over
// W = [gate | up]; 3 (EPI_PART): fp32 partial slices [S, M, N] (bias in slice 0).  -2: not taken.
extern "C" int edge_gemm_bf16_ring(const void* A, const void* W, const void* bias, void* out, int M, int N, int K,
                                   int epi, int S, hipStream_t st) {
  if (M < 1 || M > 256 || K % 64 != 0 || K <= 0 || N % 16 != 0 || (epi == EPI_GLU && N % 32 != 0)) return -2;
  if (epi != EPI_OUT && epi != EPI_GLU && epi != EPI_PART) return -2;
  if ((epi == EPI_PART) != (S > 1) || S < 1 || (S > 1 && K / 64 < 4 * S)) return -2;
  return M > 128 ? bfr_dispatch<2>(A, W, bias, out, M, N, K, epi, S, st)
                 : bfr_dispatch<1>(A, W, bias, out, M, N, K, epi, S, st);
}

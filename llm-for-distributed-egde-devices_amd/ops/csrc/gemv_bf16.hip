// Decode GEMV for bf16 weights: y[M, N] = x[M, K] . W[N, K]^T (+ bias) -> bf16, M <= 64
// (MB = 1..4 row blocks of 16: every weight fragment feeds MB MFMAs, so 17-64 decode rows read the
// weights once instead of hipBLASLt's small-M kernels).
// The fp16/bf16 evaluators (Phi-2, Pythia-1B, Llama-3.2-1B at batch 1) spend
// most of a decode step here; hipBLASLt's small-M kernels stream the weights at about 2 TB/s.
//
// Weights are read in MFMA fragment order (ops.pack_bf16_weight, a decode-only copy of the HF
// [N, K] tensor that prefill keeps using): 1 KiB tiles of 16 rows x 32 k, tile (nt, kt) at
// ((nt * K/32) + kt) * 512 elements, lane l's 8 elements = W[16 nt + (l & 15)][32 kt + 8 (l >> 4) ..]
// — the B fragment of v_mfma_f32_16x16x32_bf16.  A wave walks K in pairs of k-steps, i.e. 2 KiB
// of contiguous weights per tile per pair (the [N, K] layout gave each load instruction 16 rows x
// 64 B: 36 % more bytes fetched and 2.3 TB/s on Llama-3.2-1B's gate_up).  A workgroup = 16 waves
// on NTW 16-column tiles; wave w takes k-pairs w, w + 16, ..., keeping U pairs of weight loads in
// flight (nontemporal: each weight byte is read once per step).  The 16 partial tiles are
// reduced through LDS.  Rows >= M load a clamped row and are never stored.
//   EPI_OUT: + bias, bf16 [M, N].
//   EPI_GLU: W = [gate (F rows) | up (F rows)] (the natural gate_up concatenation); a workgroup's
//            tiles are NTW/2 gate tiles and the matching up tiles, and it writes
//            h = silu(gate) * up as bf16 [M, F] (gate and up rounded to bf16 first, as the
//            unfused GEMM output is) — the separate SwiGLU launch disappears.
//   EPI_GELU_TANH / EPI_GELU: gelu(bf16(y + bias)) -> bf16 [M, N] (Phi-2 / Pythia MLP up
//            projection; the same math as rowwise.hip::act_kernel modes 1 / 2).
//   EPI_PART: split-K, workgroup (group, ks) reduces k-pairs [KP ks / S, KP (ks + 1) / S) and
//            writes fp32 partials part[ks][M][N] (bias in slice 0) for a norm kernel that sums
//            them (the o / down projections of RMSNorm decoders; N = 2048 has only 128 tiles).
// HF: fp16 activations / weights / outputs on v_mfma_f32_16x16x32_f16 (the reference's fp16 agents,
// Phi-2 / Pythia); the same fragment layout and epilogues with fp16 roundings.
#include "common.h"

namespace {
constexpr int EPI_OUT = 0, EPI_GLU = 1, EPI_GELU_TANH = 2, EPI_GELU = 3, EPI_PART = 4;
constexpr int NW = 16;

typedef _Float16 v8h __attribute__((ext_vector_type(8)));

template <bool HF>
__device__ __forceinline__ v4f mfma_16(const v8s& a, const v8s& b, const v4f& c) {
  if constexpr (HF)
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(v8h, a), __builtin_bit_cast(v8h, b), c, 0, 0, 0);
  else return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ v8s ld_nt(const bf16_t* p) {
  return __builtin_bit_cast(v8s, __builtin_nontemporal_load(reinterpret_cast<const v4i*>(p)));
}

// Decode RMSNorm prologue for the 16-bit GEMV (NRM > 0, M <= 4 rows, K 2048 / 4096): the activation
// rows are RMSNorm(sum of S fp32 split-K slices + residual), computed in the consumer instead of a
// norm launch of its own (rowwise.hip norm_kernel<NCH, RMS, HAS_RES, !QUANT, PART>: the same
// element layout, reduction order and roundings, so the rows are bit-identical).  Four 256-thread
// groups, one row each; the normalised 16-bit rows go to LDS, where the k-loop reads its A
// fragments.  The slices, residual and gamma loads all issue before any use.  Workgroup 0 writes
// the new residual rows.  NRM = 8 * NCH + SMAX (S <= SMAX slices).
// LN (NRM >= 64): LayerNorm of x + residual with 16-bit input rows x (the parallel-residual
// decoders, Phi-2 / GPT-NeoX: norm_kernel<NCH, !RMS, HAS_RES, !QUANT, !PART>), K up to 4096.
struct NormIn16 {
  const float* part;      // [S][M][K] fp32 slices (RMS)
  const bf16_t* res;      // [M][K] residual in (null: none, a stage's first norm over the embedding)
  const bf16_t* gamma;    // [K]
  bf16_t* res_out;        // [M][K] residual out (must not alias res)
  float eps;
  int S;
  const bf16_t* x;        // [M][K] 16-bit input rows (LN)
  const bf16_t* beta;     // [K] (LN; may be null)
  bf16_t* y_out;          // [M][K] (LN; may be null): workgroup 0 also writes the normalised rows here
};
constexpr int NRM16_ROWS = 4;

template <int NCH, int SMAX, bool LN = false>
struct NormRegs16 {
  uint4 rv[NCH], gv[NCH];
  float4 pv[NCH][LN ? 1 : SMAX][2];
  uint4 xv[NCH], bv[NCH];
};

template <int NCH, int SMAX, bool LN>
__device__ __forceinline__ void norm16_load(const NormIn16& na, int H, int M, NormRegs16<NCH, SMAX, LN>& nr) {
  const int t = threadIdx.x & 255, row = threadIdx.x >> 8;
  uint4 (&rv)[NCH] = nr.rv;
  uint4 (&gv)[NCH] = nr.gv;
  auto& pv = nr.pv;
  if constexpr (LN) {
    if (row < M) {
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const int e = min((c * 256 + t) * 8, H - 8);
        nr.xv[c] = *reinterpret_cast<const uint4*>(na.x + (size_t)row * H + e);
        rv[c] = na.res != nullptr ? *reinterpret_cast<const uint4*>(na.res + (size_t)row * H + e) : uint4{0u, 0u, 0u, 0u};
        gv[c] = *reinterpret_cast<const uint4*>(na.gamma + e);
        nr.bv[c] = na.beta != nullptr ? *reinterpret_cast<const uint4*>(na.beta + e) : uint4{0u, 0u, 0u, 0u};
      }
    }
    asm volatile("" ::: "memory");
    return;
  }
  if (row < M) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int e = min((c * 256 + t) * 8, H - 8);
      rv[c] = na.res != nullptr ? *reinterpret_cast<const uint4*>(na.res + (size_t)row * H + e) : uint4{0u, 0u, 0u, 0u};
#pragma unroll
      for (int k = 0; k < SMAX; ++k)
        if (k < na.S) {
          const float4* p = reinterpret_cast<const float4*>(na.part + ((size_t)k * M + row) * H + e);
          pv[c][k][0] = p[0];
          pv[c][k][1] = p[1];
        }
      gv[c] = *reinterpret_cast<const uint4*>(na.gamma + e);
    }
  }
  asm volatile("" ::: "memory");                          // these loads issue before the weights
}

// LayerNorm form (norm_kernel's !RMS, HAS_RES, !PART path: x + residual rounded to 16 bits, the
// mean, then the variance of the rounded row, gamma and beta)
template <int NCH, bool HF>
__device__ __forceinline__ void ln16_prologue(const NormIn16& na, int H, int M, bf16_t* xs, float* nred,
                                              const NormRegs16<NCH, 1, true>& nr) {
  const int t = threadIdx.x & 255, row = threadIdx.x >> 8, w = t >> 6;
  const bool act = row < M;
  float v[NCH][8];
  float sm = 0.f;
  if (act) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int e = (c * 256 + t) * 8;
      if (e < H) {
        unpack8e<HF>(nr.xv[c], v[c]);
        float r[8];
        unpack8e<HF>(nr.rv[c], r);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] += r[j];
        const uint4 u = pack8e<HF>(v[c]);                    // the residual stream in 16 bits
        if (blockIdx.x == 0) *reinterpret_cast<uint4*>(na.res_out + (size_t)row * H + e) = u;
        unpack8e<HF>(u, v[c]);
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
  float mean = 0.f, ss = 0.f;
  if (act) {
    const float* gr = nred + 4 * row;
    mean = ((((0.f + gr[0]) + gr[1]) + gr[2]) + gr[3]) / (float)H;
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
  __syncthreads();                                        // every group has read its sums
  if (act && (t & 63) == 0) nred[4 * row + w] = ss;
  __syncthreads();
  if (act) {
    const float* gr = nred + 4 * row;
    const float rstd = rsqrtf(((((0.f + gr[0]) + gr[1]) + gr[2]) + gr[3]) / (float)H + na.eps);
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int e = (c * 256 + t) * 8;
      if (e < H) {
        float wf[8], bf[8];
        unpack8e<HF>(nr.gv[c], wf);
        unpack8e<HF>(nr.bv[c], bf);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] = (v[c][j] - mean) * rstd * wf[j] + bf[j];
        const uint4 u = pack8e<HF>(v[c]);
        *reinterpret_cast<uint4*>(xs + (size_t)row * H + e) = u;
        if (na.y_out != nullptr && blockIdx.x == 0) *reinterpret_cast<uint4*>(na.y_out + (size_t)row * H + e) = u;
      }
    }
  }
  __syncthreads();                                        // the rows are complete in LDS
}

template <int NCH, int SMAX, bool HF>
__device__ __forceinline__ void norm16_prologue(const NormIn16& na, int H, int M, bf16_t* xs, float* nred,
                                                const NormRegs16<NCH, SMAX>& nr) {
  const int t = threadIdx.x & 255, row = threadIdx.x >> 8, w = t >> 6;
  const bool act = row < M;
  const uint4* rv = nr.rv;
  const uint4* gv = nr.gv;
  const auto& pv = nr.pv;
  float v[NCH][8];
  float ss = 0.f;
  if (act) {
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
        unpack8e<HF>(pack8e<HF>(v[c]), v[c]);                 // the projection's 16-bit output
        float r[8];
        unpack8e<HF>(rv[c], r);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] += r[j];
        const uint4 u = pack8e<HF>(v[c]);                    // the residual stream in 16 bits
        if (blockIdx.x == 0) *reinterpret_cast<uint4*>(na.res_out + (size_t)row * H + e) = u;
        unpack8e<HF>(u, v[c]);
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
    if ((t & 63) == 0) nred[4 * row + w] = ss;
  }
  __syncthreads();
  if (act) {
    const float* gr = nred + 4 * row;
    const float rstd = rsqrtf((((0.f + gr[0]) + gr[1]) + gr[2] + gr[3]) / (float)H + na.eps);
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int e = (c * 256 + t) * 8;
      if (e < H) {
        float wf[8];
        unpack8e<HF>(gv[c], wf);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] = (v[c][j] - 0.f) * rstd * wf[j];
        *reinterpret_cast<uint4*>(xs + (size_t)row * H + e) = pack8e<HF>(v[c]);
      }
    }
  }
  __syncthreads();                                        // the rows are complete in LDS
}

template <int MB, int NTW, int U, int EPI, bool HF, int NRM = 0>
__global__ void __launch_bounds__(NW * 64) gemv_bf16_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
                                                            const bf16_t* __restrict__ bias, bf16_t* __restrict__ out,
                                                            int M, int N, int K, int F, int S,
                                                            const bf16_t* __restrict__ add, NormIn16 na) {
  static_assert(EPI != EPI_GLU || NTW % 2 == 0, "GLU: gate/up tile pairs");
  static_assert(MB * NTW <= 8 && MB * (EPI == EPI_GLU ? NTW / 2 : NTW) <= NW, "LDS reduction / output waves");
  static_assert(NRM == 0 || (MB == 1 && NTW <= 4 && EPI != EPI_PART), "norm prologue: up to 4 rows, LDS budget");
  __shared__ v4f red[NW][MB * NTW][64];
  // NRM: 8 NCH + SMAX (RMSNorm over split-K slices), + 64 for the LayerNorm of 16-bit rows
  constexpr bool LN_N = NRM >= 64;
  constexpr int NCH_N = (NRM % 64) / 8, SMAX_N = LN_N ? 1 : NRM % 8;
  __shared__ __attribute__((aligned(16))) bf16_t xs[NRM > 0 ? NRM16_ROWS * NCH_N * 2048 : 8];
  __shared__ float nred[16];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 15, kq = 8 * (lane >> 4);
  // output column of tile j for this lane (EPI_GLU: gate tiles then the matching up tiles)
  const int grp = EPI == EPI_PART ? (int)blockIdx.x / S : (int)blockIdx.x;
  const int ks = EPI == EPI_PART ? (int)blockIdx.x % S : 0;
  auto col_of = [&](int j) -> int {
    if constexpr (EPI == EPI_GLU) {
      const int f0 = grp * (NTW / 2) * 16;
      return j < NTW / 2 ? f0 + j * 16 + r : F + f0 + (j - NTW / 2) * 16 + r;
    } else {
      return (grp * NTW + j) * 16 + r;
    }
  };
  const int KP = K / 64;
  const int kbeg = EPI == EPI_PART ? KP * ks / S : 0, kend = EPI == EPI_PART ? KP * (ks + 1) / S : KP;
  const bf16_t* wrow[NTW];                                  // tile row of this lane's fragments
#pragma unroll
  for (int j = 0; j < NTW; ++j) wrow[j] = W + ((size_t)(min(col_of(j), N - 1) >> 4) * (2 * KP) * 64 + lane) * 8;
  const bf16_t* arow[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) arow[mb] = (NRM > 0 ? xs : A) + (size_t)min(16 * mb + r, M - 1) * K + kq;
  // NRM: the prologue's loads, then the first k-pair's weights, are in flight before the norm
  // runs (a wave's loads retire in issue order: weights first would make the norm wait for them)
  NormRegs16<(NRM > 0 ? NCH_N : 1), (NRM > 0 ? SMAX_N : 1), LN_N> nr;
  v8s b0[NTW][2];
  if constexpr (NRM > 0) {
    norm16_load(na, K, M, nr);
    const int k = min(kbeg + wave, kend - 1) * 64;
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      b0[j][0] = ld_nt(wrow[j] + (size_t)k * 16);
      b0[j][1] = ld_nt(wrow[j] + (size_t)k * 16 + 512);
    }
    if constexpr (LN_N) ln16_prologue<NCH_N, HF>(na, K, M, xs, nred, nr);
    else norm16_prologue<NCH_N, SMAX_N, HF>(na, K, M, xs, nred, nr);
  }
  v4f acc[MB][NTW];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb)
#pragma unroll
    for (int j = 0; j < NTW; ++j) acc[mb][j] = v4f{0.f, 0.f, 0.f, 0.f};
  bool first = NRM > 0;
  for (int kp = kbeg + wave; kp < kend; kp += NW * U) {
    v8s a[U][MB][2], b[U][NTW][2];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = min(kp + u * NW, kend - 1) * 64;        // clamped: loads never branch
#pragma unroll
      for (int j = 0; j < NTW; ++j) {                        // tiles 2 kp, 2 kp + 1: 2 KiB contiguous
        if (NRM > 0 && u == 0 && first) {
          b[u][j][0] = b0[j][0];
          b[u][j][1] = b0[j][1];
        } else {
          b[u][j][0] = ld_nt(wrow[j] + (size_t)k * 16);
          b[u][j][1] = ld_nt(wrow[j] + (size_t)k * 16 + 512);
        }
      }
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) {
        a[u][mb][0] = *reinterpret_cast<const v8s*>(arow[mb] + k);
        a[u][mb][1] = *reinterpret_cast<const v8s*>(arow[mb] + k + 32);
      }
    }
    first = false;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (kp + u * NW < kend) {                             // wave-uniform (scalar) guard
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
#pragma unroll
          for (int j = 0; j < NTW; ++j) {
            acc[mb][j] = mfma_16<HF>(a[u][mb][0], b[u][j][0], acc[mb][j]);
            acc[mb][j] = mfma_16<HF>(a[u][mb][1], b[u][j][1], acc[mb][j]);
          }
      }
    }
  }
#pragma unroll
  for (int mb = 0; mb < MB; ++mb)
#pragma unroll
    for (int j = 0; j < NTW; ++j) red[wave][mb * NTW + j][lane] = acc[mb][j];
  __syncthreads();
  // output units (row block, tile): wave w < MB * OUTS writes tile w % OUTS of row block w / OUTS
  constexpr int OUTS = EPI == EPI_GLU ? NTW / 2 : NTW;
  if (wave < MB * OUTS) {
    const int mb = wave / OUTS, tw = wave - mb * OUTS;
    auto total = [&](int j) {                               // 4 LDS reads in flight (bounded registers)
      v4f s = red[0][mb * NTW + j][lane];
#pragma unroll 4
      for (int w = 1; w < NW; ++w) s += red[w][mb * NTW + j][lane];
      return s;
    };
    const int c0 = col_of(tw);
    if constexpr (EPI == EPI_GLU) {
      const int c1 = col_of(tw + NTW / 2);
      const v4f g4 = total(tw), u4 = total(tw + NTW / 2);
      const float bg = bias != nullptr ? e2f<HF>(bias[c0]) : 0.f, bu = bias != nullptr ? e2f<HF>(bias[c1]) : 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = 16 * mb + 4 * (lane >> 4) + q;
        const float g = e2f<HF>(f2e<HF>(g4[q] + bg)), u = e2f<HF>(f2e<HF>(u4[q] + bu));
        if (row < M && c0 < F) out[(size_t)row * F + c0] = f2e<HF>(g / (1.f + __expf(-g)) * u);
      }
    } else if constexpr (EPI == EPI_PART) {
      const v4f s4 = total(tw);
      const float bv = bias != nullptr && c0 < N && ks == 0 ? e2f<HF>(bias[c0]) : 0.f;
      float* part = reinterpret_cast<float*>(out) + (size_t)ks * M * N;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = 16 * mb + 4 * (lane >> 4) + q;
        if (row < M && c0 < N) part[(size_t)row * N + c0] = s4[q] + bv;
      }
    } else {
      const v4f s4 = total(tw);
      const float bv = bias != nullptr && c0 < N ? e2f<HF>(bias[c0]) : 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = 16 * mb + 4 * (lane >> 4) + q;
        float v = s4[q] + bv;
        if constexpr (EPI == EPI_GELU_TANH) {
          const float a = e2f<HF>(f2e<HF>(v)), k0 = 0.7978845608028654f, k1 = 0.044715f;
          v = 0.5f * a * (1.f + tanhf(k0 * (a + k1 * a * a * a)));
        } else if constexpr (EPI == EPI_GELU) {
          const float a = e2f<HF>(f2e<HF>(v));
          v = 0.5f * a * (1.f + erff(a * 0.7071067811865476f));
        } else {
          // EPI_OUT with an addend (parallel-residual block): rnd(rnd(y) + add), the unfused add
          if (add != nullptr && row < M && c0 < N) v = e2f<HF>(f2e<HF>(v)) + e2f<HF>(add[(size_t)row * N + c0]);
        }
        if (row < M && c0 < N) out[(size_t)row * N + c0] = f2e<HF>(v);
      }
    }
  }
}

template <int MB, int NTW, int U, int EPI, bool HF, int NRM = 0>
int launch_mb(const void* A, const void* W, const void* bias, void* out, int M, int N, int K, int F, int tiles,
              hipStream_t st, int S, const void* add = nullptr, const NormIn16& na = NormIn16{}) {
  const int groups = EPI == EPI_GLU ? tiles / (NTW / 2) : (tiles + NTW - 1) / NTW;
  hipLaunchKernelGGL((gemv_bf16_kernel<MB, NTW, U, EPI, HF, NRM>), dim3(groups * S), dim3(NW * 64), 0, st,
                     (const bf16_t*)A, (const bf16_t*)W, (const bf16_t*)bias, (bf16_t*)out, M, N, K, F, S,
                     (const bf16_t*)add, na);
  return (int)hipGetLastError();
}

// NTW / U chosen for one row block; more row blocks keep U = 2 (registers) and at most 8 / MB
// tiles (the LDS reduction holds MB x NTW tiles of 16 waves)
template <int NTW, int U, int EPI, bool HF>
int launch(const void* A, const void* W, const void* bias, void* out, int M, int N, int K, int F, int tiles,
           hipStream_t st, int S = 1, const void* add = nullptr) {
  constexpr int G = EPI == EPI_GLU ? 2 : 1;                 // GLU keeps gate / up pairs
  constexpr int N2 = NTW > 4 ? 4 : (NTW < G ? G : NTW), N34 = NTW > 2 ? 2 : (NTW < G ? G : NTW);
  const int mb = (M + 15) / 16;
  if (mb <= 1) return launch_mb<1, NTW, U, EPI, HF>(A, W, bias, out, M, N, K, F, tiles, st, S, add);
  if (mb == 2) return launch_mb<2, N2, 2, EPI, HF>(A, W, bias, out, M, N, K, F, tiles, st, S, add);
  if (mb == 3) return launch_mb<3, N34, 2, EPI, HF>(A, W, bias, out, M, N, K, F, tiles, st, S, add);
  return launch_mb<4, N34, 2, EPI, HF>(A, W, bias, out, M, N, K, F, tiles, st, S, add);
}

// W: fragment-packed bf16 (ops.pack_bf16_weight).  epi 0: out bf16 [M, N] (+ the bf16 addend `add`
// [M, N] when not null: a parallel-residual block's other branch); epi 1 (GLU):
// W = [gate | up] with N = 2F, out = silu(gate) * up bf16 [M, F] (F % 16 == 0); epi 2 / 3: gelu (tanh / erf) of the bf16 output.  M <= 64, K % 64 == 0,
// N % 16 == 0.  Returns -2 for shapes it does not take.
template <bool HF>
int gemv_run(const void* A, const void* W, const void* bias, void* out, int M, int N, int K, int epi, hipStream_t st,
             const void* add) {
  if (M <= 0 || M > 64 || K % 64 != 0 || N % 16 != 0 || K <= 0) return -2;
  const int KP = K / 64;
  const int U = KP >= 64 ? 4 : 2;                            // k-pairs in flight per wave
  if (epi == EPI_GLU) {
    if (N % 32 != 0) return -2;
    const int F = N / 2, ft = F / 16;
    if (ft >= 512) return launch<4, 2, EPI_GLU, HF>(A, W, bias, out, M, N, K, F, ft, st);
    return U == 4 ? launch<2, 4, EPI_GLU, HF>(A, W, bias, out, M, N, K, F, ft, st)
                  : launch<2, 2, EPI_GLU, HF>(A, W, bias, out, M, N, K, F, ft, st);
  }
  if (epi != EPI_OUT && epi != EPI_GELU_TANH && epi != EPI_GELU) return -2;
  const int nt = N / 16;
  // ~256 workgroups: one tile each below 512 tiles, then 2 or 4
#define PICK(EP)                                                                               \
  if (nt >= 1024) return launch<4, 2, EP, HF>(A, W, bias, out, M, N, K, 0, nt, st);                \
  if (nt >= 512) return U == 4 ? launch<2, 4, EP, HF>(A, W, bias, out, M, N, K, 0, nt, st)         \
                               : launch<2, 2, EP, HF>(A, W, bias, out, M, N, K, 0, nt, st);        \
  return U == 4 ? launch<1, 4, EP, HF>(A, W, bias, out, M, N, K, 0, nt, st)                        \
                : launch<1, 2, EP, HF>(A, W, bias, out, M, N, K, 0, nt, st);
  if (epi == EPI_GELU_TANH) { PICK(EPI_GELU_TANH) }
  if (epi == EPI_GELU) { PICK(EPI_GELU) }
  // plain output, optionally + a bf16 addend [M, N]
  if (nt >= 1024) return launch<4, 2, EPI_OUT, HF>(A, W, bias, out, M, N, K, 0, nt, st, 1, add);
  if (nt >= 512) return U == 4 ? launch<2, 4, EPI_OUT, HF>(A, W, bias, out, M, N, K, 0, nt, st, 1, add)
                               : launch<2, 2, EPI_OUT, HF>(A, W, bias, out, M, N, K, 0, nt, st, 1, add);
  return U == 4 ? launch<1, 4, EPI_OUT, HF>(A, W, bias, out, M, N, K, 0, nt, st, 1, add)
                : launch<1, 2, EPI_OUT, HF>(A, W, bias, out, M, N, K, 0, nt, st, 1, add);
#undef PICK
}

// The 16-bit GEMV over RMSNorm(sum(parts) + residual) (norm16_prologue): M <= 4, K 2048 / 4096,
// S <= 4 slices; epi 0 (EPI_OUT) or 1 (EPI_GLU).  The geometry of gemv_run for one row block.
template <bool HF, int NRM>
int gemv_norm_geo(const NormIn16& na, const void* W, const void* bias, void* out, int M, int N, int K, int epi,
                  hipStream_t st) {
  const int KP = K / 64, U = KP >= 64 ? 4 : 2;
  if (epi == EPI_GLU) {
    const int F = N / 2, ft = F / 16;
    if (ft >= 512) {
      if constexpr (NRM == 20) return -2;                // 4 tiles + 3-4 held slices of K = 4096: spills
      else return launch_mb<1, 4, 2, EPI_GLU, HF, NRM>(nullptr, W, bias, out, M, N, K, F, ft, st, 1, nullptr, na);
    }
    return U == 4 ? launch_mb<1, 2, 4, EPI_GLU, HF, NRM>(nullptr, W, bias, out, M, N, K, F, ft, st, 1, nullptr, na)
                  : launch_mb<1, 2, 2, EPI_GLU, HF, NRM>(nullptr, W, bias, out, M, N, K, F, ft, st, 1, nullptr, na);
  }
  const int nt = N / 16;
#define NPICK(EP)                                                                                              \
  if (nt >= 1024) {                                                                                            \
    if constexpr (NRM == 20) return -2;                                                                        \
    else return launch_mb<1, 4, 2, EP, HF, NRM>(nullptr, W, bias, out, M, N, K, 0, nt, st, 1, nullptr, na);     \
  }                                                                                                            \
  if (nt >= 512)                                                                                               \
    return U == 4 ? launch_mb<1, 2, 4, EP, HF, NRM>(nullptr, W, bias, out, M, N, K, 0, nt, st, 1, nullptr, na)  \
                  : launch_mb<1, 2, 2, EP, HF, NRM>(nullptr, W, bias, out, M, N, K, 0, nt, st, 1, nullptr, na); \
  return U == 4 ? launch_mb<1, 1, 4, EP, HF, NRM>(nullptr, W, bias, out, M, N, K, 0, nt, st, 1, nullptr, na)    \
                : launch_mb<1, 1, 2, EP, HF, NRM>(nullptr, W, bias, out, M, N, K, 0, nt, st, 1, nullptr, na);
  if (epi == EPI_GELU_TANH) { NPICK(EPI_GELU_TANH) }
  if (epi == EPI_GELU) { NPICK(EPI_GELU) }
  NPICK(EPI_OUT)
#undef NPICK
}

// LayerNorm prologue over 16-bit rows x (+ residual): K <= 4096 (K % 64 == 0), epi 0 / 2 / 3.
template <bool HF>
int gemv_ln_run(const NormIn16& na, const void* W, const void* bias, void* out, int M, int N, int K, int epi,
                hipStream_t st) {
  if (M < 1 || M > NRM16_ROWS || K > 4096 || K % 64 != 0 || N % 16 != 0 || na.x == nullptr ||
      (epi != EPI_OUT && epi != EPI_GELU_TANH && epi != EPI_GELU) || na.res_out == nullptr || na.res == na.res_out ||
      na.x == na.res_out || na.y_out == na.x || na.y_out == na.res_out)
    return -2;
  return K <= 2048 ? gemv_norm_geo<HF, 64 + 8>(na, W, bias, out, M, N, K, epi, st)
                   : gemv_norm_geo<HF, 64 + 16>(na, W, bias, out, M, N, K, epi, st);
}

template <bool HF>
int gemv_norm_run(const NormIn16& na, const void* W, const void* bias, void* out, int M, int N, int K, int epi,
                  hipStream_t st) {
  if (M < 1 || M > NRM16_ROWS || na.S < 1 || na.S > 4 || (K != 2048 && K != 4096) || N % 16 != 0 ||
      (epi != EPI_OUT && epi != EPI_GLU) || (epi == EPI_GLU && N % 32 != 0) || na.res_out == nullptr ||
      na.res == na.res_out)
    return -2;
  if (K == 4096) return na.S <= 2 ? gemv_norm_geo<HF, 18>(na, W, bias, out, M, N, K, epi, st)
                                  : gemv_norm_geo<HF, 20>(na, W, bias, out, M, N, K, epi, st);
  return na.S <= 2 ? gemv_norm_geo<HF, 10>(na, W, bias, out, M, N, K, epi, st)
                   : gemv_norm_geo<HF, 12>(na, W, bias, out, M, N, K, epi, st);
}

// Split-K form: fp32 partial slices part [S, M, N] (bias in slice 0), one 16-column tile per group.
template <bool HF>
int gemv_splitk_run(const void* A, const void* W, const void* bias, float* part, int M, int N, int K, int S,
                    hipStream_t st) {
  if (M <= 0 || M > 64 || K % 64 != 0 || N % 16 != 0 || S < 1 || S > K / 64) return -2;
  const int nt = N / 16, kps = K / 64 / S;
  return kps >= 64 ? launch<1, 4, EPI_PART, HF>(A, W, bias, part, M, N, K, 0, nt, st, S)
                   : launch<1, 2, EPI_PART, HF>(A, W, bias, part, M, N, K, 0, nt, st, S);
}
}  // namespace

// h16: fp16 operands / outputs (fragment-packed fp16 weights), else bf16
extern "C" int edge_gemv_bf16(const void* A, const void* W, const void* bias, void* out, int M, int N, int K, int epi,
                              hipStream_t st, const void* add, int h16) {
  return h16 ? gemv_run<true>(A, W, bias, out, M, N, K, epi, st, add)
             : gemv_run<false>(A, W, bias, out, M, N, K, epi, st, add);
}

extern "C" int edge_gemv_bf16_splitk(const void* A, const void* W, const void* bias, float* part, int M, int N, int K,
                                     int S, hipStream_t st, int h16) {
  return h16 ? gemv_splitk_run<true>(A, W, bias, part, M, N, K, S, st)
             : gemv_splitk_run<false>(A, W, bias, part, M, N, K, S, st);
}

// 16-bit decode GEMV (M <= 4) over RMSNorm(sum of S fp32 slices part [S, M, K] + res) in its
// prologue; res may be null (a stage's first norm); res_out [M, K] gets the new residual rows
// (workgroup 0).  epi 0: out [M, N]; 1: SwiGLU of W = [gate | up], out [M, N / 2].  -2: not taken.
extern "C" int edge_gemv_bf16_norm(const float* part, int S, const void* res, const void* gamma, float eps,
                                   void* res_out, const void* W, const void* bias, void* out, int M, int N, int K,
                                   int epi, hipStream_t st, int h16) {
  const NormIn16 na{part, (const bf16_t*)res, (const bf16_t*)gamma, (bf16_t*)res_out, eps, S, nullptr, nullptr,
                    nullptr};
  return h16 ? gemv_norm_run<true>(na, W, bias, out, M, N, K, epi, st)
             : gemv_norm_run<false>(na, W, bias, out, M, N, K, epi, st);
}

// 16-bit decode GEMV (M <= 4) over LayerNorm(x + res) (res may be null) in its prologue; res_out
// [M, K] gets x + res (workgroup 0), y_out (when not null) the normalised rows, for a second
// consumer.  epi 0: out [M, N]; 2 / 3: gelu (tanh / erf).  -2: not taken.
extern "C" int edge_gemv_bf16_ln(const void* x, const void* res, const void* gamma, const void* beta, float eps,
                                 void* res_out, const void* W, const void* bias, void* out, int M, int N, int K,
                                 int epi, hipStream_t st, int h16, void* y_out) {
  const NormIn16 na{nullptr, (const bf16_t*)res, (const bf16_t*)gamma, (bf16_t*)res_out, eps, 0, (const bf16_t*)x,
                    (const bf16_t*)beta, (bf16_t*)y_out};
  return h16 ? gemv_ln_run<true>(na, W, bias, out, M, N, K, epi, st)
             : gemv_ln_run<false>(na, W, bias, out, M, N, K, epi, st);
}

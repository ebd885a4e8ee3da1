// W8A8 INT8 GEMM on CDNA4 MFMA (v_mfma_i32_16x16x64_i8) with fused dequant epilogue.
//   out[m][n] = (sum_k A[m][k] * W[n][k]) * a_scale[m] * w_scale[n] (+ bias[n])   -> bf16
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
// Kernels:
//   gemv:  M <= 64 per block-row (decode). HBM-bound on W: each workgroup owns one 16-column
//          panel, its 4 waves split K and keep UNROLL fragments in flight (no LDS staging:
//          the weights are read exactly once), partial sums reduced through LDS.
//   tiled: M > 64 (prefill). 128x128 block tile, BK=64, 4 waves in 2x2, A and B staged with
//          global_load_lds (16 B/lane, lane-linear fragment-ordered LDS images -> conflict-free
//          ds_read_b128), LDS double buffer.
#include "common.h"

namespace {
constexpr int NT = 256;

__device__ __forceinline__ v4i mfma_i8(const v4i& a, const v4i& b, const v4i& c) {
  return __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void store_out(bf16_t* __restrict__ out, int M, int N, int row, int col, int acc,
                                          const float* __restrict__ sa, const float* __restrict__ sw,
                                          const bf16_t* __restrict__ bias) {
  if (row < M && col < N) {
    float v = (float)acc * sa[row] * sw[col];
    if (bias) v += bf2f(bias[col]);
    out[(size_t)row * N + col] = f2bf(v);
  }
}

// ------------------------------------------------------------------------------------ gemv
// Activation scales: per token (sa[M], AG = false; int32 accumulation over all of K) or per
// (token, 64-column group) (AG = true; sa laid out [KT][Mpad], written by the fused producers —
// attention and the GLU epilogue below).  With AG each k-tile's MFMA starts from zero and is
// folded into a float accumulator with its group scale (4 cvt + 4 fma per 16x16 tile).
__device__ __forceinline__ v4f group_scales(const float* __restrict__ sa, int k, int KT, int Mpad, int r0) {
  return k < KT ? *reinterpret_cast<const v4f*>(sa + (size_t)k * Mpad + r0) : v4f{0.f, 0.f, 0.f, 0.f};
}

__device__ __forceinline__ void fold(v4f& accf, const v4i& t, const v4f& s) {
#pragma unroll
  for (int q = 0; q < 4; ++q) accf[q] += (float)t[q] * s[q];
}

__device__ __forceinline__ void store_out_f(bf16_t* __restrict__ out, int M, int N, int row, int col, float v,
                                            const float* __restrict__ sw, const bf16_t* __restrict__ bias) {
  if (row < M && col < N) {
    v *= sw[col];
    if (bias) v += bf2f(bias[col]);
    out[(size_t)row * N + col] = f2bf(v);
  }
}

// NW waves per workgroup split K; k-tile kt goes to wave kt % NW, so at each unrolled step the
// workgroup's NW waves read NW consecutive 1 KiB tiles = one contiguous NW KiB run of the panel.
// UNROLL tiles per wave are in flight before the first MFMA (nontemporal: read-once weights).
template <int MT, int UNROLL, int NW, bool AG>
__global__ void __launch_bounds__(NW * 64) w8a8_gemv_kernel(const int8_t* __restrict__ A, const float* __restrict__ sa,
                                                            const int8_t* __restrict__ Wp, const float* __restrict__ sw,
                                                            const bf16_t* __restrict__ bias, bf16_t* __restrict__ out,
                                                            int M, int N, int K, int KT, int Mpad) {
  __shared__ v4i red[NW][MT][64];
  const int nt = blockIdx.x;
  const int m0 = blockIdx.y * (16 * MT);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int arow = lane & 15, akc = 16 * (lane >> 4);

  v4i acc[MT];
  v4f accf[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) { acc[i] = v4i{0, 0, 0, 0}; accf[i] = v4f{0.f, 0.f, 0.f, 0.f}; }

  const v4i* wp = reinterpret_cast<const v4i*>(Wp + ((size_t)nt * KT) * 1024) + lane;
  const int8_t* arows[MT];
  bool aval[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int r = m0 + i * 16 + arow;
    aval[i] = r < M;
    arows[i] = A + (size_t)(aval[i] ? r : 0) * K;
  }
  const bool k16 = (K % 16) == 0;

  for (int kt = wave; kt < KT; kt += NW * UNROLL) {
    v4i b[UNROLL];
    v4i a[UNROLL][MT];
    v4f sg[UNROLL][MT];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int k = kt + u * NW;
      b[u] = (k < KT) ? __builtin_nontemporal_load(wp + (size_t)k * 64) : v4i{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int k = kt + u * NW;
      const int kk = k * 64 + akc;
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        if constexpr (AG) sg[u][i] = group_scales(sa, k, KT, Mpad, m0 + i * 16 + 4 * (lane >> 4));
        if (aval[i] && k < KT && kk + 16 <= K && k16) a[u][i] = *reinterpret_cast<const v4i*>(arows[i] + kk);
        else if (aval[i] && k < KT && kk < K) {
          int8_t t[16];  // ragged K (K % 16 != 0): byte-wise, zero padded
#pragma unroll
          for (int j = 0; j < 16; ++j) t[j] = (kk + j < K) ? arows[i][kk + j] : 0;
          a[u][i] = *reinterpret_cast<v4i*>(t);
        } else a[u][i] = v4i{0, 0, 0, 0};
      }
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        if constexpr (AG) fold(accf[i], mfma_i8(a[u][i], b[u], v4i{0, 0, 0, 0}), sg[u][i]);
        else acc[i] = mfma_i8(a[u][i], b[u], acc[i]);
      }
  }

#pragma unroll
  for (int i = 0; i < MT; ++i) {
    if constexpr (AG) red[wave][i][lane] = __builtin_bit_cast(v4i, accf[i]);
    else red[wave][i][lane] = acc[i];
  }
  __syncthreads();
  for (int i = wave; i < MT; i += NW) {
    const int col = nt * 16 + (lane & 15);
    if constexpr (AG) {
      v4f s = __builtin_bit_cast(v4f, red[0][i][lane]);
#pragma unroll
      for (int w = 1; w < NW; ++w) s += __builtin_bit_cast(v4f, red[w][i][lane]);
#pragma unroll
      for (int j = 0; j < 4; ++j) store_out_f(out, M, N, m0 + i * 16 + 4 * (lane >> 4) + j, col, s[j], sw, bias);
    } else {
      v4i s = red[0][i][lane];
#pragma unroll
      for (int w = 1; w < NW; ++w) s += red[w][i][lane];
#pragma unroll
      for (int j = 0; j < 4; ++j) store_out(out, M, N, m0 + i * 16 + 4 * (lane >> 4) + j, col, s[j], sa, sw, bias);
    }
  }
}

// NTW n-tiles per workgroup: each A fragment (one per k-tile) feeds NTW MFMAs, cutting the
// L2->CU activation traffic NTW-fold (at M = 16 an A fragment is as large as a weight fragment,
// so with NTW = 1 the kernel moves twice the bytes it must).
// For M > 16 every 16-row block is its own workgroup; the block order is XCD-grouped: dispatch
// ids b, b+8, b+16, ... land on one XCD, so the MB row blocks of a weight panel are consecutive
// ids within one XCD (id = xcd + 8 * (ks + S * (mb + MB * panel_group))) and re-read the panel
// from that XCD's L2 instead of HBM (placement is a speed assumption only, never a correctness one).
//
// Split-K (S > 1): a CU streams at most ~22 GB/s, so a grid with fewer workgroups than CUs
// cannot reach HBM speed.  S workgroups share a panel, each reducing K/S k-tiles and storing
// its partial tiles to its own scratch slot; an agent-scope acquire-release counter picks the
// last workgroup of the panel, which sums the S slots in split order (deterministic, also for
// the float AG accumulators), resets the counter for the next launch / graph replay, and runs
// the epilogue.
//
// EPI 1 (fused SwiGLU + quant, decode MLP): the gate_up weight rows are packed 64-blocked
// ([gate f0..f0+63 | up f0..f0+63] per 128 rows), so one 8-tile panel holds both halves of 64
// features.  Waves 0-3 each pair gate tile w with up tile w+4, round both to bf16 (as the
// unfused GEMM output would be), form silu(g)*u, and the panel writes int8 h with one scale per
// (token, 64 features) — exactly the per-group input the down projection's AG mode reads.
typedef uint64_t v2u64 __attribute__((ext_vector_type(2)));

struct SplitK {
  int S;
  v4i* part;     // [panels * MB][S][NTW][64 lanes] partial tiles (int32, AG: float bits)
  int* cnt;      // [panels * MB], zero between launches
};

template <int UNROLL, int NW, int NTW, bool AG, int EPI, bool FAST>
__global__ void __launch_bounds__(NW * 64) w8a8_gemv_ntw_kernel(const int8_t* __restrict__ A, const float* __restrict__ sa,
                                                                const int8_t* __restrict__ Wp, const float* __restrict__ sw,
                                                                const bf16_t* __restrict__ bias, bf16_t* __restrict__ out,
                                                                int M, int N, int K, int KT, int NTt, int Mpad,
                                                                int8_t* __restrict__ hq, float* __restrict__ hs,
                                                                SplitK sk) {
  static_assert(EPI == 0 || (NTW == 8 && NW >= 4 && !AG), "GLU epilogue: 8-tile panels, >= 4 waves");
  // tiles owned by a wave in the epilogue: EPI 0 -> wave, wave + NW, ...; EPI 1 -> wave, wave + 4
  constexpr int OWN = EPI == 1 ? 2 : (NTW + NW - 1) / NW;
  __shared__ v4i red[NW][NTW][64];
  __shared__ float gmax[4][16];
  __shared__ int last_flag;
  const int MB = (M + 15) / 16, S = sk.S;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, r = bid >> 3;
  const int ks = r % S, r2 = r / S;
  const int mb = r2 % MB, panel = xcd + 8 * (r2 / MB);
  const int nt0 = panel * NTW;
  if (nt0 >= NTt) return;                                   // grid padded to a multiple of 8 panels
  const int kt_begin = (int)((int64_t)KT * ks / S), kt_end = (int)((int64_t)KT * (ks + 1) / S);
  const int m0 = mb * 16;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int arow = m0 + (lane & 15), akc = 16 * (lane >> 4);
  v4i acc[NTW];
  v4f accf[NTW];
#pragma unroll
  for (int j = 0; j < NTW; ++j) { acc[j] = v4i{0, 0, 0, 0}; accf[j] = v4f{0.f, 0.f, 0.f, 0.f}; }
  const v4i* wp[NTW];
#pragma unroll
  for (int j = 0; j < NTW; ++j) {
    const int nt = min(nt0 + j, NTt - 1);
    wp[j] = reinterpret_cast<const v4i*>(Wp + ((size_t)nt * KT) * 1024) + lane;
  }
  const bool aval = arow < M;
  const int8_t* arow_p = A + (size_t)(aval ? arow : 0) * K;
  const bool k16 = (K % 16) == 0;

  if constexpr (FAST) {
    // K % 64 == 0: every load is unconditional (k-tile and row indices clamped to valid memory;
    // out-of-range contributions are skipped by wave-uniform guards on the MFMAs) and the next
    // group of UNROLL k-tiles is prefetched into a second register set before the current
    // group's MFMAs, so the compiler waits with a counted vmcnt instead of draining every step.
    const int8_t* ap = A + (size_t)min(arow, M - 1) * K + akc;
    const int nk = kt_end > kt_begin + wave ? (kt_end - kt_begin - wave + NW - 1) / NW : 0;
    const int ng = (nk + UNROLL - 1) / UNROLL;
    const int r0 = m0 + 4 * (lane >> 4);
    v4i b0[UNROLL][NTW], b1[UNROLL][NTW], a0[UNROLL], a1[UNROLL];
    v4f s0[UNROLL], s1[UNROLL];
    auto load = [&](v4i (&b)[UNROLL][NTW], v4i (&a)[UNROLL], v4f (&sg)[UNROLL], int g) {
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        const int k = min(kt_begin + wave + (g * UNROLL + u) * NW, kt_end - 1);
#pragma unroll
        for (int j = 0; j < NTW; ++j) b[u][j] = __builtin_nontemporal_load(wp[j] + (size_t)k * 64);
        a[u] = *reinterpret_cast<const v4i*>(ap + (size_t)k * 64);
        if constexpr (AG) sg[u] = *reinterpret_cast<const v4f*>(sa + (size_t)k * Mpad + r0);
      }
    };
    auto mma = [&](const v4i (&b)[UNROLL][NTW], const v4i (&a)[UNROLL], const v4f (&sg)[UNROLL], int g) {
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        if (g * UNROLL + u >= nk) break;                        // wave-uniform
#pragma unroll
        for (int j = 0; j < NTW; ++j) {
          if constexpr (AG) fold(accf[j], mfma_i8(a[u], b[u][j], v4i{0, 0, 0, 0}), sg[u]);
          else acc[j] = mfma_i8(a[u], b[u][j], acc[j]);
        }
      }
    };
    // ping-pong register sets, no copies: the loads of one set stay in flight while the other's
    // MFMAs run (the final prefetch re-reads the last valid group instead of branching)
    if (ng > 0) load(b0, a0, s0, 0);
    for (int g = 0; g < ng; g += 2) {
      load(b1, a1, s1, min(g + 1, ng - 1));
      mma(b0, a0, s0, g);
      load(b0, a0, s0, min(g + 2, ng - 1));
      mma(b1, a1, s1, g + 1);
    }
  } else {
    for (int kt = kt_begin + wave; kt < kt_end; kt += NW * UNROLL) {
      v4i b[UNROLL][NTW];
      v4i a[UNROLL];
      v4f sg[UNROLL];
  #pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        const int k = kt + u * NW;
  #pragma unroll
        for (int j = 0; j < NTW; ++j)
          b[u][j] = (k < kt_end) ? __builtin_nontemporal_load(wp[j] + (size_t)k * 64) : v4i{0, 0, 0, 0};
      }
  #pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        const int k = kt + u * NW;
        const int kk = k * 64 + akc;
        if constexpr (AG) sg[u] = group_scales(sa, k < kt_end ? k : KT, KT, Mpad, m0 + 4 * (lane >> 4));
        if (aval && k < kt_end && kk + 16 <= K && k16) a[u] = *reinterpret_cast<const v4i*>(arow_p + kk);
        else if (aval && k < kt_end && kk < K) {
          int8_t t[16];
  #pragma unroll
          for (int jj = 0; jj < 16; ++jj) t[jj] = (kk + jj < K) ? arow_p[kk + jj] : 0;
          a[u] = *reinterpret_cast<v4i*>(t);
        } else a[u] = v4i{0, 0, 0, 0};
      }
  #pragma unroll
      for (int u = 0; u < UNROLL; ++u)
  #pragma unroll
        for (int j = 0; j < NTW; ++j) {
          if constexpr (AG) fold(accf[j], mfma_i8(a[u], b[u][j], v4i{0, 0, 0, 0}), sg[u]);
          else acc[j] = mfma_i8(a[u], b[u][j], acc[j]);
        }
    }
  }
#pragma unroll
  for (int j = 0; j < NTW; ++j) {
    if constexpr (AG) red[wave][j][lane] = __builtin_bit_cast(v4i, accf[j]);
    else red[wave][j][lane] = acc[j];
  }
  __syncthreads();

  // ---- per-tile totals of this workgroup for the tiles this wave owns
  v4i tot[OWN];
  int tile[OWN];
#pragma unroll
  for (int o = 0; o < OWN; ++o) {
    tile[o] = EPI == 1 ? (wave < 4 ? wave + 4 * o : NTW) : wave + NW * o;
    tot[o] = v4i{0, 0, 0, 0};
    if (tile[o] < NTW) {
      if constexpr (AG) {
        v4f f = __builtin_bit_cast(v4f, red[0][tile[o]][lane]);
#pragma unroll
        for (int w = 1; w < NW; ++w) f += __builtin_bit_cast(v4f, red[w][tile[o]][lane]);
        tot[o] = __builtin_bit_cast(v4i, f);
      } else {
        v4i t = red[0][tile[o]][lane];
#pragma unroll
        for (int w = 1; w < NW; ++w) t += red[w][tile[o]][lane];
        tot[o] = t;
      }
    }
  }
  // ---- split-K: publish this split's partials; the last workgroup of the panel continues.
  // Partials go out as device-scope atomic stores (coherent across XCDs without an L2
  // writeback); each wave waits for its stores to complete before the barrier, then one relaxed
  // device-scope counter increment elects the last workgroup, which reads the partials back with
  // device-scope atomic loads.  (An agent-scope release/acquire fence here writes back the whole
  // L2 per workgroup and costs 5-6x the GEMV itself.)
  if (S > 1) {
    const size_t pbase = (size_t)(panel * MB + mb) * S;
#pragma unroll
    for (int o = 0; o < OWN; ++o) {
      if (tile[o] >= NTW) continue;
      uint64_t* p = reinterpret_cast<uint64_t*>(sk.part + ((pbase + ks) * NTW + tile[o]) * 64 + lane);
      const uint64_t* v = reinterpret_cast<const uint64_t*>(&tot[o]);
      __hip_atomic_store(p, v[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(p + 1, v[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      int* c = sk.cnt + panel * MB + mb;
      const int prev = __hip_atomic_fetch_add(c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last_flag = prev == S - 1;
      if (prev == S - 1) __hip_atomic_store(c, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!last_flag) return;
#pragma unroll
    for (int o = 0; o < OWN; ++o) {
      if (tile[o] >= NTW) continue;
      v4i parts[8];
      for (int k2 = 0; k2 < S; k2 += 8) {
        const int nk = min(8, S - k2);
        for (int i = 0; i < nk; ++i) {      // issue up to 8 slot loads before summing
          const uint64_t* p = reinterpret_cast<const uint64_t*>(sk.part + ((pbase + k2 + i) * NTW + tile[o]) * 64 + lane);
          uint64_t lo = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          uint64_t hi = __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          parts[i] = __builtin_bit_cast(v4i, (v2u64){lo, hi});
        }
        for (int i = 0; i < nk; ++i) {
          if constexpr (AG) {
            v4f f = k2 + i == 0 ? v4f{0.f, 0.f, 0.f, 0.f} : __builtin_bit_cast(v4f, tot[o]);
            tot[o] = __builtin_bit_cast(v4i, f + __builtin_bit_cast(v4f, parts[i]));
          } else {
            tot[o] = (k2 + i == 0 ? v4i{0, 0, 0, 0} : tot[o]) + parts[i];
          }
        }
      }
    }
  }

  if constexpr (EPI == 0) {
#pragma unroll
    for (int o = 0; o < OWN; ++o) {
      if (tile[o] >= NTW || nt0 + tile[o] >= NTt) continue;
      const int col = (nt0 + tile[o]) * 16 + (lane & 15);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = m0 + 4 * (lane >> 4) + q;
        if constexpr (AG) store_out_f(out, M, N, row, col, __builtin_bit_cast(v4f, tot[o])[q], sw, bias);
        else store_out(out, M, N, row, col, tot[o][q], sa, sw, bias);
      }
    }
  } else {
    const int F = N / 2;
    float h[4];
    if (wave < 4) {
      const int gcol = (nt0 + wave) * 16 + (lane & 15), ucol = (nt0 + 4 + wave) * 16 + (lane & 15);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = m0 + 4 * (lane >> 4) + q;
        const float s_a = row < M ? sa[row] : 0.f;
        float g = (float)tot[0][q] * s_a * sw[gcol], u = (float)tot[1][q] * s_a * sw[ucol];
        if (bias) { g += bf2f(bias[gcol]); u += bf2f(bias[ucol]); }
        g = bf2f(f2bf(g));
        u = bf2f(f2bf(u));
        h[q] = g / (1.f + __expf(-g)) * u;
        float m = fabsf(h[q]);
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
        if ((lane & 15) == 0) gmax[wave][4 * (lane >> 4) + q] = m;
      }
    }
    __syncthreads();
    if (wave < 4) {
      const int grp = nt0 / 8;
      const int f = grp * 64 + wave * 16 + (lane & 15);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int rr = 4 * (lane >> 4) + q, row = m0 + rr;
        const float amax = fmaxf(fmaxf(fmaxf(gmax[0][rr], gmax[1][rr]), fmaxf(gmax[2][rr], gmax[3][rr])), 1e-8f);
        if (row < M) hq[(size_t)row * F + f] = quant_i8(h[q], 127.f / amax);
        if (wave == 0 && (lane & 15) == 0) hs[(size_t)grp * Mpad + row] = amax / 127.f;
      }
    }
  }
}

// ------------------------------------------------------------------------------------ tiled
// Block tile 128 x 128, BK = 64. LDS image per buffer: A 8 x 1 KiB fragments, B 8 x 1 KiB.
constexpr int BM = 128, BN = 128;

__device__ __forceinline__ void glds16(const void* g, void* lds_base) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

__global__ void __launch_bounds__(NT) w8a8_gemm_tiled_kernel(const int8_t* __restrict__ A, const float* __restrict__ sa,
                                                             const int8_t* __restrict__ Wp, const float* __restrict__ sw,
                                                             const bf16_t* __restrict__ bias, bf16_t* __restrict__ out,
                                                             int M, int N, int K, int KT, int NTt, int grid_n) {
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];  // 2 x (8 KiB A + 8 KiB B)
  // XCD-aware remap: consecutive dispatch ids round-robin over 8 XCDs; give each XCD a
  // contiguous run of tiles along N so blocks sharing an A panel share an L2.
  const int nwg = gridDim.x;
  const int orig = blockIdx.x;
  int wgid = orig;
  if (nwg % 8 == 0) wgid = (orig % 8) * (nwg / 8) + orig / 8;
  const int bn = wgid % grid_n, bm = wgid / grid_n;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;   // 2 x 2 waves, 64 x 64 each

  // per-lane global sources for this wave's 2 A fragments and 2 B fragments
  const int8_t* asrc[2];
  const int8_t* bsrc[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int msub = wave * 2 + j;                       // 0..7
    int r = bm * BM + msub * 16 + (lane & 15);
    r = r < M ? r : M - 1;
    asrc[j] = A + (size_t)r * K + 16 * (lane >> 4);
    int ntile = bn * (BN / 16) + wave * 2 + j;            // 0..NTt-1
    ntile = ntile < NTt ? ntile : NTt - 1;
    bsrc[j] = Wp + ((size_t)ntile * KT) * 1024 + lane * 16;
  }

  auto stage = [&](int buf, int kt) {
    int8_t* base = smem + buf * 16384;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      glds16(asrc[j] + (size_t)kt * 64, base + (wave * 2 + j) * 1024);
      glds16(bsrc[j] + (size_t)kt * 1024, base + 8192 + (wave * 2 + j) * 1024);
    }
  };

  v4i acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v4i{0, 0, 0, 0};

  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int cur = 0;
  for (int kt = 0; kt < KT; ++kt) {
    if (kt + 1 < KT) stage(cur ^ 1, kt + 1);
    const int8_t* base = smem + cur * 16384;
    v4i a[4], b[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = *reinterpret_cast<const v4i*>(base + (wm * 4 + i) * 1024 + lane * 16);
#pragma unroll
    for (int j = 0; j < 4; ++j) b[j] = *reinterpret_cast<const v4i*>(base + 8192 + (wn * 4 + j) * 1024 + lane * 16);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma_i8(a[i], b[j], acc[i][j]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    cur ^= 1;
  }

#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = bn * BN + (wn * 4 + j) * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = bm * BM + (wm * 4 + i) * 16 + 4 * (lane >> 4) + r;
        store_out(out, M, N, row, col, acc[i][j][r], sa, sw, bias);
      }
    }
}
}  // namespace

static int g_gemv_nw = 0, g_gemv_unroll = 0, g_gemv_ntw = 0, g_glu_unroll = 0, g_splitk = 0, g_gemv_fast = 1;
// tuning hook (microbenchmarks): 0 = automatic choice
extern "C" void edge_w8a8_gemv_config(int nw, int unroll) { g_gemv_nw = nw; g_gemv_unroll = unroll; }
extern "C" void edge_w8a8_gemv_ntw(int ntw) { g_gemv_ntw = ntw; }
extern "C" void edge_w8a8_glu_unroll(int u) { g_glu_unroll = u; }
extern "C" void edge_w8a8_splitk(int s) { g_splitk = s; }
extern "C" void edge_w8a8_gemv_fast(int on) { g_gemv_fast = on; }

// Split-K scratch: one per device, allocated (and its counters zeroed) on first use outside a
// graph capture; every launch leaves the counters at zero again.
namespace {
constexpr size_t kPartBytes = 16u << 20;
constexpr int kCounters = 1 << 16;
struct Scratch { v4i* part = nullptr; int* cnt = nullptr; };
Scratch g_scratch[64];

Scratch* scratch(hipStream_t st) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  Scratch& s = g_scratch[dev];
  if (s.part != nullptr) return &s;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
  void *p = nullptr, *c = nullptr;
  if (hipMalloc(&p, kPartBytes) != hipSuccess) return nullptr;
  if (hipMalloc(&c, kCounters * sizeof(int)) != hipSuccess || hipMemset(c, 0, kCounters * sizeof(int)) != hipSuccess) {
    (void)hipFree(p);
    return nullptr;
  }
  s.part = (v4i*)p;
  s.cnt = (int*)c;
  return &s;
}

// Split count: opt-in (tune "splitk").  Measured on MI355X (Llama-2-7B decode shapes, M = 16)
// the partial-tile handoff on the last workgroup's critical path costs more than the extra CUs
// return (GLU 23.6 -> 29.2 us at S = 2, down 13.1 -> 16.3 us at S = 8), so the default is S = 1.
SplitK choose_split(int groups, int KT, int nw, int ntw, hipStream_t st) {
  (void)KT; (void)nw;
  const int S = g_splitk > 0 ? g_splitk : 1;
  if (S > 1) {
    Scratch* sc = scratch(st);
    if (sc != nullptr && (size_t)groups * S * ntw * 1024 <= kPartBytes && groups <= kCounters)
      return SplitK{S, sc->part, sc->cnt};
  }
  return SplitK{1, nullptr, nullptr};
}
}  // namespace

// sa: per-token [M] (a_mpad == 0) or per-group [KT][a_mpad] (a_mpad > 0, GEMV shapes only).
// glu_q/glu_s != null: fused SwiGLU + per-group quant epilogue (64-blocked gate_up weights,
// M <= 64, per-token sa): writes int8 [M, N/2] and scales [N/128][a_mpad_out] instead of `out`.
extern "C" int edge_w8a8_gemm(const void* A, const float* sa, const void* Wp, const float* sw, const void* bias,
                              void* out, int M, int N, int K, int KT, int a_mpad, void* glu_q, float* glu_s,
                              int glu_mpad, hipStream_t st) {
  if (M == 0 || N == 0) return 0;
  const int NTt = (N + 15) / 16;
  const bool ag = a_mpad > 0;
  const int mblocks16 = (M + 15) / 16;
  if (glu_q != nullptr) {
    if (ag || M > 64 || N % 128 != 0 || glu_mpad < mblocks16 * 16) return -2;
    const int groups = ((NTt / 8 + 7) / 8) * 8 * mblocks16;
    const SplitK sk = choose_split(groups, KT, 4, 8, st);
    const dim3 grid(groups * sk.S);
#define GLU(U, FA) hipLaunchKernelGGL((w8a8_gemv_ntw_kernel<U, 4, 8, false, 1, FA>), grid, dim3(256), 0, st,         \
                                      (const int8_t*)A, sa, (const int8_t*)Wp, sw, (const bf16_t*)bias, (bf16_t*)out, M, \
                                      N, K, KT, NTt, glu_mpad, (int8_t*)glu_q, glu_s, sk)
    const bool fast = (K % 64 == 0) && g_gemv_fast;
    if (g_glu_unroll >= 4) { if (fast) GLU(4, true); else GLU(4, false); }
    else { if (fast) GLU(2, true); else GLU(2, false); }
#undef GLU
    return (int)hipGetLastError();
  }
  if (ag && (M > 64 || a_mpad < mblocks16 * 16)) return -2;
  if (M > 64 && K % 64 == 0 && K / 64 == KT) {
    const int grid_n = (NTt * 16 + BN - 1) / BN;
    const int grid_m = (M + BM - 1) / BM;
    hipLaunchKernelGGL(w8a8_gemm_tiled_kernel, dim3(grid_n * grid_m), dim3(NT), 2 * 16384, st, (const int8_t*)A, sa,
                       (const int8_t*)Wp, sw, (const bf16_t*)bias, (bf16_t*)out, M, N, K, KT, NTt, grid_n);
    return (int)hipGetLastError();
  }
  // Defaults from the graph-timed cache-cold sweeps on MI355X (profiles/bench_ops_*.json):
  //   M <= 2 : one n-tile per workgroup, unroll 4 (2 with grouped scales), waves by K
  //   M <= 16: unroll 2; N >= 16K columns: 2 n-tiles x 4 waves; 8K..16K: 4 n-tiles x 8 waves;
  //            smaller N: 1 n-tile, 16 waves (K <= 8K) or 8 waves (larger K)
  //   M in (16, 64]: 4 n-tiles per workgroup (activation fragments amortised)
  int un = g_gemv_unroll > 0 ? g_gemv_unroll : (M <= 2 && !ag ? 4 : 2);
  int ntw = 1;
  if (g_gemv_ntw > 0) ntw = g_gemv_ntw;
  else if (mblocks16 > 1) ntw = 4;
  else if (M > 2 && NTt >= 1024) ntw = 2;
  else if (M > 2 && NTt >= 512) ntw = 4;
  int nw = g_gemv_nw > 0 ? g_gemv_nw : (KT >= 128 ? 16 : (KT >= 32 ? 8 : 4));
  if (g_gemv_nw <= 0 && M > 2) nw = (NTt >= 1024) ? 4 : (NTt >= 512 ? 8 : (KT >= 128 ? 8 : 16));
#define GEMV_NW(MT, U, NWV)                                                                                       \
  do {                                                                                                            \
    const dim3 g(NTt, (M + 16 * MT - 1) / (16 * MT));                                                            \
    if (ag) hipLaunchKernelGGL((w8a8_gemv_kernel<MT, U, NWV, true>), g, dim3(NWV * 64), 0, st, (const int8_t*)A,  \
                               sa, (const int8_t*)Wp, sw, (const bf16_t*)bias, (bf16_t*)out, M, N, K, KT, a_mpad); \
    else hipLaunchKernelGGL((w8a8_gemv_kernel<MT, U, NWV, false>), g, dim3(NWV * 64), 0, st, (const int8_t*)A,    \
                            sa, (const int8_t*)Wp, sw, (const bf16_t*)bias, (bf16_t*)out, M, N, K, KT, a_mpad); \
  } while (0)
#define GEMV(MT, U)                                   \
  do {                                                \
    if (nw >= 16) GEMV_NW(MT, U, 16);                 \
    else if (nw >= 8) GEMV_NW(MT, U, 8);              \
    else GEMV_NW(MT, U, 4);                           \
  } while (0)
  const bool fast = (K % 64 == 0) && g_gemv_fast;
  if (fast && nw >= 16 && (ntw >= 2 || un >= 4 && ag)) nw = 8;   // 16 waves x multi-tile spills (128-VGPR cap)
  if (ntw > 1 || fast) {
    // XCD-grouped 1-D grid: panels padded to a multiple of 8, S workgroups per (panel, 16-row block)
    const int groups = ((NTt + ntw - 1) / ntw + 7) / 8 * 8 * mblocks16;
    const SplitK sk = choose_split(groups, KT, nw, ntw, st);
#define NTWL(U, NWV, NTWV)                                                                                           \
  do {                                                                                                               \
    const dim3 g(groups * sk.S);                                                                                     \
    if (fast) {                                                                                                      \
      if (ag) hipLaunchKernelGGL((w8a8_gemv_ntw_kernel<U, NWV, NTWV, true, 0, true>), g, dim3(NWV * 64), 0, st,      \
                                 (const int8_t*)A, sa, (const int8_t*)Wp, sw, (const bf16_t*)bias, (bf16_t*)out, M, N,\
                                 K, KT, NTt, a_mpad, nullptr, nullptr, sk);                                          \
      else hipLaunchKernelGGL((w8a8_gemv_ntw_kernel<U, NWV, NTWV, false, 0, true>), g, dim3(NWV * 64), 0, st,        \
                              (const int8_t*)A, sa, (const int8_t*)Wp, sw, (const bf16_t*)bias, (bf16_t*)out, M, N, K,\
                              KT, NTt, a_mpad, nullptr, nullptr, sk);                                                \
    } else {                                                                                                         \
      if (ag) hipLaunchKernelGGL((w8a8_gemv_ntw_kernel<U, NWV, NTWV, true, 0, false>), g, dim3(NWV * 64), 0, st,     \
                                 (const int8_t*)A, sa, (const int8_t*)Wp, sw, (const bf16_t*)bias, (bf16_t*)out, M, N,\
                                 K, KT, NTt, a_mpad, nullptr, nullptr, sk);                                          \
      else hipLaunchKernelGGL((w8a8_gemv_ntw_kernel<U, NWV, NTWV, false, 0, false>), g, dim3(NWV * 64), 0, st,       \
                              (const int8_t*)A, sa, (const int8_t*)Wp, sw, (const bf16_t*)bias, (bf16_t*)out, M, N, K,\
                              KT, NTt, a_mpad, nullptr, nullptr, sk);                                                \
    }                                                                                                                \
  } while (0)
#define NTWN(NWV)                                                   \
  do {                                                              \
    if (ntw >= 4) { if (un >= 4) NTWL(4, NWV, 4); else NTWL(2, NWV, 4); } \
    else if (ntw >= 2) { if (un >= 4) NTWL(4, NWV, 2); else NTWL(2, NWV, 2); } \
    else { if (un >= 4) NTWL(4, NWV, 1); else NTWL(2, NWV, 1); }   \
  } while (0)
    if (nw >= 16) NTWN(16);
    else if (nw >= 8) NTWN(8);
    else NTWN(4);
#undef NTWN
#undef NTWL
    return (int)hipGetLastError();
  }
  const int mblocks = mblocks16;
  if (mblocks <= 1) { if (un >= 8) GEMV(1, 8); else if (un >= 4) GEMV(1, 4); else GEMV(1, 2); }
  else if (mblocks <= 2) { if (un >= 4) GEMV(2, 4); else GEMV(2, 2); }
  else GEMV(4, 2);
#undef GEMV
#undef GEMV_NW
  return (int)hipGetLastError();
}

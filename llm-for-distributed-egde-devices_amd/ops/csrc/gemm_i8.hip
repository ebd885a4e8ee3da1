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
// Kernels:
//   gemv:  M <= 64 (decode).  HBM-bound on W: a workgroup owns NTW 16-column tiles of one
//          16-row block, its NW waves split K (k-tile kt -> wave kt % NW) and keep UNROLL
//          fragments per tile in flight (no LDS staging: the weights are read exactly once,
//          nontemporal), partial sums reduced through LDS.  Activation modes:
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
//   tiled: M > 64 (prefill). 128x128 block tile, BK=64, 4 waves in 2x2, A and B staged with
//          global_load_lds (16 B/lane, lane-linear fragment-ordered LDS images -> conflict-free
//          ds_read_b128), LDS double buffer.
#include "common.h"

namespace {
constexpr int NT = 256;
constexpr int A_TOKEN = 0, A_GROUP = 1;
constexpr int EPI_OUT = 0, EPI_GLU = 1, EPI_GLUQ = 2;

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

__device__ __forceinline__ void store_out_f(bf16_t* __restrict__ out, int M, int N, int row, int col, float v,
                                            const float* __restrict__ sw, const bf16_t* __restrict__ bias) {
  if (row < M && col < N) {
    v *= sw[col];
    if (bias) v += bf2f(bias[col]);
    out[(size_t)row * N + col] = f2bf(v);
  }
}

__device__ __forceinline__ void fold(v4f& accf, const v4i& t, const v4f& s) {
#pragma unroll
  for (int q = 0; q < 4; ++q) accf[q] += (float)t[q] * s[q];
}

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
// Split-K (S > 1, opt-in): S workgroups share a tile group, each reducing K/S k-tiles; every
// wave publishes its partial tiles with device-scope (sc1, write-through) 8-byte stores, waits
// for them (vmcnt 0), and after a barrier one relaxed device-scope counter increment elects
// the last workgroup, which reads the partials back with sc1 loads, sums them in split order
// (deterministic, also for float accumulators), resets the counter and runs the epilogue.
// Measured on MI355X at Llama-2-7B decode shapes the handoff costs more than the extra CUs
// return, so the launcher uses S = 1 unless tuned ("splitk").
typedef uint64_t v2u64 __attribute__((ext_vector_type(2)));

struct SplitK {
  int S;
  v4i* part;     // [groups][S][NTW][64 lanes] partial tiles (int32, float bits for scaled modes)
  int* cnt;      // [groups], zero between launches
};

// Grid: XCD-grouped 1-D: dispatch ids b, b+8, b+16, ... land on one XCD, so the MB row blocks
// (and the S splits) of a tile group are consecutive ids within one XCD and re-read the panel
// from that XCD's L2 instead of HBM (a speed assumption only, never a correctness one).
template <int UNROLL, int NW, int NTW, int AMODE, int EPI>
__global__ void __launch_bounds__(NW * 64) w8a8_gemv_kernel(const void* __restrict__ Av, const float* __restrict__ sa,
                                                            const int8_t* __restrict__ Wp, const float* __restrict__ sw,
                                                            const bf16_t* __restrict__ bias, bf16_t* __restrict__ out,
                                                            float* __restrict__ os, int M, int N, int K, int KT,
                                                            int NTt, int Mpad, SplitK sk) {
  static_assert(EPI == EPI_OUT || (AMODE == A_TOKEN && NTW % 2 == 0 && NW >= NTW / 2),
                "GLU epilogues: gate/up tile pairs, one pair per wave, per-token A");
  static_assert(EPI != EPI_GLUQ || NTW == 8, "quantising GLU epilogue: 64 features per workgroup");
  constexpr bool SCALED = AMODE != A_TOKEN;        // float accumulation with per-k-tile scales
  constexpr bool GLU = EPI != EPI_OUT;
  constexpr int OWN = GLU ? 2 : (NTW + NW - 1) / NW;   // GLU: wave w owns tiles 2w (gate), 2w+1 (up)
  __shared__ v4i red[NW][NTW][64];
  __shared__ float gmax[4][16];
  __shared__ int last_flag;
  const int MB = (M + 15) / 16, S = sk.S;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, r = bid >> 3;
  const int ks = r % S, r2 = r / S;
  const int mb = r2 % MB, grp = xcd + 8 * (r2 / MB);
  const int nt0 = grp * NTW;
  if (nt0 >= NTt) return;                                   // grid padded to a multiple of 8 groups
  const int kt_begin = (int)((int64_t)KT * ks / S), kt_end = (int)((int64_t)KT * (ks + 1) / S);
  const int m0 = mb * 16;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int arow = m0 + (lane & 15), akc = 16 * (lane >> 4);
  const bool aval = arow < M;
  const int8_t* arow_i8 = reinterpret_cast<const int8_t*>(Av) + (size_t)(aval ? arow : 0) * K;
  const bool k16 = (K % 16) == 0;
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
      if constexpr (AMODE == A_GROUP)
        sg[u] = k < kt_end ? *reinterpret_cast<const v4f*>(sa + (size_t)k * Mpad + m0 + 4 * (lane >> 4))
                           : v4f{0.f, 0.f, 0.f, 0.f};
      a[u] = load_a_i8(arow_i8, aval, k, kt_end, akc, K, k16);
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
#pragma unroll
      for (int j = 0; j < NTW; ++j) {
        if constexpr (SCALED) fold(accf[j], mfma_i8(a[u], b[u][j], v4i{0, 0, 0, 0}), sg[u]);
        else acc[j] = mfma_i8(a[u], b[u][j], acc[j]);
      }
  }
#pragma unroll
  for (int j = 0; j < NTW; ++j) red[wave][j][lane] = SCALED ? __builtin_bit_cast(v4i, accf[j]) : acc[j];
  __syncthreads();

  // ---- per-tile totals for the tiles this wave owns (EPI_GLU: wave 0 owns the gate/up pair)
  v4i tot[OWN];
  int tile[OWN];
#pragma unroll
  for (int o = 0; o < OWN; ++o) {
    tile[o] = GLU ? (wave < NTW / 2 ? 2 * wave + o : NTW) : wave + NW * o;
    tot[o] = v4i{0, 0, 0, 0};
    if (tile[o] < NTW) {
      if constexpr (SCALED) {
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
  // ---- split-K hand-off (see SplitK)
  if (S > 1) {
    const size_t pbase = (size_t)(grp * MB + mb) * S;
#pragma unroll
    for (int o = 0; o < OWN; ++o) {
      if (tile[o] >= NTW) continue;
      uint64_t* p = reinterpret_cast<uint64_t*>(sk.part + ((pbase + ks) * NTW + tile[o]) * 64 + lane);
      const v2u64 v = __builtin_bit_cast(v2u64, tot[o]);
      __hip_atomic_store(p, v[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(p + 1, v[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      int* c = sk.cnt + grp * MB + mb;
      const int prev = __hip_atomic_fetch_add(c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last_flag = prev == S - 1;
      if (prev == S - 1) __hip_atomic_store(c, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!last_flag) return;
#pragma unroll
    for (int o = 0; o < OWN; ++o) {
      if (tile[o] >= NTW) continue;
      v4i t = v4i{0, 0, 0, 0};
      v4f f = v4f{0.f, 0.f, 0.f, 0.f};
      for (int k2 = 0; k2 < S; ++k2) {
        const uint64_t* p = reinterpret_cast<const uint64_t*>(sk.part + ((pbase + k2) * NTW + tile[o]) * 64 + lane);
        const v2u64 v = v2u64{__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                              __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)};
        if constexpr (SCALED) f += __builtin_bit_cast(v4f, v);
        else t += __builtin_bit_cast(v4i, v);
      }
      tot[o] = SCALED ? __builtin_bit_cast(v4i, f) : t;
    }
  }

  if constexpr (EPI == EPI_OUT) {
#pragma unroll
    for (int o = 0; o < OWN; ++o) {
      if (tile[o] >= NTW || nt0 + tile[o] >= NTt) continue;
      const int col = (nt0 + tile[o]) * 16 + (lane & 15);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = m0 + 4 * (lane >> 4) + q;
        if constexpr (SCALED) store_out_f(out, M, N, row, col, __builtin_bit_cast(v4f, tot[o])[q], sw, bias);
        else store_out(out, M, N, row, col, tot[o][q], sa, sw, bias);
      }
    }
  } else {
    // pair (gate tile nt0 + 2w, up tile nt0 + 2w + 1) -> feature f = (nt0/2 + w) * 16 + lane & 15
    const int F = N / 2;
    const bool owner = wave < NTW / 2 && nt0 + 2 * wave + 1 < NTt;
    const int gcol = (nt0 + 2 * wave) * 16 + (lane & 15), ucol = gcol + 16;
    const int f = (nt0 / 2 + wave) * 16 + (lane & 15);
    float h[4] = {0.f, 0.f, 0.f, 0.f};
    if (owner) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = m0 + 4 * (lane >> 4) + q;
        const float s_a = row < M ? sa[row] : 0.f;
        float g = (float)tot[0][q] * s_a * sw[gcol], u = (float)tot[1][q] * s_a * sw[ucol];
        if (bias) { g += bf2f(bias[gcol]); u += bf2f(bias[ucol]); }
        g = bf2f(f2bf(g));                // the unfused GEMM output is bf16
        u = bf2f(f2bf(u));
        h[q] = g / (1.f + __expf(-g)) * u;
        if constexpr (EPI == EPI_GLU)
          if (row < M) out[(size_t)row * F + f] = f2bf(h[q]);
      }
    }
    if constexpr (EPI == EPI_GLUQ) {
      int8_t* hq = reinterpret_cast<int8_t*>(out);
      if (owner) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float m = fabsf(h[q]);
#pragma unroll
          for (int o = 1; o < 16; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
          if ((lane & 15) == 0) gmax[wave][4 * (lane >> 4) + q] = m;
        }
      }
      __syncthreads();
      if (owner) {
        const int grp = nt0 / 8;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int rr = 4 * (lane >> 4) + q, row = m0 + rr;
          const float amax = fmaxf(fmaxf(fmaxf(gmax[0][rr], gmax[1][rr]), fmaxf(gmax[2][rr], gmax[3][rr])), 1e-8f);
          if (row < M) hq[(size_t)row * F + f] = quant_i8(h[q], 127.f / amax);
          if (wave == 0 && (lane & 15) == 0) os[(size_t)grp * Mpad + row] = row < M ? amax / 127.f : 0.f;
        }
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

static int g_gemv_nw = 0, g_gemv_unroll = 0, g_gemv_ntw = 0, g_splitk = 0;
// tuning hooks (microbenchmarks): 0 = automatic choice
extern "C" void edge_w8a8_gemv_config(int nw, int unroll) { g_gemv_nw = nw; g_gemv_unroll = unroll; }
extern "C" void edge_w8a8_gemv_ntw(int ntw) { g_gemv_ntw = ntw; }
extern "C" void edge_w8a8_splitk(int s) { g_splitk = s; }

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

SplitK choose_split(int groups, int ntw, hipStream_t st) {
  const int S = g_splitk > 0 ? g_splitk : 1;
  if (S > 1) {
    Scratch* sc = scratch(st);
    if (sc != nullptr && (size_t)groups * S * ntw * 1024 <= kPartBytes && groups <= kCounters)
      return SplitK{S, sc->part, sc->cnt};
  }
  return SplitK{1, nullptr, nullptr};
}

template <int AM, int EP>
int launch_gemv(int un, int nw, int ntw, const void* A, const float* sa, const void* Wp, const float* sw,
                const void* bias, void* out, float* os, int M, int N, int K, int KT, int Mpad, hipStream_t st) {
  const int NTt = (N + 15) / 16, mblocks = (M + 15) / 16;
  const int groups = ((NTt + ntw - 1) / ntw + 7) / 8 * 8 * mblocks;
  const SplitK sk = choose_split(groups, ntw, st);
  const dim3 g(groups * sk.S);
#define L(U, NWV, NTWV) hipLaunchKernelGGL((w8a8_gemv_kernel<U, NWV, NTWV, AM, EP>), g, dim3(NWV * 64), 0, st, A, sa, \
                                           (const int8_t*)Wp, sw, (const bf16_t*)bias, (bf16_t*)out, os, M, N, K, \
                                           KT, NTt, Mpad, sk)
#define BY_NTW(U, NWV)                                                   \
  do {                                                                   \
    if constexpr (EP == EPI_GLUQ) L(U, NWV, 8);                          \
    else if (ntw >= 4) L(U, NWV, 4);                                     \
    else if (ntw >= 2 || EP == EPI_GLU) L(U, NWV, 2);                    \
    else if constexpr (EP == EPI_OUT) L(U, NWV, 1);                      \
  } while (0)
#define BY_NW(U)                                                         \
  do {                                                                   \
    if (nw >= 16 && EP == EPI_OUT) BY_NTW(U, 16);                        \
    else if (nw >= 8) BY_NTW(U, 8);                                      \
    else BY_NTW(U, 4);                                                   \
  } while (0)
  if (un >= 4) BY_NW(4); else BY_NW(2);
#undef BY_NW
#undef BY_NTW
#undef L
  return (int)hipGetLastError();
}
}  // namespace

// sa: per-token [M] (a_mode 0) or per-group [KT][Mpad] (a_mode 1, M <= 64).
// epi 1: fused SwiGLU on 16-blocked gate/up rows, `out` is bf16 [M, N/2] (a_mode 0, M <= 64).
// epi 2: as epi 1, then per-(token, 64 features) int8 quantisation: `out` int8 [M, N/2],
//        `os` scales [N/128][Mpad] (N % 128 == 0).
extern "C" int edge_w8a8_gemm(const void* A, const float* sa, const void* Wp, const float* sw, const void* bias,
                              void* out, float* os, int M, int N, int K, int KT, int a_mode, int Mpad, int epi,
                              hipStream_t st) {
  if (M == 0 || N == 0) return 0;
  const int NTt = (N + 15) / 16;
  const int mblocks = (M + 15) / 16;
  if (a_mode != A_TOKEN && (M > 64 || (a_mode == A_GROUP && Mpad < mblocks * 16))) return -2;
  if (epi == EPI_GLU || epi == EPI_GLUQ) {
    if (a_mode != A_TOKEN || M > 64 || N % (epi == EPI_GLUQ ? 128 : 32) != 0) return -2;
    if (epi == EPI_GLUQ && (os == nullptr || Mpad < mblocks * 16)) return -2;
    const int un = g_gemv_unroll > 0 ? g_gemv_unroll : 2;
    // one gate/up pair per wave: 2 tiles (M <= 16) or 4 (activation fragments amortised over more
    // weight tiles when several row blocks re-read the panel); the quantising form needs 8
    int ntw = epi == EPI_GLUQ ? 8 : (g_gemv_ntw > 0 ? g_gemv_ntw : (mblocks > 1 ? 4 : 2));
    int nw = g_gemv_nw > 0 ? g_gemv_nw : 4;
    if (nw < ntw / 2) nw = ntw / 2;
    if (epi == EPI_GLUQ) return launch_gemv<A_TOKEN, EPI_GLUQ>(un, nw, 8, A, sa, Wp, sw, bias, out, os, M, N, K, KT, Mpad, st);
    return launch_gemv<A_TOKEN, EPI_GLU>(un, nw, ntw, A, sa, Wp, sw, bias, out, nullptr, M, N, K, KT, Mpad, st);
  }
  if (M > 64 && K % 64 == 0 && K / 64 == KT) {
    const int grid_n = (NTt * 16 + BN - 1) / BN;
    const int grid_m = (M + BM - 1) / BM;
    hipLaunchKernelGGL(w8a8_gemm_tiled_kernel, dim3(grid_n * grid_m), dim3(NT), 2 * 16384, st, (const int8_t*)A, sa,
                       (const int8_t*)Wp, sw, (const bf16_t*)bias, (bf16_t*)out, M, N, K, KT, NTt, grid_n);
    return (int)hipGetLastError();
  }
  // Defaults from the graph-timed cache-cold sweeps on MI355X (profiles/bench_ops_*.json):
  //   M <= 2 : one n-tile per workgroup, unroll 4 (2 with scaled A), waves by K
  //   M <= 16: unroll 2; N >= 16K columns: 2 n-tiles x 4 waves; 8K..16K: 4 n-tiles x 8 waves;
  //            smaller N: 1 n-tile, 16 waves (K <= 8K) or 8 waves (larger K)
  //   M in (16, 64]: 4 n-tiles per workgroup (activation fragments amortised)
  const int un = g_gemv_unroll > 0 ? g_gemv_unroll : (M <= 2 && a_mode == A_TOKEN ? 4 : 2);
  int ntw = 1;
  if (g_gemv_ntw > 0) ntw = g_gemv_ntw;
  else if (mblocks > 1) ntw = 4;
  else if (M > 2 && NTt >= 1024) ntw = 2;
  else if (M > 2 && NTt >= 512) ntw = 4;
  int nw = g_gemv_nw > 0 ? g_gemv_nw : (KT >= 128 ? 16 : (KT >= 32 ? 8 : 4));
  if (g_gemv_nw <= 0 && M > 2) nw = (NTt >= 1024) ? 4 : (NTt >= 512 ? 8 : (KT >= 128 ? 8 : 16));
  if (nw >= 16 && (ntw >= 2 || un >= 4) && a_mode != A_TOKEN) nw = 8;     // 128-VGPR cap at 16 waves
  if (a_mode == A_GROUP)
    return launch_gemv<A_GROUP, EPI_OUT>(un, nw, ntw, A, sa, Wp, sw, bias, out, nullptr, M, N, K, KT, Mpad, st);
  return launch_gemv<A_TOKEN, EPI_OUT>(un, nw, ntw, A, sa, Wp, sw, bias, out, nullptr, M, N, K, KT, Mpad, st);
}

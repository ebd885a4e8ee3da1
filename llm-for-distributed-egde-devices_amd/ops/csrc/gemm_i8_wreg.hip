// W8A8 decode GEMM for 129-256 rows with the WEIGHTS streamed global -> VGPR.
//
// Why: in ring2 / r256 (gemm_i8.hip) the weight panel of a workgroup goes through an LDS-DMA ring
// that every compute wave reads.  LDS (160 KiB per CU) then bounds the weight bytes in flight: the
// quantising gate_up (ring2<16, 2, 3, ...>) keeps 64 KiB of weights + 32 KiB of activations in
// flight per CU, and at ~2 us of loaded HBM latency that is ~45 GB/s per CU — the 36 us the kernel
// takes for 1.5 MB per workgroup.  Here the roles are swapped: every compute wave owns TPW
// DISTINCT weight tiles for ALL 128 rows of its half, so its weights are private to it and stream
// straight into its registers (one coalesced 1 KiB nontemporal load per fragment, DA stages of 2
// k-tiles ahead, the 512 KiB register file of the CU as the in-flight buffer), while the 128-row
// activation half — the operand every wave shares — goes through a small LDS-DMA ring.  Per CU in
// flight at DA = 4: 128 KiB of weights + 64 KiB of activations.
//
// Layout: weights MFMA-packed as everywhere (tile (nt, kt) = 1 KiB at ((nt KT) + kt) 1024, lane l's
// 16 B = W[16 nt + (l & 15)][64 kt + 16 (l >> 4) ..]); activations row-major [M, K] int8, staged per
// stage (2 k-tiles = 128 B of each row) as ring2's swizzled line pieces (8 rows x 128 B = 1 KiB, row
// r's 16-B chunk g at slot g ^ r).  The MFMA takes the weight fragment as its A operand, so a lane's
// accumulator holds 4 consecutive output columns (4 (lane >> 4) + q) of one row ((lane & 15) of the
// row block).
//
// Pipeline (every compute wave, the K loop fully unrolled so every register set has a name and the
// compiler's own counted vmcnt covers the weight registers): stage s's activation DMA pieces and
// weight loads are issued DA stages ahead in the order DMA(s), W(s); at the top of stage s a wave
// waits for its own DMA(s) and W(s) (a constant count: the (DA - 1) later stages' issues may stay in
// flight; the weight loads are inline asm the compiler does not track, every use pinned behind the wait),
// the barrier publishes the slot to all waves and frees the slot of stage s - 1, which DMA(s + DA)
// refills.  Nothing is issued past the last stage (the wait counts shrink there instead): an asm
// load whose result is never used would leave its register free to hipcc while the data is in flight.
// MS = 2 row halves and ring2's XCD-contiguous block mapping (both halves of a weight panel on one
// XCD: the second reader of a weight line finds it in that XCD's L2; speed only).
// Epilogues: EPI_GLUQ (gate_up: SwiGLU + int8 per (token, 64 features); a wave's tiles (2w, 2w + 1)
// are (gate, up) of 16 features, the 64-feature amax is completed across 4 waves through LDS),
// EPI_OUT (bf16 (+ bias)).
#include "gemm_i8.h"

namespace {

template <int S, int N>
struct Unroll {
  template <class F>
  __device__ __forceinline__ static void run(F&& f) {
    f(std::integral_constant<int, S>{});
    Unroll<S + 1, N>::run(f);
  }
};
template <int N>
struct Unroll<N, N> {
  template <class F>
  __device__ __forceinline__ static void run(F&&) {}
};

// A weight fragment, global -> VGPR, nontemporal; saddr form (wave-uniform base, lane offset).  Issued
// through inline asm so the compiler neither counts it nor waits for it: the kernel waits with one
// counted vmcnt per stage and pins every use behind that wait (``pin``).
__device__ __forceinline__ v4i gload_nt(const int8_t* base, uint32_t voff) {
  v4i r;
  asm volatile("global_load_dwordx4 %0, %1, %2 nt" : "=v"(r) : "v"(voff), "s"(base) : "memory");
  return r;
}
// The wait and the pin in ONE statement naming every destination "+v" (an asm load's destination
// counts as written at its ;;#ASMEND, so a separate wait would let hipcc copy it before it lands).
template <int N>
__device__ __forceinline__ void wait_vm_pin(v4i& a, v4i& b) {
  asm volatile("s_waitcnt vmcnt(%2)" : "+v"(a), "+v"(b) : "n"(N) : "memory");
}
template <int N>
__device__ __forceinline__ void wait_vm_pin(v4i& a, v4i& b, v4i& c, v4i& d) {
  asm volatile("s_waitcnt vmcnt(%4)" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "n"(N) : "memory");
}
__device__ __forceinline__ void wait_lgkm_pin(v4i& a, v4i& b, v4i& c, v4i& d) {
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) :: "memory");
}

template <int NTW, int TPW, int DA, int NSL, int EPI>
__global__ void __launch_bounds__((NTW / TPW) * 64, 1) w8a8_wreg_kernel(
    const int8_t* __restrict__ A, const float* __restrict__ sa, const int8_t* __restrict__ Wp,
    const float* __restrict__ sw, const bf16_t* __restrict__ bias, void* __restrict__ outv, float* __restrict__ os,
    int M, int N, int NTt, int Mpad, int K, int G) {
  constexpr int NCW = NTW / TPW;                      // compute waves (all of the workgroup)
  constexpr int RB = 8;                               // row blocks of a 128-row half
  constexpr int APW = 16 / NCW;                       // activation line pieces per wave per stage
  constexpr int WPS = 2 * TPW;                        // weight fragments per wave per stage
  constexpr int RA = DA + 1;                          // activation ring slots (16 KiB each)
  // vm ops a wave may leave in flight past W(s) at the top of stage s: the later stages' issues (none
  // are issued past the last stage: an unused asm load's register would be free to hipcc while the
  // load is still in flight)
  auto nwait = [](int s) constexpr { return ((s + DA - 1 < NSL - 1 ? s + DA - 1 : NSL - 1) - s) * (APW + WPS); };
  static_assert(16 % NCW == 0 && NTW % TPW == 0, "geometry");
  static_assert((DA - 1) * (APW + WPS) <= 63, "vmcnt range");
  static_assert(EPI == EPI_OUT || (EPI == EPI_GLUQ && TPW == 2 && NCW % 4 == 0), "epilogues");
  static_assert(TPW == 1 || TPW == 2, "pinned weight fragments");
  static_assert(NSL >= DA, "prologue");
  constexpr int LDS_B = RA * 16 * 1024 + NCW * RB * 16 * 4 + 2 * NTW * 16 * 4;
  static_assert(LDS_B <= 160 * 1024, "LDS budget");
  __shared__ __attribute__((aligned(1024))) int8_t lds[LDS_B];
  int8_t* const aring = lds;
  float* const xmax = reinterpret_cast<float*>(lds + RA * 16 * 1024);   // [NCW][128] row amax (GLUQ)
  float* const epi_sw = xmax + NCW * RB * 16;          // [NTW * 16] weight scales, then bias
  float* const epi_b = epi_sw + NTW * 16;

  const int x = (int)blockIdx.x & 7, jb = (int)blockIdx.x >> 3, gx = (G + 7) >> 3;
  const int row0 = (jb & 1) * 128;
  const int lbid = x * gx + (jb >> 1);
  if ((jb >> 1) >= gx || lbid >= G) return;            // whole workgroup: no barrier is left waiting
  const int Ml = min(128, M - row0);
  const int KT = K / 64;
  const int nt0 = lbid * NTW;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tw = wave * TPW;                          // the wave's first tile in the workgroup

  // ---- epilogue operands staged once in LDS (weight scales and bias of the workgroup's columns;
  // ordered for the epilogue by the stage barriers); per-token scales are read in the epilogue
  const int g4 = 4 * (lane >> 4);
  for (int c = threadIdx.x; c < NTW * 16; c += NCW * 64) {
    const int col = min(min(nt0 + (c >> 4), NTt - 1) * 16 + (c & 15), N - 1);
    epi_sw[c] = sw[col];
    epi_b[c] = bias != nullptr ? bf2f(bias[col]) : 0.f;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // ---- issue helpers
  uint32_t aoff[APW];
#pragma unroll
  for (int i = 0; i < APW; ++i)
    aoff[i] = (uint32_t)min((APW * wave + i) * 8 + (lane >> 3), Ml - 1) * (uint32_t)K + 16 * ((lane & 7) ^ (lane >> 3));
  const int8_t* const Ah = A + (size_t)row0 * K;
  auto dma = [&](int st) {                            // activation pieces of stage st
    const int8_t* ab = Ah + (size_t)st * 128;
#pragma unroll
    for (int i = 0; i < APW; ++i) glds16(ab + aoff[i], aring + ((st % RA) * 16 + APW * wave + i) * 1024);
  };
  const int8_t* wt[TPW];                              // wave-uniform panel bases
#pragma unroll
  for (int t = 0; t < TPW; ++t) wt[t] = Wp + (size_t)min(nt0 + tw + t, NTt - 1) * KT * 1024;
  const uint32_t wl = lane * 16;
  v4i wr[DA][2][TPW];
  auto loadw = [&](int st, v4i (&w)[2][TPW]) {        // the wave's weight fragments of stage st
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int t = 0; t < TPW; ++t) w[c][t] = gload_nt(wt[t] + (size_t)(2 * st + c) * 1024, wl);
  };

  v4i acc[TPW][RB];
#pragma unroll
  for (int t = 0; t < TPW; ++t)
#pragma unroll
    for (int j = 0; j < RB; ++j) acc[t][j] = v4i{0, 0, 0, 0};

  // row block j's fragment of k-tile c: line piece 2 j + ((lane & 15) >> 3), row lane & 7, chunk 4 c + (lane >> 4)
  const uint32_t a0 = lds_off(aring) + ((lane & 15) >> 3) * 1024 + (lane & 7) * 128;
  const uint32_t ax[2] = {(uint32_t)(((lane >> 4) ^ (lane & 7)) << 4), (uint32_t)(((4 + (lane >> 4)) ^ (lane & 7)) << 4)};

  // prologue: DMA(0), W(0), DMA(1), W(1), ... (the steady-state order)
  Unroll<0, DA>::run([&](auto sc) {
    constexpr int s = decltype(sc)::value;
    dma(s);
    asm volatile("" ::: "memory");
    loadw(s, wr[s]);
    asm volatile("" ::: "memory");
  });

  Unroll<0, NSL>::run([&](auto sc) {
    constexpr int s = decltype(sc)::value;
    // own DMA(s) and W(s) landed (W(s) pinned behind the wait)
    if constexpr (TPW == 1) wait_vm_pin<nwait(s)>(wr[s % DA][0][0], wr[s % DA][1][0]);
    else wait_vm_pin<nwait(s)>(wr[s % DA][0][0], wr[s % DA][0][1], wr[s % DA][1][0], wr[s % DA][1][1]);
    __builtin_amdgcn_s_barrier();                     // stage s visible to all; slot of s - 1 free
    if constexpr (s + DA < NSL) dma(s + DA);
    asm volatile("" ::: "memory");
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const uint32_t ab = a0 + (s % RA) * 16 * 1024 + ax[c];
#pragma unroll
      for (int h = 0; h < 2; ++h) {                   // 4 row blocks at a time (register budget)
        v4i af[RB / 2];
#pragma unroll
        for (int j = 0; j < RB / 2; ++j) af[j] = lds_read16(ab + (h * RB / 2 + j) * 2048);
        wait_lgkm_pin(af[0], af[1], af[2], af[3]);
#pragma unroll
        for (int t = 0; t < TPW; ++t)
#pragma unroll
          for (int j = 0; j < RB / 2; ++j)
            acc[t][h * RB / 2 + j] = mfma_i8(wr[s % DA][c][t], af[j], acc[t][h * RB / 2 + j]);
      }
    }
    asm volatile("" ::: "memory");
    if constexpr (s + DA < NSL) loadw(s + DA, wr[s % DA]);
    asm volatile("" ::: "memory");
  });
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");    // no DMA into LDS outlives the workgroup

  if constexpr (EPI == EPI_OUT) {
#pragma unroll
    for (int j = 0; j < RB; ++j) {
      const int lrow = j * 16 + (lane & 15);
      if (lrow >= Ml) continue;
      const int row = row0 + lrow;
      const float sa_j = sa[row];
#pragma unroll
      for (int t = 0; t < TPW; ++t) {
        const int col = (nt0 + tw + t) * 16 + g4;
        if (col >= N) continue;
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int cl = (tw + t) * 16 + g4 + q;
          v[q] = (float)acc[t][j][q] * sa_j * epi_sw[cl] + epi_b[cl];
        }
        bf16_t* o = reinterpret_cast<bf16_t*>(outv) + (size_t)row * N + col;
        if (col + 3 < N && (N & 3) == 0) *reinterpret_cast<uint2*>(o) = uint2{pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3])};
        else for (int q = 0; q < 4 && col + q < N; ++q) o[q] = f2bf(v[q]);
      }
    }
  } else {                                            // EPI_GLUQ: tiles (tw, tw + 1) = (gate, up) of 16 features
    const int Fo = N / 2;
    const int gw = wave & ~3;                         // first wave of this 64-feature group
    const int grp64 = (nt0 + 2 * gw) / 8;
    const bool live = nt0 + 2 * gw + 7 < NTt;
    int8_t* hq = reinterpret_cast<int8_t*>(outv);
    float h[RB][4];
#pragma unroll
    for (int j = 0; j < RB; ++j) {
      float amax = 0.f;
      const float sa_j = sa[row0 + min(j * 16 + (lane & 15), Ml - 1)];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int cg = tw * 16 + g4 + q, cu = cg + 16;
        const float g = bf2f(f2bf((float)acc[0][j][q] * sa_j * epi_sw[cg] + epi_b[cg]));   // the unfused GEMM output is bf16
        const float u = bf2f(f2bf((float)acc[1][j][q] * sa_j * epi_sw[cu] + epi_b[cu]));
        h[j][q] = g / (1.f + __expf(-g)) * u;
        amax = fmaxf(amax, fabsf(h[j][q]));
      }
      amax = fmaxf(amax, __shfl_xor(amax, 16, 64));   // the wave's 16 features of the row: lanes l ^ 16, l ^ 32
      amax = fmaxf(amax, __shfl_xor(amax, 32, 64));
      if (lane < 16) xmax[wave * 128 + j * 16 + lane] = amax;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < RB; ++j) {
      const int lrow = j * 16 + (lane & 15);
      const int row = row0 + lrow;
      float amax = 1e-8f;
#pragma unroll
      for (int i = 0; i < 4; ++i) amax = fmaxf(amax, xmax[(gw + i) * 128 + lrow]);
      const float inv = 127.f / amax;
      if (live && lrow < Ml) {
        uint32_t w = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) w |= (uint32_t)(uint8_t)quant_i8(h[j][q], inv) << (8 * q);
        const int f = ((nt0 + tw) / 2) * 16 + g4;      // output feature (4 consecutive)
        *reinterpret_cast<uint32_t*>(hq + (size_t)row * Fo + f) = w;   // Fo % 64 == 0
      }
      if (live && wave == gw && lane < 16 && row < Mpad) os[(size_t)grp64 * Mpad + row] = lrow < Ml ? amax / 127.f : 0.f;
    }
  }
}

template <int NTW, int TPW, int DA, int NSL, int EPI>
int launch_wreg(const void* A, const float* sa, const void* Wp, const float* sw, const void* bias, void* out, float* os,
                int M, int N, int K, int Mpad, hipStream_t st) {
  const int NTt = (N + 15) / 16, G = (NTt + NTW - 1) / NTW;
  hipLaunchKernelGGL((w8a8_wreg_kernel<NTW, TPW, DA, NSL, EPI>), dim3((G + 7) / 8 * 16), dim3((NTW / TPW) * 64), 0, st,
                     (const int8_t*)A, sa, (const int8_t*)Wp, sw, (const bf16_t*)bias, out, os, M, N, NTt, Mpad, K, G);
  return (int)hipGetLastError();
}

}  // namespace

// 129-256 rows, row-major int8 A with per-token scales.  epi 2 (EPI_GLUQ): 16-blocked gate_up ->
// SwiGLU -> int8 [M, N/2] + scales `os` [N/128][Mpad] (N % 256 == 0); epi 0 (EPI_OUT): bf16 [M, N]
// (+ bias).  K = 4096 (32 stages).  da: activation / weight stages in flight (4 or 6).  -2: not taken.
extern "C" int edge_w8a8_wreg(const void* A, const float* sa, const void* Wp, const float* sw, const void* bias,
                              void* out, float* os, int M, int N, int K, int Mpad, int epi, int da, hipStream_t st) {
  if (M <= 128 || M > 256 || K != 4096) return -2;
  if (epi == EPI_GLUQ) {
    if (N % 256 != 0 || os == nullptr || Mpad < M || Mpad % 16 != 0) return -2;
    // (DA = 6 spills here: 2 x 8 row blocks of accumulators + 6 stages of weights exceed 256 VGPRs, and
    // a spill's memory ops would join the counted vmcnt)
    return launch_wreg<16, 2, 4, 32, EPI_GLUQ>(A, sa, Wp, sw, bias, out, os, M, N, K, Mpad, st);
  }
  if (epi == EPI_OUT) {
    if (N % 4 != 0) return -2;
    if (da == 6) return launch_wreg<8, 1, 6, 32, EPI_OUT>(A, sa, Wp, sw, bias, out, nullptr, M, N, K, Mpad, st);
    return launch_wreg<8, 1, 4, 32, EPI_OUT>(A, sa, Wp, sw, bias, out, nullptr, M, N, K, Mpad, st);
  }
  return -2;
}

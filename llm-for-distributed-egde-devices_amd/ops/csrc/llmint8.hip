// LLM.int8() decode path without a host round trip (the reference's INT8 mode is
// bitsandbytes `Linear8bitLt`, threshold 6.0: input columns holding any |x| > threshold run in
// 16-bit against the dequantised weight columns, everything else as int8 x int8).
//
// bitsandbytes finds the outlier columns on the host (a data-dependent gather), which forces a
// device sync per projection and rules out graph capture.  Here, for decode-sized inputs
// (M <= 16 rows), one workgroup does the whole preparation on the device:
//   prep:    column outlier flags -> ordered compaction of up to CMAX outlier columns (wave
//            ballots, so the list is in column order and deterministic) -> per-token absmax over
//            the remaining columns -> int8 x with the outlier columns zeroed, the per-token
//            scales, the outlier column list and the outlier values x[:, cols].
//   the int8 GEMV (gemm_i8.hip, per-token scales) then computes the inlier part, and
//   outlier: out[m][n] += sum_j xo[m][j] * W^T[cols[j]][n] * SCB[n] / 127, reading the outlier
//            weight columns as rows of a transposed int8 copy (coalesced, N bytes per column).
// Columns past CMAX (never seen with real activations; the list holds 256) stay in the int8
// part, so nothing is dropped.  Every shape is static: the decode step is graph-capturable.
#include "common.h"

namespace {
constexpr int NT = 1024, NWV = NT / 64;
constexpr int KMAX = 32768;                 // LDS flag bitmaps: KMAX bits each

__global__ void __launch_bounds__(NT) llmint8_prep_kernel(const bf16_t* __restrict__ x, int M, int K, float thr,
                                                          int cmax, int8_t* __restrict__ q, float* __restrict__ sa,
                                                          int* __restrict__ cols, float* __restrict__ xo,
                                                          int* __restrict__ count) {
  __shared__ uint32_t flag[KMAX / 32];      // outlier columns (any row above the threshold)
  __shared__ uint32_t take[KMAX / 32];      // the accepted ones (first CMAX in column order)
  __shared__ float rmax[16][NWV];
  __shared__ int ntake;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int words = (K + 31) / 32;
  for (int w = tid; w < words; w += NT) { flag[w] = 0u; take[w] = 0u; }
  __syncthreads();
  // 1. column flags: 8 columns per thread-chunk, every row
  for (int c8 = tid * 8; c8 < K; c8 += NT * 8) {
    uint32_t bits = 0;
    for (int m = 0; m < M; ++m) {
      float v[8];
      unpack8(*reinterpret_cast<const uint4*>(x + (size_t)m * K + c8), v);
#pragma unroll
      for (int j = 0; j < 8; ++j) bits |= (fabsf(v[j]) > thr ? 1u : 0u) << j;
    }
    if (bits) atomicOr(&flag[c8 / 32], bits << (c8 % 32));
  }
  __syncthreads();
  // 2. ordered compaction by wave 0: 64 bitmap words per round, a wave prefix sum of popcounts
  if (wave == 0) {
    int base = 0;
    for (int w0 = 0; w0 < words; w0 += 64) {
      const int w = w0 + lane;
      const uint32_t f = w < words ? flag[w] : 0u;
      int pc = __popc(f), incl = pc;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(incl, o, 64);
        if (lane >= o) incl += t;
      }
      int slot = base + incl - pc;
      uint32_t acc = 0u, rest = f;
      while (rest) {
        const int b = __ffs(rest) - 1;
        rest &= rest - 1;
        if (slot < cmax) {
          cols[slot] = w * 32 + b;
          acc |= 1u << b;
        }
        ++slot;
      }
      if (w < words) take[w] = acc;
      base += __shfl(incl, 63, 64);
    }
    if (lane == 0) ntake = min(base, cmax);
  }
  __syncthreads();
  const int nt = ntake;
  if (tid == 0) *count = nt;
  // 3. per-token absmax over the columns that stay int8
  float am[16];
#pragma unroll
  for (int m = 0; m < 16; ++m) am[m] = 0.f;
  for (int c8 = tid * 8; c8 < K; c8 += NT * 8) {
    const uint32_t tk = (take[c8 / 32] >> (c8 % 32)) & 0xffu;
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      if (m < M) {
        float v[8];
        unpack8(*reinterpret_cast<const uint4*>(x + (size_t)m * K + c8), v);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (!((tk >> j) & 1u)) am[m] = fmaxf(am[m], fabsf(v[j]));
      }
    }
  }
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    float v = am[m];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    if (lane == 0) rmax[m][wave] = v;
  }
  __syncthreads();
  if (tid < M) {
    float v = 0.f;
    for (int w = 0; w < NWV; ++w) v = fmaxf(v, rmax[tid][w]);
    rmax[tid][0] = fmaxf(v, 1e-8f);
    sa[tid] = rmax[tid][0] / 127.f;
  }
  __syncthreads();
  // 4. int8 x (accepted outlier columns zeroed) and the outlier values
  for (int c8 = tid * 8; c8 < K; c8 += NT * 8) {
    const uint32_t tk = (take[c8 / 32] >> (c8 % 32)) & 0xffu;
    for (int m = 0; m < M; ++m) {
      float v[8];
      unpack8(*reinterpret_cast<const uint4*>(x + (size_t)m * K + c8), v);
      const float inv = 127.f / rmax[m][0];
      uint32_t lo = 0, hi = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) lo |= ((uint32_t)(uint8_t)((tk >> j) & 1u ? 0 : quant_i8(v[j], inv))) << (8 * j);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        hi |= ((uint32_t)(uint8_t)((tk >> (4 + j)) & 1u ? 0 : quant_i8(v[4 + j], inv))) << (8 * j);
      *reinterpret_cast<uint2*>(q + (size_t)m * K + c8) = make_uint2(lo, hi);
    }
  }
  for (int i = tid; i < M * nt; i += NT) {
    const int m = i / nt, j = i - m * nt;
    xo[(size_t)m * cmax + j] = bf2f(x[(size_t)m * K + cols[j]]);
  }
}

// out [M, N] bf16 += outlier part (fp32 sum, one rounding); a thread per output column
__global__ void __launch_bounds__(256) llmint8_outlier_kernel(bf16_t* __restrict__ out, const float* __restrict__ xo,
                                                              const int* __restrict__ cols,
                                                              const int* __restrict__ count,
                                                              const int8_t* __restrict__ wt, const float* __restrict__ scb,
                                                              int M, int N, int cmax) {
  const int nt = *count;
  if (nt == 0) return;
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  float acc[16];
#pragma unroll
  for (int m = 0; m < 16; ++m) acc[m] = 0.f;
  for (int j = 0; j < nt; ++j) {
    const float w = (float)wt[(size_t)cols[j] * N + n];
#pragma unroll
    for (int m = 0; m < 16; ++m)
      if (m < M) acc[m] += xo[(size_t)m * cmax + j] * w;
  }
  const float s = scb[n] / 127.f;
  for (int m = 0; m < M; ++m) {
    bf16_t* o = out + (size_t)m * N + n;
    *o = f2bf(bf2f(*o) + acc[m] * s);
  }
}
}  // namespace

// x bf16 [M, K] (M <= 16, K % 8 == 0, K <= 32768) -> q int8 [M, K], sa [M], cols [cmax], xo [M, cmax],
// count [1].  Returns -2 for shapes it does not take.
extern "C" int edge_llmint8_prep(const void* x, int M, int K, float thr, int cmax, void* q, float* sa, int* cols,
                                 float* xo, int* count, hipStream_t st) {
  if (M <= 0 || M > 16 || K % 8 != 0 || K > KMAX || cmax <= 0) return -2;
  hipLaunchKernelGGL(llmint8_prep_kernel, dim3(1), dim3(NT), 0, st, (const bf16_t*)x, M, K, thr, cmax, (int8_t*)q, sa,
                     cols, xo, count);
  return (int)hipGetLastError();
}

// out bf16 [M, N] += xo [M, cmax] (first *count columns) . W^T[cols] * SCB / 127; wt = int8 W^T [K, N]
extern "C" int edge_llmint8_outlier(void* out, const float* xo, const int* cols, const int* count, const void* wt,
                                    const float* scb, int M, int N, int cmax, hipStream_t st) {
  if (M <= 0 || M > 16) return -2;
  hipLaunchKernelGGL(llmint8_outlier_kernel, dim3((N + 255) / 256), dim3(256), 0, st, (bf16_t*)out, xo, cols, count,
                     (const int8_t*)wt, scb, M, N, cmax);
  return (int)hipGetLastError();
}

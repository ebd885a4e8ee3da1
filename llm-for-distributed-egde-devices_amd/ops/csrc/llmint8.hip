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
// Inputs of more rows take the uncapped multi-workgroup form below ("any rows").
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

// ---------------------------------------------------------------------------------- any rows
// The same split for prefill-sized inputs (any M), still without a host round trip, and with no
// cap: every column holding an |x| > threshold in any row goes to the 16-bit part, exactly the
// bitsandbytes split.  Four launches, all of static shape:
//   flags:   (K / 2048) x (M / 32) workgroups OR the column flags of their 32-row slab into a
//            zeroed global bitmap (one atomic per 8 flagged columns, none for clean ones);
//   compact: one wave turns the bitmap into the ordered column list + count (as in prep above);
//   quant:   one workgroup per row: absmax over the kept columns, int8 with the outliers zeroed;
//   outlier: 64 rows x 256 columns per workgroup: the rows' outlier values gathered from x into
//            LDS 32 columns at a time, W^T rows read coalesced, fp32 sums, one rounding into out.
constexpr int FR_ROWS = 32, OR_ROWS = 64, OR_COLS = 256, OR_J = 32;

__global__ void __launch_bounds__(256) llmint8_flags_kernel(const bf16_t* __restrict__ x, int M, int K, float thr,
                                                            uint32_t* __restrict__ flags) {
  const int c8 = (blockIdx.x * 256 + threadIdx.x) * 8;
  if (c8 >= K) return;
  const int m0 = blockIdx.y * FR_ROWS, m1 = min(M, m0 + FR_ROWS);
  uint32_t bits = 0;
  for (int m = m0; m < m1; ++m) {
    float v[8];
    unpack8(*reinterpret_cast<const uint4*>(x + (size_t)m * K + c8), v);
#pragma unroll
    for (int j = 0; j < 8; ++j) bits |= (fabsf(v[j]) > thr ? 1u : 0u) << j;
  }
  if (bits) atomicOr(&flags[c8 / 32], bits << (c8 % 32));
}

// one wave: ordered compaction of the flag bitmap (words = K / 32) into cols [count]; take = the
// bitmap of the accepted columns (all of them here: cmax = K)
__global__ void __launch_bounds__(64) llmint8_compact_kernel(const uint32_t* __restrict__ flags, int words, int cmax,
                                                             uint32_t* __restrict__ take, int* __restrict__ cols,
                                                             int* __restrict__ count) {
  const int lane = threadIdx.x;
  int base = 0;
  for (int w0 = 0; w0 < words; w0 += 64) {
    const int w = w0 + lane;
    const uint32_t f = w < words ? flags[w] : 0u;
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
  if (lane == 0) *count = min(base, cmax);
}

// one workgroup per row: sa[m] = absmax over the kept columns / 127, q[m] int8 (outliers zeroed)
__global__ void __launch_bounds__(256) llmint8_quant_rows_kernel(const bf16_t* __restrict__ x, int K,
                                                                 const uint32_t* __restrict__ take,
                                                                 int8_t* __restrict__ q, float* __restrict__ sa) {
  __shared__ float wmax[4];
  const int m = blockIdx.x, tid = threadIdx.x;
  const bf16_t* xr = x + (size_t)m * K;
  float am = 0.f;
  for (int c8 = tid * 8; c8 < K; c8 += 256 * 8) {
    const uint32_t tk = (take[c8 / 32] >> (c8 % 32)) & 0xffu;
    float v[8];
    unpack8(*reinterpret_cast<const uint4*>(xr + c8), v);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (!((tk >> j) & 1u)) am = fmaxf(am, fabsf(v[j]));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) am = fmaxf(am, __shfl_xor(am, o, 64));
  if ((tid & 63) == 0) wmax[tid >> 6] = am;
  __syncthreads();
  const float rm = fmaxf(fmaxf(fmaxf(wmax[0], wmax[1]), fmaxf(wmax[2], wmax[3])), 1e-8f);
  if (tid == 0) sa[m] = rm / 127.f;
  const float inv = 127.f / rm;
  for (int c8 = tid * 8; c8 < K; c8 += 256 * 8) {
    const uint32_t tk = (take[c8 / 32] >> (c8 % 32)) & 0xffu;
    float v[8];
    unpack8(*reinterpret_cast<const uint4*>(xr + c8), v);
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) lo |= ((uint32_t)(uint8_t)((tk >> j) & 1u ? 0 : quant_i8(v[j], inv))) << (8 * j);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      hi |= ((uint32_t)(uint8_t)((tk >> (4 + j)) & 1u ? 0 : quant_i8(v[4 + j], inv))) << (8 * j);
    *reinterpret_cast<uint2*>(q + (size_t)m * K + c8) = make_uint2(lo, hi);
  }
}

// out [M, N] bf16 += x[:, cols[:count]] . W^T[cols[:count]] * SCB / 127; grid (N / 256, M / 64)
__global__ void __launch_bounds__(256) llmint8_outlier_rows_kernel(bf16_t* __restrict__ out, const bf16_t* __restrict__ x,
                                                                   const int* __restrict__ cols,
                                                                   const int* __restrict__ count,
                                                                   const int8_t* __restrict__ wt,
                                                                   const float* __restrict__ scb, int M, int N, int K) {
  __shared__ float xs[OR_J][OR_ROWS];         // [outlier column][row]: a thread's 64 rows are one LDS row
  const int nt = *count;
  if (nt == 0) return;                        // uniform: the common case costs one load
  const int tid = threadIdx.x, n = blockIdx.x * OR_COLS + tid, m0 = blockIdx.y * OR_ROWS;
  const int nc = min(n, N - 1);
  float acc[OR_ROWS];
#pragma unroll
  for (int m = 0; m < OR_ROWS; ++m) acc[m] = 0.f;
  for (int j0 = 0; j0 < nt; j0 += OR_J) {
    __syncthreads();                          // previous chunk's readers are done
    for (int i = tid; i < OR_J * OR_ROWS; i += 256) {
      const int j = i / OR_ROWS, m = i - j * OR_ROWS;
      xs[j][m] = (j0 + j < nt && m0 + m < M) ? bf2f(x[(size_t)(m0 + m) * K + cols[j0 + j]]) : 0.f;
    }
    __syncthreads();
    const int jn = min(OR_J, nt - j0);
    for (int j = 0; j < jn; ++j) {
      const float w = (float)wt[(size_t)cols[j0 + j] * N + nc];
#pragma unroll
      for (int m = 0; m < OR_ROWS; ++m) acc[m] += xs[j][m] * w;
    }
  }
  if (n >= N) return;
  const float s = scb[n] / 127.f;
  const int mr = min(OR_ROWS, M - m0);
#pragma unroll
  for (int m = 0; m < OR_ROWS; ++m) {
    if (m < mr) {
      bf16_t* o = out + (size_t)(m0 + m) * N + n;
      *o = f2bf(bf2f(*o) + acc[m] * s);
    }
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

// Any-rows preparation: x bf16 [M, K] (K % 32 == 0) -> q int8 [M, K] (outlier columns zeroed),
// sa [M], cols [K] (first *count), count [1]; flags / take: scratch of K / 32 words each.
extern "C" int edge_llmint8_prep_rows(const void* x, int M, int K, float thr, void* q, float* sa, int* cols, int* count,
                                      uint32_t* flags, uint32_t* take, hipStream_t st) {
  if (M <= 0 || K % 32 != 0 || K <= 0) return -2;
  const int words = K / 32;
  hipError_t e = hipMemsetAsync(flags, 0, (size_t)words * 4, st);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(llmint8_flags_kernel, dim3((K + 2047) / 2048, (M + FR_ROWS - 1) / FR_ROWS), dim3(256), 0, st,
                     (const bf16_t*)x, M, K, thr, flags);
  hipLaunchKernelGGL(llmint8_compact_kernel, dim3(1), dim3(64), 0, st, (const uint32_t*)flags, words, K, take, cols,
                     count);
  hipLaunchKernelGGL(llmint8_quant_rows_kernel, dim3(M), dim3(256), 0, st, (const bf16_t*)x, K,
                     (const uint32_t*)take, (int8_t*)q, sa);
  return (int)hipGetLastError();
}

// out bf16 [M, N] += x[:, cols[:count]] . W^T[cols[:count]] * SCB / 127 (wt = int8 W^T [K, N]).
extern "C" int edge_llmint8_outlier_rows(void* out, const void* x, const int* cols, const int* count, const void* wt,
                                         const float* scb, int M, int N, int K, hipStream_t st) {
  if (M <= 0 || N <= 0) return -2;
  hipLaunchKernelGGL(llmint8_outlier_rows_kernel, dim3((N + OR_COLS - 1) / OR_COLS, (M + OR_ROWS - 1) / OR_ROWS),
                     dim3(256), 0, st, (bf16_t*)out, (const bf16_t*)x, cols, count, (const int8_t*)wt, scb, M, N, K);
  return (int)hipGetLastError();
}

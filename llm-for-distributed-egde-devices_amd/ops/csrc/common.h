// Shared device helpers for the edgellm CDNA4 (gfx950) kernels.
// Wave size is 64 everywhere (hard-coded: gfx950 has no wave32 mode for these kernels).
#pragma once
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#define EDGE_WAVE 64

typedef uint16_t bf16_t;                                   // raw bf16 bits in memory
typedef short    v4s  __attribute__((ext_vector_type(4)));
typedef short    v8s  __attribute__((ext_vector_type(8)));
typedef float    v4f  __attribute__((ext_vector_type(4)));
typedef float    v16f __attribute__((ext_vector_type(16)));
typedef int      v4i  __attribute__((ext_vector_type(4)));
typedef int      v16i __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float bf2f(uint32_t u16) { return __uint_as_float(u16 << 16); }
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;                      // v_cvt_pk_bf16_f32, RNE, NaN-preserving
  return __builtin_bit_cast(bf16_t, b);
}
__device__ __forceinline__ uint32_t pack_bf2(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}

// 8 bf16 packed in a uint4 <-> 8 floats
__device__ __forceinline__ void unpack8(const uint4& v, float* f) {
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
  f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xffff0000u);
  f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xffff0000u);
}
__device__ __forceinline__ uint4 pack8(const float* f) {
  uint4 v;
  v.x = pack_bf2(f[0], f[1]); v.y = pack_bf2(f[2], f[3]);
  v.z = pack_bf2(f[4], f[5]); v.w = pack_bf2(f[6], f[7]);
  return v;
}

// 16-bit float elements in memory as raw uint16 bits: bf16 (H = false, the default everywhere) or IEEE
// fp16 (H = true: the reference's fp16 agents, Code/Base Models/phi2-pythia_fp_updated.py:32).
// Kernels that move activations take a `bool H` template flag and convert through these.
template <bool H>
__device__ __forceinline__ float e2f(uint32_t u16) {
  if constexpr (H) return __half2float(__ushort_as_half((unsigned short)u16));
  else return bf2f(u16);
}
template <bool H>
__device__ __forceinline__ uint16_t f2e(float f) {
  if constexpr (H) return __half_as_ushort(__float2half(f));     // round to nearest even
  else return f2bf(f);
}
template <bool H>
__device__ __forceinline__ uint32_t pack_e2(float lo, float hi) {
  return (uint32_t)f2e<H>(lo) | ((uint32_t)f2e<H>(hi) << 16);
}
template <bool H>
__device__ __forceinline__ void unpack8e(const uint4& v, float* f) {
  if constexpr (H) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) { f[2 * i] = e2f<true>(w[i] & 0xffffu); f[2 * i + 1] = e2f<true>(w[i] >> 16); }
  } else {
    unpack8(v, f);
  }
}
template <bool H>
__device__ __forceinline__ uint4 pack8e(const float* f) {
  uint4 v;
  v.x = pack_e2<H>(f[0], f[1]); v.y = pack_e2<H>(f[2], f[3]);
  v.z = pack_e2<H>(f[4], f[5]); v.w = pack_e2<H>(f[6], f[7]);
  return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide reductions for blockDim.x == NT (multiple of 64); `red` holds NT/64 floats.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) red[w] = v;
  __syncthreads();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) r += red[i];
  __syncthreads();
  return r;
}
template <int NT>
__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) red[w] = v;
  __syncthreads();
  float r = -INFINITY;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) r = fmaxf(r, red[i]);
  __syncthreads();
  return r;
}

// Softmax exponentials use __builtin_amdgcn_exp2f (a bare v_exp_f32): the libm exp2f wraps it in a
// denormal-range fix-up (compare, select, add, multiply) per call, and softmax arguments are <= 0,
// where a result below 2^-126 may flush to zero.

__device__ __forceinline__ int8_t quant_i8(float v, float inv_scale) {
  float q = rintf(v * inv_scale);
  q = fminf(fmaxf(q, -127.f), 127.f);
  return (int8_t)(int)q;
}

// Counter-based uniform in (0,1); bit-identical to ops/_ref.py::uniform_hash.
__device__ __forceinline__ uint32_t mix32(uint32_t h) {
  h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
  return h;
}
__device__ __forceinline__ float uniform_hash(uint32_t seed, uint32_t row, uint32_t step, uint32_t idx) {
  uint32_t h = mix32((row * 0x9E3779B1u) ^ seed);
  h = mix32(h ^ (step * 0x7FEB352Du));
  h = mix32(h ^ (idx * 0x846CA68Bu));
  return (float)(((h >> 9) << 1) | 1u) * (1.0f / 16777216.0f);  // exact in f32
}

#define EDGE_CHECK_LAUNCH() do { (void)hipGetLastError(); } while (0)

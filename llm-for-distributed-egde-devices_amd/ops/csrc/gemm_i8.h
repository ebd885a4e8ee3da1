// Shared by the W8A8 GEMM kernels (gemm_i8.hip: decode, gemm_i8_prefill.hip: prefill).
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
#pragma once
#include "common.h"

namespace {
constexpr int NT = 256;
constexpr int A_TOKEN = 0, A_GROUP = 1;
constexpr int EPI_OUT = 0, EPI_GLU = 1, EPI_GLUQ = 2, EPI_PART = 3, EPI_GELUQT = 4, EPI_GELUQE = 5;
// (EPI_GELUQT / EPI_GELUQE: gelu (tanh / erf) of the bf16 output, quantised per (token, 64 columns)
// in the epilogue of a 4-tile workgroup — the GELU MLPs' (Phi-2, Pythia) up projection at <= 64 rows)

__device__ __forceinline__ v4i mfma_i8(const v4i& a, const v4i& b, const v4i& c) {
  return __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void fold(v4f& accf, const v4i& t, const v4f& s) {
#pragma unroll
  for (int q = 0; q < 4; ++q) accf[q] += (float)t[q] * s[q];
}
__device__ __forceinline__ void fold1(v4f& accf, const v4i& t, float s) {
#pragma unroll
  for (int q = 0; q < 4; ++q) accf[q] += (float)t[q] * s;
}

// zero bias for epilogues without one (a valid address for unconditional loads)
__device__ const bf16_t g_zero_bf16[8] = {0, 0, 0, 0, 0, 0, 0, 0};

// LDS-DMA helpers

__device__ __forceinline__ void glds16(const void* g, void* lds_base) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}
// streaming form (cache policy nt): weight bytes read once per step, kept out of the way of the
// L2-resident activation panel every workgroup re-reads
__device__ __forceinline__ void glds16_nt(const void* g, void* lds_base) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)lds_base, 16, 0, 2);
}

// LDS byte address of a __shared__ pointer, and a ds_read_b128 the compiler does not track (callers
// order it with explicit lgkmcnt waits; see the ring kernel below)
__device__ __forceinline__ uint32_t lds_off(const void* p) {
  return (uint32_t)(uintptr_t)((__attribute__((address_space(3))) const void*)p);
}
__device__ __forceinline__ v4i lds_read16(uint32_t addr) {
  v4i r;
  asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(addr));
  return r;
}
__device__ __forceinline__ int lds_read4(uint32_t addr) {
  int r;
  asm volatile("ds_read_b32 %0, %1" : "=v"(r) : "v"(addr));
  return r;
}

// n ds_read_b128 at addr + 1024 i (immediate offsets: no address VALU, no extra VGPRs)
template <int I, int N>
__device__ __forceinline__ void lds_read_row_(uint32_t addr, v4i (&f)[N]) {
  if constexpr (I < N) {
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(f[I]) : "v"(addr), "n"(I * 1024));
    lds_read_row_<I + 1, N>(addr, f);
  }
}
template <int N>
__device__ __forceinline__ void lds_read_row(uint32_t addr, v4i (&f)[N]) { lds_read_row_<0, N>(addr, f); }

}  // namespace

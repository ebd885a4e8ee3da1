// Fused RoPE + KV-cache write (SURVEY K4 + K6 append).
// Input: the QKV projection output [B*T, (Hq + 2*Hkv) * D] (token-major, heads contiguous).
// Rotates q and k with the HF "rotate_half" convention on the first `rot` dims (full RoPE for
// Llama, partial 32/80 for Phi-2 and 64/256 for Pythia; llama3 frequency scaling is folded into
// the host-built cos/sin table), writes q to a [B, T, Hq, D] buffer and k, v straight into the
// head-major caches [B, Hkv, S, D] (row stride D) at position start_pos[b] + t.
// HeadInfer split: kv heads h >= split_h go to a second cache (k2/v2, heads re-based to
// h - split_h) at position cpos2[b] + t — the offloaded heads' device staging rows.
// One workgroup per token; every thread moves 8 elements (16 B) per step.  HF: fp16 rows and
// caches (the reference's fp16 agents), bf16 otherwise.
#include "common.h"

namespace {
constexpr int NT = 256;

struct Cache2 {
  bf16_t* k;
  bf16_t* v;
  int64_t sb, sh;
  int S, split_h;
  const int* cpos;
};

template <bool HF>
__global__ void __launch_bounds__(NT) rope_kv_kernel(
    const bf16_t* __restrict__ qkv, const int* __restrict__ start_pos, const float* __restrict__ cs,
    bf16_t* __restrict__ q_out, bf16_t* __restrict__ kc, bf16_t* __restrict__ vc,
    int T, int Hq, int Hkv, int D, int rot, int64_t c_sb, int64_t c_sh, int S, Cache2 c2) {
  const int tok = blockIdx.x;
  const int b = tok / T, t = tok - b * T;
  const int pos = start_pos[b] + t;
  const int pos2 = (c2.cpos != nullptr ? c2.cpos[b] : start_pos[b]) + t;
  const int cpr = D / 8;                  // 8-element chunks per head
  const int nchunks = (Hq + 2 * Hkv) * cpr;
  const int half = rot / 2;
  const bf16_t* x = qkv + (size_t)tok * (Hq + 2 * Hkv) * D;
  const float2* csp = reinterpret_cast<const float2*>(cs) + (size_t)pos * half;
  for (int c = threadIdx.x; c < nchunks; c += NT) {
    const int hh = c / cpr;
    const int e0 = (c - hh * cpr) * 8;
    float v[8];
    unpack8e<HF>(*reinterpret_cast<const uint4*>(x + (size_t)hh * D + e0), v);
    const bool is_v = hh >= Hq + Hkv;
    if (!is_v && e0 < rot) {
      const bool lo = e0 < half;
      const int pe = lo ? e0 + half : e0 - half;
      const int fi = lo ? e0 : e0 - half;
      float p[8];
      unpack8e<HF>(*reinterpret_cast<const uint4*>(x + (size_t)hh * D + pe), p);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float2 r = csp[fi + j];
        v[j] = lo ? (v[j] * r.x - p[j] * r.y) : (v[j] * r.x + p[j] * r.y);
      }
    }
    const uint4 o = pack8e<HF>(v);
    if (hh < Hq) {
      *reinterpret_cast<uint4*>(q_out + ((size_t)tok * Hq + hh) * D + e0) = o;
      continue;
    }
    const int h = is_v ? hh - Hq - Hkv : hh - Hq;
    if (h < c2.split_h) {
      if (pos < S) {  // host checks capacity; never write out of the cache
        bf16_t* dst = (is_v ? vc : kc) + b * c_sb + h * c_sh + (size_t)pos * D + e0;
        *reinterpret_cast<uint4*>(dst) = o;
      }
    } else if (pos2 < c2.S) {
      bf16_t* dst = (is_v ? c2.v : c2.k) + b * c2.sb + (h - c2.split_h) * c2.sh + (size_t)pos2 * D + e0;
      *reinterpret_cast<uint4*>(dst) = o;
    }
  }
}
}  // namespace

extern "C" int edge_rope_kv_write(const void* qkv, const int* start_pos, const float* cs, void* q_out,
                                  void* k_cache, void* v_cache, int B, int T, int Hq, int Hkv, int D, int rot,
                                  int64_t c_sb, int64_t c_sh, int S, void* k2, void* v2, int64_t c2_sb,
                                  int64_t c2_sh, int S2, int split_h, const int* cpos2, int h16, hipStream_t st) {
  if (D % 8 || (rot % 16 && rot != 0) || rot > D) return -2;
  if (B * T == 0) return 0;
  Cache2 c2{(bf16_t*)k2, (bf16_t*)v2, c2_sb, c2_sh, S2, split_h < 0 ? Hkv : split_h, cpos2};
  if (h16)
    hipLaunchKernelGGL(rope_kv_kernel<true>, dim3(B * T), dim3(NT), 0, st, (const bf16_t*)qkv, start_pos, cs,
                       (bf16_t*)q_out, (bf16_t*)k_cache, (bf16_t*)v_cache, T, Hq, Hkv, D, rot, c_sb, c_sh, S, c2);
  else
    hipLaunchKernelGGL(rope_kv_kernel<false>, dim3(B * T), dim3(NT), 0, st, (const bf16_t*)qkv, start_pos, cs,
                       (bf16_t*)q_out, (bf16_t*)k_cache, (bf16_t*)v_cache, T, Hq, Hkv, D, rot, c_sb, c_sh, S, c2);
  return (int)hipGetLastError();
}

// Causal flash-attention forward for prefill / chunked prefill on bf16 MFMA.
//
// q [B, T, Hq, D] for positions start_pos[b] + t; K/V from the head-major caches [B, Hkv, S, D]
// (already written by rope_kv_write), keys [0, start_pos[b] + T).  GQA: kv head = h / (Hq/Hkv).
// D in {64, 80, 128, 256}; D=80 (Phi-2) is zero-padded to 96 on the reduction side.
//
// Workgroup = 4 waves = 64 query rows of one (batch, head); each wave owns 16 rows.
// Per 64-key tile:  S = Q.K^T   v_mfma_f32_16x16x32_bf16, Q fragments resident in VGPRs,
//                               K fragments by ds_read_b128 from a padded-row LDS image
//                               (row stride 2*DP + 16 B -> the 16 rows of a lane group land on
//                               16 distinct 16-B slots: conflict-free)
//                   online softmax in the log2 domain, rows spread over 16 lanes (xor-shuffles)
//                   P -> per-wave LDS (bf16, padded rows) -> A fragments by ds_read_b128
//                   O += P.V     V fragments by ds_read_b64_tr_b16 (hardware transpose read of
//                               the row-major V tile: no transposed copy)
// The next tile's K/V are loaded into registers while the current tile computes (async-STAGE
// split: issue early, ds_write after the barrier).
#include "common.h"

namespace {
constexpr int NT = 256;
constexpr int QT = 64;   // query rows per workgroup
constexpr int KT = 64;   // keys per tile

typedef __attribute__((address_space(3))) v4s lds_v4s;

__device__ __forceinline__ v4f mfma_bf16(const v8s& a, const v8s& b, const v4f& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

template <int D>
struct Geo {
  static constexpr int DP = (D + 31) / 32 * 32;       // reduction-padded head dim
  static constexpr int KS = DP * 2 + 16;              // K LDS row stride (bytes)
  static constexpr int VS = D * 2 + 16;               // V LDS row stride (bytes)
  static constexpr int PS = KT * 2 + 16;              // P LDS row stride (bytes)
  static constexpr int KCH = DP / 8;                  // 16-B chunks per K LDS row
  static constexpr int VCH = D / 8;                   // 16-B chunks per V row
  static constexpr int K_BYTES = KT * KS;
  static constexpr int V_BYTES = KT * VS;
  static constexpr int P_BYTES = 16 * PS;             // per wave
  static constexpr int LDS = K_BYTES + V_BYTES + 4 * P_BYTES;
  static constexpr int KLOADS = (KT * KCH + NT - 1) / NT;  // uint4 per thread per K tile
  static constexpr int VLOADS = (KT * VCH + NT - 1) / NT;
  static constexpr int NDT = D / 16;                  // output d-tiles
  static constexpr int NKK = DP / 32;                 // QK^T k-steps
};

template <int D, bool CAUSAL>
__global__ void __launch_bounds__(NT) prefill_attn_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc, int64_t c_sb,
    int64_t c_sh, const int* __restrict__ start_pos, bf16_t* __restrict__ out, int T, int Hq, int Hkv,
    float scale_log2) {
  using G = Geo<D>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* k_lds = smem;
  char* v_lds = smem + G::K_BYTES;
  const int qtile = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int kvh = h / (Hq / Hkv);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  char* p_lds = smem + G::K_BYTES + G::V_BYTES + wave * G::P_BYTES;
  const int s0 = start_pos[b];
  const int nkeys = s0 + T;
  const int q0 = qtile * QT;                           // first query row (within T) of the WG
  const int wq0 = q0 + wave * 16;                      // first row of this wave
  const int g4 = lane >> 4, c16 = lane & 15;

  // ---- Q fragments (A operand): lane <- Q[row = wq0 + c16][d = kk*32 + 8*g4 .. +8]
  v8s qf[G::NKK];
  {
    const int t = wq0 + c16;
#pragma unroll
    for (int kk = 0; kk < G::NKK; ++kk) {
      const int d = kk * 32 + 8 * g4;
      if (t < T && d < D) {
        qf[kk] = *reinterpret_cast<const v8s*>(q + (((size_t)b * T + t) * Hq + h) * D + d);
      } else {
        qf[kk] = v8s{0, 0, 0, 0, 0, 0, 0, 0};
      }
    }
  }

  v4f o[G::NDT];
#pragma unroll
  for (int i = 0; i < G::NDT; ++i) o[i] = v4f{0.f, 0.f, 0.f, 0.f};
  float m_i[4], l_i[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) { m_i[i] = -INFINITY; l_i[i] = 0.f; }

  // keys this workgroup needs: causal -> up to the last query row's position
  const int last_q = min(q0 + QT, T) - 1;
  const int kend = CAUSAL ? min(nkeys, s0 + last_q + 1) : nkeys;
  const int ntiles = (kend + KT - 1) / KT;

  const bf16_t* kbase = kc + b * c_sb + kvh * c_sh;
  const bf16_t* vbase = vc + b * c_sb + kvh * c_sh;

  uint4 kreg[G::KLOADS], vreg[G::VLOADS];
  auto load_tile = [&](int kt) {
#pragma unroll
    for (int i = 0; i < G::KLOADS; ++i) {
      const int idx = threadIdx.x + i * NT;
      const int r = idx / G::KCH, ch = idx - r * G::KCH;
      const int key = kt * KT + r;
      kreg[i] = (r < KT && key < kend && ch * 8 < D) ? *reinterpret_cast<const uint4*>(kbase + (size_t)key * D + ch * 8)
                                                     : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < G::VLOADS; ++i) {
      const int idx = threadIdx.x + i * NT;
      const int r = idx / G::VCH, ch = idx - r * G::VCH;
      const int key = kt * KT + r;
      vreg[i] = (r < KT && key < kend) ? *reinterpret_cast<const uint4*>(vbase + (size_t)key * D + ch * 8)
                                       : make_uint4(0, 0, 0, 0);
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int i = 0; i < G::KLOADS; ++i) {
      const int idx = threadIdx.x + i * NT;
      const int r = idx / G::KCH, ch = idx - r * G::KCH;
      if (r < KT) *reinterpret_cast<uint4*>(k_lds + r * G::KS + ch * 16) = kreg[i];
    }
#pragma unroll
    for (int i = 0; i < G::VLOADS; ++i) {
      const int idx = threadIdx.x + i * NT;
      const int r = idx / G::VCH, ch = idx - r * G::VCH;
      if (r < KT) *reinterpret_cast<uint4*>(v_lds + r * G::VS + ch * 16) = vreg[i];
    }
  };

  if (ntiles > 0) load_tile(0);
  for (int kt = 0; kt < ntiles; ++kt) {
    __syncthreads();           // every wave is done reading the previous tile
    store_tile();
    __syncthreads();
    if (kt + 1 < ntiles) load_tile(kt + 1);   // in flight during this tile's math

    // ---- S = Q K^T : 4 key sub-tiles of 16
    v4f s[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      s[nt] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < G::NKK; ++kk) {
        const v8s kf = *reinterpret_cast<const v8s*>(k_lds + (nt * 16 + c16) * G::KS + (kk * 32 + 8 * g4) * 2);
        s[nt] = mfma_bf16(qf[kk], kf, s[nt]);
      }
    }
    // ---- online softmax; lane holds S[row = 4*g4 + i][key = nt*16 + c16]
    float alpha[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int qpos = s0 + wq0 + 4 * g4 + i;
      float mx = -INFINITY;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int kpos = kt * KT + nt * 16 + c16;
        float v = s[nt][i] * scale_log2;
        const bool masked = (kpos >= kend) || (CAUSAL && kpos > qpos);
        v = masked ? -INFINITY : v;
        s[nt][i] = v;
        mx = fmaxf(mx, v);
      }
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) mx = fmaxf(mx, __shfl_xor(mx, off, 64));
      const float mnew = fmaxf(m_i[i], mx);
      const float msafe = (mnew == -INFINITY) ? 0.f : mnew;
      alpha[i] = exp2f(m_i[i] - msafe);
      float rs = 0.f;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const float p = exp2f(s[nt][i] - msafe);
        s[nt][i] = p;
        rs += p;
      }
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) rs += __shfl_xor(rs, off, 64);
      l_i[i] = l_i[i] * alpha[i] + rs;
      m_i[i] = mnew;
    }
#pragma unroll
    for (int dt = 0; dt < G::NDT; ++dt)
#pragma unroll
      for (int i = 0; i < 4; ++i) o[dt][i] *= alpha[i];

    // ---- P -> LDS (bf16), row-major [16][64] with padded rows
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        *reinterpret_cast<bf16_t*>(p_lds + (4 * g4 + i) * G::PS + (nt * 16 + c16) * 2) = f2bf(s[nt][i]);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's P writes landed
    __builtin_amdgcn_wave_barrier();

    // ---- O += P V : 2 k-steps of 32 keys
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const v8s pf = *reinterpret_cast<const v8s*>(p_lds + c16 * G::PS + (ks * 32 + 8 * g4) * 2);
      const int key0 = ks * 32 + 8 * g4;
      const int qq = c16 >> 2, pp = c16 & 3;
#pragma unroll
      for (int dt = 0; dt < G::NDT; ++dt) {
        const char* a0 = v_lds + (key0 + qq) * G::VS + (dt * 16 + 4 * pp) * 2;
        const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(a0));
        const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(a0 + 4 * G::VS));
        const v8s vf = v8s{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        o[dt] = mfma_bf16(pf, vf, o[dt]);
      }
    }
  }

  // ---- epilogue: O / l -> out[b][t][h][d]
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int t = wq0 + 4 * g4 + i;
    if (t < T) {
      const float inv = l_i[i] > 0.f ? 1.f / l_i[i] : 0.f;
#pragma unroll
      for (int dt = 0; dt < G::NDT; ++dt)
        out[(((size_t)b * T + t) * Hq + h) * D + dt * 16 + c16] = f2bf(o[dt][i] * inv);
    }
  }
}
}  // namespace

extern "C" int edge_prefill_attn(const void* q, const void* k_cache, const void* v_cache, int64_t c_sb, int64_t c_sh,
                                 const int* start_pos, void* out, int B, int T, int Hq, int Hkv, int D, float scale,
                                 int causal, hipStream_t st) {
  if (B * T == 0) return 0;
  if (Hq % Hkv) return -2;
  const float sl2 = scale * 1.4426950408889634f;
  const dim3 grid((T + QT - 1) / QT, Hq, B);
#define PL(DD)                                                                                                    \
  do {                                                                                                            \
    static bool attr_set = false; /* >64 KiB dynamic LDS (D=256): raise the per-kernel cap once */                \
    if (!attr_set && Geo<DD>::LDS > 65536) {                                                                      \
      (void)hipFuncSetAttribute((const void*)prefill_attn_kernel<DD, true>,                                        \
                                hipFuncAttributeMaxDynamicSharedMemorySize, Geo<DD>::LDS);                         \
      (void)hipFuncSetAttribute((const void*)prefill_attn_kernel<DD, false>,                                       \
                                hipFuncAttributeMaxDynamicSharedMemorySize, Geo<DD>::LDS);                         \
    }                                                                                                             \
    attr_set = true;                                                                                              \
    if (causal)                                                                                                   \
      hipLaunchKernelGGL((prefill_attn_kernel<DD, true>), grid, dim3(NT), Geo<DD>::LDS, st, (const bf16_t*)q,       \
                         (const bf16_t*)k_cache, (const bf16_t*)v_cache, c_sb, c_sh, start_pos, (bf16_t*)out, T, Hq, \
                         Hkv, sl2);                                                                               \
    else                                                                                                          \
      hipLaunchKernelGGL((prefill_attn_kernel<DD, false>), grid, dim3(NT), Geo<DD>::LDS, st, (const bf16_t*)q,      \
                         (const bf16_t*)k_cache, (const bf16_t*)v_cache, c_sb, c_sh, start_pos, (bf16_t*)out, T, Hq, \
                         Hkv, sl2);                                                                               \
  } while (0)
  switch (D) {
    case 64: PL(64); break;
    case 80: PL(80); break;
    case 128: PL(128); break;
    case 256: PL(256); break;
    default: return -4;
  }
#undef PL
  return (int)hipGetLastError();
}

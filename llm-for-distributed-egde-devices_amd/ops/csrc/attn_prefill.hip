// Causal flash-attention forward for prefill / chunked prefill on bf16 MFMA (fp16
// MFMA for the fp16 agents: template flag HF, same tiling — the f16 MFMAs run at the bf16 rate).
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

#include <type_traits>

namespace {
constexpr int NT = 256;
constexpr int QT = 64;   // query rows per workgroup
constexpr int KT = 64;   // keys per tile

typedef __attribute__((address_space(3))) v4s lds_v4s;

typedef _Float16 v8h __attribute__((ext_vector_type(8)));

template <bool HF>
__device__ __forceinline__ v4f mfma_16(const v8s& a, const v8s& b, const v4f& c) {
  if constexpr (HF)
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(v8h, a), __builtin_bit_cast(v8h, b), c, 0, 0, 0);
  else return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void glds16_fa(const void* g, void* lds_base) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

// max / sum over lanes i and i ^ 32 by one v_permlane32_swap instead of a ds_bpermute round trip
// (+0.5-1.4 % on the flash kernel, profiles/fa_v2_forms_ab_r5.json): the swap of x with itself
// leaves the low half's values in r[0] and the high half's in r[1] on every lane.  Same operands,
// same order as the shuffle form: bit-identical
__device__ __forceinline__ float half_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float half_sum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// Transposed V reads in inline asm.  Through the builtin, the compiler's wait-count pass cannot tell
// them from reads of the slot an LDS-DMA is still filling and puts an s_waitcnt vmcnt(0) before every
// P.V: each tile then waits for the DMA of tile t + 2 it has just issued.  The ring's own counted
// vmcnt + barrier already orders every V read after its tile's DMA; here the reads are counted by
// lgkmcnt, and the wait names every destination ("+v") so nothing reads them early (sched_barrier:
// no MFMA hoisted above the wait).  The step's rows go in the immediate offset (P.V address work
// 26 -> 11 vector instructions per tile).  Measured on one box against the builtin form: within 1 %
// (profiles/fa_tr_asm_vs_builtin_ab_r5.json, prefill_ttft_32k_tr_ab_r5.jsonl) - the ~1-2 tiles
// of look-ahead still covered the DMA's L2-hit latency.
template <int OFF>
__device__ __forceinline__ v4s ds_tr16(uint32_t addr) {
  v4s r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
  return r;
}
template <int N>
__device__ __forceinline__ void wait_tr(v4s (&lo)[N], v4s (&hi)[N]) {
  if constexpr (N == 4)
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(lo[0]), "+v"(lo[1]), "+v"(lo[2]), "+v"(lo[3]), "+v"(hi[0]), "+v"(hi[1]),
                 "+v"(hi[2]), "+v"(hi[3]));
  else
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(lo[0]), "+v"(lo[1]), "+v"(hi[0]), "+v"(hi[1]));
  __builtin_amdgcn_sched_barrier(0);
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

template <int D, bool CAUSAL, bool HF>
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
        s[nt] = mfma_16<HF>(qf[kk], kf, s[nt]);
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
      alpha[i] = __builtin_amdgcn_exp2f(m_i[i] - msafe);
      float rs = 0.f;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const float p = __builtin_amdgcn_exp2f(s[nt][i] - msafe);
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

    // ---- P -> LDS (16-bit), row-major [16][64] with padded rows
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        *reinterpret_cast<bf16_t*>(p_lds + (4 * g4 + i) * G::PS + (nt * 16 + c16) * 2) = f2e<HF>(s[nt][i]);
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
        o[dt] = mfma_16<HF>(pf, vf, o[dt]);
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
        out[(((size_t)b * T + t) * Hq + h) * D + dt * 16 + c16] = f2e<HF>(o[dt][i] * inv);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// fa_kernel: the D = 64 / 128 flash-attention forward (Llama-2 / -3 / -3.2 / Mistral heads), rebuilt for
// CDNA4 around three choices the 16-row kernel above lacks:
//  * 256 query rows per workgroup, 8 waves x 32 rows on v_mfma_f32_32x32x16_bf16, computed
//    TRANSPOSED: S^T = K Q^T (A = K rows from LDS by ds_read_b128, B = Q^T resident in VGPRs) puts
//    one query per lane (32 of the 64 keys of a tile in the lane, the other 32 in lane ^ 32), so
//    the row max / sum are in-lane reductions plus ONE cross-half shuffle, the rescale of O is a
//    per-lane multiply, and the S^T accumulator converts to the B operand (P^T) of O^T = V^T P^T
//    in place — no P round trip through LDS.  V^T comes from the row-major V tile by
//    ds_read_b64_tr_b16 (the key order inside a 16-key step is permuted identically on both
//    operands, which leaves the sum unchanged).
//  * K/V tiles (64 keys, 8 / 16 KiB each) move global -> LDS by LDS-DMA (global_load_lds_dwordx4,
//    no VGPR staging) into a 3-slot ring: tile t + 2 is issued right after the one barrier of
//    tile t, which also retires tile t - 1's slot — one s_barrier per tile, two tiles in flight.
//  * XOR-swizzled 16-byte chunks (slot = chunk ^ f(key)) chosen so both the K reads (16 keys x
//    one chunk per lane group) and the transposed V reads (4 keys x 4 chunks) are conflict-free;
//    the DMA realises the swizzle by choosing each lane's global source address.
// Causal tiles above a wave's last query are skipped by that wave (it still joins the barrier);
// workgroups are dispatched longest-first.  Keys past the cache end are clamped to a valid row
// and masked, so a tile never reads outside the cache.
constexpr int FA_W = 8, FA_NT = FA_W * 64, FA_QT = FA_W * 32, FA_KT = 64, FA_RING = 3;
template <int D>
struct FaGeo {
  static constexpr int ROWB = D * 2;                     // bytes per key row
  static constexpr int CH = D / 8;                       // 16-byte chunks per row
  static constexpr int KK = D / 16;                      // S^T k-steps
  static constexpr int DB = D / 32;                      // O^T 32-row blocks
  static constexpr int TILE = FA_KT * ROWB;              // one K (or V) tile
  static constexpr int SLOT = 2 * TILE;
  static constexpr int LDS = FA_RING * SLOT;             // 96 KiB (D 128) / 48 KiB (D 64)
  static constexpr int LDS_STG = (FA_RING + 1) * SLOT;   // the staggered form's 4-slot ring
  static constexpr int RPP = 1024 / ROWB;                // key rows per 1 KiB DMA piece
  static constexpr int PIECES = TILE / 1024;             // per K (or V) tile
  static constexpr int PPW = 2 * PIECES / FA_W;          // pieces per wave per tile
  // chunk swizzle: K reads (16 keys, one chunk) and transposed V reads (4 keys x 4 chunks) hit
  // distinct banks.  D 128: one row = all 64 banks, 16 chunks; D 64: two rows per bank window
  __device__ static __forceinline__ int swz(int kr) {
    if constexpr (D == 128) return ((kr & 3) << 2) | ((kr >> 2) & 3);
    else { const int v = (kr >> 1) & 7; return ((v & 1) << 2) | (v >> 1); }
  }
};

template <bool HF>
__device__ __forceinline__ v16f mfma_32(const v8s& a, const v8s& b, const v16f& c) {
  if constexpr (HF)
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(v8h, a), __builtin_bit_cast(v8h, b), c, 0, 0, 0);
  else return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// STG (stagger): waves 4-7 (the partners of waves 0-3 on the same SIMDs) defer each tile's O^T += V^T
// P^T to the next tile's interval, so on every SIMD one wave's softmax VALU runs beside the other's
// MFMAs instead of both waves hitting the same phase after each barrier (MI355X microarch item 9).
// The deferred V tile stays readable one barrier longer, so the ring grows to 4 slots.
template <int D, bool CAUSAL, bool STG, bool HF>
__global__ void __launch_bounds__(FA_NT, 1) fa_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc, int64_t c_sb,
    int64_t c_sh, const int* __restrict__ start_pos, bf16_t* __restrict__ out, int T, int Hq, int Hkv,
    float scale_log2, int order, int prio, float thr) {
  using G = FaGeo<D>;
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  // one-dimensional grid, longest (causal) query tile first over ALL heads and batch rows: the CUs
  // that finish short tiles pick up the remaining long ones, so no long tile starts near the end
  // (per-head longest-first left the last heads' longest tiles as a tail: ~11 % of the attention
  // time of a 32K prompt in 4K chunks, 29 % at an 8K causal prompt, by a dispatch model).  Within a
  // tile index the heads of one KV group go to one XCD (workgroups b and b + 8 share an XCD), so
  // they read that group's K / V through the same L2.  order 0: the per-head form (A/B).
  const int nqt = (T + FA_QT - 1) / FA_QT, nhb = (int)gridDim.x / nqt;   // grid = nqt x Hq x B
  int qtile, h, b;
  if (order == 0) {
    qtile = nqt - 1 - (int)blockIdx.x % nqt;
    h = (int)blockIdx.x / nqt % Hq;
    b = (int)blockIdx.x / nqt / Hq;
  } else {
    const int r = (int)blockIdx.x % nhb;
    qtile = nqt - 1 - (int)blockIdx.x / nhb;
    b = r / Hq;
    const int hr = r % Hq;
    h = (Hq & 7) == 0 ? (hr & 7) * (Hq >> 3) + (hr >> 3) : hr;
  }
  const int kvh = h / (Hq / Hkv);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ql = lane & 31, hf = lane >> 5;                    // query column / half of the wave
  const int s0 = start_pos[b];
  const int nkeys = s0 + T;
  const int q0 = qtile * FA_QT;
  const int wq0 = q0 + wave * 32;
  const int tq = wq0 + ql;                                     // this lane's query row (within T)
  const int qpos = s0 + tq;
  const int last_q = min(q0 + FA_QT, T) - 1;
  const int kend = CAUSAL ? min(nkeys, s0 + last_q + 1) : nkeys;
  const int ntiles = (kend + FA_KT - 1) / FA_KT;
  const bf16_t* kbase = kc + b * c_sb + kvh * c_sh;
  const bf16_t* vbase = vc + b * c_sb + kvh * c_sh;

  // ---- Q^T fragments (B operand): lane <- Q[tq][16 kk + 8 hf .. +8]
  v8s qf[G::KK];
#pragma unroll
  for (int kk = 0; kk < G::KK; ++kk)
    qf[kk] = tq < T ? *reinterpret_cast<const v8s*>(q + (((size_t)b * T + tq) * Hq + h) * D + kk * 16 + hf * 8)
                    : v8s{0, 0, 0, 0, 0, 0, 0, 0};

  // ---- LDS-DMA of tile t into ring slot t % RING: 1 KiB pieces of RPP key rows, PPW per wave
  constexpr int RING = STG ? FA_RING + 1 : FA_RING;
  auto issue = [&](int t) {
    char* slot = smem + (t % RING) * G::SLOT;
#pragma unroll
    for (int j = 0; j < G::PPW; ++j) {
      const int p = wave * G::PPW + j;                         // [0, PIECES) K, then V
      const bool isv = p >= G::PIECES;
      const int pp = isv ? p - G::PIECES : p;
      const int kr = pp * G::RPP + lane / G::CH;               // tile-relative key row
      const int key = min(t * FA_KT + kr, kend - 1);
      const int ch = (lane % G::CH) ^ G::swz(kr);              // source chunk for this LDS slot
      // wave-uniform base (K or V rows: the piece index is the wave's) + a 32-bit lane offset: the
      // SADDR form of the DMA, no 64-bit lane arithmetic per piece (23 vs 29 vector instructions
      // per tile; +0.1-0.8 %, profiles/fa_saddr_ab_r5.json)
      const uint64_t bp = reinterpret_cast<uint64_t>(isv ? vbase : kbase);
      const char* base = reinterpret_cast<const char*>(
          ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(bp >> 32)) << 32) |
          (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)bp));
      glds16_fa(base + (uint32_t)(key * G::ROWB + ch * 16), slot + (isv ? G::TILE : 0) + pp * 1024);
    }
  };

  v16f o[G::DB];
#pragma unroll
  for (int i = 0; i < G::DB; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[i][r] = 0.f;
  float m_i = -INFINITY, l_i = 0.f;

  // O rescale (only when some query's running max moved: alpha != 1; multiplying by exactly 1 is the
  // identity, so the skip is bit-exact and past the first tiles a new maximum is rare), then
  // O^T += V^T P^T: per 16-key step, lane group g reads keys {4 hf .. +3} and {8 + 4 hf .. +3}
  auto pv = [&](const char* vl, const v8s (&pb)[2][2], float alpha) {
    if (__any(alpha != 1.f)) {
#pragma unroll
      for (int i = 0; i < G::DB; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[i][r] *= alpha;
    }
    const int c16 = lane & 15, qq = c16 >> 2, pq = c16 & 3, g2 = (lane >> 4) & 1;
    const uint32_t vb = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) const char*)vl);
    // the swizzle of key row 32 kb + 16 ks + r is r's (it repeats every 16 rows): per lane one
    // address per (d-block, key quad), the step's rows as the instruction's immediate offset
    uint32_t va[G::DB][2];
#pragma unroll
    for (int db = 0; db < G::DB; ++db)
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const int kr = 4 * hf + qq + 8 * h2, d0 = db * 32 + g2 * 16 + 4 * pq;
        va[db][h2] = vb + kr * G::ROWB + (((d0 >> 3) ^ G::swz(kr)) << 4) + (d0 & 7) * 2;
      }
    auto step = [&](auto kbc, auto ksc) {
      constexpr int kb = decltype(kbc)::value, ks = decltype(ksc)::value, OFF = (kb * 32 + ks * 16) * G::ROWB;
      v4s lo[G::DB], hi[G::DB];
#pragma unroll
      for (int db = 0; db < G::DB; ++db) {
        lo[db] = ds_tr16<OFF>(va[db][0]);
        hi[db] = ds_tr16<OFF>(va[db][1]);
      }
      wait_tr<G::DB>(lo, hi);
#pragma unroll
      for (int db = 0; db < G::DB; ++db) {
        const v8s vf = v8s{lo[db][0], lo[db][1], lo[db][2], lo[db][3], hi[db][0], hi[db][1], hi[db][2], hi[db][3]};
        o[db] = mfma_32<HF>(vf, pb[kb][ks], o[db]);
      }
    };
    step(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{});
    step(std::integral_constant<int, 0>{}, std::integral_constant<int, 1>{});
    step(std::integral_constant<int, 1>{}, std::integral_constant<int, 0>{});
    step(std::integral_constant<int, 1>{}, std::integral_constant<int, 1>{});
  };
  const bool late = STG && wave >= FA_W / 2;                   // wave-uniform
  bool pend = false;
  // the staggered half's pending P lives in one of two named register sets that swap roles every
  // tile (the loop body runs twice per iteration) instead of being copied each tile: ~30 fewer
  // register moves per tile, +0.7-2 % (profiles/fa_pingpong_p_ab_r5.json)
  v8s pbA[2][2], pbB[2][2];
  float alpha_p = 1.f;
  const char* vl_p = smem;

  // static priority for the younger wave half (waves 4-7 lose VALU arbitration to their SIMD
  // partners otherwise; the guard must be provably wave-uniform for s_setprio): A/B knob, 5 % slower
  // with the staggered schedule (profiles/fa_softmax_knobs_ab_r5.json)
  if (prio && __builtin_amdgcn_readfirstlane(threadIdx.x) >= FA_NT / 2) __builtin_amdgcn_s_setprio(1);
  if (ntiles > 0) issue(0);
  if (ntiles > 1) issue(1);
  // one key tile; pb receives this tile's P, pq holds the previous tile's (the staggered half's
  // deferred P.V)
  auto tile = [&](int t, v8s (&pb)[2][2], v8s (&pq)[2][2]) {
    if (t + 1 < ntiles) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::PPW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();                              // tile t landed; slot of t - 1 free
    if (t + 2 < ntiles) issue(t + 2);
    if constexpr (STG) {
      if (late && pend) {                                      // the previous tile's O^T += V^T P^T
        pv(vl_p, pq, alpha_p);
        pend = false;
      }
    }
    const int k0 = t * FA_KT;
    if (wq0 >= T || (CAUSAL && k0 > s0 + wq0 + 31)) return;    // nothing visible for this wave
    const char* kl = smem + (t % RING) * G::SLOT;
    const char* vl = kl + G::TILE;

    // ---- S^T = K Q^T for the two 32-key blocks
    v16f sacc[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
      for (int r = 0; r < 16; ++r) sacc[kb][r] = 0.f;
      const int kr = kb * 32 + ql;
#pragma unroll
      for (int kk = 0; kk < G::KK; ++kk) {
        const v8s kf = *reinterpret_cast<const v8s*>(kl + kr * G::ROWB + (((2 * kk + hf) ^ G::swz(kr)) << 4));
        sacc[kb] = mfma_32<HF>(kf, qf[kk], sacc[kb]);
      }
      asm volatile("" ::: "memory");                           // K fragments: one 32-key block in flight
    }
    // ---- mask, online softmax (one query per lane).  The max runs over the raw scores (the scale
    // is positive), and the scale folds into each exponent's fma: exp2(s * scale - m)
    const bool full = (k0 + FA_KT <= kend) && (!CAUSAL || k0 + FA_KT - 1 <= s0 + wq0);
    float mx = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float v = sacc[kb][r];
        if (!full) {
          const int key = k0 + kb * 32 + 8 * (r >> 2) + 4 * hf + (r & 3);
          if (key >= kend || (CAUSAL && key > qpos)) v = -INFINITY;
        }
        sacc[kb][r] = v;
        mx = fmaxf(mx, v);
      }
    mx = half_max(mx);
    // the running max moves only when some query of the wave exceeds it by more than thr (log2
    // units): below that the probabilities stay <= 2^thr against the old max and the O rescale is
    // skipped.  thr = 0 (the default) is the exact online softmax: a rescale whenever a max moved
    const float cand = mx * scale_log2;
    const float mnew = __all(cand <= m_i + thr) ? m_i : fmaxf(m_i, cand);
    const float msafe = mnew == -INFINITY ? 0.f : mnew;
    // v_exp_f32 directly: exp2f adds a denormal-range fix-up (compare, select, add, multiply) to
    // every exponential; arguments here are <= 0 and a probability below 2^-126 may flush to 0
    const float alpha = __builtin_amdgcn_exp2f(m_i - msafe);
    float rs = 0.f;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[kb][8 * ks + j], scale_log2, -msafe));
          rs += pv;
          pb[kb][ks][j] = (short)f2e<HF>(pv);
        }
    rs = half_sum(rs);
    l_i = l_i * alpha + rs;
    m_i = mnew;
    if constexpr (STG) {
      if (late) {                                              // O^T update deferred one tile
        alpha_p = alpha;
        vl_p = vl;
        pend = true;
        return;
      }
    }
    pv(vl, pb, alpha);
  };
  int t = 0;
  for (; t + 1 < ntiles; t += 2) {
    tile(t, pbA, pbB);
    tile(t + 1, pbB, pbA);
  }
  if (t < ntiles) tile(t, pbA, pbB);
  if constexpr (STG) {                                         // no DMA after the last tile: slot intact
    if (late && pend) {                                        // the last tile's P: pbA if ntiles is odd
      if (ntiles & 1) pv(vl_p, pbA, alpha_p);
      else pv(vl_p, pbB, alpha_p);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");             // no DMA outlives the workgroup

  // ---- epilogue: lane holds O^T[d = 32 db + 8 j + 4 hf + 0..3][tq]
  if (tq < T) {
    const float inv = l_i > 0.f ? 1.f / l_i : 0.f;
    bf16_t* orow = out + (((size_t)b * T + tq) * Hq + h) * D;
#pragma unroll
    for (int db = 0; db < G::DB; ++db)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        uint2 w;
        w.x = pack_e2<HF>(o[db][4 * j] * inv, o[db][4 * j + 1] * inv);
        w.y = pack_e2<HF>(o[db][4 * j + 2] * inv, o[db][4 * j + 3] * inv);
        *reinterpret_cast<uint2*>(orow + db * 32 + 8 * j + 4 * hf) = w;
      }
  }
}
}  // namespace

static int g_prefill_fa = 1;           // tune key "prefill_fa": 0 = the 16-row kernel only, 1 = auto, 2 = fa_kernel always
static int g_prefill_fa_stag = 1;      // tune key "prefill_fa", second value: 1 = staggered wave halves, 0 = lockstep (A/B)
static int g_prefill_fa_order = 1;     // tune key "prefill_fa_order": 1 = longest tiles first over all heads, 0 = per head (A/B)
static int g_prefill_fa_prio = 0;      // tune key "prefill_fa_sm": a = static s_setprio 1 for waves 4-7 (A/B)
static float g_prefill_fa_thr = 0.f;   // tune key "prefill_fa_sm": b = deferred-max threshold, log2 units (A/B)
extern "C" void edge_prefill_fa(int v, int stag) { g_prefill_fa = v; g_prefill_fa_stag = stag; }
extern "C" void edge_prefill_fa_order(int v) { g_prefill_fa_order = v; }
extern "C" void edge_prefill_fa_sm(int prio, int thr) { g_prefill_fa_prio = prio; g_prefill_fa_thr = (float)thr; }

namespace {
template <bool HF>
int run_prefill(const void* q, const void* k_cache, const void* v_cache, int64_t c_sb, int64_t c_sh,
                const int* start_pos, void* out, int B, int T, int Hq, int Hkv, int D, float sl2, int causal,
                hipStream_t st) {
#define ARGS (const bf16_t*)q, (const bf16_t*)k_cache, (const bf16_t*)v_cache, c_sb, c_sh, start_pos, (bf16_t*)out, T, \
             Hq, Hkv, sl2
  // fa_kernel takes 256 queries per workgroup: below ~128 workgroups (short prompts, few heads) the
  // 64-row kernel keeps more CUs busy (tools/bench_ops.py --only prefill, D 128: T 512 x 32 heads
  // 23.4 vs 27.6 us, T 1024 54.8 vs 50.2, T 2048 198 vs 98, 4K chunk over 28K cached keys 6.09 vs
  // 2.78 ms)
  const bool fa_fills = (int64_t)((T + FA_QT - 1) / FA_QT) * Hq * B >= 128;
  if ((D == 128 || D == 64) && (g_prefill_fa == 2 || (g_prefill_fa == 1 && fa_fills))) {
#define FA(DD)                                                                                                     \
  do {                                                                                                             \
    static bool fa_attr = false;                                                                                   \
    if (!fa_attr) {                                                                                                \
      (void)hipFuncSetAttribute((const void*)fa_kernel<DD, true, false, HF>,                                       \
                                hipFuncAttributeMaxDynamicSharedMemorySize, FaGeo<DD>::LDS);                       \
      (void)hipFuncSetAttribute((const void*)fa_kernel<DD, false, false, HF>,                                      \
                                hipFuncAttributeMaxDynamicSharedMemorySize, FaGeo<DD>::LDS);                       \
      (void)hipFuncSetAttribute((const void*)fa_kernel<DD, true, true, HF>,                                        \
                                hipFuncAttributeMaxDynamicSharedMemorySize, FaGeo<DD>::LDS_STG);                   \
      (void)hipFuncSetAttribute((const void*)fa_kernel<DD, false, true, HF>,                                       \
                                hipFuncAttributeMaxDynamicSharedMemorySize, FaGeo<DD>::LDS_STG);                   \
      fa_attr = true;                                                                                              \
    }                                                                                                              \
    const dim3 g((T + FA_QT - 1) / FA_QT * Hq * B);                                                                   \
    if (g_prefill_fa_stag) {                                                                                       \
      if (causal) hipLaunchKernelGGL((fa_kernel<DD, true, true, HF>), g, dim3(FA_NT), FaGeo<DD>::LDS_STG, st, ARGS, g_prefill_fa_order, g_prefill_fa_prio, g_prefill_fa_thr); \
      else hipLaunchKernelGGL((fa_kernel<DD, false, true, HF>), g, dim3(FA_NT), FaGeo<DD>::LDS_STG, st, ARGS, g_prefill_fa_order, g_prefill_fa_prio, g_prefill_fa_thr);     \
      break;                                                                                                       \
    }                                                                                                              \
    if (causal) hipLaunchKernelGGL((fa_kernel<DD, true, false, HF>), g, dim3(FA_NT), FaGeo<DD>::LDS, st, ARGS, g_prefill_fa_order, g_prefill_fa_prio, g_prefill_fa_thr);    \
    else hipLaunchKernelGGL((fa_kernel<DD, false, false, HF>), g, dim3(FA_NT), FaGeo<DD>::LDS, st, ARGS, g_prefill_fa_order, g_prefill_fa_prio, g_prefill_fa_thr);          \
  } while (0)
    if (D == 128) FA(128);
    else FA(64);
#undef FA
    return (int)hipGetLastError();
  }
  const dim3 grid((T + QT - 1) / QT, Hq, B);
#define PL(DD)                                                                                                    \
  do {                                                                                                            \
    static bool attr_set = false; /* >64 KiB dynamic LDS (D=256): raise the per-kernel cap once */                \
    if (!attr_set && Geo<DD>::LDS > 65536) {                                                                      \
      (void)hipFuncSetAttribute((const void*)prefill_attn_kernel<DD, true, HF>,                                    \
                                hipFuncAttributeMaxDynamicSharedMemorySize, Geo<DD>::LDS);                         \
      (void)hipFuncSetAttribute((const void*)prefill_attn_kernel<DD, false, HF>,                                   \
                                hipFuncAttributeMaxDynamicSharedMemorySize, Geo<DD>::LDS);                         \
    }                                                                                                             \
    attr_set = true;                                                                                              \
    if (causal) hipLaunchKernelGGL((prefill_attn_kernel<DD, true, HF>), grid, dim3(NT), Geo<DD>::LDS, st, ARGS);   \
    else hipLaunchKernelGGL((prefill_attn_kernel<DD, false, HF>), grid, dim3(NT), Geo<DD>::LDS, st, ARGS);         \
  } while (0)
  switch (D) {
    case 64: PL(64); break;
    case 80: PL(80); break;
    case 128: PL(128); break;
    case 256: PL(256); break;
    default: return -4;
  }
#undef PL
#undef ARGS
  return (int)hipGetLastError();
}
}  // namespace

// h16: q, caches and out are fp16 (fp16 MFMA), else bf16
extern "C" int edge_prefill_attn(const void* q, const void* k_cache, const void* v_cache, int64_t c_sb, int64_t c_sh,
                                 const int* start_pos, void* out, int B, int T, int Hq, int Hkv, int D, float scale,
                                 int causal, int h16, hipStream_t st) {
  if (B * T == 0) return 0;
  if (Hq % Hkv) return -2;
  const float sl2 = scale * 1.4426950408889634f;
  return h16 ? run_prefill<true>(q, k_cache, v_cache, c_sb, c_sh, start_pos, out, B, T, Hq, Hkv, D, sl2, causal, st)
             : run_prefill<false>(q, k_cache, v_cache, c_sb, c_sh, start_pos, out, B, T, Hq, Hkv, D, sl2, causal, st);
}

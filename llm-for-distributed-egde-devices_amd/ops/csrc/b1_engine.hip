// Batch-1 W8A8 decode of a whole Llama-family decoder stack in ONE persistent launch (SURVEY K11,
// the reference's own workload: single-stream generate, combine_model_fp_updated.py:86-110).
//
// Why: at batch 1 every projection is a weight stream (Llama-2-7B: 202 MB of int8 per layer), and
// the launch-per-op decode (qkv GEMV, fused attention, o, gate_up + SwiGLU, down: 57.6 us/layer)
// loses ~20 us/layer to kernel boundaries, ramps and tails.  A weight byte never depends on the
// activation, so here the weights stream continuously across ALL ops and layers of the step, and the
// dependency waits (the "seams": each projection needs the whole output of the one before) overlap
// the weight stream instead of stopping it (the CDNA guide's prefetch-credit engine).
//
// Work split (grid = one workgroup per CU, G of them; all resident by construction: > 80 KiB of LDS
// per workgroup).  Eight waves per workgroup:
//   * waves 0-3 stream.  Every projection's output columns are cut into 16-column units (gate_up:
//     8 features = their 8 gate + 8 up rows), units spread evenly over the G CUs; each streaming wave
//     owns a quarter of K.  A wave's weights for the whole step are ONE contiguous stream of 1 KiB
//     fragments (16 columns x 64 k; lane l <- W[col 4 (l >> 2)..][k 16 (l & 3)..+16]) in the order it
//     consumes them, laid out by the host (engine/b1_engine.py).  Fragments land by LDS-DMA in a
//     per-wave ring of D slots: the wave waits for fragment g (vmcnt(D - 1): the D - 1 later ones stay
//     in flight), reads it with its int8 activation chunk, refills the slot with fragment g + D, and
//     sums 4 v_dot4 per fragment (int32 per unit; grouped-scale inputs fold one fp32 scale each);
//   * waves 4-7 (the seam waves) do every global read of a seam: they issue no weight DMA, so their
//     loads do not retire behind ~100 KiB of a streaming wave's prefetch (vmcnt retires in order).
//     They gather the producers' values into LDS, with the norm weights and the epilogue scales, and
//     all eight waves then normalise / quantise from LDS;
//   * attention: head h on CU h (RoPE, KV append, scores, softmax, P.V over the bf16 cache), its
//     output quantised per (token, 64) like the fused decode-attention kernel.
// Seams: a producer stores its values as 8-byte granules {3 x bf16 or 6 bytes, 16-bit tag} with
// relaxed agent-scope atomic stores (no fence, no drain: the data is the flag); the seam wave re-reads
// its granules (relaxed agent-scope loads, bypassing stale L1 lines) until every tag is the current
// one (CDNA guide, Guideline 16 recipe R2).  Tags are unique per (launch, layer, kind): a device salt
// advanced by every launch, so granule buffers are never re-zeroed.  Every spin is bounded: on
// give-up the launch's abort word is raised, every waiter leaves, and ctl[2] holds the failing seam.
// Numerics follow the launch-per-op path: bf16 residual stream (HF), RMSNorm in fp32, per-token int8
// for qkv / gate_up inputs, per-(token, 64) int8 for o / down inputs, bf16 q / k / v / attention out /
// g / u / h.
#include <type_traits>

#include "common.h"
#include "b1_engine.h"

namespace {

constexpr int B1_NS = 256;                 // streaming threads (waves 0-3)
constexpr int B1_NT = 512;                 // + the seam waves (4-7)
constexpr int B1_MAXCU = 8;                // 16-column units per CU and projection
constexpr int B1_MAXG = 512;               // CUs (workgroups) a launch may have
constexpr int B1_GB = 8;                   // granules per seam-wave thread per sweep batch
constexpr unsigned B1_SPIN_LIMIT = 1u << 22;

// B1Params: b1_engine.h (shared with the host bindings)

__device__ __forceinline__ uint64_t g_ld(uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void g_st(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int c_ld(int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void c_st(int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t gran(uint64_t payload, uint32_t tag) {
  return (payload & 0xFFFFFFFFFFFFull) | ((uint64_t)tag << 48);
}

// LDS barrier: the wave's own LDS ops complete first (a bare s_barrier waits for no counter); the
// in-flight weight DMA (vmcnt) is left running
__device__ __forceinline__ void bar() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// first unit of CU c under the even split (c NU < 2^31: 32-bit division; the seams read the
// per-launch LDS tables of these instead of dividing)
__device__ __forceinline__ int u0_of(int c, int NU, int G) { return (int)(((unsigned)c * (unsigned)NU) / (unsigned)G); }
// CU owning unit u, from a table u0[0..G] of first units
__device__ __forceinline__ int owner_in(const int* u0, int u, int NU, int G) {
  int c = (int)(((unsigned)u * (unsigned)G) / (unsigned)NU);
  while (c + 1 < G && u0[c + 1] <= u) ++c;
  while (c > 0 && u0[c] > u) --c;
  return c;
}
// floor(i / d) for 0 <= i < 2^20 and small d, by one multiply: (i + 1/2) / d is at least 1 / (2 d) from
// an integer, far above the float rounding error
__device__ __forceinline__ int fdiv(int i, float inv_d) { return (int)(((float)i + 0.5f) * inv_d); }

__device__ __forceinline__ float bfr(float x) { return bf2f(f2bf(x)); }   // round to bf16

__device__ __forceinline__ float wave_max64(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

template <int D, int HD>
__global__ void __launch_bounds__(B1_NT, 1) b1_decode_kernel(B1Params p) {
  extern __shared__ __attribute__((aligned(1024))) int8_t smem[];
  const int G = (int)gridDim.x, c = (int)blockIdx.x;
  const int t = (int)threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const bool seamw = w >= 4;                          // a seam wave
  const int sidx = t - B1_NS;                          // its thread index among the seam waves
  const int L = p.L, H = p.H, Hq = p.Hq, Hkv = p.Hkv, F = p.F, NQ = p.NQ;
  constexpr int NGR = HD / 64;                       // 64-groups per head

  // ---- LDS carve (the host sizes it with edge_b1_lds_bytes)
  int8_t* const ring = smem;                          // [4][D] x 1 KiB
  int8_t* const xq = ring + 4 * D * 1024;             // int8 activations of the current projection
  float* const sx = reinterpret_cast<float*>(xq + p.xqb);       // per-64 activation scales
  int8_t* const scr = reinterpret_cast<int8_t*>(sx + p.sxn);    // seam staging / attention scratch
  int* const red = reinterpret_cast<int*>(scr + p.scb);         // [4][B1_MAXCU * 16] partial sums
  float* const misc = reinterpret_cast<float*>(red + 4 * B1_MAXCU * 16);   // [64]
  bf16_t* const ov = reinterpret_cast<bf16_t*>(misc + 64);       // [B1_MAXCU * 16] epilogue values
  int* const flag = reinterpret_cast<int*>(ov + B1_MAXCU * 16);  // [4]: [0] abort seen
  int* const tu0 = flag + 4;                                      // [3][B1_MAXG + 1] first units per CU
  float* const swl = reinterpret_cast<float*>(tu0 + 3 * (B1_MAXG + 1));   // [2][B1_MAXCU * 16] scales
  const int gs_off = (int)(reinterpret_cast<int8_t*>(swl + 2 * B1_MAXCU * 16) - smem);
  bf16_t* const gs = reinterpret_cast<bf16_t*>(smem + ((gs_off + 15) & ~15));   // [H] next norm's weights (16-B aligned)

  // ---- unit splits (units of 16 columns; gate_up: 8 features)
  const int NUq = NQ / 16, NUh = H / 16, NUf = F / 8;
  const int uq0 = u0_of(c, NUq, G), nuq = u0_of(c + 1, NUq, G) - uq0;
  const int uh0 = u0_of(c, NUh, G), nuh = u0_of(c + 1, NUh, G) - uh0;
  const int uf0 = u0_of(c, NUf, G), nuf = u0_of(c + 1, NUf, G) - uf0;
  const int kbq = H / 256, kbo = Hq * HD / 256, kbd = F / 256;    // k-blocks of 64 per wave
  int* const u0q = tu0;
  int* const u0h = tu0 + (B1_MAXG + 1);
  int* const u0f = tu0 + 2 * (B1_MAXG + 1);
  for (int i = t; i <= G; i += B1_NT) {
    u0q[i] = u0_of(i, NUq, G);
    u0h[i] = u0_of(i, NUh, G);
    u0f[i] = u0_of(i, NUf, G);
  }
  if (t == 0) flag[0] = 0;
  const float inv_gx = 1.f / (float)p.gpc_x, inv_gh = 1.f / (float)p.gpc_h;

  // ---- a streaming wave's weight stream and its ring
  const long long per_layer = (long long)(nuq + nuf) * kbq + (long long)nuh * (kbo + kbd);
  const long long T = per_layer * L;                  // fragments in each streaming wave's stream
  const int ws_w = seamw ? 0 : w;
  const int8_t* const wsb = p.ws + ((long long)(c * 4 + ws_w) * p.fmax) * 1024 + lane * 16;
  int8_t* const wring = ring + ws_w * D * 1024;
  const uint32_t ring_lds = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) void*)wring) + lane * 16;
  long long gcur = 0;                                 // next fragment to consume
  int slot = 0;                                       // gcur % D
  auto issue = [&](long long g, int s) {
    const long long gg = g < T ? g : (T > 0 ? T - 1 : 0);   // past the end: re-load the last (never read)
    __builtin_amdgcn_global_load_lds(wsb + gg * 1024, (__attribute__((address_space(3))) void*)(wring + s * 1024),
                                     16, 0, 2);       // nontemporal: read once per step
  };
  if (!seamw) {
#pragma unroll
    for (int s = 0; s < D; ++s) issue(s, s);
  }
  bar();

  const int salt = c_ld(p.ctl);
  auto tag_of = [&](int l, int kind) -> uint32_t {
    return 1u + (uint32_t)(((unsigned long long)(unsigned)salt * (unsigned)(5 * L + 2) + (unsigned)(l * 5 + kind)) % 65535ull);
  };
  int* const ctl = p.ctl;
  // profiling stamps (p.stamps): thread 0 records s_memrealtime (100 MHz) at phase boundaries
  long long* const stp = p.stamps != nullptr ? p.stamps + (long long)c * L * 24 : nullptr;
  auto stamp = [&](int l, int i) {
    if (stp != nullptr && t == 0) stp[l * 24 + i] = (long long)__builtin_amdgcn_s_memrealtime();
  };
  auto aborted = [&]() -> bool { return flag[0] != 0; };

  // ---- streaming GEMV (waves 0-3) over the current activation (xq [, sx]): nu units x kbw fragments
  // per wave, the wave's k-blocks [w kbw, (w + 1) kbw); unit partials to red[w][u * 16 + col]
  const uint32_t xq_lds = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) void*)xq) + (lane & 3) * 16;
  const uint32_t sx_lds = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) void*)sx);
  auto stream = [&](int nu, int kbw, bool grouped) {
    if (seamw) return;
    // every older vector-memory op of this wave retires first, so vmcnt(D - 1) below counts this
    // stream's DMAs only (a profiling stamp is a store).  The seam before lasted longer than the
    // prefetch's landing, so this costs nothing
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int kw0 = w * kbw;
    for (int u = 0; u < nu; ++u) {
      int acc = 0;
      float facc = 0.f;
      for (int kb = 0; kb < kbw; ++kb) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D - 1) : "memory");   // fragment gcur landed
        v4i wf, xf;
        float s;
        asm volatile(
            "ds_read_b128 %0, %3\n\t"
            "ds_read_b128 %1, %4\n\t"
            "ds_read_b32 %2, %5\n\t"
            "s_waitcnt lgkmcnt(0)"
            : "=v"(wf), "=v"(xf), "=v"(s)
            : "v"(ring_lds + slot * 1024), "v"(xq_lds + (kw0 + kb) * 64), "v"(sx_lds + (kw0 + kb) * 4)
            : "memory");
        issue(gcur + D, slot);                        // the slot is free: refill it D fragments ahead
        ++gcur;
        slot = slot + 1 == D ? 0 : slot + 1;
        if (grouped) {
          int d = __builtin_amdgcn_sdot4(wf[0], xf[0], 0, false);
          d = __builtin_amdgcn_sdot4(wf[1], xf[1], d, false);
          d = __builtin_amdgcn_sdot4(wf[2], xf[2], d, false);
          d = __builtin_amdgcn_sdot4(wf[3], xf[3], d, false);
          facc = fmaf((float)d, s, facc);
        } else {
          acc = __builtin_amdgcn_sdot4(wf[0], xf[0], acc, false);
          acc = __builtin_amdgcn_sdot4(wf[1], xf[1], acc, false);
          acc = __builtin_amdgcn_sdot4(wf[2], xf[2], acc, false);
          acc = __builtin_amdgcn_sdot4(wf[3], xf[3], acc, false);
        }
      }
      int v;
      if (grouped) {
        float f = facc;
        f += __shfl_xor(f, 1, 64);
        f += __shfl_xor(f, 2, 64);
        v = __float_as_int(f);
      } else {
        v = acc + __shfl_xor(acc, 1, 64);
        v += __shfl_xor(v, 2, 64);
      }
      if ((lane & 3) == 0) red[w * (B1_MAXCU * 16) + u * 16 + (lane >> 2)] = v;
    }
  };

  // ---- publish n values from ov[] as granules of 3 (bf16), block `blk` (the seam waves store: no
  // vector-memory op joins a streaming wave's DMA count)
  auto publish3 = [&](uint64_t* blk, int n, uint32_t tag) {
    const int ng = (n + 2) / 3;
    if (seamw && sidx < ng) {
      const int i = 3 * sidx;
      uint64_t pl = (uint64_t)ov[i];
      if (i + 1 < n) pl |= (uint64_t)ov[i + 1] << 16;
      if (i + 2 < n) pl |= (uint64_t)ov[i + 2] << 32;
      g_st(blk + sidx, gran(pl, tag));
    }
  };

  // ---- the seam waves' gather: granule slots i = sidx + 256 k (batches of B1_GB per thread, all loads
  // of a batch in flight at once); idx(i) -> the granule's offset from `base`, or -1 (nothing to wait
  // for); every pass re-reads the still-stale ones, then sleeps; consume(i, granule) once the whole
  // batch carries `tag`.  Returns false on give-up.
  auto gather = [&](uint64_t* base, int nslots, uint32_t tag, int code, auto&& idx, auto&& consume) -> bool {
    for (int b0 = 0; b0 < nslots; b0 += B1_NS * B1_GB) {
      uint64_t gv[B1_GB];
      int ix[B1_GB];
      unsigned pend = 0;
#pragma unroll
      for (int k = 0; k < B1_GB; ++k) {
        const int i = b0 + sidx + B1_NS * k;
        ix[k] = i < nslots ? idx(i) : -1;
        if (ix[k] >= 0) {
          gv[k] = g_ld(base + ix[k]);
          pend |= 1u << k;
        }
      }
      for (unsigned it = 0;; ++it) {
#pragma unroll
        for (int k = 0; k < B1_GB; ++k)
          if (((pend >> k) & 1u) && (uint32_t)(gv[k] >> 48) == tag) pend &= ~(1u << k);
        if (!__any(pend != 0)) break;
        if ((it & 15) == 15) {
          if (c_ld(ctl + 1)) return false;
          if (it >= B1_SPIN_LIMIT) {
            c_st(ctl + 2, code);
            c_st(ctl + 1, 1);
            return false;
          }
        }
        __builtin_amdgcn_s_sleep(1);
#pragma unroll
        for (int k = 0; k < B1_GB; ++k)
          if ((pend >> k) & 1u) gv[k] = g_ld(base + ix[k]);
      }
#pragma unroll
      for (int k = 0; k < B1_GB; ++k)
        if (ix[k] >= 0) consume(b0 + sidx + B1_NS * k, gv[k]);
    }
    return true;
  };

  // ---- RMSNorm + per-token int8 of a residual-stream vector into xq (returns the token scale).
  // The seam wave stages the vector (bf16, from granules: G blocks of gpc_x, block c' holding the
  // 16 nuh(c') values of its units; layer 0: the dense embedding x0) and the norm weights in LDS.
  bf16_t* const xs = reinterpret_cast<bf16_t*>(scr);          // [H]
  float* const rsum = misc + 8;                                // [8] sums, [8] maxima
  // the seam waves stage the next norm's weights during a seam, never while the streaming waves
  // stream: staging beside the streams produced wrong fragments on random CUs in the measurements
  // (cause not isolated; docs/BENCHMARKS.md, Round 6)
  auto stage_gamma = [&](const bf16_t* gam) {
    if (seamw)
      for (int v = sidx * 8; v < H; v += 8 * B1_NS) *reinterpret_cast<uint4*>(gs + v) = *reinterpret_cast<const uint4*>(gam + v);
  };
  auto norm_seam = [&](uint64_t* gblk, uint32_t tag, int code) -> float {
    float ss = 0.f, am = 0.f;
    if (seamw) {
      bool ok = true;
      if (gblk == nullptr) {
        for (int v = sidx; v < H; v += B1_NS) {
          const float x = bf2f(p.x0[v]);
          xs[v] = p.x0[v];
          ss = fmaf(x, x, ss);
          am = fmaxf(am, fabsf(x * bf2f(gs[v])));
        }
      } else {
        ok = gather(gblk, G * p.gpc_x, tag, code,
                    [&](int i) -> int {
                      const int cb = fdiv(i, inv_gx), j = i - cb * p.gpc_x;
                      return 3 * j < 16 * (u0h[cb + 1] - u0h[cb]) ? i : -1;
                    },
                    [&](int i, uint64_t v) {
                      const int cb = fdiv(i, inv_gx), j = i - cb * p.gpc_x;
                      const int base = 16 * u0h[cb], nv = 16 * u0h[cb + 1] - base;
                      for (int e = 0; e < 3 && 3 * j + e < nv; ++e) {
                        const int vi = base + 3 * j + e;
                        const float x = bf2f((uint32_t)(v >> (16 * e)) & 0xffffu);
                        xs[vi] = (bf16_t)(v >> (16 * e));
                        ss = fmaf(x, x, ss);
                        am = fmaxf(am, fabsf(x * bf2f(gs[vi])));
                      }
                    });
      }
      if (!ok && lane == 0) flag[0] = 1;
      ss = wave_sum(ss);
      am = wave_max64(am);
      if (lane == 0) { rsum[w - 4] = ss; rsum[8 + w - 4] = am; }
    }
    bar();
    float S = 0.f, A = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) { S += rsum[i]; A = fmaxf(A, rsum[8 + i]); }
    const float r = rsqrtf(S / (float)H + p.eps);
    const float sa = fmaxf(A * r, 1e-8f) / 127.f;
    const float inv = r / sa;
    for (int v = t; v < H; v += B1_NT) xq[v] = quant_i8(bf2f(xs[v]) * bf2f(gs[v]), inv);
    bar();
    return sa;
  };
  // the seam wave stages n epilogue scales src[0..n) (and src2[0..n) when given) into swl
  auto stage_scales = [&](const float* src, const float* src2, int n) {
    if (seamw) {
      for (int i = sidx; i < n; i += B1_NS) {
        swl[i] = src[i];
        if (src2 != nullptr) swl[B1_MAXCU * 16 + i] = src2[i];
      }
    }
  };

  // ---- own residual columns (o / down units), kept in registers of the epilogue threads
  float xres = 0.f, h2res = 0.f;
  if (t < 16 * nuh) xres = bf2f(p.x0[16 * uh0 + t]);

  stage_gamma(p.gam1);
  bar();
  for (int l = 0; l < L; ++l) {
    // ================= qkv
    stamp(l, 0);
    stage_scales(p.sw_q + (long long)l * NQ + 16 * uq0, nullptr, 16 * nuq);
    const float sa_q = norm_seam(l == 0 ? nullptr : p.gx + (long long)l * G * p.gpc_x, tag_of(l, 0), 1);
    if (aborted()) break;
    stamp(l, 1);
    stream(nuq, kbq, false);
    stamp(l, 2);
    bar();
    if (t < 16 * nuq) {
      int tot = 0;
#pragma unroll
      for (int ww = 0; ww < 4; ++ww) tot += red[ww * (B1_MAXCU * 16) + t];
      ov[t] = f2bf((float)tot * sa_q * swl[t]);
    }
    bar();
    publish3(p.gq + ((long long)l * G + c) * p.gpc_q, 16 * nuq, tag_of(l, 1));
    stamp(l, 3);

    // ================= attention: head c on CU c
    if (c < Hq) {
      float* const qs = reinterpret_cast<float*>(scr);        // [3 HD] q, k, v as read
      float* const qr = qs + 3 * HD;                           // [HD] rotated q (bf16-rounded)
      float* const kr = qr + HD;                               // [HD] rotated k (bf16-rounded)
      float* const ored = kr + HD;                             // [4][HD]
      float* const sc = ored + 4 * HD;                         // [ctx] scores, then probabilities
      const int grp = Hq / Hkv, g = c / grp;
      const int pos = *p.pos;
      const int ctx = pos + 1;
      const uint32_t tq = tag_of(l, 1);
      bf16_t* const kl = p.kc + (long long)l * p.kv_l + (long long)g * p.kv_h;
      bf16_t* const vl = p.vc + (long long)l * p.kv_l + (long long)g * p.kv_h;
      const int jmax = pos > 0 ? pos - 1 : 0;                  // last cached key (loads clamp to it)
      // scores: 16 lanes per key (DPL dims each), 4 keys per wave, SB steps; P.V: LPK lanes per key
      // (4 dims each), KPW keys per wave, PB steps.  The cached rows do not depend on this step: the
      // streaming waves load their first batches while the seam wave gathers q / k / v.
      constexpr int DPL = HD / 16, SB = 8, KB = 16 * SB;
      constexpr int LPK = HD / 4, KPW = 64 / LPK, PB = HD == 128 ? 8 : 16, VB = 4 * KPW * PB;
      using KT = typename std::conditional<DPL == 8, uint4, uint2>::type;
      const int lg = lane >> 4, li = lane & 15;
      const int kh = lane / LPK, dl = (lane % LPK) * 4;
      const int aw = w & 3;                                    // a seam wave's index among the four
      KT kk[SB];
      uint2 vv[PB];
      auto load_k = [&](int j0) {
#pragma unroll
        for (int r = 0; r < SB; ++r) {
          const int j = min(j0 + r * 16 + aw * 4 + lg, jmax);
          kk[r] = *reinterpret_cast<const KT*>(kl + (long long)j * HD + li * DPL);
        }
      };
      auto load_v = [&](int j0) {
#pragma unroll
        for (int r = 0; r < PB; ++r) {
          const int j = min(j0 + r * 4 * KPW + aw * KPW + kh, jmax);
          vv[r] = *reinterpret_cast<const uint2*>(vl + (long long)j * HD + dl);
        }
      };
      if (seamw) {
        load_k(0);                                             // in flight during the q / k / v gather
        load_v(0);
        const bool ok = gather(p.gq + (long long)l * G * p.gpc_q, 3 * HD, tq, 2,
            [&](int i) -> int {
              const int vi = i < HD ? c * HD + i : (i < 2 * HD ? (Hq + g) * HD + i - HD : (Hq + Hkv + g) * HD + i - 2 * HD);
              const int cb = owner_in(u0q, vi >> 4, NUq, G);
              return cb * p.gpc_q + (vi - 16 * u0q[cb]) / 3;
            },
            [&](int i, uint64_t v) {
              const int vi = i < HD ? c * HD + i : (i < 2 * HD ? (Hq + g) * HD + i - HD : (Hq + Hkv + g) * HD + i - 2 * HD);
              const int cb = owner_in(u0q, vi >> 4, NUq, G);
              qs[i] = bf2f((uint32_t)(v >> (16 * ((vi - 16 * u0q[cb]) % 3))) & 0xffffu);
            });
        if (!ok && lane == 0) flag[0] = 1;
      }
      stamp(l, 14);
      bar();
      if (aborted()) break;
      if (t < HD / 2) {
        const float* cs = p.rope + ((long long)pos * (HD / 2) + t) * 2;
        const float co = cs[0], sn = cs[1];
        const float q1 = qs[t], q2 = qs[t + HD / 2], k1 = qs[HD + t], k2 = qs[HD + t + HD / 2];
        qr[t] = bfr(q1 * co - q2 * sn);                        // bf16 q, as the rotated qkv tensor
        qr[t + HD / 2] = bfr(q2 * co + q1 * sn);
        kr[t] = bfr(k1 * co - k2 * sn);
        kr[t + HD / 2] = bfr(k2 * co + k1 * sn);
      }
      bar();
      if (c % grp == 0 && seamw && sidx < 64) {                // the group's first head appends k / v
        for (int d = sidx; d < HD; d += 64) {
          kl[(long long)pos * HD + d] = f2bf(kr[d]);
          vl[(long long)pos * HD + d] = f2bf(qs[2 * HD + d]);
        }
      }
      if (seamw) {
        float qv[DPL];
#pragma unroll
        for (int d = 0; d < DPL; ++d) qv[d] = qr[li * DPL + d];
        for (int j0 = 0; j0 < ctx; j0 += KB) {
          if (j0 > 0) load_k(j0);
#pragma unroll
          for (int r = 0; r < SB; ++r) {
            const int j = j0 + r * 16 + aw * 4 + lg;
            float sv = 0.f;
            if constexpr (DPL == 8) {
              float kf[8];
              unpack8(reinterpret_cast<const uint4&>(kk[r]), kf);
#pragma unroll
              for (int e = 0; e < 8; ++e) sv = fmaf(qv[e], kf[e], sv);
            } else {
              const uint2 k2 = reinterpret_cast<const uint2&>(kk[r]);
              sv = qv[0] * bf2f(k2.x & 0xffffu) + qv[1] * bf2f(k2.x >> 16) + qv[2] * bf2f(k2.y & 0xffffu) +
                   qv[3] * bf2f(k2.y >> 16);
            }
            if (j == pos) {                                    // the new key, from LDS
              sv = 0.f;
#pragma unroll
              for (int d = 0; d < DPL; ++d) sv = fmaf(qv[d], kr[li * DPL + d], sv);
            }
            sv += __shfl_xor(sv, 8, 64);
            sv += __shfl_xor(sv, 4, 64);
            sv += __shfl_xor(sv, 2, 64);
            sv += __shfl_xor(sv, 1, 64);
            if (li == 0 && j < ctx) sc[j] = sv * p.scale;
          }
        }
      }
      bar();
      stamp(l, 15);
      float m = -INFINITY;
      for (int j = t; j < ctx; j += B1_NT) m = fmaxf(m, sc[j]);
      m = wave_max64(m);
      if (lane == 0) rsum[w] = m;
      bar();
      m = rsum[0];
#pragma unroll
      for (int i = 1; i < 8; ++i) m = fmaxf(m, rsum[i]);
      float ls = 0.f;
      for (int j = t; j < ctx; j += B1_NT) {
        const float e = __expf(sc[j] - m);
        sc[j] = e;
        ls += e;
      }
      ls = wave_sum(ls);
      if (lane == 0) rsum[8 + w] = ls;
      bar();
      float lsum = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) lsum += rsum[8 + i];
      stamp(l, 16);
      if (seamw) {
        float o4[4] = {0.f, 0.f, 0.f, 0.f};
        for (int j0 = 0; j0 < ctx; j0 += VB) {
          if (j0 > 0) load_v(j0);
#pragma unroll
          for (int r = 0; r < PB; ++r) {
            const int j = j0 + r * 4 * KPW + aw * KPW + kh;
            if (j < pos) {
              const float pj = sc[j];
              o4[0] = fmaf(pj, bf2f(vv[r].x & 0xffffu), o4[0]);
              o4[1] = fmaf(pj, bf2f(vv[r].x >> 16), o4[1]);
              o4[2] = fmaf(pj, bf2f(vv[r].y & 0xffffu), o4[2]);
              o4[3] = fmaf(pj, bf2f(vv[r].y >> 16), o4[3]);
            } else if (j == pos) {
              const float pj = sc[j];
#pragma unroll
              for (int d = 0; d < 4; ++d) o4[d] = fmaf(pj, qs[2 * HD + dl + d], o4[d]);
            }
          }
        }
#pragma unroll
        for (int d = 0; d < 4; ++d) {
#pragma unroll
          for (int o = LPK; o < 64; o <<= 1) o4[d] += __shfl_xor(o4[d], o, 64);
        }
        if (kh == 0) {
#pragma unroll
          for (int d = 0; d < 4; ++d) ored[aw * HD + dl + d] = o4[d];
        }
      }
      bar();
      stamp(l, 17);
      // quantise per 64 dims: wave gi < NGR takes group gi; its record (64 int8 + fp32 scale) goes
      // out as 12 granules: 10 x 6 bytes, 4 bytes, the scale
      if (seamw && aw < NGR) {
        const int dd = aw * 64 + lane;
        const float o_ = bfr((ored[dd] + ored[HD + dd] + ored[2 * HD + dd] + ored[3 * HD + dd]) / lsum);   // bf16 out
        const float amx = wave_max64(fabsf(o_));
        const float s = fmaxf(amx, 1e-8f) / 127.f;
        int8_t* const rec = reinterpret_cast<int8_t*>(sc + ctx + 64) + aw * 80;
        rec[lane] = quant_i8(o_, 1.f / s);
        if (lane == 0) *reinterpret_cast<float*>(rec + 64) = s;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane < 12) {
          uint64_t pl = 0;
          if (lane < 10) {
#pragma unroll
            for (int b = 0; b < 6; ++b) pl |= (uint64_t)(uint8_t)rec[6 * lane + b] << (8 * b);
          } else if (lane == 10) {
#pragma unroll
            for (int b = 0; b < 4; ++b) pl |= (uint64_t)(uint8_t)rec[60 + b] << (8 * b);
          } else {
            pl = (uint64_t)__float_as_uint(*reinterpret_cast<const float*>(rec + 64));
          }
          g_st(p.ga + (((long long)l * Hq + c) * NGR + aw) * 12 + lane, gran(pl, tag_of(l, 2)));
        }
      }
    }
    stamp(l, 4);

    // ================= o projection (grouped-scale input from the attention granules)
    stage_scales(p.sw_o + (long long)l * H + 16 * uh0, nullptr, 16 * nuh);
    stage_gamma(p.gam2 + (long long)l * H);                    // for the gate_up norm, in this seam
    if (seamw) {
      const int n = Hq * NGR * 12;
      uint64_t* const gb = p.ga + (long long)l * n;
      const bool ok = gather(gb, n, tag_of(l, 2), 3, [&](int i) -> int { return i; },
                             [&](int i, uint64_t v) {
                               const int grp64 = i / 12, j = i - grp64 * 12;
                               if (j < 11) {
                                 const int nb = j < 10 ? 6 : 4;
                                 for (int b = 0; b < nb; ++b) xq[grp64 * 64 + 6 * j + b] = (int8_t)(uint8_t)(v >> (8 * b));
                               } else {
                                 sx[grp64] = __uint_as_float((uint32_t)v);
                               }
                             });
      if (!ok && lane == 0) flag[0] = 1;
    }
    bar();
    if (aborted()) break;
    stamp(l, 5);
    stream(nuh, kbo, true);
    stamp(l, 6);
    bar();
    if (t < 16 * nuh) {
      float tot = 0.f;
#pragma unroll
      for (int ww = 0; ww < 4; ++ww) tot += __int_as_float(red[ww * (B1_MAXCU * 16) + t]);
      h2res = bfr(tot * swl[t] + xres);
      ov[t] = f2bf(h2res);
    }
    bar();
    publish3(p.gr + ((long long)l * G + c) * p.gpc_x, 16 * nuh, tag_of(l, 3));
    stamp(l, 7);

    // ================= gate_up + SwiGLU
    stage_scales(p.sw_gu + (long long)l * 2 * F + 8 * uf0, p.sw_gu + (long long)l * 2 * F + F + 8 * uf0, 8 * nuf);
    const float sa_g = norm_seam(p.gr + (long long)l * G * p.gpc_x, tag_of(l, 3), 4);
    if (aborted()) break;
    stamp(l, 8);
    stream(nuf, kbq, false);
    stamp(l, 9);
    bar();
    if (t < 8 * nuf) {
      const int u = t >> 3, i = t & 7;
      int tg = 0, tu = 0;
#pragma unroll
      for (int ww = 0; ww < 4; ++ww) {
        tg += red[ww * (B1_MAXCU * 16) + u * 16 + i];
        tu += red[ww * (B1_MAXCU * 16) + u * 16 + 8 + i];
      }
      const float gg = bfr((float)tg * sa_g * swl[t]), uu = bfr((float)tu * sa_g * swl[B1_MAXCU * 16 + t]);
      ov[t] = f2bf(gg / (1.f + __expf(-gg)) * uu);
    }
    bar();
    publish3(p.gh + ((long long)l * G + c) * p.gpc_h, 8 * nuf, tag_of(l, 4));
    stamp(l, 10);

    // ================= down (grouped-scale input: h quantised per 64 features here)
    stage_scales(p.sw_d + (long long)l * H + 16 * uh0, nullptr, 16 * nuh);
    if (l + 1 < L) stage_gamma(p.gam1 + (long long)(l + 1) * H);   // for the next qkv norm, in this seam
    {
      bf16_t* const hv = reinterpret_cast<bf16_t*>(scr);
      if (seamw) {
        uint64_t* const gb = p.gh + (long long)l * G * p.gpc_h;
        const bool ok = gather(gb, G * p.gpc_h, tag_of(l, 4), 5,
                               [&](int i) -> int {
                                 const int cb = fdiv(i, inv_gh), j = i - cb * p.gpc_h;
                                 return 3 * j < 8 * (u0f[cb + 1] - u0f[cb]) ? i : -1;
                               },
                               [&](int i, uint64_t v) {
                                 const int cb = fdiv(i, inv_gh), j = i - cb * p.gpc_h;
                                 const int f0 = 8 * u0f[cb], nv = 8 * u0f[cb + 1] - f0;
                                 for (int e = 0; e < 3 && 3 * j + e < nv; ++e) hv[f0 + 3 * j + e] = (bf16_t)(v >> (16 * e));
                               });
        if (!ok && lane == 0) flag[0] = 1;
      }
      stamp(l, 18);
      bar();
      if (aborted()) break;
      stamp(l, 19);
      // 16 lanes x 4 features per 64-group, 4 groups per wave step (all eight waves)
      const int NG = F / 64;
      for (int gb0 = w * 4; gb0 < NG; gb0 += 32) {
        const int gb = gb0 + (lane >> 4), li = lane & 15;
        float hf[4] = {0.f, 0.f, 0.f, 0.f};
        if (gb < NG) {
          const uint2 hh = *reinterpret_cast<const uint2*>(hv + gb * 64 + li * 4);
          hf[0] = bf2f(hh.x & 0xffffu); hf[1] = bf2f(hh.x >> 16); hf[2] = bf2f(hh.y & 0xffffu); hf[3] = bf2f(hh.y >> 16);
        }
        float a = fmaxf(fmaxf(fabsf(hf[0]), fabsf(hf[1])), fmaxf(fabsf(hf[2]), fabsf(hf[3])));
        a = fmaxf(a, __shfl_xor(a, 8, 64));
        a = fmaxf(a, __shfl_xor(a, 4, 64));
        a = fmaxf(a, __shfl_xor(a, 2, 64));
        a = fmaxf(a, __shfl_xor(a, 1, 64));
        if (gb < NG) {
          const float s = fmaxf(a, 1e-8f) / 127.f, inv = 1.f / s;
          const uint32_t q = (uint32_t)(uint8_t)quant_i8(hf[0], inv) | ((uint32_t)(uint8_t)quant_i8(hf[1], inv) << 8) |
                             ((uint32_t)(uint8_t)quant_i8(hf[2], inv) << 16) | ((uint32_t)(uint8_t)quant_i8(hf[3], inv) << 24);
          *reinterpret_cast<uint32_t*>(xq + gb * 64 + li * 4) = q;
          if (li == 0) sx[gb] = s;
        }
      }
    }
    stamp(l, 20);
    bar();
    if (l == L - 1 && c == 0 && t == 0) c_st(p.ctl, salt + 1);   // every CU read the salt long ago
    stamp(l, 11);
    stream(nuh, kbd, true);
    stamp(l, 12);
    bar();
    if (t < 16 * nuh) {
      float tot = 0.f;
#pragma unroll
      for (int ww = 0; ww < 4; ++ww) tot += __int_as_float(red[ww * (B1_MAXCU * 16) + t]);
      xres = bfr(tot * swl[t] + h2res);
      ov[t] = f2bf(xres);
    }
    bar();
    if (l == L - 1 && seamw && sidx < 16 * nuh) p.xout[16 * uh0 + sidx] = ov[sidx];
    if (l + 1 < L) publish3(p.gx + ((long long)(l + 1) * G + c) * p.gpc_x, 16 * nuh, tag_of(l + 1, 0));
    stamp(l, 13);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");    // no DMA outlives the workgroup
}

}  // namespace

// LDS bytes of a launch (the carve at the top of the kernel)
extern "C" int edge_b1_lds_bytes(int D, int xqb, int sxn, int scb) {
  return 4 * D * 1024 + xqb + 4 * sxn + scb + 4 * 4 * B1_MAXCU * 16 + 4 * 64 + 2 * B1_MAXCU * 16 + 16 +
         4 * 3 * (B1_MAXG + 1) + 4 * 2 * B1_MAXCU * 16 + 16 + 2 * xqb;
}

template <int D, int HD>
static int b1_launch(const B1Params& p, int G, int lds, hipStream_t st) {
  static int set = -1;
  if (set != lds) {
    if (hipFuncSetAttribute((const void*)b1_decode_kernel<D, HD>, hipFuncAttributeMaxDynamicSharedMemorySize, lds) !=
        hipSuccess)
      return -3;
    set = lds;
  }
  hipLaunchKernelGGL((b1_decode_kernel<D, HD>), dim3(G), dim3(B1_NT), lds, st, p);
  return (int)hipGetLastError();
}

// -1: no instantiation for (D, HD); -3: the LDS request was refused
extern "C" int edge_b1_decode(const B1Params* p, int G, int D, int HD, int lds, hipStream_t st) {
  if (lds > 160 * 1024) return -3;
  if (HD == 128) {
    if (D == 16) return b1_launch<16, 128>(*p, G, lds, st);
    if (D == 24) return b1_launch<24, 128>(*p, G, lds, st);
  } else if (HD == 64) {
    if (D == 16) return b1_launch<16, 64>(*p, G, lds, st);
    if (D == 24) return b1_launch<24, 64>(*p, G, lds, st);
  }
  return -1;
}

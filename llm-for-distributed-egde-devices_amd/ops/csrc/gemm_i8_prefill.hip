// W8A8 prefill GEMMs (M > 64 rows, K % 64 == 0, N % 8 == 0): the 128 x 256 LDS-DMA ring kernel
// and the 256 x 256 32x32-MFMA kernel, with the optional fragment-packed A (pack_a_kernel).  The
// operand layout and the epilogue math are those of the decode kernels (gemm_i8.h).
#include "gemm_i8.h"

namespace {
// ------------------------------------------------------------------------------------ big
// Prefill GEMM (M > 128, K % 64 == 0, N % 8 == 0): BM x 256 block tile (BM = 256, or 128 when
// 256-row tiles would leave CUs idle), 8 waves as 2 (M) x 4 (N), BK = 64, one block per CU.
//  * Both operands go global -> LDS by global_load_lds into a ring of R = 4 stages (BM/16 + 16 KiB
//    each; 128 KiB at BM = 256): 3 stages of DMA stay in flight across every barrier (counted
//    vmcnt, bare s_barrier, LDS reads by inline asm so the compiler never drains the ring with a
//    vmcnt(0) — the structure of the 128-row decode ring kernel below).
//  * Fragments are double-buffered in registers: iteration s reads stage s + 1's fragments while
//    the MFMAs consume stage s's, so LDS latency hides under 32 MFMAs per wave.
//  * Operands are swapped in the MFMA (W tile as the A operand, activations as B), so the
//    accumulator of a lane holds 4 consecutive output COLUMNS of one row: the epilogue scales,
//    packs 4 bf16 into 8 bytes, and restages the wave's tile through LDS (XOR-swizzled 16-B
//    chunks) to write full 128-B row segments with 16-B stores.
//  * blockIdx -> tile: bijective XCD remap (each XCD gets a contiguous range), then groups of 4
//    row tiles walked column-major, so an XCD's ~32 resident blocks share 4 A panels and 8 W panels
//    in its L2.
//  * APK: A arrives fragment-packed (pack_a_kernel: 1 KiB = 16 rows x 64 k per (row block, k-tile),
//    the layout of the packed weights), so an A piece is 1 KiB of contiguous bytes instead of 16
//    rows x 64 B — the pattern tools/ingest_bw.hip measured at ~18 B/clk/CU L2 -> LDS against
//    ~60 for contiguous pieces.  The LDS image is identical, only the DMA source offsets change.
//  * A k-tile's DMA pieces are interleaved into its MFMA stream (piece g after MFMA group g: a glds
//    that stalls on a full memory queue then holds back only the MFMAs behind it; 1-3 % ahead of
//    issuing them before the fragment reads or after the MFMAs on the Llama-2-7B shapes).
template <int BMV, bool APK = false>
__global__ void __launch_bounds__(512, 1) w8a8_gemm_big_kernel(const int8_t* __restrict__ A, const float* __restrict__ sa,
                                                              const int8_t* __restrict__ Wp, const float* __restrict__ sw,
                                                              const bf16_t* __restrict__ bias, bf16_t* __restrict__ out,
                                                              int M, int N, int K, int KT, int NTt, int grid_m, int grid_n) {
  constexpr int R = 4, BNV = 256, NWV = 8;
  constexpr int AP = BMV / 16, BP = BNV / 16, PIECES = AP + BP, PPW = PIECES / NWV, STAGE = PIECES * 1024;
  constexpr int MI = BMV / 32, NJ = 4;                        // row blocks / column tiles per wave
  static_assert(PIECES % NWV == 0, "pieces per wave");
  static_assert(R * STAGE <= 160 * 1024 && NWV * (BMV / 4) * 256 <= R * STAGE, "LDS budget");
  __shared__ __attribute__((aligned(1024))) int8_t ring[R * STAGE];

  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  constexpr int GM = 4;
  const int per_group = GM * grid_n;
  const int grp = wgid / per_group, gm0 = grp * GM, gsz = min(GM, grid_m - gm0);
  const int inr = wgid - grp * per_group;
  const int bm = gm0 + inr % gsz, bn = inr / gsz;

  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 2, wn = wave & 3;

  // this wave's DMA pieces p = wave + 8 i: A row block p (p < AP) or W tile p - AP.  Per-lane
  // 32-bit offsets from the (wave-uniform) operand base: one VGPR per piece, SGPR base + VGPR
  // offset addressing (M * K and the packed W stay below 4 GiB)
  uint32_t off[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int p = wave + NWV * i;
    if (p < AP && APK) {
      const int rb = min(bm * (BMV / 16) + p, (M + 15) / 16 - 1);
      off[i] = (uint32_t)rb * (uint32_t)KT * 1024u + lane * 16;
    } else if (p < AP) {
      const int row = min(bm * BMV + p * 16 + (lane & 15), M - 1);
      off[i] = (uint32_t)row * (uint32_t)K + 16 * (lane >> 4);
    } else {
      const int t = min(bn * BP + (p - AP), NTt - 1);
      off[i] = (uint32_t)t * (uint32_t)KT * 1024u + lane * 16;
    }
  }
  // DMA of stage st into slot st % R.  Stages past the last k-tile re-load the last k-tile into
  // their slot (never read again: every stage still to be read sits in another slot), so every
  // stage is PPW pieces per wave, the loop is branch-free and the vmcnt counts are constants.
  auto issue_piece = [&](int st, int i) {
    const int kt = min(st, KT - 1);
    const bool isa = wave + NWV * i < AP;
    glds16((isa ? A + (size_t)kt * (APK ? 1024 : 64) : Wp + (size_t)kt * 1024) + off[i],
           ring + (st % R) * STAGE + (wave + NWV * i) * 1024);
  };
  auto issue = [&](int st) {
#pragma unroll
    for (int i = 0; i < PPW; ++i) issue_piece(st, i);
  };
  // fragment reads: one VGPR base per operand and slot, immediate offsets
  const uint32_t ring0 = lds_off(ring) + lane * 16;
  const uint32_t wbase = ring0 + (AP + wn * NJ) * 1024, abase = ring0 + wm * MI * 1024;
  auto read_frags = [&](int st, v4i (&fw)[NJ], v4i (&fa)[MI]) {
    const uint32_t so = (st % R) * STAGE;
    const uint32_t wb = wbase + so, ab = abase + so;
    lds_read_row<NJ>(wb, fw);
    lds_read_row<MI>(ab, fa);
  };
  auto pin = [&](v4i (&fw)[NJ], v4i (&fa)[MI]) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) asm volatile("" : "+v"(fw[j]));
#pragma unroll
    for (int i = 0; i < MI; ++i) asm volatile("" : "+v"(fa[i]));
  };

  v4i acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = v4i{0, 0, 0, 0};
  // fragments pinned after the reads that precede this call, accumulators pinned after the
  // MFMAs: the MFMAs sit between the fragment reads and the next lgkmcnt wait (left alone,
  // hipcc hoists the wait above them and the LDS latency is exposed every k-tile)
  auto mma = [&](v4i (&fw)[NJ], v4i (&fa)[MI]) {
    pin(fw, fa);
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = mfma_i8(fw[j], fa[i], acc[i][j]);
  };
  auto pin_acc = [&]() {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) asm volatile("" : "+v"(acc[i][j]));
  };

  // prologue: R stages in flight, stage 0's fragments in registers
#pragma unroll
  for (int st = 0; st < R; ++st) issue(st);
  v4i w0[NJ], a0[MI], w1[NJ], a1[MI];
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"((R - 1) * PPW) : "memory");
  __builtin_amdgcn_s_barrier();
  read_frags(0, w0, a0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");

  // k-tile s < KT - 1: stage s + 1's fragments -> (wx, ax) while the MFMAs consume (wc, ac):
  // reads -> MFMAs -> lgkmcnt(0), the wave's own MFMAs cover the LDS latency (measured 3-8 %
  // faster than reads -> lgkmcnt(0) -> MFMAs, where only the SIMD's other wave covers it)
  auto full = [&](int s, v4i (&wc)[NJ], v4i (&ac)[MI], v4i (&wx)[NJ], v4i (&ax)[MI]) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((R - 2) * PPW) : "memory");   // own DMA of s + 1
    __builtin_amdgcn_s_barrier();                     // stage s + 1 landed everywhere; slot of s free
    read_frags(s + 1, wx, ax);
    pin(wc, ac);
    constexpr int TOT = MI * NJ, GRP = TOT / (PPW + 1);
#pragma unroll
    for (int f = 0; f < TOT; ++f) {                   // DMA pieces interleaved into the MFMA stream
      const int i = f / NJ, j = f % NJ;
      acc[i][j] = mfma_i8(wc[j], ac[i], acc[i][j]);
      if ((f + 1) % GRP == 0 && (f + 1) / GRP <= PPW) {
        asm volatile("" : "+v"(acc[i][j])::"memory");   // this MFMA issued before the piece
        issue_piece(s + R, (f + 1) / GRP - 1);
      }
    }
    pin_acc();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };
  int s = 0;
  for (; s + 2 < KT; s += 2) {
    full(s, w0, a0, w1, a1);
    full(s + 1, w1, a1, w0, a0);
  }
  if (s + 1 < KT) {
    full(s, w0, a0, w1, a1);
    mma(w1, a1);
  } else {
    mma(w0, a0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the re-load stages past the end

  // epilogue: lane holds int32 out[row = rb*16 + (lane & 15)][col = tile*16 + 4 (lane >> 4) + r].
  // The raw accumulators go to LDS first (one 16-B write per tile, freeing their registers), in
  // halves of MI/2 row blocks per wave ([MI*8 rows][64 cols] int32, 256-B rows, 16-B chunk c of
  // row m at c ^ (m & 15): conflict-free); each lane then owns 8 consecutive columns (its scales
  // and bias loaded once), scales, packs bf16 and writes 16 B.
  const int r16 = lane & 15, g4 = lane >> 4, c8 = lane & 7;
  const int col0 = bn * BNV + wn * 64 + c8 * 8;
  const bf16_t* bp = bias != nullptr ? bias : g_zero_bf16;
  float swv[8], bv[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int col = min(col0 + e, N - 1);
    swv[e] = sw[col];
    bv[e] = bf2f(bp[bias != nullptr ? col : 0]);        // absent bias: a zero word, no branch
  }
  __syncthreads();                                    // every wave is done with the ring
  int8_t* wt = ring + wave * (MI * 8 * 256);
  constexpr int HALF = MI / 2;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int i = 0; i < HALF; ++i) {
      const int m = i * 16 + r16;
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        *reinterpret_cast<v4i*>(wt + m * 256 + (((4 * j + g4) ^ (m & 15)) << 4)) = acc[h * HALF + i][j];
    }
    // (a wave's LDS operations complete in issue order: no wait between its writes and reads)
#pragma unroll
    for (int it = 0; it < HALF * 2; ++it) {
      const int m = it * 8 + (lane >> 3);
      const int row = bm * BMV + wm * MI * 16 + h * HALF * 16 + m;
      const float sr = sa[min(row, M - 1)];
      const v4i lo = *reinterpret_cast<const v4i*>(wt + m * 256 + (((2 * c8) ^ (m & 15)) << 4));
      const v4i hi = *reinterpret_cast<const v4i*>(wt + m * 256 + (((2 * c8 + 1) ^ (m & 15)) << 4));
      float v[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = (float)lo[e] * sr * swv[e] + bv[e];
        v[e + 4] = (float)hi[e] * sr * swv[e + 4] + bv[e + 4];
      }
      if (row < M && col0 < N) *reinterpret_cast<uint4*>(out + (size_t)row * N + col0) = pack8(v);   // N % 8 == 0
    }
  }
}

// Fragment-pack A [M, K] int8 for the APK prefill GEMM: piece (rb, kt) = 1 KiB at
// (rb * KT + kt) * 1024, lane l's 16 B = A[16 rb + (l & 15)][64 kt + 16 (l >> 4) ..] (rows past M
// repeat row M - 1; the GEMM never stores them).  One thread per 16 B; writes are contiguous.
__global__ void __launch_bounds__(256) pack_a_kernel(const int8_t* __restrict__ A, int8_t* __restrict__ Ap, int M, int K,
                                                     int KT, int64_t total) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= total) return;
  const int64_t piece = t >> 6;
  const int lane = (int)(t & 63);
  const int rb = (int)(piece / KT), kt = (int)(piece - (int64_t)rb * KT);
  const int row = min(rb * 16 + (lane & 15), M - 1);
  *reinterpret_cast<uint4*>(Ap + t * 16) =
      *reinterpret_cast<const uint4*>(A + (size_t)row * K + (size_t)kt * 64 + 16 * (lane >> 4));
}

// ------------------------------------------------------------------------------------ x32
// Prefill GEMM on v_mfma_i32_32x32x32_i8 with 256 x 256 block tiles (M >= 256, K % 64 == 0,
// N % 8 == 0).  The LDS image is the big kernel's (1 KiB pieces of 16 rows x 64 k, activations
// row-major or fragment-packed, weights packed), 4 stages of 32 KiB; what changes is the MFMA:
//  * 8 waves as 2 (tokens) x 4 (columns), each 128 tokens x 64 columns = 4 x 2 blocks of 32 x 32.
//    Per 32-k step a wave reads 6 fragments (4 activation + 2 weight blocks) for 8 MFMAs, so the
//    LDS reads per MFMA-cycle are those of a 128 x 64 wave tile: the big kernel's 16x16x64 form
//    holds its 64 x 64 tile's k-tile fragments (32 VGPRs) x 2 buffers + 64 accumulators, and at
//    128 x 64 it spilled; a 32-k step's fragments are 24 VGPRs, so 128 accumulators + two steps of
//    fragments fit, and a k-tile costs 1024 MFMA cycles per CU against 32 KiB of DMA (31 B/clk)
//    and ~125 B/clk of LDS traffic.
//  * A 32 x 32 x 32 operand of 32 rows = two stacked 16-row pieces: lane l reads piece 2 b +
//    ((l >> 4) & 1), 16 B of lane slot (l & 15) + 16 (2 s + (l >> 5)) — row l & 31, k 32 s + 16 (l >> 5)
//    of the 64-k tile (conflict-free: each 16-lane group covers the 64 banks once).
//  * Operands swapped as in the big kernel (weights = A operand): a lane's accumulator holds one
//    token (l & 31) and 4 runs of 4 consecutive columns 8 q + 4 (l >> 5).  The epilogue restages
//    32 tokens x 64 columns per wave at a time (int32, XOR-swizzled 16-B chunks) and writes 16-B
//    bf16 row chunks.
//  * The two waves of each SIMD are de-phased: waves 0-3 issue a stage's LDS-DMA pieces right after
//    the barrier, waves 4-7 after their second MFMA step, so after every barrier one wave per SIMD
//    runs MFMAs while the other issues DMA (+4-10 % over issuing together).
//  * Measured against the 128 x 256 16x16x64 kernel (tools/bench_ops.py --only x32, Llama-2-7B shapes):
//    2.17-2.30 vs 2.10-2.15 POPS at M = 16384, behind it at <= 384 tiles (qkv at M = 2048: 1.77 vs
//    2.05), so the launcher takes it from 512 tiles (two full rounds of the 256 CUs).  The same
//    kernel on bf16 operands (v_mfma_f32_32x32x16_bf16) ran 1.19-1.24 PF against hipBLASLt's
//    1.46-1.61 PF and was dropped.
// GLU: the gate_up projection of a 16-blocked SwiGLU layer (columns [gate(16) | up(16)] per 16
// features, quant.linear.W8A8Linear.glu_blocked): the epilogue writes h = silu(g) * u in bf16 [M, N / 2]
// instead of g / u [M, N], with g and u rounded to bf16 first, as the unfused path stores them.
template <bool APK, bool GLU = false>
__global__ void __launch_bounds__(512, 1) w8a8_gemm_x32_kernel(const int8_t* __restrict__ A, const float* __restrict__ sa,
                                                              const int8_t* __restrict__ Wp, const float* __restrict__ sw,
                                                              const bf16_t* __restrict__ bias, bf16_t* __restrict__ out,
                                                              int M, int N, int K, int KT, int NTt, int grid_m, int grid_n) {
  constexpr int R = 4, BMV = 256, BNV = 256, NWV = 8;
  constexpr int AP = BMV / 16, BP = BNV / 16, PIECES = AP + BP, PPW = PIECES / NWV, STAGE = PIECES * 1024;
  static_assert(R * STAGE <= 160 * 1024 && NWV * 32 * 256 <= R * STAGE, "LDS budget");
  __shared__ __attribute__((aligned(1024))) int8_t ring[R * STAGE];

  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  constexpr int GM = 4;
  const int per_group = GM * grid_n;
  const int grp = wgid / per_group, gm0 = grp * GM, gsz = min(GM, grid_m - gm0);
  const int inr = wgid - grp * per_group;
  const int bm = gm0 + inr % gsz, bn = inr / gsz;

  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const bool late = wave >= 4;                        // DMA after the second MFMA step (see above)
  uint32_t off[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int p = wave + NWV * i;
    if (p < AP && APK) {
      const int rb = min(bm * (BMV / 16) + p, (M + 15) / 16 - 1);
      off[i] = (uint32_t)rb * (uint32_t)KT * 1024u + lane * 16;
    } else if (p < AP) {
      const int row = min(bm * BMV + p * 16 + (lane & 15), M - 1);
      off[i] = (uint32_t)row * (uint32_t)K + 16 * (lane >> 4);
    } else {
      const int t = min(bn * BP + (p - AP), NTt - 1);
      off[i] = (uint32_t)t * (uint32_t)KT * 1024u + lane * 16;
    }
  }
  auto issue = [&](int st) {
    const int kt = min(st, KT - 1);
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const bool isa = wave + NWV * i < AP;
      glds16((isa ? A + (size_t)kt * (APK ? 1024 : 64) : Wp + (size_t)kt * 1024) + off[i],
             ring + (st % R) * STAGE + (wave + NWV * i) * 1024);
    }
  };
  // lane's byte in a 32-row operand block: piece offset ((l >> 4) & 1) KiB, lane slot
  // (l & 15) + 16 (l >> 5) = row l & 15 of the piece, 16-B k chunk l >> 5 (k-step 0; k-step 1 is
  // chunks 2, 3: 32 slots = 512 B further)
  const uint32_t lo = (((lane >> 4) & 1) << 10) + (((lane & 15) + 16 * (lane >> 5)) << 4);
  const uint32_t ring0 = lds_off(ring) + lo;
  const uint32_t abase = ring0 + (wm * 8) * 1024, wbase = ring0 + (AP + wn * 4) * 1024;
  // fragments of stage st, k-step ks: fa[c] = activation block c (tokens 32 c..), fw[b] = weight block b
  auto read_frags = [&](int st, int ks, v4i (&fa)[4], v4i (&fw)[2]) {
    const uint32_t so = (st % R) * STAGE + ks * 512;
    const uint32_t ab = abase + so, wb = wbase + so;
    asm volatile("ds_read_b128 %0, %1 offset:0" : "=v"(fa[0]) : "v"(ab));
    asm volatile("ds_read_b128 %0, %1 offset:2048" : "=v"(fa[1]) : "v"(ab));
    asm volatile("ds_read_b128 %0, %1 offset:4096" : "=v"(fa[2]) : "v"(ab));
    asm volatile("ds_read_b128 %0, %1 offset:6144" : "=v"(fa[3]) : "v"(ab));
    asm volatile("ds_read_b128 %0, %1 offset:0" : "=v"(fw[0]) : "v"(wb));
    asm volatile("ds_read_b128 %0, %1 offset:2048" : "=v"(fw[1]) : "v"(wb));
  };
  v16i acc[4][2];
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[c][b][r] = 0;
  auto mma = [&](v4i (&fa)[4], v4i (&fw)[2]) {
#pragma unroll
    for (int c = 0; c < 4; ++c) asm volatile("" : "+v"(fa[c]));
#pragma unroll
    for (int b = 0; b < 2; ++b) asm volatile("" : "+v"(fw[b]));
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        acc[c][b] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fw[b], fa[c], acc[c][b], 0, 0, 0);
      }
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int b = 0; b < 2; ++b) asm volatile("" : "+v"(acc[c][b]));
  };

#pragma unroll
  for (int st = 0; st < R; ++st) issue(st);
  v4i xa[4], xw[2], ya[4], yw[2];
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"((R - 1) * PPW) : "memory");
  __builtin_amdgcn_s_barrier();
  read_frags(0, 0, xa, xw);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  for (int kt = 0; kt < KT; ++kt) {                   // x: (kt, step 0) in registers
    read_frags(kt, 1, ya, yw);
    mma(xa, xw);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (kt + 1 < KT) {                                // wave-uniform
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((R - 2) * PPW) : "memory");   // own DMA of kt + 1
      __builtin_amdgcn_s_barrier();                   // kt + 1 landed everywhere; slot of kt free
      if (!late) issue(kt + R);
      read_frags(kt + 1, 0, xa, xw);
    }
    mma(ya, yw);
    if (late && kt + 1 < KT) issue(kt + R);           // waves 4-7: behind this k-tile's second MFMA step
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the re-load stages past the end

  if constexpr (GLU) {
    // the wave's 64 columns are two 32-column blocks [gate(16) | up(16)] = 32 features.  Lane:
    // features (lane & 3) * 8 .. + 8 of the wave's 32 (block b = (lane & 3) >> 1; gate columns c0 ..
    // c0 + 7, up 16 further), tokens it * 16 + (lane >> 2).  int32 restaged as below.
    const int qg = lane & 3, bb = qg >> 1, c0 = bb * 32 + (qg & 1) * 8;
    const int gcol = bn * BNV + wn * 64 + c0, F = N / 2;
    const int f0 = (bn * BNV + wn * 64 + bb * 32) / 2 + (qg & 1) * 8;
    const bf16_t* bp = bias != nullptr ? bias : g_zero_bf16;
    float swg[8], swu[8], bgv[8], buv[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int cg = min(gcol + e, N - 1), cu = min(gcol + 16 + e, N - 1);
      swg[e] = sw[cg];
      swu[e] = sw[cu];
      bgv[e] = bf2f(bp[bias != nullptr ? cg : 0]);
      buv[e] = bf2f(bp[bias != nullptr ? cu : 0]);
    }
    __syncthreads();                                  // every wave is done with the ring
    int8_t* wt = ring + wave * (32 * 256);
    const int tl = lane & 31, hi = lane >> 5;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int k16 = 8 * b + 2 * q + hi;
          const v4i v4 = v4i{acc[c][b][4 * q], acc[c][b][4 * q + 1], acc[c][b][4 * q + 2], acc[c][b][4 * q + 3]};
          *reinterpret_cast<v4i*>(wt + tl * 256 + ((k16 ^ (tl & 15)) << 4)) = v4;
        }
#pragma unroll
      for (int it = 0; it < 2; ++it) {
        const int t = it * 16 + (lane >> 2);
        const int row = bm * BMV + wm * 128 + c * 32 + t;
        const float sr = sa[min(row, M - 1)];
        const int kg = c0 >> 2, ku = (c0 + 16) >> 2;
        const v4i g0 = *reinterpret_cast<const v4i*>(wt + t * 256 + ((kg ^ (t & 15)) << 4));
        const v4i g1 = *reinterpret_cast<const v4i*>(wt + t * 256 + (((kg + 1) ^ (t & 15)) << 4));
        const v4i u0 = *reinterpret_cast<const v4i*>(wt + t * 256 + ((ku ^ (t & 15)) << 4));
        const v4i u1 = *reinterpret_cast<const v4i*>(wt + t * 256 + (((ku + 1) ^ (t & 15)) << 4));
        float h[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int gi = e < 4 ? g0[e] : g1[e - 4], ui = e < 4 ? u0[e] : u1[e - 4];
          const float g = bf2f(f2bf((float)gi * sr * swg[e] + bgv[e]));
          const float u = bf2f(f2bf((float)ui * sr * swu[e] + buv[e]));
          h[e] = g / (1.f + __expf(-g)) * u;
        }
        if (row < M && gcol < N) *reinterpret_cast<uint4*>(out + (size_t)row * F + f0) = pack8(h);
      }
    }
    return;
  }
  // epilogue: acc[c][b] register r -> token wm*128 + 32 c + (l & 31), column
  // wn*64 + 32 b + 8 (r >> 2) + 4 (l >> 5) + (r & 3).  Per c: the wave's 32 tokens x 64 columns of
  // int32 go to its LDS block (256-B rows, 16-B chunk k of token t at k ^ (t & 15)), then each lane
  // takes 8 consecutive columns (chunk pair lane & 7) of tokens it * 8 + (lane >> 3).
  const int c8 = lane & 7, tl = lane & 31, hi = lane >> 5;
  const int col0 = bn * BNV + wn * 64 + c8 * 8;
  const bf16_t* bp = bias != nullptr ? bias : g_zero_bf16;
  float swv[8], bv[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int col = min(col0 + e, N - 1);
    swv[e] = sw[col];
    bv[e] = bf2f(bp[bias != nullptr ? col : 0]);
  }
  __syncthreads();                                    // every wave is done with the ring
  int8_t* wt = ring + wave * (32 * 256);
#pragma unroll
  for (int c = 0; c < 4; ++c) {
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int k16 = 8 * b + 2 * q + hi;           // 16-B chunk (4 int32 columns) of the 64
        const v4i v4 = v4i{acc[c][b][4 * q], acc[c][b][4 * q + 1], acc[c][b][4 * q + 2], acc[c][b][4 * q + 3]};
        *reinterpret_cast<v4i*>(wt + tl * 256 + ((k16 ^ (tl & 15)) << 4)) = v4;
      }
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int t = it * 8 + (lane >> 3);
      const int row = bm * BMV + wm * 128 + c * 32 + t;
      const float sr = sa[min(row, M - 1)];
      const v4i lo4 = *reinterpret_cast<const v4i*>(wt + t * 256 + (((2 * c8) ^ (t & 15)) << 4));
      const v4i hi4 = *reinterpret_cast<const v4i*>(wt + t * 256 + (((2 * c8 + 1) ^ (t & 15)) << 4));
      float v[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = (float)lo4[e] * sr * swv[e] + bv[e];
        v[e + 4] = (float)hi4[e] * sr * swv[e + 4] + bv[e + 4];
      }
      if (row < M && col0 < N) *reinterpret_cast<uint4*>(out + (size_t)row * N + col0) = pack8(v);   // N % 8 == 0
    }
  }
}

}  // namespace

// the 256 x 256 x32 kernel: g_prefill_x32 0 never, 1 from 512 tiles (default), 2 from 192 tiles (tests)
static int g_prefill_apack = 1, g_prefill_x32 = 1;
static bool x32_takes(int M, int grid_n) {
  const int64_t tiles = (int64_t)((M + 255) / 256) * grid_n;
  return g_prefill_x32 && M >= 256 && tiles >= (g_prefill_x32 == 2 ? 192 : 512);
}
// prefill_x32: 0 off, 1 the 256 x 256 32x32x32 kernel when the grid fills >= 1 round of CUs (M >= 256)
extern "C" void edge_w8a8_prefill_x32(int v) { g_prefill_x32 = v; }
extern "C" void edge_w8a8_prefill_apack(int v) { g_prefill_apack = v; }

// Row-major A (per-token scales sa [M]) -> bf16 out [M, N] (+ bias).  128 x 256 tiles.  (The 256 x 256
// form of the ring kernel measured 2.21 vs 2.11 POPS on the K = 11008 down projection at M = 16384,
// but at 256 VGPRs it spilled ~290 B per lane, and spill traffic joins the ring's counted vmcnt — the
// same hazard that broke a decode kernel — so it is gone; the x32 kernel takes the big grids.)
extern "C" int edge_w8a8_prefill(const void* A, const float* sa, const void* Wp, const float* sw, const void* bias,
                                 void* out, int M, int N, int K, int KT, hipStream_t st) {
  if (M <= 64 || K % 64 != 0 || K / 64 != KT || N % 8 != 0) return -2;
  const int NTt = (N + 15) / 16;
  const int grid_n = (NTt * 16 + 255) / 256;
  const int grid_m = (M + 127) / 128;
  if (x32_takes(M, grid_n)) {
    const int gm2 = (M + 255) / 256;
    hipLaunchKernelGGL((w8a8_gemm_x32_kernel<false>), dim3(gm2 * grid_n), dim3(512), 0, st, (const int8_t*)A, sa,
                       (const int8_t*)Wp, sw, (const bf16_t*)bias, (bf16_t*)out, M, N, K, KT, NTt, gm2, grid_n);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL((w8a8_gemm_big_kernel<128>), dim3(grid_m * grid_n), dim3(512), 0, st, (const int8_t*)A, sa,
                     (const int8_t*)Wp, sw, (const bf16_t*)bias, (bf16_t*)out, M, N, K, KT, NTt, grid_m, grid_n);
  return (int)hipGetLastError();
}

// Prefill GEMM with A fragment-packed first (APK form of w8a8_gemm_big_kernel).  Ap: scratch of
// (M + 15) / 16 * 16 * K bytes from the caller's (stream-ordered) allocator.  Returns -2 when the
// shape does not take the ring GEMM (the caller then runs edge_w8a8_gemm).
// g_prefill_apack: 0 off, 1 automatic, 2 always.  Automatic = wide N at >= 2048 rows, where every A
// panel is re-read by >= 32 column blocks (tools/bench_ops.py pgemm, Llama-2-7B shapes: gate_up
// 1.91 -> 2.10 POPS and qkv 1.96 -> 2.04 at M = 16384; at N = 4096 or M = 512 the extra pass over
// A costs more than the contiguous pieces save, o at M = 2048 1.85 -> 1.69)
extern "C" int edge_w8a8_apack_ok(int M, int N, int K, int KT) {
  const bool want = g_prefill_apack == 2 || (g_prefill_apack == 1 && N >= 8192 && M >= 2048);
  return want && M > 128 && K % 64 == 0 && K / 64 == KT && N % 8 == 0 &&
         (int64_t)((M + 15) / 16) * KT * 1024 < (int64_t)1 << 32;
}

extern "C" int edge_w8a8_gemm_apk(const void* A, void* Ap, const float* sa, const void* Wp, const float* sw,
                                  const void* bias, void* out, int M, int N, int K, int KT, hipStream_t st) {
  if (!edge_w8a8_apack_ok(M, N, K, KT)) return -2;
  const int64_t total = (int64_t)((M + 15) / 16) * KT * 64;
  hipLaunchKernelGGL(pack_a_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, (const int8_t*)A,
                     (int8_t*)Ap, M, K, KT, total);
  const int NTt = (N + 15) / 16;
  const int grid_n = (NTt * 16 + 255) / 256;
  const int grid_m = (M + 127) / 128;
  if (x32_takes(M, grid_n)) {
    const int gm2 = (M + 255) / 256;
    hipLaunchKernelGGL((w8a8_gemm_x32_kernel<true>), dim3(gm2 * grid_n), dim3(512), 0, st, (const int8_t*)Ap, sa,
                       (const int8_t*)Wp, sw, (const bf16_t*)bias, (bf16_t*)out, M, N, K, KT, NTt, gm2, grid_n);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL((w8a8_gemm_big_kernel<128, true>), dim3(grid_m * grid_n), dim3(512), 0, st, (const int8_t*)Ap,
                     sa, (const int8_t*)Wp, sw, (const bf16_t*)bias, (bf16_t*)out, M, N, K, KT, NTt, grid_m, grid_n);
  return (int)hipGetLastError();
}

// gate_up of a 16-blocked SwiGLU layer with the SwiGLU in the epilogue (x32 kernel, GLU): h = silu(g)
// * u, bf16 [M, N / 2].  A row-major (per-token scales sa [M]); Ap: scratch of (M + 15) / 16 * 16 * K
// bytes for the fragment-packed copy when edge_w8a8_apack_ok.  -2: the shape does not take the x32
// kernel (the caller runs the GEMM and the blocked activation kernel instead).
extern "C" int edge_w8a8_prefill_glu(const void* A, void* Ap, const float* sa, const void* Wp, const float* sw,
                                     const void* bias, void* out, int M, int N, int K, int KT, hipStream_t st) {
  if (M <= 64 || K % 64 != 0 || K / 64 != KT || N % 256 != 0) return -2;
  const int NTt = N / 16, grid_n = N / 256;
  if (!x32_takes(M, grid_n)) return -2;
  const int gm2 = (M + 255) / 256;
  if (Ap != nullptr && edge_w8a8_apack_ok(M, N, K, KT)) {
    const int64_t total = (int64_t)((M + 15) / 16) * KT * 64;
    hipLaunchKernelGGL(pack_a_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, (const int8_t*)A,
                       (int8_t*)Ap, M, K, KT, total);
    hipLaunchKernelGGL((w8a8_gemm_x32_kernel<true, true>), dim3(gm2 * grid_n), dim3(512), 0, st, (const int8_t*)Ap,
                       sa, (const int8_t*)Wp, sw, (const bf16_t*)bias, (bf16_t*)out, M, N, K, KT, NTt, gm2, grid_n);
  } else {
    hipLaunchKernelGGL((w8a8_gemm_x32_kernel<false, true>), dim3(gm2 * grid_n), dim3(512), 0, st, (const int8_t*)A,
                       sa, (const int8_t*)Wp, sw, (const bf16_t*)bias, (bf16_t*)out, M, N, K, KT, NTt, gm2, grid_n);
  }
  return (int)hipGetLastError();
}

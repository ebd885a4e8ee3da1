// How fast can a CU take in L2-resident bytes?  The decode GEMVs at 65-128 rows and the prefill
// GEMM both re-read operand panels that sit in L2; this measures the chip-wide rate of that path
// alone (no MFMA), for the two load forms the kernels use:
//   mode 0: global_load_dwordx4 into VGPRs (U loads in flight per wave, XOR-folded)
//   mode 1: global_load_lds_dwordx4 into an LDS ring (U pieces in flight per wave, counted vmcnt)
//   mode 2: as 1, each piece 16 rows x 64 B of a row-major [256][4096] int8 matrix (the GEMV's
//           activation fragments) instead of 1 KiB contiguous
//   mode 3: as 2 with 8 rows x 128 B (whole lines) per piece
// Every workgroup streams the same L2-resident buffer (A_KB per workgroup offset so XCDs see
// different lines), `iters` 1 KiB wave-pieces per wave.  Prints TB/s and B/clk/CU at 2.1 GHz.
//   hipcc -O3 --offload-arch=gfx950 tools/ingest_bw.hip -o build/ingest_bw && ./build/ingest_bw
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef int v4i __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <int U>
__global__ void __launch_bounds__(512) vgpr_kernel(const v4i* __restrict__ buf, int pieces, int iters, int* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v4i acc = v4i{0, 0, 0, 0};
  int p = (blockIdx.x * 7 + wave * 3) % pieces;
  for (int it = 0; it < iters; it += U) {
    v4i b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int q = (p + u * nw) % pieces;
      b[u] = buf[(size_t)q * 64 + lane];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= b[u];
    p = (p + U * nw) % pieces;
  }
  if ((acc[0] ^ acc[1] ^ acc[2] ^ acc[3]) == 0x7fffffff) out[0] = 1;
}

// ROWS: a piece is 16 rows x 64 B of a [rows][4096] int8 matrix (the GEMV activation-fragment
// pattern: lane l -> row l & 15, bytes 16 (l >> 4)); otherwise 1 KiB contiguous.
template <int U, int ROWS>
__global__ void __launch_bounds__(512) glds_kernel(const int8_t* __restrict__ buf, int pieces, int iters, int* out) {
  __shared__ __attribute__((aligned(1024))) int8_t ring[8 * U * 1024];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  int p = (blockIdx.x * 7 + wave * 3) % pieces;
  int slot = 0;
  for (int it = 0; it < iters; ++it) {
    // ROWS 1: 16 rows x 64 B; 2: 8 rows x 128 B (full lines, chunk XOR-swizzled by row)
    const size_t src = ROWS == 1 ? (size_t)(p >> 6) * 16 * 4096 + (size_t)(lane & 15) * 4096 + (p & 63) * 64 + 16 * (lane >> 4)
                     : ROWS == 2 ? (size_t)(p >> 5) * 8 * 4096 + (size_t)(lane >> 3) * 4096 + (p & 31) * 128 +
                                       16 * ((lane & 7) ^ (lane >> 3))
                                 : (size_t)p * 1024 + lane * 16;
    __builtin_amdgcn_global_load_lds(buf + src,
                                     (__attribute__((address_space(3))) void*)(ring + (wave * U + slot) * 1024), 16, 0, 0);
    if (it >= U - 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(U - 1) : "memory");
    slot = slot + 1 == U ? 0 : slot + 1;
    p = p + nw >= pieces ? p + nw - pieces : p + nw;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (ring[threadIdx.x] == 0x7f && ring[threadIdx.x + 1] == 0x7e && ring[threadIdx.x + 2] == 0x11) out[0] = 1;
}

int main() {
  const int KB = 1024;                       // buffer: 1 MiB, L2-resident after the first touch
  const int pieces = KB;                     // 1 KiB pieces
  int8_t* buf;
  int* out;
  CK(hipMalloc(&buf, (size_t)pieces * 1024));
  CK(hipMalloc(&out, 4));
  CK(hipMemset(buf, 1, (size_t)pieces * 1024));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int iters = 4096;
  printf("mode,grid,waves,U,us,TBps,B_per_clk_per_CU\n");
  for (int mode = 0; mode < 4; ++mode)
    for (int grid : {256, 512})
      for (int waves : {4, 8})
        for (int U : {2, 4, 8}) {
          auto launch = [&]() {
#define L(UV)                                                                                                        \
  if (U == UV) {                                                                                                     \
    if (mode == 0) hipLaunchKernelGGL(vgpr_kernel<UV>, dim3(grid), dim3(waves * 64), 0, 0, (const v4i*)buf, pieces, iters, out); \
    else if (mode == 1) hipLaunchKernelGGL((glds_kernel<UV, 0>), dim3(grid), dim3(waves * 64), 0, 0, buf, pieces, iters, out); \
    else if (mode == 2) hipLaunchKernelGGL((glds_kernel<UV, 1>), dim3(grid), dim3(waves * 64), 0, 0, buf, pieces, iters, out); \
    else hipLaunchKernelGGL((glds_kernel<UV, 2>), dim3(grid), dim3(waves * 64), 0, 0, buf, pieces, iters, out); \
  }
            L(2) L(4) L(8)
#undef L
          };
          launch();
          CK(hipDeviceSynchronize());
          CK(hipEventRecord(e0));
          const int reps = 5;
          for (int r = 0; r < reps; ++r) launch();
          CK(hipEventRecord(e1));
          CK(hipEventSynchronize(e1));
          float ms;
          CK(hipEventElapsedTime(&ms, e0, e1));
          const double us = ms * 1e3 / reps;
          const double bytes = (double)grid * waves * iters * 1024;
          const double tbps = bytes / us / 1e6;
          const double cus = grid < 256 ? grid : 256;
          printf("%d,%d,%d,%d,%.1f,%.2f,%.1f\n", mode, grid, waves, U, us, tbps, bytes / us / 1e-6 / cus / 2.1e9);
        }
  return 0;
}

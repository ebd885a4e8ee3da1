// Streaming-read microbenchmark for decode-GEMV grid design on MI355X (gfx950).
// Each workgroup reads a contiguous slice of T bytes (1 KiB wave-chunks interleaved over its
// waves, U chunks in flight per wave, nontemporal 16 B/lane loads), cache-cold (the slice base
// rotates through a 2 GiB buffer so nothing is served by the 256 MiB Infinity Cache).
// Prints us and TB/s per (T, workgroups, waves, unroll).
//   hipcc -O3 --offload-arch=gfx950 tools/membw.hip -o build/membw && ./build/membw
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

typedef int v4i __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <int U>
__global__ void stream_kernel(const v4i* __restrict__ buf, size_t slice_chunks, size_t total_chunks, int* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  // XCD-spread: consecutive ids land on different XCDs already; slices are id-ordered
  const size_t c0 = (size_t)blockIdx.x * slice_chunks;
  const size_t c1 = c0 + slice_chunks < total_chunks ? c0 + slice_chunks : total_chunks;
  v4i acc = v4i{0, 0, 0, 0};
  for (size_t c = c0 + wave; c < c1; c += (size_t)nw * U) {
    v4i b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t cc = c + (size_t)u * nw;
      b[u] = cc < c1 ? __builtin_nontemporal_load(buf + cc * 64 + lane) : v4i{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= b[u];
  }
  if ((acc[0] ^ acc[1] ^ acc[2] ^ acc[3]) == 0x7fffffff) out[0] = 1;
}

// Same stream plus R reads of a small shared buffer (an activation matrix every workgroup
// re-reads from L2) per weight chunk: does L2-served A traffic cost HBM-stream time?
template <int U, int R>
__global__ void stream_a_kernel(const v4i* __restrict__ buf, const v4i* __restrict__ abuf, int achunks,
                                size_t slice_chunks, size_t total_chunks, int* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const size_t c0 = (size_t)blockIdx.x * slice_chunks;
  const size_t c1 = c0 + slice_chunks < total_chunks ? c0 + slice_chunks : total_chunks;
  v4i acc = v4i{0, 0, 0, 0};
  for (size_t c = c0 + wave; c < c1; c += (size_t)nw * U) {
    v4i b[U], a[U][R > 0 ? R : 1];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t cc = c + (size_t)u * nw;
      b[u] = cc < c1 ? __builtin_nontemporal_load(buf + cc * 64 + lane) : v4i{0, 0, 0, 0};
#pragma unroll
      for (int r = 0; r < R; ++r) a[u][r] = abuf[(size_t)(((cc - c0) * R + r) % achunks) * 64 + lane];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      acc ^= b[u];
#pragma unroll
      for (int r = 0; r < R; ++r) acc += a[u][r];
    }
  }
  if ((acc[0] ^ acc[1] ^ acc[2] ^ acc[3]) == 0x7fffffff) out[0] = 1;
}

template <int U, int R>
float run_a(const char* base, const char* abase, int achunks, size_t buf_bytes, size_t T, int G, int W, int iters) {
  const size_t chunks = T / 1024, slice = (chunks + G - 1) / G, nrot = buf_bytes / T;
  int* out;
  CK(hipMalloc(&out, 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i)
    stream_a_kernel<U, R><<<G, W * 64>>>((const v4i*)(base + (i % nrot) * T), (const v4i*)abase, achunks, slice, chunks, out);
  CK(hipDeviceSynchronize());
  std::vector<float> ts;
  for (int it = 0; it < iters; ++it) {
    CK(hipEventRecord(e0));
    for (int r = 0; r < 10; ++r)
      stream_a_kernel<U, R><<<G, W * 64>>>((const v4i*)(base + ((it * 10 + r + 3) % nrot) * T), (const v4i*)abase,
                                           achunks, slice, chunks, out);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ts.push_back(ms / 10);
  }
  std::sort(ts.begin(), ts.end());
  CK(hipFree(out));
  return ts[ts.size() / 2] * 1e3f;
}

template <int U>
float run(const char* base, size_t buf_bytes, size_t T, int G, int W, int iters) {
  const size_t chunks = T / 1024;
  const size_t slice = (chunks + G - 1) / G;
  int* out;
  CK(hipMalloc(&out, 4));
  const size_t nrot = buf_bytes / T;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i)
    stream_kernel<U><<<G, W * 64>>>((const v4i*)(base + (i % nrot) * T), slice, chunks, out);
  CK(hipDeviceSynchronize());
  std::vector<float> ts;
  for (int it = 0; it < iters; ++it) {
    CK(hipEventRecord(e0));
    for (int r = 0; r < 10; ++r)
      stream_kernel<U><<<G, W * 64>>>((const v4i*)(base + ((it * 10 + r + 3) % nrot) * T), slice, chunks, out);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ts.push_back(ms / 10);
  }
  std::sort(ts.begin(), ts.end());
  CK(hipFree(out));
  return ts[ts.size() / 2] * 1e3f;
}

int main(int argc, char** argv) {
  const size_t buf_bytes = 2ull << 30;
  char* base;
  CK(hipMalloc(&base, buf_bytes));
  CK(hipMemset(base, 1, buf_bytes));
  const size_t Ts[] = {16ull << 20, 50ull << 20, 90ull << 20, 1ull << 30};
  const int Gs[] = {128, 172, 192, 256, 344, 512, 688, 768, 1024, 2048};
  const int Ws[] = {4, 8, 16};
  if (argc > 1 && argv[1][0] == 'a') {
    // T = 16 / 50 MB weight streams, 256 workgroups x 16 waves, U = 2; A = 64 KB or 256 KB shared
    char* abase;
    CK(hipMalloc(&abase, 1 << 20));
    CK(hipMemset(abase, 2, 1 << 20));
    printf("T_MB,A_KB,R,us,TBps_weights\n");
    for (size_t T : {16ull << 20, 50ull << 20})
      for (int akb : {64, 256}) {
        const int ac = akb;   // 1 KiB chunks
        float t0 = run_a<2, 0>(base, abase, ac, buf_bytes, T, 256, 16, 20);
        float t1 = run_a<2, 1>(base, abase, ac, buf_bytes, T, 256, 16, 20);
        float t2 = run_a<2, 2>(base, abase, ac, buf_bytes, T, 256, 16, 20);
        float t4 = run_a<2, 4>(base, abase, ac, buf_bytes, T, 256, 16, 20);
        printf("%zu,%d,0,%.2f,%.2f\n%zu,%d,1,%.2f,%.2f\n%zu,%d,2,%.2f,%.2f\n%zu,%d,4,%.2f,%.2f\n", T >> 20, akb, t0,
               T / t0 * 1e-6, T >> 20, akb, t1, T / t1 * 1e-6, T >> 20, akb, t2, T / t2 * 1e-6, T >> 20, akb, t4,
               T / t4 * 1e-6);
      }
    CK(hipFree(abase));
    CK(hipFree(base));
    return 0;
  }
  printf("T_MB,G,W,U,us,TBps\n");
  for (size_t T : Ts)
    for (int G : Gs)
      for (int W : Ws)
        for (int U : {2, 4, 8}) {
          if (W * 64 * 4 > 1024 && U == 8) continue;
          float us = U == 2 ? run<2>(base, buf_bytes, T, G, W, 20)
                   : U == 4 ? run<4>(base, buf_bytes, T, G, W, 20) : run<8>(base, buf_bytes, T, G, W, 20);
          printf("%zu,%d,%d,%d,%.2f,%.2f\n", T >> 20, G, W, U, us, T / us * 1e-6);
        }
  CK(hipFree(base));
  return 0;
}

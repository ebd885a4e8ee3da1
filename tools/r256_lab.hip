// 256-row W8A8 decode GEMM data-flow lab (standalone, round 5).
//
// Times the production 256-row kernels (ring2: both operands through LDS) against the
// packed-activation kernel w8a8_r256_kernel (ops/csrc/gemm_i8.hip: activations fragment-packed and
// loaded global -> VGPR by the compute waves that own the rows; only the shared weight panel goes
// through the LDS-DMA ring), on the Llama-2-7B decode shapes at 256 rows, and checks that the
// outputs are bit-identical where the two compute the same thing (same split-K slices and epilogue).
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I llm-for-distributed-egde-devices_amd/ops/csrc \
//         tools/r256_lab.hip -o tools/.bin/r256_lab && ./tools/.bin/r256_lab
// Weights are rotated over > 256 MiB of copies, so every call streams them from HBM as in a decode
// step.  One JSON line per (shape, variant, round).
#include "gemm_i8.hip"
#include <functional>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

namespace lab {
// W [N, K] int8 -> MFMA-packed 1 KiB tiles (ops.pack_int8_weight's layout)
__global__ void pack_w_kernel(const int8_t* __restrict__ W, int8_t* __restrict__ Wp, int N, int K) {
  const int KT = K / 64;
  const int64_t total = (int64_t)((N + 15) / 16) * KT * 64;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int l = (int)(i & 63);
    const int64_t tile = i >> 6;
    const int kt = (int)(tile % KT), nt = (int)(tile / KT);
    const int n = min(nt * 16 + (l & 15), N - 1), k0 = kt * 64 + 16 * (l >> 4);
    *reinterpret_cast<v4i*>(Wp + tile * 1024 + l * 16) = *reinterpret_cast<const v4i*>(W + (size_t)n * K + k0);
  }
}
}  // namespace lab

template <typename T>
static T* dev_rand(size_t n, int lo, int hi, float scale = 1.f) {
  std::vector<T> h(n);
  for (auto& v : h) v = (T)(scale * (float)(lo + rand() % (hi - lo + 1)));
  T* d;
  CK(hipMalloc(&d, n * sizeof(T)));
  CK(hipMemcpy(d, h.data(), n * sizeof(T), hipMemcpyHostToDevice));
  return d;
}

static size_t mismatches(const void* a, const void* b, size_t bytes) {
  std::vector<uint8_t> x(bytes), y(bytes);
  CK(hipMemcpy(x.data(), a, bytes, hipMemcpyDeviceToHost));
  CK(hipMemcpy(y.data(), b, bytes, hipMemcpyDeviceToHost));
  size_t bad = 0;
  for (size_t i = 0; i < bytes; ++i) bad += x[i] != y[i];
  return bad;
}

struct Case {
  std::string shape, variant;
  std::function<void(int w)> run;     // w: weight copy index
};

int main() {
  const int M = 256, Mpad = 256;
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  struct Shape { const char* name; int N, K, epi; bool sc; };
  // epi: 0 bf16 out, 2 quantising SwiGLU (gate_up), 3 fp32 split-K slices (o / down, grouped scales)
  const Shape shapes[] = {{"qkv", 12288, 4096, 0, false}, {"gate_up_gluq", 22016, 4096, 2, false},
                          {"o", 4096, 4096, 3, true}, {"down", 4096, 11008, 3, true}};
  for (const Shape& sh : shapes) {
    const int N = sh.N, K = sh.K, KT = K / 64;
    int8_t* A = dev_rand<int8_t>((size_t)M * K, -127, 127);
    int8_t* Ap;
    CK(hipMalloc(&Ap, (size_t)Mpad * K));
    {
      const int64_t total = (int64_t)(Mpad / 16) * KT * 64;
      hipLaunchKernelGGL(pack_a_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, A, Ap, M, K, KT, total);
    }
    float* sa = sh.sc ? dev_rand<float>((size_t)KT * Mpad, 1, 17, 1e-3f) : dev_rand<float>(Mpad, 1, 17, 1e-3f);
    float* sw = dev_rand<float>(N, 1, 13, 1e-3f);
    int8_t* W = dev_rand<int8_t>((size_t)N * K, -127, 127);
    const size_t wbytes = (size_t)((N + 15) / 16) * 16 * K;
    const int copies = (int)((size_t)400 * 1024 * 1024 / wbytes) + 1;
    std::vector<int8_t*> Wp(copies);
    for (int c = 0; c < copies; ++c) {
      CK(hipMalloc(&Wp[c], wbytes));
      hipLaunchKernelGGL(lab::pack_w_kernel, dim3(1024), dim3(256), 0, st, W, Wp[c], N, K);
    }
    const size_t obytes = sh.epi == 3 ? (size_t)4 * M * N * 4 : (size_t)M * N * 2;
    void *o_ref, *o_var;
    float *s_ref = nullptr, *s_var = nullptr;
    CK(hipMalloc(&o_ref, obytes));
    CK(hipMalloc(&o_var, obytes));
    CK(hipMalloc(&s_ref, (size_t)(N / 128 + 1) * Mpad * 4));
    CK(hipMalloc(&s_var, (size_t)(N / 128 + 1) * Mpad * 4));
    std::vector<Case> cases;
    auto chk = [](int rc, const char* what) { if (rc) { printf("%s: rc %d\n", what, rc); exit(1); } };
    if (sh.epi == 0) {
      cases.push_back({sh.name, "production ring2", [&](int w) {
        chk(edge_w8a8_gemm(A, sa, Wp[w], sw, nullptr, o_ref, nullptr, M, N, K, KT, 0, Mpad, 0, st), "prod"); }});
      cases.push_back({sh.name, "r256 NTW6 RG4 RW7 DA3", [&](int w) {
        chk(launch_r256x<6, 4, 1, 2, 7, 3, 2, 32, EPI_OUT, false>(Ap, sa, Wp[w], sw, nullptr, o_var, nullptr, M, N, K, Mpad, 1, st), "r256"); }});
      cases.push_back({sh.name, "r256 NTW6 RG4 RW9 DA4", [&](int w) {
        chk(launch_r256x<6, 4, 1, 2, 9, 4, 2, 32, EPI_OUT, false>(Ap, sa, Wp[w], sw, nullptr, o_var, nullptr, M, N, K, Mpad, 1, st), "r256"); }});
    } else if (sh.epi == 2) {
      cases.push_back({sh.name, "production ring2 gluq", [&](int w) {
        chk(edge_w8a8_gemm(A, sa, Wp[w], sw, nullptr, o_ref, s_ref, M, N, K, KT, 0, Mpad, 2, st), "prod"); }});
      cases.push_back({sh.name, "r256 gluq NTW8 RG4 MS2 RW8", [&](int w) {
        chk(launch_r256x<8, 4, 1, 2, 8, 3, 2, 32, EPI_GLUQ, false>(Ap, sa, Wp[w], sw, nullptr, o_var, s_var, M, N, K, Mpad, 1, st), "r256"); }});
      cases.push_back({sh.name, "r256 gluq NTW16 RG4 TG2 MS2 RW4", [&](int w) {
        chk(launch_r256x<16, 4, 2, 2, 4, 3, 2, 32, EPI_GLUQ, false>(Ap, sa, Wp[w], sw, nullptr, o_var, s_var, M, N, K, Mpad, 1, st), "r256"); }});
      cases.push_back({sh.name, "r256 gluq NTW8 RG8 MS1 RW8", [&](int w) {
        chk(launch_r256x<8, 8, 1, 2, 8, 3, 1, 32, EPI_GLUQ, false>(Ap, sa, Wp[w], sw, nullptr, o_var, s_var, M, N, K, Mpad, 1, st), "r256"); }});
      cases.push_back({sh.name, "r256 gluq NTW8 RG8 MS1 RW8 NWL4", [&](int w) {
        chk(launch_r256x<8, 8, 1, 4, 8, 3, 1, 32, EPI_GLUQ, false>(Ap, sa, Wp[w], sw, nullptr, o_var, s_var, M, N, K, Mpad, 1, st), "r256"); }});
    } else if (K == 4096) {
      cases.push_back({sh.name, "production ring2 splitk S2", [&](int w) {
        chk(edge_w8a8_gemm_splitk(A, sa, Wp[w], sw, nullptr, (float*)o_ref, M, N, K, KT, 1, Mpad, 2, st), "prod"); }});
      cases.push_back({sh.name, "r256 part S2 NTW4 RW8", [&](int w) {
        chk(launch_r256x<4, 4, 1, 2, 8, 3, 2, 16, EPI_PART, true>(Ap, sa, Wp[w], sw, nullptr, o_var, nullptr, M, N, K, Mpad, 2, st), "r256"); }});
      cases.push_back({sh.name, "r256 part S2 NTW2 RW14", [&](int w) {
        chk(launch_r256x<2, 4, 1, 2, 14, 3, 2, 16, EPI_PART, true>(Ap, sa, Wp[w], sw, nullptr, o_var, nullptr, M, N, K, Mpad, 2, st), "r256"); }});
      cases.push_back({sh.name, "r256 out(no split) NTW2 RW14", [&](int w) {
        chk(launch_r256x<2, 4, 1, 2, 14, 3, 2, 32, EPI_OUT, true>(Ap, sa, Wp[w], sw, nullptr, o_var, nullptr, M, N, K, Mpad, 1, st), "r256"); }});
    } else {
      cases.push_back({sh.name, "production ring2 splitk S4", [&](int w) {
        chk(edge_w8a8_gemm_splitk(A, sa, Wp[w], sw, nullptr, (float*)o_ref, M, N, K, KT, 1, Mpad, 4, st), "prod"); }});
      cases.push_back({sh.name, "r256 part S4 NTW8 RW5", [&](int w) {
        chk(launch_r256x<8, 4, 1, 2, 5, 3, 2, 22, EPI_PART, true>(Ap, sa, Wp[w], sw, nullptr, o_var, nullptr, M, N, K, Mpad, 4, st), "r256"); }});
      cases.push_back({sh.name, "r256 part S4 NTW4 RW8", [&](int w) {
        chk(launch_r256x<4, 4, 1, 2, 8, 3, 2, 22, EPI_PART, true>(Ap, sa, Wp[w], sw, nullptr, o_var, nullptr, M, N, K, Mpad, 4, st), "r256"); }});
      cases.push_back({sh.name, "r256 part S2 NTW4 RW8", [&](int w) {
        chk(launch_r256x<4, 4, 1, 2, 8, 3, 2, 43, EPI_PART, true>(Ap, sa, Wp[w], sw, nullptr, o_var, nullptr, M, N, K, Mpad, 2, st), "r256"); }});
    }
    // exactness: variants that compute the production kernel's exact output (same epilogue, same
    // split-K slices) must match it byte for byte
    cases[0].run(0);
    for (size_t v = 1; v < cases.size(); ++v) {
      const std::string& nm = cases[v].variant;
      // (down: production cuts its 43 stages 10 / 11 / 11 / 11, the r256 slices 11 / 11 / 11 / 10)
      const bool same = sh.epi != 3 || (K == 4096 && nm.find("part S2") != std::string::npos);
      if (!same) continue;
      CK(hipMemsetAsync(o_var, 0, obytes, st));
      CK(hipMemsetAsync(s_var, 0, (size_t)(N / 128 + 1) * Mpad * 4, st));
      cases[v].run(0);
      CK(hipStreamSynchronize(st));
      const size_t ob = sh.epi == 2 ? (size_t)M * (N / 2) : sh.epi == 3 ? (size_t)2 * M * N * 4 : obytes;
      size_t bad = mismatches(o_ref, o_var, ob);
      if (sh.epi == 2) bad += mismatches(s_ref, s_var, (size_t)(N / 128) * Mpad * 4);
      double maxrel = 0.0, ref_err = 0.0, var_err = 0.0;
      if (sh.epi == 3 && bad) {
        // fp32 slices: how far apart, and which is closer to the exact (double) slice sums
        std::vector<float> a(2 * (size_t)M * N), b(2 * (size_t)M * N), hs((size_t)KT * Mpad), hw(N);
        std::vector<int8_t> hA((size_t)M * K), hW((size_t)N * K);
        CK(hipMemcpy(a.data(), o_ref, a.size() * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(b.data(), o_var, b.size() * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hs.data(), sa, hs.size() * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hw.data(), sw, hw.size() * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hA.data(), A, hA.size(), hipMemcpyDeviceToHost));
        CK(hipMemcpy(hW.data(), W, hW.size(), hipMemcpyDeviceToHost));
        double amax = 0.0;
        for (size_t i = 0; i < a.size(); ++i) amax = fmax(amax, fabs((double)a[i]));
        int shown = 0;
        for (size_t i = 0; i < a.size(); ++i) {
          maxrel = fmax(maxrel, fabs((double)a[i] - b[i]) / amax);
          if (a[i] != b[i] && shown < 6) {
            ++shown;
            const int ks = (int)(i / ((size_t)M * N)), row = (int)(i / N % M), col = (int)(i % N);
            printf("  diff ks %d row %d col %d: prod %.6g r256 %.6g\n", ks, row, col, a[i], b[i]);
          }
        }
        for (int ks = 0; ks < 2; ++ks)
          for (int row = 0; row < M; row += 37)
            for (int col = 0; col < N; col += 101) {
              double ex = 0.0;
              for (int kt = ks * KT / 2; kt < (ks + 1) * KT / 2; ++kt) {
                long long d = 0;
                for (int k = kt * 64; k < kt * 64 + 64; ++k) d += (long long)hA[(size_t)row * K + k] * hW[(size_t)col * K + k];
                ex += (double)d * hs[(size_t)kt * Mpad + row];
              }
              ex *= hw[col];
              const size_t i = ((size_t)ks * M + row) * N + col;
              ref_err = fmax(ref_err, fabs(a[i] - ex) / amax);
              var_err = fmax(var_err, fabs(b[i] - ex) / amax);
            }
      }
      printf("{\"shape\": \"%s\", \"variant\": \"%s\", \"mismatched_bytes\": %zu, \"max_rel_diff\": %.3g, "
             "\"prod_rel_err\": %.3g, \"var_rel_err\": %.3g}\n", sh.name, nm.c_str(), bad, maxrel, ref_err, var_err);
      fflush(stdout);
      if (bad && sh.epi != 3) exit(2);
    }
    const int iters = 64;
    for (int round = 0; round < 3; ++round)
      for (auto& c : cases) {
        for (int w = 0; w < 6; ++w) c.run(w % copies);
        CK(hipEventRecord(e0, st));
        for (int it = 0; it < iters; ++it) c.run(it % copies);
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("{\"shape\": \"%s\", \"N\": %d, \"K\": %d, \"variant\": \"%s\", \"round\": %d, \"us\": %.2f}\n", sh.name,
               N, K, c.variant.c_str(), round, ms * 1e3f / iters);
        fflush(stdout);
      }
    for (int c = 0; c < copies; ++c) CK(hipFree(Wp[c]));
    CK(hipFree(W));
    CK(hipFree(A));
    CK(hipFree(Ap));
    CK(hipFree(sa));
    CK(hipFree(sw));
    CK(hipFree(o_ref));
    CK(hipFree(o_var));
    CK(hipFree(s_ref));
    CK(hipFree(s_var));
  }
  return 0;
}

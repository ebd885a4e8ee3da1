// HeadInfer offload transfers: strided host<->device copies of KV head blocks on a side stream.
//
// A head block is [B, c heads, L positions, D] carved out of a head-major cache [B, H, S, D]
// (pinned host pool or device staging buffer): for each (batch row, head) it is L*D contiguous
// elements, with a head pitch of S*D elements and a batch pitch of H*S*D.
//
// Two transports:
//  * kernel (default): ONE launch per block. Pinned host memory is mapped into the GPU's address
//    space (hipPointerGetAttributes -> devicePointer), so a grid of B*c workgroups streams the
//    rows with 16-byte vector loads/stores over PCIe/xGMI.  At decode the write-back of the new
//    token is B*c rows of D*2 bytes; issuing those as per-row DMA requests cost ~10 us each
//    (16k requests per step for Llama-3-8B at B=128), so the launch count, not bandwidth, bound
//    the step.  Measured: see docs/BENCHMARKS.md (HeadInfer row).
//  * dma (EDGE_HEADINFER_COPY=dma, or when a pointer is not device-mapped / not 16B aligned):
//    one hipMemcpy2DAsync per batch row on the copy engines.
// Auto choice (mode 0): rows of >= 64 KiB (the history prefetches of long contexts: a 32K-token
// head row is 8 MiB) go to the copy engines (SDMA), so the CUs keep computing attention over the
// resident heads while the next chunk streams in; short rows (the decode write-back of one new
// token per head) take the one-launch kernel.  The return value reports the transport used
// (1 kernel, 2 dma) so tests and the offload statistics can tell them apart.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

namespace {

__global__ void __launch_bounds__(256) head_block_copy_kernel(uint4* __restrict__ dst, int64_t dst_sb, int64_t dst_sh,
                                                              const uint4* __restrict__ src, int64_t src_sb,
                                                              int64_t src_sh, int heads, int64_t row_vec) {
  // strides are in uint4 units; blockIdx.x = b * heads + h
  const int b = blockIdx.x / heads, h = blockIdx.x - b * heads;
  uint4* d = dst + b * dst_sb + h * dst_sh;
  const uint4* s = src + b * src_sb + h * src_sh;
  for (int64_t i = threadIdx.x; i < row_vec; i += blockDim.x) d[i] = s[i];
}

// p itself when the GPU can dereference it (device memory, or pinned host memory mapped at the
// same virtual address under ROCm's unified addressing), else null -> DMA path.
void* device_alias(const void* p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return a.devicePointer == p ? const_cast<void*>(p) : nullptr;
}

bool use_kernel() {
  static int v = [] {
    const char* e = getenv("EDGE_HEADINFER_COPY");
    return (e && strcmp(e, "dma") == 0) ? 0 : 1;
  }();
  return v != 0;
}

}  // namespace

extern "C" int edge_copy_head_block(void* dst, int64_t dst_sb, int64_t dst_sh, const void* src, int64_t src_sb,
                                    int64_t src_sh, int B, int heads, int64_t row_bytes, int elem_bytes,
                                    hipStream_t st, int mode, int* used) {
  *used = 0;
  if (B == 0 || heads == 0 || row_bytes == 0) return 0;
  const int64_t sb_d = dst_sb * elem_bytes, sh_d = dst_sh * elem_bytes;
  const int64_t sb_s = src_sb * elem_bytes, sh_s = src_sh * elem_bytes;
  const bool want_kernel = mode == 1 || (mode == 0 && use_kernel() && row_bytes < (64 << 10));
  if (want_kernel && (row_bytes | sb_d | sh_d | sb_s | sh_s) % 16 == 0) {
    void* dd = device_alias(dst);
    const void* ds = device_alias(src);
    if (dd && ds && (((uintptr_t)dd | (uintptr_t)ds) & 15) == 0 && (int64_t)B * heads <= INT32_MAX) {
      const int64_t row_vec = row_bytes / 16;
      const int threads = row_vec >= 256 ? 256 : (row_vec >= 64 ? 64 : (int)((row_vec + 63) / 64) * 64);
      hipLaunchKernelGGL(head_block_copy_kernel, dim3((unsigned)(B * heads)), dim3(threads), 0, st, (uint4*)dd,
                         sb_d / 16, sh_d / 16, (const uint4*)ds, sb_s / 16, sh_s / 16, heads, row_vec);
      *used = 1;
      return (int)hipGetLastError();
    }
  }
  for (int b = 0; b < B; ++b) {
    char* d = (char*)dst + (size_t)b * sb_d;
    const char* s = (const char*)src + (size_t)b * sb_s;
    hipError_t e = hipMemcpy2DAsync(d, (size_t)sh_d, s, (size_t)sh_s, (size_t)row_bytes, (size_t)heads,
                                    hipMemcpyDefault, st);
    if (e != hipSuccess) return (int)e;
  }
  *used = 2;
  return 0;
}


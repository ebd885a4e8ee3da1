// HeadInfer offload transfers: strided host<->device copies of KV head blocks on a side stream.
//
// A head block is [B, c heads, L positions, D] carved out of a head-major cache [B, H, S, D]
// (pinned host pool or device staging buffer): for each batch row it is c rows of L*D contiguous
// elements with a pitch of S*D elements — one hipMemcpy2DAsync per batch row, no gather/scatter
// kernel and no intermediate host copy (torch would stage a non-contiguous pinned view through
// an unpinned temporary).  DMA engines do the PCIe/xGMI work while the CUs run attention.
#include <hip/hip_runtime.h>
#include <stdint.h>

extern "C" int edge_copy_head_block(void* dst, int64_t dst_sb, int64_t dst_sh, const void* src, int64_t src_sb,
                                    int64_t src_sh, int B, int heads, int64_t row_bytes, int elem_bytes,
                                    hipStream_t st) {
  if (B == 0 || heads == 0 || row_bytes == 0) return 0;
  for (int b = 0; b < B; ++b) {
    char* d = (char*)dst + (size_t)b * dst_sb * elem_bytes;
    const char* s = (const char*)src + (size_t)b * src_sb * elem_bytes;
    hipError_t e = hipMemcpy2DAsync(d, (size_t)dst_sh * elem_bytes, s, (size_t)src_sh * elem_bytes, (size_t)row_bytes,
                                    (size_t)heads, hipMemcpyDefault, st);
    if (e != hipSuccess) return (int)e;
  }
  return 0;
}

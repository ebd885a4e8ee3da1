// Kernel arguments of the batch-1 persistent decode (b1_engine.hip), shared with the host bindings.
#pragma once
#include <stdint.h>

typedef uint16_t b1_bf16_t;

struct B1Params {
  const int8_t* ws;                        // weight streams [G][4][fmax] x 1 KiB
  long long fmax;                          // fragments per wave stream (allocation stride)
  const float* sw_q;                       // [L][NQ] per-output-channel weight scales
  const float* sw_o;                       // [L][H]
  const float* sw_gu;                      // [L][2F] canonical [gate | up] order
  const float* sw_d;                       // [L][H]
  const b1_bf16_t* gam1;                   // [L][H] RMSNorm weights (SmoothQuant smoothing folded in)
  const b1_bf16_t* gam2;
  const float* rope;                       // [max_pos][HD / 2][2] cos, sin
  const b1_bf16_t* x0;                     // [H] embedding of the token
  b1_bf16_t* xout;                         // [H] residual stream after the last layer
  b1_bf16_t* kc;                           // KV cache of batch row 0, layer 0 ([L][B][Hkv][S][HD])
  b1_bf16_t* vc;
  long long kv_l, kv_h;                    // element strides of a layer / a kv head
  const int* pos;                          // position of the new token
  uint64_t* gx;                            // granules: layer inputs x_l      [L][G][gpc_x]
  uint64_t* gq;                            //           qkv                   [L][G][gpc_q]
  uint64_t* ga;                            //           attention out (int8)  [L][Hq][HD / 64][12]
  uint64_t* gr;                            //           h2 = x + o            [L][G][gpc_x]
  uint64_t* gh;                            //           SwiGLU h              [L][G][gpc_h]
  int* ctl;                                // [0] salt, [1] abort, [2] error code
  int L, H, Hq, Hkv, F, NQ;
  float eps, scale;
  int gpc_x, gpc_q, gpc_h;
  int xqb, sxn, scb;                       // LDS carve: activation bytes, scale floats, scratch bytes
  long long* stamps;                       // optional [G][L][24] s_memrealtime stamps (profiling)
};

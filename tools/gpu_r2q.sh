#!/bin/bash
# Round 2 (q): batch-1 Llama-2-7B W8A8 decode latency under launcher variants (EDGELLM_TUNE).
set -o pipefail
mkdir -p gpurun_out/r2q
run() { name=$1; shift; env "$@" timeout -k 10 300 python -u bench.py --micro-batch 1 --lanes 1 --steps 128 --warmup 8 --latency-point off \
  > gpurun_out/r2q/$name.log 2>&1 || { tail -5 gpurun_out/r2q/$name.log; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/r2q/$name.log') if l.startswith('{')][-1]); print('$name', d['value'], d['ms_per_step'], d['p50_token_latency_ms'], d['p90_token_latency_ms'])"; }
run default EDGELLM_TUNE=
run attn_direct EDGELLM_TUNE=decode_attn=32
run gluq8 EDGELLM_TUNE=gemv=8
run default2 EDGELLM_TUNE=

#!/bin/bash
# Round 2 (s): prefill GEMM DMA-issue placement variants (tests + sweep), then the batch-1 job.
set -o pipefail
mkdir -p gpurun_out/r2s
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "prefill" > gpurun_out/r2s/tests.log 2>&1 || { tail -30 gpurun_out/r2s/tests.log; exit 1; }
tail -1 gpurun_out/r2s/tests.log
timeout -k 10 600 python -u tools/bench_ops.py --only pgemm --out gpurun_out/r2s/pgemm.json > gpurun_out/r2s/pgemm.log 2>&1 || exit 1
python3 - <<'PY'
import json
for r in json.load(open('gpurun_out/r2s/pgemm.json')):
    print(r['shape'], r['M'], ' '.join(f"{k[:-5]}={v}" for k, v in r.items() if k.endswith('_TOPs')))
PY
bash tools/gpu_r2r.sh

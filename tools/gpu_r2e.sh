set -o pipefail
mkdir -p gpurun_out/r2e
timeout -k 10 120 python tools/dbg_quant_append.py > gpurun_out/r2e/dbg_qa.log 2>&1; echo dbg rc=$?; cat gpurun_out/r2e/dbg_qa.log | tail -12
timeout -k 10 300 python tools/attn_bench.py --out gpurun_out/r2e/attn_bench.json > gpurun_out/r2e/attn_bench.log 2>&1; echo attn rc=$?; cat gpurun_out/r2e/attn_bench.log | tail -14

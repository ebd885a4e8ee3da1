set -o pipefail
mkdir -p gpurun_out/r2f
timeout -k 10 120 python tools/dbg_quant_append.py > gpurun_out/r2f/dbg_qa.log 2>&1; echo dbg rc=$?; tail -8 gpurun_out/r2f/dbg_qa.log
timeout -k 10 200 python -u -m pytest tests/test_kv_int8.py -v --timeout 100 --timeout-method thread > gpurun_out/r2f/pytest.log 2>&1; rc=$?; echo pytest rc=$rc; grep -E "PASS|FAIL" gpurun_out/r2f/pytest.log | tail -20; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/attn_bench.py --shapes 128x160,128x512,64x160,256x160 --out gpurun_out/r2f/attn_bench.json > gpurun_out/r2f/attn_bench.log 2>&1; echo attn rc=$?; grep op gpurun_out/r2f/attn_bench.log

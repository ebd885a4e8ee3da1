set -o pipefail
mkdir -p gpurun_out/r2h
timeout -k 10 200 python -u -m pytest tests/test_kv_int8.py -q --timeout 100 --timeout-method thread > gpurun_out/r2h/pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -3 gpurun_out/r2h/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/attn_bench.py --shapes 128x160,128x512,64x160,16x2048,1x160 --out gpurun_out/r2h/attn_bench.json > gpurun_out/r2h/attn_bench.log 2>&1; echo attn rc=$?; grep op gpurun_out/r2h/attn_bench.log

# Round 6: pipeline-serving GPU tests and the serving-under-load record (world-1 RCCL vs Generator)
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r6b; mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_pp_slots_gpu.py tests/test_multiproc_gpu.py tests/test_rccl_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1 || exit $?
timeout -k 10 600 python -u tools/serve_load.py --model llama-2-7b --quant w8a8_smoothquant --requests 64 --rate 8 --out $D/serve_load.jsonl > $D/serve_load.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/serve_load.py --model llama-2-7b --quant w8a8_smoothquant --requests 128 --rate 32 --max-batch 128 --out $D/serve_load.jsonl > $D/serve_load_hi.log 2>&1 || exit $?

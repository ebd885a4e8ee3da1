set -o pipefail
mkdir -p gpurun_out/r2l
timeout -k 10 300 python -u -m pytest tests/test_headinfer.py -q --timeout 200 --timeout-method thread > gpurun_out/r2l/pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -3 gpurun_out/r2l/pytest.log; [ $rc -le 1 ] || exit $rc
run() { name=$1; shift; timeout -k 10 400 "$@" > gpurun_out/r2l/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; grep metric gpurun_out/r2l/$name.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ('value','p50_token_latency_ms','prefill_tokens_per_s','ttft_ms','peak_mem_gb','kv_gpu_gb','kv_host_gb','offload')})"; [ $rc -eq 0 ] || exit $rc; }
run l3_32k_res python bench.py --model llama-3-8b --micro-batch 1 --lanes 1 --prompt-len 32768 --steps 8 --warmup 2 --latency-point off
run l3_32k_hi1 python bench.py --model llama-3-8b --micro-batch 1 --lanes 1 --prompt-len 32768 --steps 8 --warmup 2 --latency-point off --headinfer-heads 1 --prefill-chunk 4096
EDGELLM_HEADINFER_COPY_MODE=1 run l3_32k_hi1_kernel python bench.py --model llama-3-8b --micro-batch 1 --lanes 1 --prompt-len 32768 --steps 8 --warmup 2 --latency-point off --headinfer-heads 1 --prefill-chunk 4096
run l3_128k_hi1 python bench.py --model llama-3-8b --micro-batch 1 --lanes 1 --prompt-len 131072 --steps 4 --warmup 1 --latency-point off --headinfer-heads 1 --prefill-chunk 8192

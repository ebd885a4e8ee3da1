# Llama-3-8B W8A8 at a 32K prompt, batch 1, final round-5 tree: resident bf16 KV, and HeadInfer with 7 of 8
# KV heads per layer offloaded (int8 KV) — BASELINE config 4's long-context shape on one GPU
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r5zh; mkdir -p $D
timeout -k 10 400 python3 bench.py --model llama-3-8b --micro-batch 1 --lanes 1 --prompt-len 32768 --steps 8 --warmup 2 --latency-point off > $D/resident.log 2>&1 || exit $?
timeout -k 10 500 python3 bench.py --model llama-3-8b --micro-batch 1 --lanes 1 --prompt-len 32768 --headinfer-heads 1 --kv-dtype int8 --steps 8 --warmup 2 --latency-point off > $D/headinfer_int8.log 2>&1 || exit $?

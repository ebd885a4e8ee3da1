set -o pipefail
D=gpurun_out/r5zi; mkdir -p $D
for r in 1 2; do
timeout -k 10 500 python3 bench.py --model llama-3-8b --micro-batch 1 --lanes 1 --prompt-len 32768 --headinfer-heads 1 --kv-dtype int8 --steps 8 --warmup 2 --latency-point off > $D/hi_$r.log 2>&1 || exit $?
done

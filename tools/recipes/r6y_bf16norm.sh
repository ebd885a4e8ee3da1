# Round 6: 16-bit decode GEMV with the RMSNorm in its prologue — exactness tests, the model test,
# and batch-1 bf16 A/B (ab_old/: norm kernels) on Llama-3.2-1B and Llama-2-7B
set -o pipefail
export PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/r6y; mkdir -p $D
cd $R
timeout -k 10 400 python -u -m pytest tests/test_fused_gpu.py -k "gemv_bf16_norm or norm_fused or split_k or bf16" -x -q --timeout 120 --timeout-method thread > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for m in llama-3.2-1b llama-2-7b; do
for i in 1 2; do
  for v in old new; do
    if [ $v = old ]; then cd $R/ab_old; else cd $R; fi
    timeout -k 10 300 python3 bench.py --model $m --quant none --micro-batch 1 --lanes 1 --steps 64 --warmup 8 --latency-point off > $D/b_${m}_${v}_$i.log 2>&1 || { tail -20 $D/b_${m}_${v}_$i.log; exit 1; }
    echo "$m $v $i $(grep '^{' $D/b_${m}_${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
done

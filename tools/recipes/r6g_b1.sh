# Round 6: the batch-1 persistent decode engine on the GPU: numerics tests, then an interleaved A/B of
# the batch-1 bench (engine on / off)
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r6g; mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_b1_engine_gpu.py -x -v --timeout 300 --timeout-method thread > $D/tests.log 2>&1
rc=$?
tail -15 $D/tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for e in 1 0; do
    EDGELLM_B1_ENGINE=$e timeout -k 10 300 python bench.py --micro-batch 1 --lanes 1 --steps 64 --warmup 8 --latency-point off > $D/bench_b1_e${e}_$i.log 2>&1 || { tail -20 $D/bench_b1_e${e}_$i.log; exit 1; }
    echo "engine=$e run=$i $(grep '^{' $D/bench_b1_e${e}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("p50_token_latency_ms"))')"
  done
done

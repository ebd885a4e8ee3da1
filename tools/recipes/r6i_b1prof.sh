# Round 6: the batch-1 engine: numerics tests, phase timing (in-kernel clocks), batch-1 bench A/B
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r6i; mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_b1_engine_gpu.py -x -q --timeout 300 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -2 $D/tests.log
timeout -k 10 400 python -u tools/b1_profile.py --out $D/prof.json > $D/prof.log 2>&1 || { tail -30 $D/prof.log; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r6i/prof.json"))
print("wall", round(d["wall_ms_mean"], 3), "layer", round(d["layer_us_cu0"], 2))
for k, v in d["phases_us"].items(): print(f"{k:14s}", v)
print("attention", d["attention_us"])
print("down seam", d["down_seam_us"])
for k, v in d["seam_after_last_publish_us"].items(): print("after last publish:", k, v)
PY
for e in 1 0; do
  EDGELLM_B1_ENGINE=$e timeout -k 10 300 python bench.py --micro-batch 1 --lanes 1 --steps 64 --warmup 8 --latency-point off > $D/bench_e$e.log 2>&1 || { tail -20 $D/bench_e$e.log; exit 1; }
  echo "engine=$e $(grep '^{' $D/bench_e$e.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("p50_token_latency_ms"))')"
done

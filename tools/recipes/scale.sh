#!/usr/bin/env bash
# Scaling curve of the headline bench on one node: N = 1, 2, 4, 8 (or the counts given in NS),
# each run `python bench.py --gpus N` (the script starts its own N rank processes, one per GPU,
# RCCL over xGMI) under its own time limit; one JSON line per N appended to OUT.
#   NS="1 2 4 8" STEPS=20 WARMUP=5 OUT=gpurun_out/scale.jsonl bash tools/recipes/scale.sh
# Each line carries world_size, per_rank (compute / P2P wait / bubble / host issue per tick) and
# the modelled stage_cost_spread; efficiency = value(N) / (N * value(1)) is left to the reader.
set -o pipefail
NS=${NS:-"1 2 4 8"}
STEPS=${STEPS:-20}
WARMUP=${WARMUP:-5}
OUT=${OUT:-gpurun_out/scale.jsonl}
LIMIT=${LIMIT:-900}
mkdir -p "$(dirname "$OUT")"
for n in $NS; do
  log="$(dirname "$OUT")/scale_n${n}.log"
  echo "[scale] N=$n -> $log"
  if ! timeout -k 10 "$LIMIT" python bench.py --gpus "$n" --steps "$STEPS" --warmup "$WARMUP" >"$log" 2>&1; then
    echo "[scale] N=$n failed (exit $?); stopping" >&2
    tail -20 "$log" >&2
    exit 1
  fi
  grep '^{' "$log" | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({k: d.get(k) for k in ("n_gpus","world_size","value","ms_per_step","p50_token_latency_ms","bubble_frac_max","stage_cost_spread","per_rank","config")}))' >>"$OUT"
  tail -1 "$OUT"
done

# Round 6: decode-attention occupancy A/B on the default bench (2 x 256)
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r6k; mkdir -p $D
for i in 1 2; do
  for occ in 4 5; do
    EDGELLM_TUNE="decode_attn_occ=$occ" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --latency-point off > $D/b_occ${occ}_$i.log 2>&1 || { tail -20 $D/b_occ${occ}_$i.log; exit 1; }
    echo "occ=$occ run=$i $(grep '^{' $D/b_occ${occ}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done

# Round 6: decode attention microbenchmark (tools/bench_ops.py attn_fused) with the persistent
# direct grid at 0 / 1024 / 2048 / 4096 workgroups
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r6v; mkdir -p $D
for p in 0 1024 2048 4096; do
  timeout -k 10 300 python3 tools/bench_ops.py --only attn_fused --tune decode_attn_pers=$p > $D/p$p.log 2>&1 || { tail -20 $D/p$p.log; exit 1; }
  grep "occ': 4, 'early': 1" $D/p$p.log | sed "s/^/pers=$p /" | sort -u
done

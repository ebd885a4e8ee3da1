# Round 6: persistent direct decode attention (decode_attn_pers = workgroups) on the default bench:
# ab_old/ (before the change) vs this tree with pers 0 / 1024 / 2048, same box, alternating;
# plus the decode-attention tests
set -o pipefail
export PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/r6u; mkdir -p $D
cd $R
timeout -k 10 400 python -u -m pytest tests/test_fused_gpu.py tests/test_kernels_gpu.py -k "decode_attn or attention" -x -q --timeout 120 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for i in 1 2; do
  for v in old p0 p1024 p2048; do
    if [ $v = old ]; then cd $R/ab_old; T=""; else cd $R; T="decode_attn_pers=${v#p}"; fi
    EDGELLM_TUNE="$T" timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --latency-point off > $D/b_${v}_$i.log 2>&1 || { tail -20 $D/b_${v}_$i.log; exit 1; }
    echo "$v $i $(grep '^{' $D/b_${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done

# Round 6: the reference's batch-1 configs on the final tree (+ the one-launch engine on the Llama
# rows), and kernel traces of one batch-1 decode step: launch-per-op path vs the engine
set -o pipefail
export PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/r6l; mkdir -p $D
cd $R
timeout -k 10 500 python3 tools/bench_reference_config.py --modes none,w8a8_smoothquant --repeats 2 > $D/ref.jsonl 2> $D/ref.err || { tail -20 $D/ref.err; exit 1; }
EDGELLM_B1_ENGINE=1 timeout -k 10 300 python3 tools/bench_reference_config.py --models llama-3.2-1b --modes w8a8_smoothquant --repeats 2 > $D/ref_b1.jsonl 2> $D/ref_b1.err || { tail -20 $D/ref_b1.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
for e in 0 1; do
  EDGELLM_B1_ENGINE=$e timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/prof_e$e -o run -- python3 $R/bench.py --micro-batch 1 --lanes 1 --steps 8 --warmup 3 --latency-point off > $D/prof_e$e.log 2>&1 || { tail -20 $D/prof_e$e.log; exit 1; }
done
cd $R
ls -R $D | head -30

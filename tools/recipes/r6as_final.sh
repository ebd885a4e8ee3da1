# Round 6 final tree: the whole GPU suite, smoke(), the default bench (the driver's round-end
# sequence), the reference batch-1 configs and a kernel-stats profile of the default bench
set -o pipefail
export PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/r6as; mkdir -p $D
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -30 $D/gpu_tests.log; exit 1; }
tail -1 $D/gpu_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $D/bench.log 2>&1 || { tail -20 $D/bench.log; exit 1; }
grep '^{' $D/bench.log | cut -c1-300
timeout -k 10 500 python3 tools/bench_reference_config.py --modes none,w8a8_smoothquant --repeats 2 > $D/ref.jsonl 2> $D/ref.err || { tail -20 $D/ref.err; exit 1; }
cat $D/ref.jsonl | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 $R/bench.py --steps 10 --warmup 3 --latency-point off > $D/prof.log 2>&1 || { tail -20 $D/prof.log; exit 1; }
ls $D/prof
cd $R && N=64 bash tools/recipes/r6aq_table3_b1.sh > $D/table3.log 2>&1 || { tail -20 $D/table3.log; exit 1; }
grep -E "rc=|Tokens/Sec" $D/table3.log

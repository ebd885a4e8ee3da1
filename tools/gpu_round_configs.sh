set -o pipefail
mkdir -p gpurun_out/r1b
run() { name=$1; shift; timeout -k 10 240 "$@" > gpurun_out/r1b/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; tail -1 gpurun_out/r1b/$name.log | cut -c1-600; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run l3_8b_int8 python bench.py --model llama-3-8b --steps 32 --warmup 4
run l3_8b_int8_hi4 python bench.py --model llama-3-8b --steps 32 --warmup 4 --headinfer-heads 4
run l2_7b_bf16 python bench.py --quant none --steps 32 --warmup 4
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r1b/prof_hi -o hi -- python3 bench.py --model llama-3-8b --steps 16 --warmup 4 --headinfer-heads 4 > gpurun_out/r1b/prof_hi.log 2>&1; echo prof rc=$?

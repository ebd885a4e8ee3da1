# Round-4: kernel table of Llama-3.2-1B W8A8 at batch 1 (the reference's config, 200 new tokens)
set -o pipefail
export PYTHONUNBUFFERED=1
D=${D:-gpurun_out/r4p1b}; mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- python3 tools/bench_reference_config.py --models llama-3.2-1b --modes w8a8_smoothquant --repeats 2 > $D/prof.log 2>&1 || exit $?

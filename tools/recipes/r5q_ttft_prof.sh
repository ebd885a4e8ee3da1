# kernel table of the 32K-token Llama-3-8B W8A8 prefill (after the all-heads FA order)
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r5q; mkdir -p $D
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/prefill_profile.py --model llama-3-8b --prompt-len 32768 --reps 1 > $GRAFT_REPO_ROOT/$D/ttft.log 2>&1 || exit $?

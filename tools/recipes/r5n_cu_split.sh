# Round 5: CU-partition lab (attention and the 256-row GEMMs on CU-masked streams)
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r5n; mkdir -p $D
timeout -k 10 300 python3 tools/cu_split_lab.py --ctx 150 --reps 8 --splits 48,64,80,96,128 > $D/block.jsonl 2> $D/block.err || exit $?
timeout -k 10 300 python3 tools/cu_split_lab.py --ctx 150 --reps 8 --splits 64,96 --layout stride > $D/stride.jsonl 2> $D/stride.err || exit $?

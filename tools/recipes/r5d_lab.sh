# Round 5: 256-row decode GEMM data-flow lab (tools/r256_lab.hip, built on the CPU side)
set -o pipefail
D=gpurun_out/r5d; mkdir -p $D
timeout -k 10 300 ./tools/.bin/r256_lab > $D/lab.jsonl 2> $D/lab.err || exit $?

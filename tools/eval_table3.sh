#!/bin/bash
# Table-3 single-model rows on one MI355X: the reference's per-sample loop (generate 200 tokens at
# batch 1 + the 7 quality metrics) through cli/evaluate, per precision.  Random-init weights of the
# reference's architectures; questions = the bundled NQ sample (no dataset offline).
set -o pipefail
mkdir -p gpurun_out/eval
E="python3 -m edgellm.cli.evaluate --config configs/single.yaml --num_samples ${N:-10}"
run() { name=$1; shift; timeout -k 10 ${T:-400} "$@" > gpurun_out/eval/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; grep -E "Evaluating|Tokens/Sec|Time Taken|Memory" gpurun_out/eval/$name.log | tail -12; [ $rc -eq 0 ] || exit $rc; }
run fp_bf16   $E
run llm_int8  $E --quant llm_int8
run w8a8      $E --quant w8a8_smoothquant

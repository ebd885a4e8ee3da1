# Round 6: weights-in-VGPR 256-row GEMM (numerics vs ring2, interleaved A/B) + decode attention unroll A/B
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r6c; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_rows256_gpu.py -m gpu -x -q -k "wreg" --timeout 120 --timeout-method thread > $D/tests_wreg.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_fused_gpu.py -m gpu -x -q -k "unroll" --timeout 120 --timeout-method thread > $D/tests_unroll.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/wreg_ab.py --rounds 5 --out $D/wreg_ab.jsonl > $D/wreg_ab.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/attn_bench.py --shapes 256x150,256x200,128x160,64x512 --only bf16,bf16u8,bf16,bf16u8 --out $D/attn_unroll.json > $D/attn_unroll.log 2>&1 || exit $?

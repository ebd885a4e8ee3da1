# Round 5: persistent decode-attention grid — exactness, then the 2-lane A/B on the headline config
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r5a; mkdir -p $D
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_gpu.py -k "persistent or decode_attention_fused" > $D/pytest.log 2>&1 || exit $?
timeout -k 10 900 python3 tools/lane_ab.py --knobs "none;decode_attn_persist=1;decode_attn_persist=2;decode_attn_persist=3" --lanes 2,1 --rounds 2 > $D/lane_ab.jsonl 2> $D/lane_ab.err || exit $?

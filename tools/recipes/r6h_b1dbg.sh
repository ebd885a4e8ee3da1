# Round 6: stage-by-stage check of the batch-1 engine against an fp32 emulation, the HIP launch path
# and the torch reference ops
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r6h; mkdir -p $D
timeout -k 10 300 python -u tools/b1_debug.py --layers 1 > $D/dbg1.log 2>&1 || { tail -30 $D/dbg1.log; exit 1; }
timeout -k 10 300 python -u tools/b1_debug.py --layers 1 --ref > $D/dbg1r.log 2>&1 || { tail -30 $D/dbg1r.log; exit 1; }
tail -20 $D/dbg1r.log
timeout -k 10 300 python -u tools/b1_debug.py --layers 2 --model llama-3-8b --ref > $D/dbg2r.log 2>&1 || { tail -30 $D/dbg2r.log; exit 1; }
tail -30 $D/dbg2r.log

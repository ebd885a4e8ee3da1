set -o pipefail
mkdir -p gpurun_out/r2g
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P1=SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_INSTS_VALU,SQ_INSTS_VMEM_RD,SQ_INSTS_LDS
P2=FETCH_SIZE,GRBM_GUI_ACTIVE,GRBM_COUNT,SQ_BUSY_CYCLES,SQ_WAVES,SQ_INSTS_SALU,SQ_ACTIVE_INST_LDS
timeout -s KILL 120 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d gpurun_out/r2g/p1 -o p1 -- python3 tools/attn_bench.py --shapes 128x160 > gpurun_out/r2g/p1.log 2>&1; echo p1 rc=$?
timeout -s KILL 120 rocprofv3 --pmc $P2 --kernel-trace --output-format csv -d gpurun_out/r2g/p2 -o p2 -- python3 tools/attn_bench.py --shapes 128x160 > gpurun_out/r2g/p2.log 2>&1; echo p2 rc=$?
ls -R gpurun_out/r2g | head -20

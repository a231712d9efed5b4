#!/bin/bash
# PMC passes over K9r (one pass per counter group, each under its own time limit).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
export PYTHONPATH="$GRAFT_REPO_ROOT${PYTHONPATH:+:$PYTHONPATH}"
mkdir -p gpurun_out/r3/pmc
P="python3 scripts/mb_k9r_pmc.py 20000000 256 256 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3/pmc/trace -o k9r -- $P > gpurun_out/r3/pmc/trace.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/r3/pmc/p1 -o p1 -- $P > gpurun_out/r3/pmc/p1.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC -d gpurun_out/r3/pmc/p2 -o p2 -- $P > gpurun_out/r3/pmc/p2.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d gpurun_out/r3/pmc/p3 -o p3 -- $P > gpurun_out/r3/pmc/p3.log 2>&1 || exit 4
echo done

#!/bin/bash
# 32x32 vs 16x16 K9r: ablation (dbg bits) and PMC pass 1 for each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
export PYTHONPATH="$GRAFT_REPO_ROOT${PYTHONPATH:+:$PYTHONPATH}"
mkdir -p gpurun_out/r3/pmc32
timeout -k 10 200 python -u scripts/mb_assign_rr_dbg.py 20000000 256 256 > gpurun_out/r3/ablation_m32.log 2>&1 || exit 1
CML_KMEANS_RR_M32=0 timeout -k 10 200 python -u scripts/mb_assign_rr_dbg.py 20000000 256 256 > gpurun_out/r3/ablation_m16.log 2>&1 || exit 2
P="python3 scripts/mb_k9r_pmc.py 20000000 256 256 0"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/r3/pmc32/p1 -o p1 -- $P > gpurun_out/r3/pmc32/p1.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC -d gpurun_out/r3/pmc32/p2 -o p2 -- $P > gpurun_out/r3/pmc32/p2.log 2>&1 || exit 4
cat gpurun_out/r3/ablation_m32.log gpurun_out/r3/ablation_m16.log

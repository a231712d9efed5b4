set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmc/p1 -o p1 -- python3 scripts/mb_assign_pmc.py > gpurun_out/pmc/p1.log 2>&1 || { tail -5 gpurun_out/pmc/p1.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_COEXEC_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmc/p2 -o p2 -- python3 scripts/mb_assign_pmc.py > gpurun_out/pmc/p2.log 2>&1 || { tail -5 gpurun_out/pmc/p2.log; exit 1; }
find gpurun_out/pmc -name "*.csv" | head

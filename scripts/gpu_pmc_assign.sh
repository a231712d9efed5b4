# PMC passes over the K9 / K9r assign (scripts/mb_assign_pmc.py). usage: bash scripts/gpu_pmc_assign.sh TAG VARIANT N D K [RR_DEBUG]
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-k9}; V=${2:-0}; N=${3:-20000000}; D=${4:-256}; KC=${5:-256}; DBG=${6:-0}
mkdir -p gpurun_out/pmc_$TAG
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmc_$TAG/p1 -o p1 -- python3 scripts/mb_assign_pmc.py $V $N $D $KC $DBG > gpurun_out/pmc_$TAG/p1.log 2>&1 || { tail -5 gpurun_out/pmc_$TAG/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace --output-format csv -d gpurun_out/pmc_$TAG/p2 -o p2 -- python3 scripts/mb_assign_pmc.py $V $N $D $KC $DBG > gpurun_out/pmc_$TAG/p2.log 2>&1 || { tail -5 gpurun_out/pmc_$TAG/p2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum --kernel-trace --output-format csv -d gpurun_out/pmc_$TAG/p3 -o p3 -- python3 scripts/mb_assign_pmc.py $V $N $D $KC $DBG > gpurun_out/pmc_$TAG/p3.log 2>&1 || { tail -5 gpurun_out/pmc_$TAG/p3.log; exit 1; }
find gpurun_out/pmc_$TAG -name "*.csv" | head

set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/benches
CML_TRACE=1 timeout -k 10 600 python bench.py --workload pipeline --steps 2 --warmup 1 > gpurun_out/benches/pipeline_trace.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/benches/pipeline_trace.log | tail -25 | cut -c1-200
exit $rc

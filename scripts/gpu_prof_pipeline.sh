set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_pipe
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pipe -o pipe -- python3 bench.py --workload pipeline --steps 1 --warmup 0 > gpurun_out/prof_pipe/pipe.log 2>&1
rc=$?; grep metric gpurun_out/prof_pipe/pipe.log | cut -c1-300
exit $rc

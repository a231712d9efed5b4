set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_bench
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o bench -- python3 bench.py --steps 10 --warmup 2 > gpurun_out/prof_bench/bench.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/prof_bench/bench.log | tail -3
for f in $(find gpurun_out/prof_bench -name "*kernel_stats.csv"); do cut -d, -f1-8 $f | head -16 | cut -c1-220; done
exit $rc

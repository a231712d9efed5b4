set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/benches
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload pipeline --rows-per-gpu 20000000 --steps 1 --warmup 1 > gpurun_out/benches/pipeline_20M.log 2>&1; rc=$?
tail -3 gpurun_out/benches/pipeline_20M.log | cut -c1-900
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --workload pipeline --steps 2 --warmup 1 > gpurun_out/benches/pipeline_125M.log 2>&1; rc=$?
tail -3 gpurun_out/benches/pipeline_125M.log | cut -c1-900
grep '^{' gpurun_out/benches/pipeline_125M.log > gpurun_out/benches/pipeline_125Mx512_fp8.json
exit $rc

# The 8-GPU shard (12.5M rows of the headline) on one GPU through the multi-rank code path
# (CML_COMM_SELF=1: a one-rank RCCL group whose collectives run): kernel+runtime trace of the timed fit.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4shard
export CML_COMM_SELF=1
timeout -k 10 300 python3 bench.py --rows 12500000 --warmup 3 --no-overlap --breakdown > gpurun_out/r4shard/bench.json 2> gpurun_out/r4shard/bench.err || { tail -5 gpurun_out/r4shard/bench.err; exit 1; }
cut -c1-1500 gpurun_out/r4shard/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --runtime-trace -d gpurun_out/r4shard/tr -o tr -- python3 bench.py --rows 12500000 --warmup 3 --no-overlap > gpurun_out/r4shard/tr.log 2>&1 || { tail -5 gpurun_out/r4shard/tr.log; exit 1; }
python3 scripts/rocpd_stats.py gpurun_out/r4shard/tr/tr_results.db --marker row_pass_kernel --index 1 --top 25

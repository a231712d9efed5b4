#!/bin/bash
# The multi-rank code path on one GPU (CML_COMM_SELF=1: a one-rank RCCL group whose collectives run):
# per-rank shard of the 8-GPU strong-scaling point (12.5M rows), multi-rank path vs single-rank path,
# and kernel traces of the pruned step (graph | RCCL all-reduce | graph) and of the 2-chunk full step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH="$GRAFT_REPO_ROOT${PYTHONPATH:+:$PYTHONPATH}"
out=gpurun_out/selfcomm
mkdir -p $out
timeout -k 10 200 python -u bench.py --rows 12500000 --breakdown > $out/single_rank_12.5M.log 2>&1 || exit 3
tail -1 $out/single_rank_12.5M.log | cut -c1-200
export CML_COMM_SELF=1
timeout -k 10 200 python -u bench.py --rows 12500000 --breakdown > $out/self_rccl_12.5M.log 2>&1 || exit 4
tail -1 $out/self_rccl_12.5M.log | cut -c1-200
timeout -k 10 200 python -u bench.py --rows 12500000 --prune off --chunks 2 > $out/self_rccl_12.5M_full_2chunks.log 2>&1 || exit 5
tail -1 $out/self_rccl_12.5M_full_2chunks.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/$out/prof_pruned" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --rows 12500000 --steps 20 --warmup 1 > "$GRAFT_REPO_ROOT/$out/prof_pruned.log" 2>&1 || exit 6
timeout -k 10 240 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/$out/prof_2chunk" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --rows 12500000 --prune off --chunks 2 --steps 8 --warmup 1 > "$GRAFT_REPO_ROOT/$out/prof_2chunk.log" 2>&1 || exit 7
cd "$GRAFT_REPO_ROOT"
for t in pruned 2chunk; do
  python scripts/rocpd_timeline.py $out/prof_$t/run_results.db --after row_pass_kernel --skip 1 --limit 600 > $out/timeline_$t.txt
  python scripts/rocpd_timeline.py $out/prof_$t/run_results.db --after row_pass_kernel --skip 1 --stats --limit 40 > $out/stats_$t.txt
  python scripts/rocpd_streams.py $out/prof_$t/run_results.db > $out/streams_$t.txt || true
  rm -rf $out/prof_$t
done
echo done

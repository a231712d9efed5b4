# One driver for every GPU-box job (run from the repo root on the box, e.g. through gpurun):
#
#   bash scripts/gpu.sh JOB OUT [args...]      results under gpurun_out/OUT/
#
# JOB:
#   tests [files...]      pytest -m gpu (all of tests/ by default), one process, per-test timeout
#   final                 whole GPU suite, smoke(), headline bench, config-2 f32 fit, config-5 pipeline (trace)
#   bench [bench args]    python bench.py ARGS -> bench.json (+ stderr)
#   pipeline [args]       config-5 pipeline bench with the CML_TRACE stage table
#   profile [bench args]  rocprofv3 kernel trace of bench.py ARGS: per-kernel table of the timed fit
#   shard [bench args]    the 8-GPU shard (12.5M rows) on a one-rank RCCL group: fit breakdown, merged
#                         kernel / blocking-call / roctx timeline, kernel table, host syncs, sync audit
#   strong                strong-scaling emulation: per-rank shards of the headline (100M / N rows)
#   workflow              the reference workflow end to end on 4M uploaded rows (examples/)
#   ovtl [seeded|full]    2-rank gloo timeline of the seeded step's overlapped accumulate, or of the split
#                         full-pass step on overlapping data (rocprofv3 per rank)
#   clock                 K9r clock / MFMA busy share, rows from HBM vs from L2 (one rocprofv3 --pmc pass)
#   drivers               every scripts/mb_*.py subcommand once at a small size, prof.py on a fresh trace
#   mb SCRIPT [args]      a microbenchmark script (scripts/mb_*.py ...) -> SCRIPT.log
#
# Every GPU step runs under its own `timeout -k 10`; steps are chained so a failure ends the job.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=$PWD
JOB=${1:?job}
O=gpurun_out/${2:-$1}
shift 2 || shift $#
mkdir -p "$O"

fit_line() {  # one summary line of a bench.py JSON result
  tail -1 "$1" | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); e = d.get('extra', {}); b = e.get('breakdown') or {}
print(d['metric'][:60], '| value', d['value'], '| ms/step', round(d['ms_per_step'], 3),
      '| fit ms', round(1000 * e.get('fit_s', 0), 2), '| engine', e.get('engine_fit_ms'),
      '| init', b.get('init_ms'), '| steady', e.get('steady_state_ms_per_step'),
      '| overlap fit', (e.get('overlap') or {}).get('fit_ms'))"
}

case "$JOB" in
tests)
  T=${*:-tests}
  timeout -k 10 1100 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu $T \
    > "$O/tests.log" 2>&1 || { tail -40 "$O/tests.log"; exit 1; }
  tail -3 "$O/tests.log"
  ;;
final)
  timeout -k 10 1100 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    > "$O/pytest_gpu.log" 2>&1
  rc=$?
  tail -2 "$O/pytest_gpu.log"
  grep -E "FAILED|Error" "$O/pytest_gpu.log" | head -20
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1 \
    || { tail -5 "$O/smoke.log"; exit 1; }
  tail -1 "$O/smoke.log"
  timeout -k 10 500 python3 bench.py > "$O/bench.json" 2> "$O/bench.err" || { tail -5 "$O/bench.err"; exit 1; }
  fit_line "$O/bench.json"
  timeout -k 10 300 python3 bench.py --rows 10000000 --dim 128 --k 64 --dtype f32 --warmup 1 --steps 20 \
    > "$O/cfg2_f32.json" 2> "$O/cfg2_f32.err" || { tail -5 "$O/cfg2_f32.err"; exit 1; }
  fit_line "$O/cfg2_f32.json"
  CML_TRACE=1 timeout -k 10 600 python3 bench.py --workload pipeline --steps 2 --warmup 1 > "$O/pipe.json" \
    2> "$O/pipe.err" || { tail -20 "$O/pipe.err"; exit 1; }
  cut -c1-240 "$O/pipe.json"
  grep -A12 "^range" "$O/pipe.err"
  ;;
bench)
  timeout -k 10 900 python3 bench.py "$@" > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
  cut -c1-400 "$O/bench.json"
  ;;
pipeline)
  CML_TRACE=1 timeout -k 10 900 python3 bench.py --workload pipeline --steps 2 --warmup 1 "$@" > "$O/pipe.json" \
    2> "$O/pipe.err" || { tail -20 "$O/pipe.err"; exit 1; }
  cut -c1-400 "$O/pipe.json"
  grep -A16 "^range" "$O/pipe.err"
  ;;
profile)
  timeout -k 10 900 rocprofv3 --kernel-trace --stats -d /tmp/pf -o pf -- python3 bench.py "$@" > "$O/run.log" 2>&1 \
    || { tail -20 "$O/run.log"; exit 1; }
  tail -1 "$O/run.log" | cut -c1-400
  python3 scripts/prof.py stats /tmp/pf/pf_results.db --top 50 > "$O/kernel_stats.txt"
  python3 scripts/prof.py stats /tmp/pf/pf_results.db --marker row_pass_kernel --index 1 --top 40 \
    > "$O/kernel_stats_timed_fit.txt"
  head -30 "$O/kernel_stats.txt"
  [ -z "$KEEPDB" ] || cp /tmp/pf/pf_results.db "$O/"  # KEEPDB=1: the trace itself, for scripts/prof.py here
  ;;
shard)
  export CML_COMM_SELF=1
  timeout -k 10 300 python3 bench.py --rows 12500000 --warmup 3 --no-overlap --breakdown "$@" > "$O/shard.json" \
    2> "$O/shard.err" || { tail -5 "$O/shard.err"; exit 1; }
  fit_line "$O/shard.json"
  timeout -k 10 300 rocprofv3 --kernel-trace --runtime-trace --marker-trace -d /tmp/sh -o sh -- python3 bench.py \
    --rows 12500000 --warmup 3 --no-overlap "$@" > "$O/sh.log" 2>&1 || { tail -5 "$O/sh.log"; exit 1; }
  python3 scripts/prof.py timeline /tmp/sh/sh_results.db --marker row_pass_kernel --index 1 --gap-apis 80 --gap-detail 250 \
    > "$O/timeline.txt"
  python3 scripts/prof.py stats /tmp/sh/sh_results.db --marker row_pass_kernel --index 1 --top 40 > "$O/stats.txt"
  python3 scripts/prof.py syncs /tmp/sh/sh_results.db --marker row_pass_kernel --index 1 --show 5 > "$O/syncs.txt"
  timeout -k 10 300 python3 scripts/sync_audit.py --rows 2000000 > "$O/sync_audit.txt" 2>&1 \
    || { tail -20 "$O/sync_audit.txt"; exit 1; }
  head -3 "$O/syncs.txt"
  grep "^window" "$O/timeline.txt"
  head -1 "$O/sync_audit.txt"
  ;;
strong)
  for n in 50000000 25000000 12500000; do
    timeout -k 10 240 python3 bench.py --rows $n --chunks 2 --steps 20 --warmup 3 --no-overlap > "$O/c2_$n.json" \
      2> "$O/c2_$n.err" || { tail -5 "$O/c2_$n.err"; exit 1; }
    CML_COMM_SELF=1 timeout -k 10 240 python3 bench.py --rows $n --steps 20 --warmup 3 --no-overlap \
      > "$O/self_$n.json" 2> "$O/self_$n.err" || { tail -5 "$O/self_$n.err"; exit 1; }
    fit_line "$O/c2_$n.json"
    fit_line "$O/self_$n.json"
  done
  ;;
workflow)
  python3 -c "
import sys; sys.path.insert(0, 'examples')
import hospital_resource_prediction as h
h.synth_uploads('/tmp/wfsrc/hospitals/incoming', n_files=4, rows=1000000)
" || exit 1
  rm -rf /tmp/wf && mkdir -p /tmp/wf && cp -r /tmp/wfsrc/hospitals /tmp/wf/
  t0=$(date +%s.%N)
  timeout -k 10 400 python3 examples/hospital_resource_prediction.py --master mi355x --out /tmp/wf --trace \
    > "$O/workflow.log" 2>&1 || { tail -20 "$O/workflow.log"; exit 1; }
  t1=$(date +%s.%N)
  python3 -c "print('workflow wall s', round($t1 - $t0, 3))"
  grep -A24 "^range" "$O/workflow.log"
  ;;
ovtl)
  # two gloo ranks on the one GPU, one rocprofv3 process each: the seeded step's split accumulate and the
  # order of chunk 0's all-reduce copies against chunk 1's kernels (scripts/overlap_timeline.py)
  P=$((29500 + RANDOM % 400))
  W=${1:-seeded}  # seeded | full
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d /tmp/ov0 -o r0 -- \
    python3 scripts/overlap_timeline.py rank 0 2 $P $W > "$O/r0.log" 2>&1 &
  P0=$!
  S1=0
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d /tmp/ov1 -o r1 -- \
    python3 scripts/overlap_timeline.py rank 1 2 $P $W > "$O/r1.log" 2>&1 || S1=$?
  S0=0
  wait $P0 || S0=$?
  [ $S0 -eq 0 ] && [ $S1 -eq 0 ] || { tail -20 "$O/r0.log" "$O/r1.log"; exit 1; }
  python3 scripts/overlap_timeline.py show /tmp/ov0/r0_results.db /tmp/ov1/r1_results.db > "$O/timeline.txt"
  head -80 "$O/timeline.txt"
  ;;
clock)
  # K9r clock and MFMA busy share with rows from HBM vs from L2 (one PMC pass, kernel trace only)
  R=$PWD
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES \
    --kernel-trace -d /tmp/ck -o ck --output-format csv -- python3 "$R/scripts/mb_k9r.py" clock) > "$O/run.log" 2>&1 \
    || { tail -20 "$O/run.log"; exit 1; }
  python3 scripts/mb_k9r.py clock-show /tmp/ck > "$O/clock.txt"
  cat "$O/clock.txt"
  ;;
drivers)
  # every microbenchmark / trace-reader subcommand once at a small size (a smoke test of the scripts themselves)
  R=$PWD
  M="timeout -k 10 180 python3 -u scripts/mb_k9r.py"
  $M rr 2000000 256 256 0,8 > $O/rr.log 2>&1 && tail -4 $O/rr.log &&
  $M dbg 2000000 > $O/dbg.log 2>&1 && tail -3 $O/dbg.log &&
  $M modes 2000000 > $O/modes.log 2>&1 && tail -3 $O/modes.log &&
  $M pmc-mode 2000000 256 256 1 > $O/pm.log 2>&1 && tail -1 $O/pm.log &&
  $M sched 2000000 0,1 > $O/sched.log 2>&1 && tail -3 $O/sched.log &&
  $M ablate 0 8 > $O/ablate.log 2>&1 && tail -3 $O/ablate.log &&
  (cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace -d /tmp/drv -o p -- python3 "$R/scripts/mb_k9r.py" pmc 8 2000000) > $O/prof.log 2>&1 &&
  python3 scripts/prof.py stats /tmp/drv/p_results.db --top 5 > $O/stats.txt && cat $O/stats.txt &&
  bash scripts/gpu.sh clock "${O#gpurun_out/}/clock" &&
  K="timeout -k 10 180 python3 -u scripts/mb_kmeans.py"
  $K accum --scale 0.02 > $O/accum.log 2>&1 && tail -2 $O/accum.log &&
  $K segacc --rows 2000000 > $O/segacc.log 2>&1 && tail -2 $O/segacc.log &&
  $K overlap --rows 2000000 > $O/overlap.log 2>&1 && tail -1 $O/overlap.log &&
  $K rowpass --rows 4000000 > $O/rowpass.log 2>&1 && tail -1 $O/rowpass.log &&
  $K prune --rows 2000000 --steps 2 --warmup 1 > $O/prune.log 2>&1 && grep untraced $O/prune.log &&
  $K bounds --rows 2000000 > $O/bounds.log 2>&1 && tail -2 $O/bounds.log &&
  $K churn --rows 1000000 --iters 3 > $O/churn.log 2>&1 && tail -1 $O/churn.log &&
  $K graph --rows 1000000 --steps 3 > $O/graph.log 2>&1 && tail -1 $O/graph.log &&
  $K cert --rows 500000 --reps 1 > $O/cert.log 2>&1 && tail -1 $O/cert.log &&
  $K fp8-mx --rows 1000000 --steps 2 > $O/fp8mx.log 2>&1 && tail -1 $O/fp8mx.log &&
  $K host --rows 500000 --iters 3 --top 5 > $O/host.log 2>&1 && head -1 $O/host.log &&
  L="timeout -k 10 180 python3 -u scripts/mb_ml.py"
  $L glm --scale 0.02 > $O/glm.log 2>&1 && tail -1 $O/glm.log &&
  $L glm-fp8 --rows 1000000 > $O/glmfp8.log 2>&1 && tail -1 $O/glmfp8.log &&
  $L logreg --scale 0.02 > $O/logreg.log 2>&1 && tail -1 $O/logreg.log &&
  $L trees --scale 0.02 > $O/trees.log 2>&1 && tail -1 $O/trees.log &&
  $L tree-transform --rows 100000 > $O/tt.log 2>&1 && tail -1 $O/tt.log &&
  Q="timeout -k 10 180 python3 -u scripts/mb_sql.py"
  $Q frame --rows 4000000 --reps 2 > $O/frame.log 2>&1 && tail -2 $O/frame.log | cut -c1-200 &&
  $Q groupby --rows 1000000 > $O/groupby.log 2>&1 && tail -2 $O/groupby.log | cut -c1-200 &&
  $Q relational --rows 1000000 --host-rows 20000 > $O/rel.log 2>&1 && tail -1 $O/rel.log | cut -c1-200 &&
  $Q window --rows 1000000 --host-rows 20000 > $O/win.log 2>&1 && tail -1 $O/win.log &&
  $Q dropna --rows 100000 --reps 1 --dir /tmp/mbd > $O/dropna.log 2>&1 && tail -1 $O/dropna.log &&
  echo ALL_OK
  ;;
mb)
  S=${1:?script}
  shift
  timeout -k 10 600 python3 -u "$S" "$@" > "$O/$(basename "$S" .py).log" 2>&1 \
    || { tail -20 "$O/$(basename "$S" .py).log"; exit 1; }
  grep -v amdgpu.ids "$O/$(basename "$S" .py).log" | tail -40
  ;;
*)
  echo "unknown job $JOB" >&2
  exit 2
  ;;
esac

#!/bin/bash
# Forest shapes of SURVEY §2.3 (20 trees, depth 5, 32 bins; 10M x 4 and 2M x 64): fit times and a kernel
# trace of the histogram / split / route kernels.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH="$GRAFT_REPO_ROOT${PYTHONPATH:+:$PYTHONPATH}"
out=gpurun_out/trees; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/$out/prof" -o run -- python3 "$GRAFT_REPO_ROOT/scripts/mb_trees.py" > "$GRAFT_REPO_ROOT/$out/mb_trees.log" 2>&1 || exit 3
cd "$GRAFT_REPO_ROOT"
grep -E "^RF|^GBT" $out/mb_trees.log
python scripts/rocpd_timeline.py $out/prof/run_results.db --stats --limit 30 > $out/kernel_stats.txt
python - "$out/prof/run_results.db" > $out/hist_kernels.txt <<'PY'
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
q = ("select name, count(*), sum(end-start)/1e6, avg(end-start)/1e3, max(end-start)/1e3, avg(grid_x*grid_y*grid_z/workgroup_x), "
     "avg(lds_size), avg(vgpr_count) from kernels where name like '%tree%' group by name order by 3 desc")
print("kernel | calls | total ms | avg us | max us | avg workgroups | LDS B | VGPRs")
for r in c.execute(q):
    print(f"{r[0][:70]} | {r[1]} | {r[2]:.3f} | {r[3]:.1f} | {r[4]:.1f} | {r[5]:.0f} | {r[6]:.0f} | {r[7]:.0f}")
PY
cat $out/hist_kernels.txt
rm -rf $out/prof

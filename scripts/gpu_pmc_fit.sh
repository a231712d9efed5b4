#!/bin/bash
# PMC passes over one whole headline fit (2 Lloyd steps, no warm-up fit): bytes fetched / L2 hits, and
# SQ busy / wait / VALU counts of the gathered-row kernels (segmented sums, near list, K9r candidate pass),
# the row pass and the bounds pass. One counter group per run (rocprofv3 does not split passes).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH="$GRAFT_REPO_ROOT${PYTHONPATH:+:$PYTHONPATH}"
out="$GRAFT_REPO_ROOT/gpurun_out/pmc_fit"; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum --kernel-trace -d $out/p1 -o p1 -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 0 > $out/p1.log 2>&1 || exit 3
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_ANY --kernel-trace -d $out/p2 -o p2 -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 0 > $out/p2.log 2>&1 || exit 4
cd "$GRAFT_REPO_ROOT"
for kname in kmeans_segacc init_near_list row_pass_kernel kmeans_prune_bounds "kmeans_assign_rr<256, 4, false, 2" "kmeans_assign_rr<256, 5, false, 0" kmeans_scatter init_classify; do
  echo "== $kname"
  python scripts/rocpd_pmc.py $out/p1/p1_results.db $out/p2/p2_results.db --kernel "$kname" 2>&1 | tail -14
done > $out/summary.txt
rm -rf $out/p1 $out/p2
cat $out/summary.txt | head -80

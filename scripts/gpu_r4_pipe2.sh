# Config-5 pipeline: k-means|| per-row path limit and pruned init on/off
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4pipe2}
mkdir -p $O
for v in "CML_KMEANS_INIT_LMAX=0" "CML_KMEANS_INIT_LMAX=2" "CML_KMEANS_INIT_LMAX=8" "CML_KMEANS_INIT_PRUNE=0"; do
  env $v CML_TRACE=1 timeout -k 10 500 python3 bench.py --workload pipeline --steps 2 --warmup 1 > $O/pipe.json 2> $O/pipe.err || { tail -20 $O/pipe.err; exit 1; }
  echo "== $v"; grep -E "Pipeline.fit|kmeans.init|KMeans.fit" $O/pipe.err
done

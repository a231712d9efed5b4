# Config-5 pipeline: 32x32 MFMA K9r variant and a longer pruned-step backoff
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4pipe3}
mkdir -p $O
for v in "CML_KMEANS_RR_M32=1" "CML_KMEANS_PRUNE_BACKOFF=8" "CML_KMEANS_RR_M32=0"; do
  env $v CML_TRACE=1 timeout -k 10 500 python3 bench.py --workload pipeline --steps 2 --warmup 1 > $O/pipe.json 2> $O/pipe.err || { tail -20 $O/pipe.err; exit 1; }
  echo "== $v"; grep -E "Pipeline.fit|kmeans.init|kmeans.step|LogisticRegression.fit" $O/pipe.err
done

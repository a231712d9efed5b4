#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH="$GRAFT_REPO_ROOT${PYTHONPATH:+:$PYTHONPATH}"
mkdir -p gpurun_out/rowpass
for p in 0 0; do
  CML_ROWPASS_PACKED=$p timeout -k 10 200 python -u scripts/mb_rowpass.py >> gpurun_out/rowpass/ab.log 2>&1 || exit 3
done
grep row_pass gpurun_out/rowpass/ab.log


set -o pipefail
cd $GRAFT_REPO_ROOT
python -c "import __graft_entry__ as g; g.build()" > /dev/null 2>&1 || exit 1
timeout -k 10 300 python -m pytest tests -x -q -m gpu 2>&1 | tail -3
PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 300 python scripts/mb_accum.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 400 python bench.py --steps 20 --warmup 3 2>&1 | grep -v amdgpu.ids | tail -2

set -o pipefail
cd $GRAFT_REPO_ROOT
python -c "import __graft_entry__ as g; g.build()" > /dev/null 2>&1 || exit 1
PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 300 python scripts/mb_assign_ablate.py ${VARIANTS} 2>&1 | grep -v amdgpu.ids

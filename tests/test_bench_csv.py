"""BASELINE config 1 plumbing (bench.py --workload csv): CSV -> VectorAssembler -> KMeans k=5 on
local[2] CPU emits one JSON line whose centres equal a numpy Lloyd fixed point."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_csv_workload():
    env = dict(os.environ, CML_FORCE_CPU="1", PYTHONPATH=ROOT)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--workload", "csv", "--steps", "1",
                          "--warmup", "0"], capture_output=True, text=True, env=env, timeout=300, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1]
    res = json.loads(line)
    assert res["config"]["model"] == "KMeans k=5" and res["config"]["dim"] == 16
    assert res["value"] > 0 and res["extra"]["max_center_err_vs_numpy_lloyd"] < 1e-9


def test_bench_two_ranks_cpu_contract():
    """The driver's N > 1 launch (torch.distributed.run, one rank per device) on CPU/gloo: rank 0
    prints exactly one JSON line with the whole-job value, n_gpus = 2 and the headline fields."""
    env = dict(os.environ, CML_FORCE_CPU="1", PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", str(29500 + os.getpid() % 1000),
                          os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
                          "--rows", "20000", "--dim", "16", "--k", "8"],
                         capture_output=True, text=True, env=env, timeout=600, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 0 and res["config"]["parallelism"] == "dp2"  # CPU ranks: no GPUs claimed
    assert res["steps"] == 2 and res["warmup"] == 1 and res["value"] > 0
    for key in ("metric", "unit", "ms_per_step", "higher_is_better", "scaling", "vs_baseline", "dtype", "data",
                "config"):
        assert key in res

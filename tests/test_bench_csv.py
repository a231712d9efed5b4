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

"""The reference script's full intended workflow (examples/hospital_resource_prediction.py)."""
import importlib.util
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load():
    spec = importlib.util.spec_from_file_location("hosp_example",
                                                  os.path.join(ROOT, "examples", "hospital_resource_prediction.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _run(master, tmp_path):
    mod = _load()
    out = mod.main(["--master", master, "--out", str(tmp_path / "hdfs"), "--plots", str(tmp_path / "plots")])
    assert out["lr_rmse"] < 0.6 and out["rf_rmse"] < out["dt_rmse"] * 1.2
    assert out["dt_accuracy"] > 0.85 and out["rf_accuracy"] > 0.85
    assert len(out["batches"]) >= 1
    for m in ("lr", "dt", "rf"):
        assert os.path.exists(tmp_path / "hdfs" / "hospitals" / "models" / "latest_model" / m / "metadata" /
                              "part-00000")
    assert os.path.exists(tmp_path / "plots" / "residuals.png")
    return out


def test_reference_workflow_local(tmp_path):
    _run("local[2]", tmp_path)


@pytest.mark.gpu
def test_reference_workflow_gpu_matches_local(tmp_path):
    gpu = _run("mi355x", tmp_path / "g")
    cpu = _run("local[2]", tmp_path / "c")
    assert abs(gpu["lr_rmse"] - cpu["lr_rmse"]) < 1e-6
    assert abs(gpu["dt_rmse"] - cpu["dt_rmse"]) < 0.05 * cpu["dt_rmse"]
    assert abs(gpu["rf_accuracy"] - cpu["rf_accuracy"]) < 0.03

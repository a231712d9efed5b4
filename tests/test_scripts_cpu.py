"""The measurement scripts stay runnable: scripts/prof.py on synthetic rocprofv3 databases and CSVs, the CPU-capable
scripts/mb_sql.py subcommands at a tiny size, scripts/mb_k9r.py clock-show on a synthetic counter CSV, and every
driver's subcommand list."""
import csv
import importlib.util
import os
import sqlite3
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, "scripts", name + ".py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.fixture()
def trace_db(tmp_path):
    """Two fits opened by a row-pass marker: kernels on queues 1 and 2 (one RCCL kernel), runtime regions."""
    db = str(tmp_path / "t_results.db")
    c = sqlite3.connect(db)
    c.execute("create table kernels(name text, start int, end int, queue_id int)")
    c.execute("create table regions(name text, start int, end int)")
    us = 1000
    ks = [("void (anonymous namespace)::row_pass_kernel<32>(float*)", 0, 100 * us, 1),
          ("kmeans_assign_rr<256, 4>", 150 * us, 400 * us, 1),
          ("ncclDevKernel_AllReduce_Sum_f64", 200 * us, 300 * us, 2),
          ("void (anonymous namespace)::row_pass_kernel<32>(float*)", 1000 * us, 1100 * us, 1),
          ("kmeans_assign_rr<256, 4>", 1200 * us, 1500 * us, 1)]
    c.executemany("insert into kernels values (?,?,?,?)", ks)
    c.executemany("insert into regions values (?,?,?)", [("hipStreamSynchronize", 110 * us, 140 * us),
                                                        ("hipLaunchKernel", 120 * us, 125 * us),
                                                        ("hipMemcpy", 1110 * us, 1190 * us)])
    c.execute("create table counters_collection(dispatch_id int, kernel_name text, counter_name text, value real, "
              "duration int, vgpr_count int, accum_vgpr_count int, sgpr_count int, lds_block_size int)")
    c.executemany("insert into counters_collection values (?,?,?,?,?,?,?,?,?)",
                  [(1, "kmeans_assign_rr", "SQ_BUSY_CYCLES", 10.0, 5, 128, 0, 40, 0),
                   (1, "kmeans_assign_rr", "SQ_BUSY_CYCLES", 5.0, 5, 128, 0, 40, 0),
                   (2, "kmeans_assign_rr", "SQ_BUSY_CYCLES", 30.0, 5, 128, 0, 40, 0)])
    c.commit()
    c.close()
    return db


def test_prof_views(trace_db, capsys):
    prof = load("prof")
    prof.main(["stats", trace_db, "--marker", "row_pass", "--index", "0"])
    out = capsys.readouterr().out
    assert "window: 3 dispatches" in out and "row_pass_kernel<32>" in out and "anonymous" not in out
    prof.main(["timeline", trace_db, "--marker", "row_pass", "--index", "0", "--gap-apis", "10"])
    out = capsys.readouterr().out
    assert "[hipStreamSynchronize]" in out and "gap" in out and "hipLaunchKernel x1" in out
    prof.main(["syncs", trace_db, "--marker", "row_pass", "--index", "1"])
    out = capsys.readouterr().out
    assert "'hipMemcpy': 1" in out and "GPU idle gaps > 20 us after 0 ms: 1" in out
    prof.main(["streams", trace_db, "--after", "row_pass", "--skip", "0"])
    out = capsys.readouterr().out
    assert "1 collective kernels" in out and "(100.0%)" in out
    prof.main(["longcalls", trace_db, "--min-ms", "0.05"])
    assert "hipMemcpy" in capsys.readouterr().out
    prof.main(["pmc", trace_db, "--kernel", "assign"])
    out = capsys.readouterr().out
    assert "dispatches 2" in out and "mean" in out and "22.5" in out  # (15 + 30) / 2


def test_prof_csv_views(tmp_path, capsys):
    prof = load("prof")
    run = tmp_path / "pmc" / "run0"
    run.mkdir(parents=True)
    with open(run / "x_counter_collection.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Dispatch_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp", "VGPR_Count", "Counter_Name",
                    "Counter_Value"])
        w.writerow([7, "kmeans_assign_rr<256>", 0, 1_000_000, 128, "GRBM_GUI_ACTIVE", 8 * 2.0e6])
        w.writerow([7, "kmeans_assign_rr<256>", 0, 1_000_000, 128, "SQ_VALU_MFMA_BUSY_CYCLES", 1024 * 1.0e6])
    prof.main(["pmccsv", str(tmp_path / "pmc"), "assign"])
    out = capsys.readouterr().out
    assert "clock 2.00 GHz" in out and "MFMA busy 50%" in out
    stats = tmp_path / "kernel_stats.csv"
    with open(stats, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "AverageNs", "TotalDurationNs", "Percentage"])
        w.writerow(["void (anonymous namespace)::k<1>(int)", 3, 2e6, 6e6, 75.0])
    prof.main(["kcsv", str(stats), "5"])
    out = capsys.readouterr().out
    assert out.startswith("k<1>") and "6.00 ms" in out


def test_k9r_clock_show(tmp_path, capsys):
    mb = load("mb_k9r")
    with open(tmp_path / "ck_counter_collection.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Dispatch_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp", "Counter_Name", "Counter_Value"])
        for did in range(1, 8):
            w.writerow([did, "rr::kmeans_assign_rr<256>", 0, 1_000_000, "GRBM_GUI_ACTIVE", 8 * 2.0e6])
            w.writerow([did, "rr::kmeans_assign_rr<256>", 0, 1_000_000, "SQ_VALU_MFMA_BUSY_CYCLES", 1024 * 1.3e6])
    mb.cmd_clock_show([str(tmp_path)])
    lines = capsys.readouterr().out.splitlines()
    assert len(lines) == 7 and "rows from HBM" in lines[0] and "rows from L2" in lines[6]
    assert "clock 2.00 GHz, MFMA busy 65.0%" in lines[0]


def test_sql_drivers_on_cpu(capsys):
    mb = load("mb_sql")
    mb.cmd_groupby(["--rows", "3000", "--master", "local[2]"])
    mb.cmd_relational(["--rows", "3000", "--host-rows", "500", "--master", "local[2]"])
    mb.cmd_window(["--rows", "3000", "--host-rows", "500", "--master", "local[2]"])
    out = capsys.readouterr().out
    assert '"path": "python-merge"' in out and '"path": "row-loop"' in out and '"speedup_same_rows"' in out


@pytest.mark.parametrize("name", ["mb_k9r", "mb_kmeans", "mb_ml", "mb_sql"])
def test_driver_lists_subcommands(name):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", name + ".py")], capture_output=True, text=True,
                       timeout=300, cwd=ROOT)
    assert r.returncode == 2 and f"python scripts/{name}.py" in r.stdout


def test_prof_kres_parses_hipcc_remarks(capsys):
    if not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("no hipcc")
    prof = load("prof")
    prof.main(["kres", os.path.join(ROOT, "clustermachinelearningforhospitalnetworks_apache_spark_amd", "_native",
                                    "csrc", "group.hip"), "group_reduce"])
    out = capsys.readouterr().out
    assert "group_reduce_kernel" in out and "vgpr=" in out and "spill=0" in out

"""N0 launcher: rank environment, a distributed job end to end, and failure detection (one dead
rank takes the job down instead of leaving its peers blocked in a collective)."""
import os
import sys
import textwrap
import time

from clustermachinelearningforhospitalnetworks_apache_spark_amd import launch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _script(tmp_path, body):
    p = tmp_path / "app.py"
    p.write_text("import sys\nsys.path.insert(0, %r)\n" % ROOT + textwrap.dedent(body))
    return str(p)


def test_launch_runs_spmd_job(tmp_path):
    out = tmp_path / "out"
    out.mkdir()
    app = _script(tmp_path, f"""
        import os
        from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession
        spark = SparkSession.builder.master("local[1]").getOrCreate()
        df = spark.range(1000)
        n = df.count()
        open(os.path.join({str(out)!r}, f"rank{{spark.rank}}"), "w").write(f"{{spark.world_size}} {{n}}")
        spark.stop()
    """)
    rc = launch.main(["--nproc-per-node", "3", app])
    assert rc == 0
    got = sorted((p.name, p.read_text()) for p in out.iterdir())
    assert got == [("rank0", "3 1000"), ("rank1", "3 1000"), ("rank2", "3 1000")]


def test_launch_failure_stops_peers(tmp_path):
    app = _script(tmp_path, """
        import os, sys, time
        import torch.distributed as dist
        dist.init_process_group("gloo", init_method="env://")
        if int(os.environ["RANK"]) == 1:
            sys.exit(3)
        dist.barrier()          # would block until the collective timeout without the launcher
        time.sleep(600)
    """)
    t0 = time.time()
    rc = launch.main(["--nproc-per-node", "3", "--grace", "2", app])
    assert rc == 3
    assert time.time() - t0 < 60


def test_launch_restarts_failed_job(tmp_path):
    marker = tmp_path / "attempted"
    app = _script(tmp_path, f"""
        import os, sys
        m = {str(marker)!r}
        if os.environ["RANK"] == "0" and not os.path.exists(m):
            open(m, "w").close()
            sys.exit(5)
    """)
    assert launch.main(["--nproc-per-node", "2", "--max-restarts", "1", app]) == 0
    assert marker.exists()


def test_visible_gpu_count_from_kfd_sysfs(tmp_path, monkeypatch):
    """The launcher counts GPUs from the KFD topology (nodes with SIMDs), never through the HIP runtime,
    and honours the *_VISIBLE_DEVICES masks."""
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.launch import visible_gpu_count
    for i, simds in enumerate([0, 0, 1024, 1024, 1024]):  # two CPU nodes, three GPUs
        d = tmp_path / str(i)
        d.mkdir()
        (d / "properties").write_text(f"cpu_cores_count 0\nsimd_count {simds}\nmax_waves_per_simd 8\n")
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(var, raising=False)
    assert visible_gpu_count(str(tmp_path)) == 3
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,2")
    assert visible_gpu_count(str(tmp_path)) == 2
    assert visible_gpu_count(str(tmp_path / "missing")) == 2
    monkeypatch.delenv("HIP_VISIBLE_DEVICES")
    assert visible_gpu_count(str(tmp_path / "missing")) == 0

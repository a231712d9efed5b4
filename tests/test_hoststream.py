"""Host-side pieces of the out-of-core row stream (utils/hoststream.py): chunk boundaries and the HBM
budget knob. The streamed passes themselves run in tests/test_kmeans_stream_gpu.py."""
import torch

from clustermachinelearningforhospitalnetworks_apache_spark_amd.utils.hoststream import (HostRowStream,
                                                                                          hbm_budget_bytes)


def test_chunk_bounds_cover_rows_on_aligned_steps():
    for n, rows in ((100, 32), (0, 32), (1, 1000), (1_000_003, 40_000), (64, 64), (65, 50)):
        b = HostRowStream.chunk_bounds(n, rows)
        assert b[0] == 0 and b[-1] == n
        assert all(b[i] <= b[i + 1] for i in range(len(b) - 1))
        step = max(32, rows // 32 * 32)
        assert all(b[i] % 32 == 0 and b[i] - b[i - 1] == step for i in range(1, len(b) - 1))
        assert len(b) - 1 == max(1, -(-n // step))


def test_budget_knob(monkeypatch):
    cpu = torch.device("cpu")
    assert hbm_budget_bytes(cpu, "12345") == 12345
    assert hbm_budget_bytes(cpu, "1e6") == 1_000_000
    monkeypatch.setenv("CML_HBM_BUDGET_BYTES", "4096")
    assert hbm_budget_bytes(cpu) == 4096
    monkeypatch.delenv("CML_HBM_BUDGET_BYTES")
    assert hbm_budget_bytes(cpu) >= 1 << 60  # no device memory to bound on the CPU


def test_cpu_session_keeps_vector_columns_as_given():
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession
    spark = SparkSession.builder.master("local[1]").getOrCreate()
    spark.conf.set("cml.hbm.budgetBytes", "16")
    try:
        df = spark.createDataFrameFromTensors({"features": torch.randn(100, 4, dtype=torch.float64)})
        assert df._feature_matrix("features").shape == (100, 4)
    finally:
        spark.conf.unset("cml.hbm.budgetBytes")

"""Out-of-core KMeans (utils/hoststream.py): rows in pinned host memory streamed through two
device buffers give the resident fit bit for bit — the k-means|| init picks, every Lloyd step's centres
and labels — for bf16 and fp8 rows, chunk sizes that leave a partial last chunk, and through the public
API with a forced small ``cml.hbm.budgetBytes``."""
import numpy as np
import pytest
import torch

from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine
from clustermachinelearningforhospitalnetworks_apache_spark_amd.utils.hoststream import HostRowStream

pytestmark = pytest.mark.gpu


def _blobs(n, d, k, seed, dtype):
    g = torch.Generator().manual_seed(seed)
    cen = torch.randn(k, d, generator=g) * 3
    x = cen[torch.randint(0, k, (n,), generator=g)] + torch.randn(n, d, generator=g)
    return x.to(dtype)


@pytest.fixture(autouse=True)
def _unpruned_init(monkeypatch):
    # the streamed init runs the unpruned candidate passes; the resident one matches them exactly with
    # its pruned passes off (pruned passes agree only up to near-tie rounding)
    monkeypatch.setenv("CML_KMEANS_INIT_PRUNE", "0")


@pytest.mark.parametrize("n,d,k,dtype,chunk", [(300_001, 256, 64, torch.bfloat16, 40_000),
                                               (120_017, 512, 128, torch.float8_e4m3fn, 16_384),
                                               (50_000, 100, 20, torch.bfloat16, 1 << 20)])
def test_streamed_fit_equals_resident(n, d, k, dtype, chunk):
    xh = _blobs(n, d, k, seed=n, dtype=dtype)
    res = LloydEngine(xh.cuda(), d, k)
    st = LloydEngine(xh, d, k, device=torch.device("cuda"), stream_chunk_rows=chunk)
    assert st._hs is not None and st.x.is_pinned() and not st.x.is_cuda
    assert st.row_chunks == len(HostRowStream.chunk_bounds(n, chunk)) - 1
    i_res = res.init_kmeans_parallel(seed=3)
    i_st = st.init_kmeans_parallel(seed=3)
    assert np.array_equal(i_res, i_st)
    res.set_centers(i_res)
    st.set_centers(i_st)
    for it in range(6):
        res.step()
        st.step()
        torch.cuda.synchronize()
        assert torch.equal(res.centers, st.centers), f"step {it}"
        assert torch.equal(res.labels[:n], st.labels[:n]), f"step {it}"
    # same labels and centres; the resident fit evaluates the cost by the exact f64 cost pass, the streamed
    # full steps sum the assign's per-row f32 distances
    assert st.training_cost() == pytest.approx(res.training_cost(), rel=1e-6)
    lab_r, d_r = res.assign()
    lab_s, d_s = st.assign()
    assert torch.equal(lab_r[:n], lab_s[:n]) and torch.equal(d_r[:n], d_s[:n])
    assert st._hs.passes >= 8 and st._hs.bytes >= 8 * n * st.dp * st.x.element_size()


def test_streamed_h2d_rate_reported():
    n, d, k = 400_000, 512, 32
    st = LloydEngine(_blobs(n, d, k, 1, torch.float8_e4m3fn), d, k, device=torch.device("cuda"),
                     stream_chunk_rows=65_536)
    st.set_centers(st.init_random(seed=1))
    rows = 0
    for _, r0, r1, xc in st._hs.chunks(st.bounds, timed=True):
        rows += xc.shape[0]
    assert rows == n
    gbps = st._hs.last_h2d_gbps()
    assert gbps is not None and gbps > 1.0


def test_budget_conf_streams_the_feature_column():
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.clustering import KMeans
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession
    spark = SparkSession.builder.master("mi355x").getOrCreate()
    n, d, k = 200_003, 64, 12
    xh = _blobs(n, d, k, seed=9, dtype=torch.bfloat16)
    out = {}
    for name, budget in (("resident", None), ("streamed", 1 << 20)):
        if budget is None:
            spark.conf.unset("cml.hbm.budgetBytes")
        else:
            spark.conf.set("cml.hbm.budgetBytes", str(budget))
        df = spark.createDataFrameFromTensors({"features": xh})
        assert df._feature_matrix("features").is_cuda == (budget is None)
        m = KMeans(k=k, seed=4, maxIter=8, tol=0.0).fit(df)
        pred = m.transform(df)
        out[name] = (np.array(m.clusterCenters()), m.summary.clusterSizes, m.summary.trainingCost,
                     pred._numeric("prediction").cpu())
    spark.conf.unset("cml.hbm.budgetBytes")
    assert np.array_equal(out["resident"][0], out["streamed"][0])
    assert out["resident"][1] == out["streamed"][1]
    assert out["streamed"][2] == pytest.approx(out["resident"][2], rel=1e-6)  # cost formulas differ (above)
    assert torch.equal(out["resident"][3], out["streamed"][3])


def test_f32_out_of_core_column_converted_once():
    """an f32 out-of-core column is converted to the pinned bf16 layout ONCE — fit, transform
    and computeCost reuse that copy (and its stream buffers) instead of making a bf16 copy plus a pinned
    copy per call; the host RSS growth over repeated transforms stays far below one matrix."""
    import psutil
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.clustering import KMeans
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession
    spark = SparkSession.builder.master("mi355x").getOrCreate()
    n, d, k = 400_000, 200, 16
    xh = _blobs(n, d, k, seed=12, dtype=torch.float32)
    spark.conf.set("cml.hbm.budgetBytes", str(1 << 20))
    try:
        df = spark.createDataFrameFromTensors({"features": xh})
        col = df._feature_matrix("features")
        assert not col.is_cuda and col.dtype == torch.float32
        m = KMeans(k=k, seed=4, maxIter=4, tol=0.0).fit(df)
        layout = col._cml_hostlayout[2]
        assert layout.is_pinned() and layout.dtype == torch.bfloat16 and layout.shape == (n, 256)
        ptr = layout.data_ptr()
        m.transform(df)._numeric("prediction")
        proc = psutil.Process()
        rss0 = proc.memory_info().rss
        for _ in range(3):
            m.transform(df)._numeric("prediction")
            m.computeCost(df)
        grown = proc.memory_info().rss - rss0
        assert col._cml_hostlayout[2].data_ptr() == ptr
        assert len(layout._cml_streams) == 1
        assert grown < 0.25 * layout.numel() * layout.element_size(), grown
    finally:
        spark.conf.unset("cml.hbm.budgetBytes")

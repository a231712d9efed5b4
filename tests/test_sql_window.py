"""Window functions (sql/window.py) and the extra aggregates against pandas oracles, on one process
and on 2 gloo ranks (partitions spanning ranks)."""
import numpy as np
import pandas as pd
import pytest

from helpers import hospital_frame, hospital_schema, session
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import Window
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import functions as F


def _df(n=300, seed=0):
    s = session()
    pdf = hospital_frame(n, seed=seed)
    pdf = pdf.astype({"emergency_visits": "object"})
    pdf.loc[pdf.index[::17], "emergency_visits"] = None  # real nulls (a float NaN is a value in Spark)
    return s.createDataFrame(pdf, schema=hospital_schema()), pdf


def _collect(df, cols):
    out = df.toPandas()
    return out.sort_values(["hospital_id", "event_time", "admission_count"]).reset_index(drop=True)[cols]


def test_ranking_and_offsets():
    df, pdf = _df()
    w = Window.partitionBy("hospital_id").orderBy("event_time", "admission_count")
    got = _collect(df.select("hospital_id", "event_time", "admission_count", "current_occupancy",
                             F.row_number().over(w).alias("rn"), F.rank().over(w).alias("rk"),
                             F.dense_rank().over(w).alias("dr"), F.lag("current_occupancy", 1).over(w).alias("prev"),
                             F.lead("current_occupancy", 2, -1).over(w).alias("nxt2"),
                             F.percent_rank().over(w).alias("pr"), F.ntile(3).over(w).alias("nt")),
                   ["hospital_id", "event_time", "admission_count", "current_occupancy", "rn", "rk", "dr", "prev",
                    "nxt2", "pr", "nt"])
    ref = pdf.sort_values(["hospital_id", "event_time", "admission_count"]).reset_index(drop=True)
    g = ref.groupby("hospital_id")
    np.testing.assert_array_equal(got.rn.values, g.cumcount().values + 1)
    keys = list(zip(ref.event_time, ref.admission_count))
    ref["k"] = pd.Series(range(len(ref)))
    # ties on (event_time, admission_count) are rare; rank == row_number where unique
    np.testing.assert_array_equal(got.rk.values[~pd.Series(keys).duplicated(keep=False).values],
                                  got.rn.values[~pd.Series(keys).duplicated(keep=False).values])
    prev = g.current_occupancy.shift(1)
    assert got.prev.isna().sum() == ref.hospital_id.nunique()
    np.testing.assert_array_equal(got.prev.dropna().values, prev.dropna().values)
    np.testing.assert_array_equal(got.nxt2.values, g.current_occupancy.shift(-2).fillna(-1).values)
    sizes = g.hospital_id.transform("size").values
    np.testing.assert_allclose(got.pr.values, np.where(sizes > 1, (got.rk.values - 1) / np.maximum(sizes - 1, 1), 0))
    assert set(got.nt.unique()) == {1, 2, 3}


def test_running_and_sliding_aggregates():
    df, pdf = _df()
    w = Window.partitionBy("hospital_id").orderBy("event_time", "admission_count")
    w3 = w.rowsBetween(-2, 0)
    wall = Window.partitionBy("hospital_id")
    got = _collect(df.select("hospital_id", "event_time", "admission_count",
                             F.sum("admission_count").over(w).alias("run_sum"),
                             F.avg("emergency_visits").over(w3).alias("ma3"),
                             F.max("current_occupancy").over(wall).alias("hmax"),
                             F.count("emergency_visits").over(w).alias("cnt"),
                             F.first("admission_count").over(w).alias("first")),
                   ["hospital_id", "run_sum", "ma3", "hmax", "cnt", "first"])
    ref = pdf.sort_values(["hospital_id", "event_time", "admission_count"]).reset_index(drop=True)
    g = ref.groupby("hospital_id")
    np.testing.assert_array_equal(got.run_sum.values, g.admission_count.cumsum().values)
    ma3 = g.emergency_visits.transform(lambda s: s.astype(float).rolling(3, min_periods=1).mean())
    ma3 = ma3.astype(float)
    np.testing.assert_allclose(got.ma3.astype(float).values, ma3.values, rtol=1e-12)
    np.testing.assert_array_equal(got.hmax.values, g.current_occupancy.transform("max").values)
    np.testing.assert_array_equal(got.cnt.values, g.emergency_visits.transform(lambda s: s.notna().cumsum()).values)
    np.testing.assert_array_equal(got["first"].values, g.admission_count.transform("first").values)


def test_range_frame_and_peers():
    s = session()
    pdf = pd.DataFrame({"g": ["a"] * 6 + ["b"] * 3, "t": [1, 2, 2, 4, 7, 8, 1, 1, 5],
                        "v": [1.0, 2.0, 3.0, 4.0, 5.0, 6.0, 10.0, 20.0, 30.0]})
    df = s.createDataFrame(pdf)
    w = Window.partitionBy("g").orderBy("t")
    got = df.select("g", "t", "v", F.sum("v").over(w).alias("run"),
                    F.sum("v").over(w.rangeBetween(-2, 0)).alias("r2"),
                    F.rank().over(w).alias("rk"), F.cume_dist().over(w).alias("cd")).toPandas()
    got = got.sort_values(["g", "t", "v"]).reset_index(drop=True)
    # RANGE default frame includes peers (t = 2 twice; t = 1 twice in b)
    assert got.run.tolist() == [1.0, 6.0, 6.0, 10.0, 15.0, 21.0, 30.0, 30.0, 60.0]
    assert got.r2.tolist() == [1.0, 6.0, 6.0, 9.0, 5.0, 11.0, 30.0, 30.0, 30.0]
    assert got.rk.tolist() == [1, 2, 2, 4, 5, 6, 1, 1, 3]
    np.testing.assert_allclose(got.cd.tolist(), [1 / 6, 3 / 6, 3 / 6, 4 / 6, 5 / 6, 1.0, 2 / 3, 2 / 3, 1.0])


def test_extra_aggregates():
    df, pdf = _df(200, seed=3)
    out = df.groupBy("hospital_id").agg(F.collect_list("admission_count").alias("l"),
                                        F.collect_set("hospital_id").alias("s"),
                                        F.last("current_occupancy").alias("lst"),
                                        F.percentile_approx("current_occupancy", 0.5).alias("med"),
                                        F.percentile_approx("current_occupancy", [0.25, 0.75]).alias("q"),
                                        F.approx_count_distinct("admission_count").alias("nd")).toPandas()
    for _, r in out.iterrows():
        sub = pdf[pdf.hospital_id == r.hospital_id]
        assert sorted(r.l) == sorted(sub.admission_count.tolist())
        assert list(r.s) == [r.hospital_id]
        srt = np.sort(sub.current_occupancy.values)
        assert r.med == srt[int(np.ceil(0.5 * len(srt))) - 1]
        assert list(r.q) == [srt[int(np.ceil(q * len(srt))) - 1] for q in (0.25, 0.75)]
        assert r.nd == sub.admission_count.nunique()


def test_time_window_groupby_tumbling_and_sliding():
    s = session()
    ts = pd.to_datetime(["2025-03-31 21:31:00", "2025-03-31 21:39:59", "2025-03-31 21:40:00",
                         "2025-03-31 21:55:00", "2025-03-31 22:07:30"])
    pdf = pd.DataFrame({"hospital_id": ["H1", "H1", "H2", "H1", "H2"], "event_time": ts,
                        "admission_count": [1, 2, 3, 4, 5]})
    df = s.createDataFrame(pdf)
    tum = (df.groupBy(F.window("event_time", "10 minutes")).agg(F.sum("admission_count").alias("s"))
           .toPandas())
    got = {(r.window.start.strftime("%H:%M"), r.window.end.strftime("%H:%M")): r.s for _, r in tum.iterrows()}
    assert got == {("21:30", "21:40"): 3, ("21:40", "21:50"): 3, ("21:50", "22:00"): 4, ("22:00", "22:10"): 5}
    sl = (df.groupBy("hospital_id", F.window("event_time", "20 minutes", "10 minutes"))
          .agg(F.count("*").alias("n")).toPandas())
    got = {(r.hospital_id, r.window.start.strftime("%H:%M")): r.n for _, r in sl.iterrows()}
    # every row lands in 2 overlapping 20-minute windows
    assert sum(got.values()) == 2 * len(pdf)
    assert got[("H1", "21:20")] == 2 and got[("H1", "21:30")] == 2 and got[("H1", "21:40")] == 1
    assert got[("H2", "21:30")] == 1 and got[("H2", "21:40")] == 1
    one = df.select(F.window("event_time", "1 hour").alias("w")).toPandas()
    assert one.w.iloc[0].start.strftime("%H:%M") == "21:00" and one.w.iloc[-1].end.strftime("%H:%M") == "23:00"


def test_sql_over_clause():
    df, pdf = _df(150, seed=4)
    df.createOrReplaceTempView("ev")
    s = session()
    df.createOrReplaceTempView("ev")
    got = s.sql("SELECT hospital_id, event_time, admission_count, "
                "ROW_NUMBER() OVER (PARTITION BY hospital_id ORDER BY event_time, admission_count) AS rn, "
                "SUM(admission_count) OVER (PARTITION BY hospital_id ORDER BY event_time, admission_count "
                "ROWS BETWEEN 1 PRECEDING AND CURRENT ROW) AS s2, "
                "LAG(admission_count, 1, 0) OVER (PARTITION BY hospital_id ORDER BY event_time, admission_count) AS p "
                "FROM ev").toPandas()
    got = got.sort_values(["hospital_id", "event_time", "admission_count"]).reset_index(drop=True)
    ref = pdf.sort_values(["hospital_id", "event_time", "admission_count"]).reset_index(drop=True)
    g = ref.groupby("hospital_id")
    np.testing.assert_array_equal(got.rn.values, g.cumcount().values + 1)
    np.testing.assert_array_equal(got.s2.values, g.admission_count.transform(lambda v: v.rolling(2, min_periods=1).sum()))
    np.testing.assert_array_equal(got.p.values, g.admission_count.shift(1).fillna(0).values)

"""Stateful structured streaming: groupBy().agg() in complete / update / append (windowed, watermark)
output modes, streaming dropDuplicates, late-row dropping, and exactly-once replay of the state."""
import os

import pandas as pd
import pytest

from helpers import hospital_frame, hospital_schema, session, write_csv_files
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import functions as F


@pytest.fixture()
def spark(tmp_path):
    s = session()
    s.conf.set("spark.sql.warehouse.dir", str(tmp_path / "warehouse"))
    return s


def _src(spark, d):
    return spark.readStream.option("header", True).schema(hospital_schema()).csv(d)


def _run(sdf, ckpt, mode, sink=None, name="agg", fn=None):
    w = sdf.writeStream.outputMode(mode).option("checkpointLocation", ckpt).trigger(availableNow=True)
    if fn is not None:
        w = w.foreachBatch(fn)
    else:
        w = w.format("memory").queryName(name)
    q = w.start()
    q.awaitTermination()
    return q


def test_complete_mode_counts_accumulate(spark, tmp_path):
    src, ck = str(tmp_path / "in"), str(tmp_path / "ck")
    pdf = hospital_frame(200)
    write_csv_files(pdf.iloc[:120], src, nfiles=2, prefix="a")
    agg = _src(spark, src).groupBy("hospital_id").agg(F.count("*").alias("n"), F.sum("admission_count").alias("adm"),
                                                       F.avg("length_of_stay").alias("los"))
    _run(agg, ck, "complete")
    got = {r.hospital_id: (r.n, r.adm) for r in spark.table("agg").collect()}
    ref = pdf.iloc[:120].groupby("hospital_id").agg(n=("hospital_id", "size"), adm=("admission_count", "sum"))
    assert got == {h: (int(r.n), int(r.adm)) for h, r in ref.iterrows()}
    write_csv_files(pdf.iloc[120:], src, nfiles=1, prefix="b")
    _run(agg, ck, "complete")  # restart: the state is reloaded from the checkpoint
    rows = spark.table("agg").collect()
    ref = pdf.groupby("hospital_id").agg(n=("hospital_id", "size"), adm=("admission_count", "sum"),
                                         los=("length_of_stay", "mean"))
    assert {r.hospital_id: (r.n, r.adm) for r in rows} == {h: (int(r.n), int(r.adm)) for h, r in ref.iterrows()}
    for r in rows:
        assert r.los == pytest.approx(ref.loc[r.hospital_id, "los"], rel=1e-12)
    assert len(os.listdir(os.path.join(ck, "state"))) >= 1


def test_update_mode_emits_touched_groups(spark, tmp_path):
    src, ck = str(tmp_path / "in"), str(tmp_path / "ck")
    pdf = hospital_frame(140)
    first = pdf[pdf.hospital_id.isin(["H0", "H1", "H2"])]
    second = pdf[pdf.hospital_id == "H1"]
    write_csv_files(first, src, nfiles=1, prefix="a")
    out = []
    agg = _src(spark, src).groupBy("hospital_id").agg(F.count("*").alias("n"))
    _run(agg, ck, "update", fn=lambda df, bid: out.append((bid, sorted((r.hospital_id, r.n) for r in df.collect()))))
    write_csv_files(second, src, nfiles=1, prefix="b")
    _run(agg, ck, "update", fn=lambda df, bid: out.append((bid, sorted((r.hospital_id, r.n) for r in df.collect()))))
    c = first.hospital_id.value_counts()
    assert out[0] == (0, sorted((h, int(c[h])) for h in ["H0", "H1", "H2"]))
    assert out[1] == (1, [("H1", int(c["H1"]) + len(second))])


def test_append_mode_windows_close_with_watermark(spark, tmp_path):
    src, ck = str(tmp_path / "in"), str(tmp_path / "ck")
    base = hospital_frame(1)
    mk = lambda times: pd.DataFrame([dict(base.iloc[0], event_time=pd.Timestamp(t)) for t in times])  # noqa: E731
    write_csv_files(mk(["2025-04-01 10:01:00", "2025-04-01 10:05:00", "2025-04-01 10:12:00"]), src, 1, "a")
    out = []
    agg = (_src(spark, src).withWatermark("event_time", "5 minutes")
           .groupBy(F.window("event_time", "10 minutes")).agg(F.count("*").alias("n")))
    cb = lambda df, bid: out.append((bid, sorted((str(r.window.start), r.n) for r in df.collect())))  # noqa: E731
    _run(agg, ck, "append", fn=cb)
    # batch 0 starts with watermark 0: nothing is final yet; the watermark becomes 10:12 - 5 min = 10:07
    assert out == [(0, [])]
    # batch 1 starts with watermark 10:07: still nothing ends by then; the late 10:02 row is dropped
    write_csv_files(mk(["2025-04-01 10:02:00", "2025-04-01 10:31:00"]), src, 1, "b")
    _run(agg, ck, "append", fn=cb)
    assert out[-1] == (1, [])
    # batch 2 starts with watermark 10:26: windows [10:00, 10:10) and [10:10, 10:20) are final
    write_csv_files(mk(["2025-04-01 10:33:00"]), src, 1, "c")
    _run(agg, ck, "append", fn=cb)
    assert out[-1] == (2, [("2025-04-01 10:00:00", 2), ("2025-04-01 10:10:00", 1)])


def test_streaming_dedup_and_replay(spark, tmp_path):
    src, ck = str(tmp_path / "in"), str(tmp_path / "ck")
    pdf = hospital_frame(60)
    write_csv_files(pdf, src, nfiles=1, prefix="a")
    write_csv_files(pdf.iloc[:30], src, nfiles=1, prefix="b")  # re-upload of half the rows
    dd = _src(spark, src).dropDuplicates(["hospital_id", "event_time", "admission_count"])
    q = dd.writeStream.format("memory").queryName("dd").option("checkpointLocation", ck).trigger(
        availableNow=True).start()
    q.awaitTermination()
    n_unique = len(pdf.drop_duplicates(["hospital_id", "event_time", "admission_count"]))
    assert spark.table("dd").count() == n_unique
    # complete-mode aggregation: crash before the last commit, replay recomputes from the saved state
    ck2 = str(tmp_path / "ck2")
    agg = _src(spark, src).groupBy("hospital_id").agg(F.count("*").alias("n"))
    _run(agg, ck2, "complete", name="cnt")
    before = {r.hospital_id: r.n for r in spark.table("cnt").collect()}
    last = max(int(f) for f in os.listdir(os.path.join(ck2, "commits")) if f.isdigit())
    os.remove(os.path.join(ck2, "commits", str(last)))
    _run(agg, ck2, "complete", name="cnt")
    assert {r.hospital_id: r.n for r in spark.table("cnt").collect()} == before


def test_output_mode_validation(spark, tmp_path):
    src = str(tmp_path / "in")
    write_csv_files(hospital_frame(10), src, nfiles=1)
    agg = _src(spark, src).groupBy("hospital_id").count()
    with pytest.raises(ValueError):
        agg.writeStream.outputMode("append").format("memory").queryName("x").option(
            "checkpointLocation", str(tmp_path / "c")).start()
    with pytest.raises(ValueError):
        _src(spark, src).writeStream.outputMode("complete").format("memory").queryName("y").option(
            "checkpointLocation", str(tmp_path / "c2")).start()


def _session_rows(df):
    return sorted((r.hospital_id, str(r.session_window.start), str(r.session_window.end), r.n) for r in df.collect())


def test_session_window_merges_across_batches(spark, tmp_path):
    """Streaming session_window: a later event bridges two sessions of earlier batches; complete
    mode equals the batch groupBy over everything seen, update mode emits only merged / new sessions."""
    src, ck = str(tmp_path / "in"), str(tmp_path / "ck")
    base = hospital_frame(1)
    mk = lambda hs: pd.DataFrame([dict(base.iloc[0], hospital_id=h, event_time=pd.Timestamp(t))  # noqa: E731
                                  for h, t in hs])
    b1 = mk([("H0", "2025-04-01 10:00:00"), ("H0", "2025-04-01 10:03:00"), ("H0", "2025-04-01 10:20:00"),
             ("H1", "2025-04-01 10:00:00")])
    b2 = mk([("H0", "2025-04-01 10:11:00"), ("H1", "2025-04-01 11:00:00")])
    b3 = mk([("H0", "2025-04-01 10:24:00")])
    sess = F.session_window("event_time", "10 minutes")
    agg = _src(spark, src).groupBy("hospital_id", sess).agg(F.count("*").alias("n"))
    outs = {"complete": [], "update": []}
    for mode in outs:
        d = str(tmp_path / f"in_{mode}")
        ckm = ck + mode
        for i, b in enumerate((b1, b2, b3)):
            write_csv_files(b, d, 1, f"p{i}")
            a = _src(spark, d).groupBy("hospital_id", sess).agg(F.count("*").alias("n"))
            _run(a, ckm, mode, fn=lambda df, bid, m=mode: outs[m].append(_session_rows(df)))
    allrows = pd.concat([b1, b2, b3])
    batch = spark.createDataFrame(allrows[["hospital_id", "event_time"]])
    ref = _session_rows(batch.groupBy("hospital_id", sess).agg(F.count("*").alias("n")))
    assert outs["complete"][-1] == ref
    # 10:00, 10:03 | 10:20 merge through 10:11 -> one session [10:00, 10:30); 10:24 extends it to 10:34
    assert ("H0", "2025-04-01 10:00:00", "2025-04-01 10:34:00", 5) in ref
    assert outs["update"][1] == [("H0", "2025-04-01 10:00:00", "2025-04-01 10:30:00", 4),
                                 ("H1", "2025-04-01 11:00:00", "2025-04-01 11:10:00", 1)]
    assert outs["update"][2] == [("H0", "2025-04-01 10:00:00", "2025-04-01 10:34:00", 5)]
    assert agg.isStreaming


def test_session_window_append_mode_emits_closed_sessions(spark, tmp_path):
    src, ck = str(tmp_path / "in"), str(tmp_path / "ck")
    base = hospital_frame(1)
    mk = lambda ts: pd.DataFrame([dict(base.iloc[0], hospital_id="H0", event_time=pd.Timestamp(t))  # noqa: E731
                                  for t in ts])
    out = []
    for i, ts in enumerate((["2025-04-01 10:00:00", "2025-04-01 10:04:00"], ["2025-04-01 10:30:00"],
                            ["2025-04-01 11:00:00"], ["2025-04-01 11:30:00"])):
        write_csv_files(mk(ts), src, 1, f"p{i}")
        a = (_src(spark, src).withWatermark("event_time", "5 minutes")
             .groupBy("hospital_id", F.session_window("event_time", "10 minutes")).agg(F.count("*").alias("n")))
        _run(a, ck, "append", fn=lambda df, bid: out.append(_session_rows(df)))
    emitted = [r for b in out for r in b]
    # a session closes in the first batch whose watermark (max event of earlier batches - 5 min)
    # has passed its end: 10:00-10:14 in batch 2, 10:30-10:40 in batch 3
    assert ("H0", "2025-04-01 10:00:00", "2025-04-01 10:14:00", 2) in emitted
    assert ("H0", "2025-04-01 10:30:00", "2025-04-01 10:40:00", 1) in emitted
    assert len(emitted) == len(set(emitted)) == 2 and out[0] == []

"""Property test of the streaming ingest path (ref.py:75-118): any sequence of CSV uploads, micro-batch
runs and crashes (a lost checkpoint commit, with or without the sink's table version) leaves every
uploaded row in the unbounded table exactly once."""
import os
import shutil
import tempfile

from hypothesis import given, settings
from hypothesis import strategies as st

from helpers import hospital_frame, hospital_schema, session, write_csv_files
from clustermachinelearningforhospitalnetworks_apache_spark_amd.io import table as tbl
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import functions as F

_op = st.one_of(
    st.tuples(st.just("upload"), st.integers(1, 40), st.integers(1, 3)),  # rows, files
    st.tuples(st.just("run"), st.just(0), st.just(0)),
    st.tuples(st.just("crash_commit"), st.just(0), st.just(0)),   # crash after the sink commit
    st.tuples(st.just("crash_sink"), st.just(0), st.just(0)),     # crash before the sink commit
)


def _run(spark, src, ckpt, table):
    sdf = (spark.readStream.option("header", True).schema(hospital_schema()).csv(src)
           .withWatermark("event_time", "10 minutes").withColumn("ingest_time", F.current_timestamp()))
    return (sdf.writeStream.format("delta").outputMode("append").option("checkpointLocation", ckpt)
            .trigger(availableNow=True).toTable(table))


@settings(max_examples=int(os.environ.get("CML_PROP_EXAMPLES", 12)), deadline=None)
@given(ops=st.lists(_op, min_size=1, max_size=8))
def test_stream_exactly_once_under_crashes(ops):
    spark = session()
    root = tempfile.mkdtemp(prefix="cml_prop_stream_")
    spark.conf.set("spark.sql.warehouse.dir", os.path.join(root, "wh"))
    src, ckpt = os.path.join(root, "in"), os.path.join(root, "ck")
    os.makedirs(src)
    table = "prop_stream_" + os.path.basename(root).replace("-", "_").lower()
    uploaded, n_up, ran = 0, 0, False
    try:
        for kind, rows, files in ops + [("run", 0, 0)]:
            if kind == "upload":
                write_csv_files(hospital_frame(rows, seed=n_up), src, nfiles=min(files, rows), prefix=f"u{n_up}")
                uploaded += rows
                n_up += 1
            elif kind == "run":
                _run(spark, src, ckpt, table)
                ran = True
            elif ran and os.path.isdir(os.path.join(ckpt, "commits")):
                commits = sorted(int(c) for c in os.listdir(os.path.join(ckpt, "commits")) if c.isdigit())
                if not commits:
                    continue
                os.remove(os.path.join(ckpt, "commits", str(commits[-1])))
                if kind == "crash_sink":
                    tr = spark.catalog._table_path(table)
                    vs = tbl.versions(tr)
                    if vs:
                        os.remove(os.path.join(tr, "_txn_log", f"{vs[-1]:020d}.json"))
        assert spark.table(table).count() == uploaded
        got = sorted(r["length_of_stay"] for r in spark.table(table).select("length_of_stay").collect())
        want = sorted(float(v) for i in range(n_up) for v in
                      hospital_frame([r for k, r, _ in ops if k == "upload"][i], seed=i)["length_of_stay"])
        assert len(got) == len(want) and all(abs(a - b) <= 1e-9 * max(1.0, abs(b)) for a, b in zip(got, want))
    finally:
        spark.catalog.dropTable(table) if hasattr(spark.catalog, "dropTable") else None
        shutil.rmtree(root, ignore_errors=True)

"""Native CSV number parsing: the fast integer / Clinger fast-path double parsers must agree bit for
bit with Python's float() / int() (the strtod/strtoll fallback covers the rest); malformed cells are
null (Spark PERMISSIVE)."""
import numpy as np

from clustermachinelearningforhospitalnetworks_apache_spark_amd.io.csv import parse_csv_bytes, record_starts
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import types as T

CELLS = ["0.1", "1e-5", "123456789012345678901", "1.7976931348623157e308", "-0", "5e-324", ".5", "5.", "+3",
         "3.14159265358979323846", "9007199254740993", "1e22", "1e23", "4.35", "0.000001234", "-2.5E+3", "1e",
         "e5", "abc", "1.2.3", "nan", "inf", "  7.25  ", "", "12345678.123456789", "2.2250738585072014e-308"]


def _py(v):
    v = v.strip()
    try:
        return float(v)
    except ValueError:
        return None


def test_doubles_match_python():
    buf = ("x\n" + "\n".join(c if c else '""' for c in CELLS) + "\n").encode()
    # quoted empty string "" is a non-null empty cell for strings but invalid for doubles
    out, n = parse_csv_bytes(buf, T.StructType([T.StructField("x", T.DoubleType())]), header=True)
    vals, valid = out["x"]
    assert n == len(CELLS)
    for c, v, ok in zip(CELLS, vals, valid):
        ref = _py(c)
        if ref is None:
            assert not ok, c
        else:
            assert ok, c
            assert np.float64(v).tobytes() == np.float64(ref).tobytes() or (np.isnan(v) and np.isnan(ref)), c


def test_ints_and_index():
    cells = ["0", "-17", "+42", "2147483647", "2147483648", "-2147483648", "9223372036854775807", "1.0", "x", " 5 "]
    buf = ("i,l\n" + "\n".join(f"{c},{c}" for c in cells)).encode()  # no trailing newline
    sch = T.StructType([T.StructField("i", T.IntegerType()), T.StructField("l", T.LongType())])
    out, n = parse_csv_bytes(buf, sch, header=True)
    i, iv = out["i"]
    l, lv = out["l"]
    want_i = [0, -17, 42, 2147483647, None, -2147483648, None, None, None, 5]
    want_l = [0, -17, 42, 2147483647, 2147483648, -2147483648, 9223372036854775807, None, None, 5]
    assert [int(a) if ok else None for a, ok in zip(i, iv)] == want_i
    assert [int(a) if ok else None for a, ok in zip(l, lv)] == want_l
    # quoted newlines do not split records, in both the serial and the multithreaded index
    q = b'a,b\n"x\ny",1\n"p""q",2\n\n3,4\n'
    assert list(record_starts(q, True)) == [4, 12, 22]
    big = q[4:] * 100000
    st = record_starts(b"a,b\n" + big, True, nthreads=8)
    assert st.shape[0] == 300000 and st[1] - st[0] == 8

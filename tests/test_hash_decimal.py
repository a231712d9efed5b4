"""hash()/xxhash64() of DecimalType like Spark: the unscaled value as a long (precision <= 18) or the
unscaled BigInteger's two's-complement big-endian bytes (precision > 18); host and device agree."""
from decimal import Decimal

from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import functions as F
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import types as T
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql.hashing import (hash_value, m3_bytes, m3_long,
                                                                                     xx_bytes, xx_long)


def test_decimal_hash_uses_unscaled_value():
    dt = T.DecimalType(10, 2)
    assert hash_value(Decimal("1.10"), dt, 42, "murmur3") == m3_long(110, 42)
    assert hash_value(1.1, dt, 42, "xxhash64") == xx_long(110, 42)
    assert hash_value(Decimal("-3.07"), dt, 42, "murmur3") == m3_long(-307, 42)
    wide = T.DecimalType(30, 3)
    v = Decimal("123456789012345678901.234")
    u = 123456789012345678901234
    assert hash_value(v, wide, 42, "murmur3") == m3_bytes(u.to_bytes((u.bit_length() + 8) // 8, "big", signed=True),
                                                          42)
    assert hash_value(Decimal("-1.000"), wide, 42, "xxhash64") == xx_bytes(b"\xfc\x18", 42)  # -1000
    # BigInteger.toByteArray is minimal for negative powers of two: -128 -> [0x80], -32768 -> [0x80, 0x00]
    w2 = T.DecimalType(38, 2)
    assert hash_value(Decimal("-1.28"), w2, 42, "murmur3") == m3_bytes(b"\x80", 42)
    assert hash_value(Decimal("-327.68"), w2, 42, "xxhash64") == xx_bytes(b"\x80\x00", 42)
    assert hash_value(Decimal("-1.29"), w2, 42, "murmur3") == m3_bytes(b"\xff\x7f", 42)
    assert hash_value(Decimal("1.28"), w2, 42, "murmur3") == m3_bytes(b"\x00\x80", 42)


def test_decimal_column_hash_matches_host():
    spark = SparkSession.builder.master("local[1]").getOrCreate()
    schema = T.StructType([T.StructField("d", T.DecimalType(10, 2))])
    df = spark.createDataFrame([(Decimal("1.10"),), (Decimal("-3.07"),), (None,)], schema)
    got = [r[0] for r in df.select(F.hash("d")).collect()]
    want = [hash_value(v, T.DecimalType(10, 2), 42, "murmur3") for v in (Decimal("1.10"), Decimal("-3.07"))]
    want = [w - (1 << 32) if w >= (1 << 31) else w for w in want] + [42]
    assert got == want

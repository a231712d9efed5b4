"""Checkpointed streaming state is tagged JSON (no pickle): every state value type round-trips, and a
file that is not a state record (e.g. a planted pickle) is refused instead of executed."""
import datetime as dt
import math
import os
import pickle
from decimal import Decimal

import numpy as np
import pytest

from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql.types import Row
from clustermachinelearningforhospitalnetworks_apache_spark_amd.utils import jsonstate


def test_round_trip_of_state_values():
    st = {0: {("h1", dt.datetime(2024, 1, 2, 3, 4, 5, 6)): [1, 2.5, None, math.inf, "x"],
              (Decimal("1.25"), dt.date(2024, 2, 29)): (Row(a=1, b="z"), Row(3, 4)),
              (1, (2, 3)): {frozenset({1, 2}), "s"} and [b"\x00\x01", dt.timedelta(days=1, microseconds=7)]},
          3: {"arr": np.arange(6, dtype=np.float32).reshape(2, 3), "nan": float("nan"), "t": True}}
    back = jsonstate.loads(jsonstate.dumps(st))
    assert set(back) == {0, 3}
    a = back[0]
    assert a[("h1", dt.datetime(2024, 1, 2, 3, 4, 5, 6))][:3] == [1, 2.5, None]
    assert math.isinf(a[("h1", dt.datetime(2024, 1, 2, 3, 4, 5, 6))][3])
    r1, r2 = a[(Decimal("1.25"), dt.date(2024, 2, 29))]
    assert r1.asDict() == {"a": 1, "b": "z"} and tuple(r2) == (3, 4)
    assert a[(1, (2, 3))] == [b"\x00\x01", dt.timedelta(days=1, microseconds=7)]
    assert back[3]["arr"].dtype == np.float32 and back[3]["arr"].tolist() == [[0, 1, 2], [3, 4, 5]]
    assert math.isnan(back[3]["nan"]) and back[3]["t"] is True


def test_unknown_types_fail_at_save():
    with pytest.raises(TypeError):
        jsonstate.dumps({0: object()})


def test_streaming_refuses_non_json_state(tmp_path):
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql.streaming import StreamingQuery  # noqa: F401
    p = tmp_path / "state"
    p.write_bytes(pickle.dumps({0: {}}))
    with pytest.raises(ValueError):
        jsonstate.loads(p.read_bytes().decode("utf-8", errors="strict"))

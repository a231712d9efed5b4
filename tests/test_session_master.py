"""master("mi355x[N]") honours N: a session whose world size differs fails loudly, naming the launcher
(the reference's .master(...) picks the cluster, ref.py:55-58)."""
import pytest

from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql.session import SparkSession, parse_master


def test_parse_master_forms():
    assert parse_master("mi355x[8]") == ("gpu", 8)
    assert parse_master("local[2]") == ("local", 2)
    assert parse_master("mi355x")[1] is None


def test_mi355x_n_requires_matching_world_size(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "1")
    with pytest.raises(ValueError, match="launch --nproc-per-node 8"):
        SparkSession({"spark.master": "mi355x[8]"})
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("RANK", "1")
    with pytest.raises(ValueError, match="WORLD_SIZE=2"):
        SparkSession({"spark.master": "mi355x[4]"})

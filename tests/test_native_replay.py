"""Recorded launch sequences (_native.recording / Recorded, used by the device pruned Lloyd step): calls made
through the wrappers while recording are kept with their arguments converted once, not run; replaying them
calls the same entry points and raises on a non-zero status."""
import ctypes

import pytest

from clustermachinelearningforhospitalnetworks_apache_spark_amd import _native
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import kmeans_ops as K  # noqa: F401  (sigs)


def test_recording_keeps_calls_and_replays_them():
    lib = _native.kernels()
    before = lib.cml_kmeans_set_fp8_mx(-1)  # query, no change
    with _native.recording() as rec:
        assert _native.kernels() is not lib
        st = _native.kernels().cml_kmeans_set_fp8_mx(0)
        assert st == 0  # recorded, not run
    assert _native.kernels() is lib
    assert lib.cml_kmeans_set_fp8_mx(-1) == before  # nothing ran while recording
    assert len(rec.calls) == 1
    fn, conv, name = rec.calls[0]
    assert name == "cml_kmeans_set_fp8_mx" and isinstance(conv[0], ctypes.c_int) and conv[0].value == 0
    seq = _native.Recorded(rec.calls)
    if before:  # replaying "set to 0" returns the previous setting (1): a non-zero status raises
        with pytest.raises(_native.NativeError):
            seq()
    else:
        seq()
    assert lib.cml_kmeans_set_fp8_mx(-1) == 0
    lib.cml_kmeans_set_fp8_mx(before)

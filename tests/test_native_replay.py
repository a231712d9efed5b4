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


class _Holder:
    pass


def test_replay_guard_tracks_buffers_temporaries_and_torch_ops():
    import torch
    h = _Holder()
    h.a = torch.zeros(64, dtype=torch.float32)
    h.parts = [torch.zeros(8, dtype=torch.int32)]
    lib = _native.kernels()

    def rec_of(ptrs):
        r = _native._Recorder(lib)
        r.calls = [(None, tuple(ctypes.c_void_p(p) for p in ptrs), "x")]
        r.torch_ops = []
        return r

    g = _native.ReplayGuard(rec_of([h.a[16:].data_ptr(), h.parts[0].data_ptr(), 0xABC0]), [h], stream=0xABC0)
    assert g.ok and g.valid() and len(g.watch) == 2
    h.parts = [h.parts[0].clone()]  # a re-allocated buffer: the recording is stale
    assert not g.valid()
    tmp = torch.zeros(4)
    g2 = _native.ReplayGuard(rec_of([tmp.data_ptr()]), [h], stream=0)
    assert not g2.ok and "temporary" in g2.why
    with _native.recording() as rec:
        torch.zeros(3).add_(1)  # torch work inside a recording runs now, never on replay
        h.a[:4]  # a view is fine
    assert rec.torch_ops and not _native.ReplayGuard(rec, [h], stream=0).ok


def _engine_fit(x, steps, stream_after=None, realloc_after=None):
    import torch
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine
    eng = LloydEngine(x, x.shape[1], 48)
    eng.set_centers(eng.init_kmeans_parallel(seed=3, as_device=True))
    for it in range(steps):
        if realloc_after is not None and it == realloc_after:
            eng.msgs = eng.msgs.clone()
            eng._pst.ub = eng._pst.ub.clone()
        if stream_after is not None and it >= stream_after:
            side = stream_after_stream[0]
            side.wait_stream(torch.cuda.default_stream())  # (stream semantics: the caller orders the switch)
            with torch.cuda.stream(side):
                eng.step()
        else:
            eng.step()
    torch.cuda.synchronize()
    return eng


stream_after_stream = [None]


@pytest.mark.gpu
def test_replayed_steps_follow_the_stream_and_reallocated_buffers():
    """the recorded pruned-step launches froze the stream and the buffer pointers. A fit
    continued under a non-default stream, and one whose step buffers are re-allocated mid-fit, must re-record
    and give the default fit bit for bit; the default path's sequences must be replayable (no refusal)."""
    import torch
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    c = torch.randn(48, 128, generator=g, device=dev) * 5
    x = (c[torch.randint(0, 48, (300_000,), generator=g, device=dev)]
         + torch.randn(300_000, 128, generator=g, device=dev)).to(torch.bfloat16)
    ref = _engine_fit(x, 10)
    assert ref._pdev
    st = ref._pst
    assert st.replay_refused is None, st.replay_refused
    assert st.replay and all(ent[1].ok for ent in st.replay.values())
    stream_after_stream[0] = torch.cuda.Stream(device=dev)
    side = _engine_fit(x, 10, stream_after=5)
    streams = {k[1] for k in side._pst.replay}
    assert len(streams) == 2, streams
    assert torch.equal(side.centers, ref.centers) and torch.equal(side.labels, ref.labels)
    re = _engine_fit(x, 10, realloc_after=6)
    assert torch.equal(re.centers, ref.centers) and torch.equal(re.labels, ref.labels)
    assert side.training_cost() == ref.training_cost() == re.training_cost()

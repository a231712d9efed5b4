"""K25 group_reduce (_native/csrc/group.hip) against the torch scatter oracle of ops/group_ops.py:
sum / min / max over f64 / f32 / i32 / i64 / u8 columns and the row index, with and without a
mask, group counts 1..2048, and run-to-run bitwise determinism of the f64 sums."""
import pytest
import torch

from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import group_ops


def test_cpu_oracle_matches_python():
    g = torch.tensor([0, 1, 0, 2, 1, 0])
    v = torch.tensor([1.0, 2.0, 3.0, float("nan"), 5.0, -1.0])
    m = ~torch.isnan(v)
    assert group_ops.group_reduce(g, v, 3, "sum", mask=m).tolist() == [3.0, 7.0, 0.0]
    assert group_ops.group_reduce(g, v, 3, "max", mask=m).tolist() == [3.0, 5.0, float("-inf")]
    assert group_ops.group_reduce(g, None, 3, "min", mask=m, floating=False).tolist()[:2] == [0, 1]


@pytest.mark.gpu
@pytest.mark.parametrize("G", [1, 7, 500, 2048])
def test_group_reduce_matches_torch(G):
    dev = torch.device("cuda")
    gen = torch.Generator(device=dev).manual_seed(G)
    n = 1_000_003
    gid = torch.randint(0, G, (n,), device=dev, generator=gen)
    mask = torch.rand(n, device=dev, generator=gen) < 0.9
    cols = {"f64": torch.randn(n, device=dev, dtype=torch.float64, generator=gen) * 100,
            "f32": torch.randn(n, device=dev, generator=gen),
            "i32": torch.randint(-1000, 1000, (n,), device=dev, dtype=torch.int32, generator=gen),
            "i64": torch.randint(-2**40, 2**40, (n,), device=dev, generator=gen),
            "u8": (torch.rand(n, device=dev, generator=gen) < 0.5).to(torch.uint8)}
    for name, v in cols.items():
        for op in ("sum", "min", "max"):
            for mk in (None, mask):
                got = group_ops.group_reduce(gid, v, G, op, mask=mk)
                ref = group_ops._torch_reduce(gid, v, G, op, mk, v.is_floating_point(), n)
                if op == "sum" and v.is_floating_point():
                    torch.testing.assert_close(got, ref, rtol=1e-12, atol=1e-9)
                else:
                    assert torch.equal(got, ref), (name, op)
    for op in ("min", "max"):
        got = group_ops.group_reduce(gid, None, G, op, mask=mask, floating=False)
        assert torch.equal(got, group_ops._torch_reduce(gid, None, G, op, mask, False, n))


@pytest.mark.gpu
def test_group_reduce_deterministic_sums():
    dev = torch.device("cuda")
    gen = torch.Generator(device=dev).manual_seed(3)
    n = 4_000_000
    gid = torch.randint(0, 300, (n,), device=dev, generator=gen)
    v = torch.randn(n, device=dev, dtype=torch.float64, generator=gen) * 1e3
    a = group_ops.group_reduce(gid, v, 300, "sum")
    b = group_ops.group_reduce(gid, v, 300, "sum")
    assert torch.equal(a, b)  # fixed block ranges, wave-private LDS copies, fixed trees


@pytest.mark.gpu
def test_group_reduce_rejects_out_of_range_ids():
    gid = torch.full((1 << 15,), 5, device="cuda", dtype=torch.int64)
    with pytest.raises(ValueError):
        group_ops.group_reduce(gid, torch.ones(1 << 15, device="cuda", dtype=torch.float64), 5, "sum")


@pytest.mark.gpu
@pytest.mark.parametrize("G,d", [(3, 4), (10, 128), (256, 8)])
def test_group_sum_rows_matches_torch(G, d):
    dev = torch.device("cuda")
    gen = torch.Generator(device=dev).manual_seed(G * d)
    n = 300_001
    gid = torch.randint(0, G, (n,), device=dev, generator=gen)
    for dt in (torch.float64, torch.float32):
        x = torch.randn(n, d, device=dev, dtype=dt, generator=gen)
        mask = torch.rand(n, device=dev, generator=gen) < 0.8
        got = group_ops.group_sum_rows(gid, x, G, mask=mask)
        ref = torch.zeros(G, d, dtype=torch.float64, device=dev).index_add_(
            0, gid, torch.where(mask[:, None], x.double(), torch.zeros_like(x.double())))
        torch.testing.assert_close(got, ref, rtol=1e-11, atol=1e-9)
        assert torch.equal(got, group_ops.group_sum_rows(gid, x, G, mask=mask))

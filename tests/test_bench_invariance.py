"""The strong-scaling bench fits ONE problem at every rank count.

bench.py generates every row from its global row index (utils/synth.py) and the fit is
partition-invariant: the k-means|| sampling rate and the training cost are integer-limb sums
(exactsum.hip), the Lloyd sums are exact. So the N-rank launch (torch.distributed.run, one rank per
device — here gloo ranks sharing the CPU or cuda:0) must print the same trainingCost bits and the
same cluster-size histogram as N = 1.
"""
import json
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(n: int, extra, port: int, timeout: int = 300) -> dict:
    env = dict(os.environ, CML_COMM_BACKEND="gloo", PYTHONPATH=ROOT)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", str(n), *extra]
    out = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=timeout, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[0])


def _check(res):
    base = res[0]["extra"]
    for r in res[1:]:
        e = r["extra"]
        assert e["training_cost_hex"] == base["training_cost_hex"], (r["config"]["parallelism"], e, base)
        assert e["cluster_sizes_digest"] == base["cluster_sizes_digest"]
        assert e["iterations"] == base["iterations"]


def test_synth_rows_shards_are_rows_of_one_table():
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.utils import synth
    c = synth.synth_rows(0, 5, 7, seed=3, stream=1) * 4
    whole, lab = synth.synth_rows(0, 1000, 7, seed=1, centres=c, with_labels=True)
    parts = [synth.synth_rows(r0, r1 - r0, 7, seed=1, centres=c) for r0, r1 in
             (synth.shard_range(1000, r, 3) for r in range(3))]
    assert torch.equal(torch.cat(parts), whole)
    assert int(lab.min()) >= 0 and int(lab.max()) < 5 and len(set(lab.tolist())) == 5
    u = synth.synth_rows(10, 4000, 3, seed=2, mode="uniform")
    assert float(u.min()) >= -2.0 and float(u.max()) < 2.0
    z = synth.synth_rows(0, 20000, 4, seed=9)
    assert abs(float(z.mean())) < 0.03 and abs(float(z.std()) - 1.0) < 0.03


def test_bench_cpu_same_problem_at_1_2_ranks():
    extra = ["--steps", "3", "--warmup", "0", "--rows", "30000", "--dim", "16", "--k", "8"]
    _check([_run(n, extra, 29800 + n + os.getpid() % 50) for n in (1, 2)])


@pytest.mark.gpu
def test_bench_gpu_same_problem_at_1_2_4_ranks():
    """The headline bench path (pruned k-means|| init, seeded step, pruned steps) at 2M x 256, k = 256, on
    1, 2 and 4 gloo ranks sharing cuda:0: identical trainingCost bits and cluster sizes."""
    extra = ["--steps", "6", "--warmup", "1", "--rows", "2000000", "--no-overlap"]
    res = [_run(n, extra, 29850 + n + os.getpid() % 50, timeout=110) for n in (1, 2, 4)]
    _check(res)
    assert res[2]["config"]["parallelism"] == "dp4"


@pytest.mark.gpu
def test_synth_rows_kernel_matches_host_twin_and_shards():
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.utils import synth
    dev = torch.device("cuda", 0)
    n, d, ld = 50_000, 33, 40
    c = synth.synth_rows(0, 6, d, seed=3, stream=1, device=dev) * 4
    whole, lab = synth.synth_rows(0, n, d, seed=1, centres=c, dtype=torch.bfloat16, device=dev, ld=ld,
                                  with_labels=True)
    parts = [synth.synth_rows(r0, r1 - r0, d, seed=1, centres=c, dtype=torch.bfloat16, device=dev, ld=ld)
             for r0, r1 in (synth.shard_range(n, r, 4) for r in range(4))]
    assert torch.equal(torch.cat(parts), whole)
    assert not whole[:, d:].any()
    ref, lab_h = synth.synth_rows(0, n, d, seed=1, centres=c.cpu(), dtype=torch.float64, with_labels=True)
    assert torch.equal(lab.cpu(), lab_h)
    err = (whole[:, :d].cpu().double() - ref).abs()
    assert bool((err <= ref.abs() * 2.0 ** -8 + 1e-4).all())


@pytest.mark.gpu
def test_fixsum_exact_and_split_invariant():
    import math
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import kmeans_ops as K
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    v = (torch.rand(1_000_003, generator=g, device=dev) ** 3 * 1000).to(torch.float32)
    v64 = v.double()
    lab = torch.randint(0, 37, (v.numel(),), generator=g, device=dev, dtype=torch.int32)
    bound = v.max().reshape(1)
    whole = K.fixsum(v, v.numel(), bound, 1.0)
    cuts = [0, 1, 400_000, 400_017, v.numel()]
    parts = torch.zeros(2, dtype=torch.int64, device=dev)
    for a, b in zip(cuts[:-1], cuts[1:]):
        parts += K.fixsum(v[a:b].contiguous(), b - a, bound, 1.0)
    # the limbs are not canonical (where a sum is split into 31-bit limbs depends on the partition), their value
    # hi·2^31 + lo is — and so is the finalized f64
    def val(lm, j=0, k=1):
        lm = lm.cpu().tolist()
        return lm[k + j] * 2 ** 31 + lm[j]
    assert val(whole) == val(parts)
    assert torch.equal(K.fixsum_finalize(whole, 1, bound), K.fixsum_finalize(parts, 1, bound))
    tot = float(K.fixsum_finalize(whole, 1, bound)[0])
    exact = math.fsum(v64.cpu().tolist())
    assert abs(tot - exact) <= 1e-13 * exact
    lw = K.fixsum(v64, v.numel(), bound, 1.0, lab=lab, k=37)
    lp = torch.zeros(74, dtype=torch.int64, device=dev)
    for a, b in zip(cuts[:-1], cuts[1:]):
        lp += K.fixsum(v64[a:b].contiguous(), b - a, bound, 1.0, lab=lab[a:b].contiguous(), k=37)
    assert all(val(lw, j, 37) == val(lp, j, 37) for j in range(37))
    assert torch.equal(K.fixsum_finalize(lw, 37, bound), K.fixsum_finalize(lp, 37, bound))
    q = K.fixsum_finalize(lw, 37, bound).cpu()
    for j in (0, 17, 36):
        ex = math.fsum(v64[lab == j].cpu().tolist())
        assert abs(float(q[j]) - ex) <= 1e-13 * ex

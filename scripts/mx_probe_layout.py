"""Operand and scale layout of v_mfma_scale_f32_16x16x128_f8f6f4 on MI355X, through the one-wave probe
kernel (kmeans_mx.hip cml_mx_probe): which output element each A/B byte position feeds, which lane's E8M0
scale applies to each byte, and the scale-value semantics. What it found is what kmeans_rr.h compute_mx and
kmeans_mx_snap_kernel rely on; tests/test_kmeans_mx_gpu.py pins it.

    python scripts/mx_probe_layout.py [layout|values|owners|all]
"""
import sys

import torch

from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import kmeans_ops as K

dev = torch.device("cuda", 0)
ONE = int(torch.tensor([1.0]).to(torch.float8_e4m3fn).view(torch.uint8).item())
ao = torch.full((16, 128), ONE, dtype=torch.uint8)
bo = ao
u = torch.full((64,), 127, dtype=torch.int32)


def run(a, b, sa=None, sb=None):
    sa = u if sa is None else sa
    sb = u if sb is None else sb
    return K.mx_probe(a.to(dev), b.to(dev), sa.to(dev), sb.to(dev)).cpu()


def dec(x):
    return x.view(torch.float8_e4m3fn).double()


def layout():
    # the probe buffer: lane l = (r, g) reads A[r, 32g : 32g + 32] (byte j of its 32 = A[r, 32g + j])
    g = torch.Generator().manual_seed(3)
    a = (torch.randn(16, 128, generator=g) * 8).to(torch.float8_e4m3fn).view(torch.uint8)
    b = (torch.randn(16, 128, generator=g) * 8).to(torch.float8_e4m3fn).view(torch.uint8)
    out = run(a, b).double()
    ref = dec(a) @ dec(b).t()
    print("unit scales: max rel err (out vs A B^T)", ((out - ref).abs() / (dec(a).abs() @ dec(b).abs().t())).max().item())
    print("unit scales: max rel err (out^T vs A B^T)",
          ((out.t() - ref).abs() / (dec(a).abs() @ dec(b).abs().t())).max().item())

    # one-hot A byte at (r, k) against B = ones: which output entries light up
    bo = torch.full((16, 128), ONE, dtype=torch.uint8)
    for (r, k) in [(0, 0), (1, 0), (0, 1), (0, 31), (0, 32), (0, 64), (5, 100), (15, 127)]:
        a1 = torch.zeros(16, 128, dtype=torch.uint8)
        a1[r, k] = ONE
        o = run(a1, bo)
        nz = (o != 0).nonzero().tolist()
        print(f"A one-hot (r={r}, k={k}) -> out nonzero rows {sorted(set(i for i, _ in nz))} cols {len(set(j for _, j in nz))}")
    # one-hot B byte against A = ones
    ao = torch.full((16, 128), ONE, dtype=torch.uint8)
    for (r, k) in [(0, 0), (1, 0), (0, 32), (7, 64)]:
        b1 = torch.zeros(16, 128, dtype=torch.uint8)
        b1[r, k] = ONE
        o = run(ao, b1)
        nz = (o != 0).nonzero().tolist()
        print(f"B one-hot (r={r}, k={k}) -> out nonzero cols {sorted(set(j for _, j in nz))} rows {len(set(i for i, _ in nz))}")
    # k pairing: A one-hot (0, ka), B one-hot (0, kb)
    pairs = []
    for ka in [0, 1, 16, 31, 32, 33, 64, 96, 127]:
        a1 = torch.zeros(16, 128, dtype=torch.uint8)
        a1[0, ka] = ONE
        hits = []
        for kb in range(128):
            b1 = torch.zeros(16, 128, dtype=torch.uint8)
            b1[0, kb] = ONE
            if run(a1, b1)[0, 0].item() != 0:
                hits.append(kb)
        pairs.append((ka, hits))
    print("A k -> B k pairing (row 0, col 0):", pairs)
    # scales: A = ones, B = ones, one lane of sa set to 128 (x2): which outputs double
    for lane in [0, 1, 16, 17, 32, 48, 63]:
        sa = torch.full((64,), 127, dtype=torch.int32)
        sa[lane] = 128
        o = run(ao, bo, sa=sa)
        base = run(ao, bo)
        ch = (o != base).nonzero().tolist()
        print(f"sa[{lane}] = 2: changed rows {sorted(set(i for i, _ in ch))} cols {sorted(set(j for _, j in ch))[:4]}.. "
              f"value {o[ch[0][0], ch[0][1]].item() if ch else None} (base {base[0, 0].item()})")
    for lane in [0, 1, 16, 32]:
        sb = torch.full((64,), 127, dtype=torch.int32)
        sb[lane] = 128
        o = run(ao, bo, sb=sb)
        base = run(ao, bo)
        ch = (o != base).nonzero().tolist()
        print(f"sb[{lane}] = 2: changed rows {sorted(set(i for i, _ in ch))[:4]}.. cols {sorted(set(j for _, j in ch))} "
              f"value {o[ch[0][0], ch[0][1]].item() if ch else None}")


def values():
    g = torch.Generator().manual_seed(3)
    u = torch.full((64,), 127, dtype=torch.int32)
    for v in [100, 118, 120, 126, 127, 128, 130, 135, 140, 160, 200]:
        sa = u.clone()
        sa[0] = v
        o = run(ao, ao, sa, u)
        print(f"sa[0] = {v}: out[0,0] = {o[0, 0].item()} (expect {96 + 32 * 2.0 ** (v - 127)})")
    for v in [118, 126, 128, 135]:
        sa = torch.full((64,), v, dtype=torch.int32)
        o = run(ao, ao, sa, u)
        print(f"all sa = {v}: out[0,0] = {o[0, 0].item()} (expect {128 * 2.0 ** (v - 127)})")
    g = torch.Generator().manual_seed(3)
    sa = torch.randint(118, 136, (64,), generator=g, dtype=torch.int32)
    o = run(ao, ao, sa, u)
    exp = torch.tensor([sum(2.0 ** (sa[r + 16 * q].item() - 127) * 32 for q in range(4)) for r in range(16)])
    print("random sa, ones: out[:,0]", o[:, 0].tolist())
    print("expected        ", exp.tolist())
    sb = torch.randint(118, 136, (64,), generator=g, dtype=torch.int32)
    o = run(ao, ao, u, sb)
    exp = torch.tensor([sum(2.0 ** (sb[r + 16 * q].item() - 127) * 32 for q in range(4)) for r in range(16)])
    print("random sb, ones: out[0,:]", o[0, :].tolist())
    print("expected        ", exp.tolist())

    # random values, unit scales, then random scales: per-output error
    a = (torch.randn(16, 128, generator=g) * 8).to(torch.float8_e4m3fn).view(torch.uint8)
    b = (torch.randn(16, 128, generator=g) * 8).to(torch.float8_e4m3fn).view(torch.uint8)
    lane = torch.arange(16)[:, None] + 16 * (torch.arange(128)[None, :] // 32)
    for name, sa, sb in [("unit", u, u), ("sa random", torch.randint(118, 136, (64,), generator=g, dtype=torch.int32), u),
                         ("sa in 126..128", torch.randint(126, 129, (64,), generator=g, dtype=torch.int32), u)]:
        o = run(a, b, sa, sb).double()
        A = a.view(torch.float8_e4m3fn).double() * torch.pow(2.0, (sa[lane] - 127).double())
        B = b.view(torch.float8_e4m3fn).double() * torch.pow(2.0, (sb[lane] - 127).double())
        ref = A @ B.t()
        mag = A.abs() @ B.abs().t()
        e = (o - ref).abs() / mag
        print(name, "max rel", e.max().item(), "median", e.median().item(), "o[0,:3]", o[0, :3].tolist(), "ref", ref[0, :3].tolist())


def owners():
    for which in ("A", "B"):
        for r in (0, 3):
            owner = []
            for k in range(128):
                x = torch.zeros(16, 128, dtype=torch.uint8)
                x[r, k] = ONE
                hit = []
                for g in range(4):
                    s = u.clone()
                    s[r + 16 * g] = 128
                    o = run(x, ao, s, u) if which == "A" else run(ao, x, u, s)
                    v = o[r, 0].item() if which == "A" else o[0, r].item()
                    if v == 2.0:
                        hit.append(g)
                owner.append(hit[0] if len(hit) == 1 else tuple(hit))
            print(which, "row", r, "scale lane group by buffer k:", owner)


if __name__ == "__main__":
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    for name, fn in (("layout", layout), ("values", values), ("owners", owners)):
        if what in (name, "all"):
            print(f"--- {name}", flush=True)
            fn()

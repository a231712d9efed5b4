"""Layout / scale semantics of v_mfma_scale_f32_16x16x128_f8f6f4 (kmeans_mx.hip cml_mx_probe): which output
element each A/B byte position feeds, and which lane's E8M0 scale applies to it.

    python scripts/r5/mx_probe_diag.py
"""
import torch

from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import kmeans_ops as K

dev = torch.device("cuda", 0)
ONE = int(torch.tensor([1.0]).to(torch.float8_e4m3fn).view(torch.uint8).item())
TWO = int(torch.tensor([2.0]).to(torch.float8_e4m3fn).view(torch.uint8).item())


def run(a, b, sa=None, sb=None):
    sa = torch.full((64,), 127, dtype=torch.int32) if sa is None else sa
    sb = torch.full((64,), 127, dtype=torch.int32) if sb is None else sb
    return K.mx_probe(a.to(dev), b.to(dev), sa.to(dev), sb.to(dev)).cpu()


def dec(x):
    return x.view(torch.float8_e4m3fn).double()


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

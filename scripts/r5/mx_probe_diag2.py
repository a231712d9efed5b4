"""Scale-value semantics of the MX MFMA probe (see mx_probe_diag.py)."""
import torch

from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import kmeans_ops as K

dev = torch.device("cuda", 0)
ONE = int(torch.tensor([1.0]).to(torch.float8_e4m3fn).view(torch.uint8).item())
ao = torch.full((16, 128), ONE, dtype=torch.uint8)


def run(a, b, sa, sb):
    return K.mx_probe(a.to(dev), b.to(dev), sa.to(dev), sb.to(dev)).cpu()


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

"""Which lane's E8M0 scale applies to each byte position of the MX MFMA operands (mx_probe_diag.py)."""
import torch

from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import kmeans_ops as K

dev = torch.device("cuda", 0)
ONE = int(torch.tensor([1.0]).to(torch.float8_e4m3fn).view(torch.uint8).item())
ao = torch.full((16, 128), ONE, dtype=torch.uint8)
u = torch.full((64,), 127, dtype=torch.int32)


def run(a, b, sa, sb):
    return K.mx_probe(a.to(dev), b.to(dev), sa.to(dev), sb.to(dev)).cpu()


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

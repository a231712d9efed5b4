"""Why does the split screen certify fewer rows in some passes? Records every screened pass of a k-means||
init on config-2-shaped data (2M x 128 f32) — the K9r labels and bounds and the certificate's centre
constants as the engine produced them — and reports against exact distances on a sample of rows how loose
the bounds are, and the per-row slack E."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from bench import make_blobs  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import kmeans_ops as K  # noqa: E402

n, d, k = 2_000_000, 128, 64
m = 200_000
x = make_blobs(n, d, k, seed=1000, device=torch.device("cuda"), dtype=torch.float32)
recs = []
orig_sl, orig_rr, orig_cert = LloydEngine._screen_labels, K.assign_rr_ext, K.screen_cert_split


def rec_sl(self, C, lab, best=None):
    recs.append({"C": C.detach().to(torch.float64).clone()})
    return orig_sl(self, C, lab, best)


def rec_rr(mode, *a, **kw):
    r = orig_rr(mode, *a, **kw)
    if mode == 1 and recs and "lab" not in recs[-1]:
        lab, ub, lb = a[7], a[9], a[10]
        recs[-1].update(lab=lab[:m].clone(), ub=ub[:m].clone(), lb=lb[:m].clone())
    return r


def rec_cert(ub, lb, ea, eb, en, cst, n_, lst, count, u_out, l_out, stream=None):
    recs[-1].update(cst=cst.clone(), E=(2 * (ea[:m].double() * cst[0] + eb[:m].double() * cst[1]
                                            + 1.01 * en[:m].double() * cst[2])))
    return orig_cert(ub, lb, ea, eb, en, cst, n_, lst, count, u_out, l_out, stream)


LloydEngine._screen_labels = rec_sl
K.assign_rr_ext = rec_rr
K.screen_cert_split = rec_cert
eng = LloydEngine(x, d, k, precision="screen")
eng.track_prune = True
init = eng.init_kmeans_parallel(seed=42)
torch.cuda.synchronize()
print("rechecked per pass:", eng._scr.rechecked, "tau", eng._scr.tau, flush=True)
q = torch.tensor([0.0, 0.01, 0.5, 0.99, 1.0], device="cuda", dtype=torch.float64)
for i, r in enumerate(recs):
    C = r["C"]
    kc = int(C.shape[0])
    lab = r["lab"]
    lo_, hi_ = int(lab.min()), int(lab.max())
    print(f"pass {i}: kc={kc} labels [{lo_}, {hi_}] cst={[float(v) for v in r['cst']]}", flush=True)
    if lo_ < 0 or hi_ >= kc:
        print("   labels out of range: skipped", flush=True)
        continue
    D = torch.cdist(x[:m].double(), C)
    li = lab.long()[:, None]
    own = D.gather(1, li)[:, 0]
    exact_best = D.min(1).values
    other = D.scatter(1, li, float("inf")).min(1).values
    ub, lb = r["ub"].double(), r["lb"].double()
    print("   ub-own   ", [round(v, 5) for v in torch.quantile(ub - own, q).tolist()])
    print("   other-lb ", [round(v, 5) for v in torch.quantile(other - lb, q).tolist()])
    print("   own-best ", [round(v, 6) for v in torch.quantile(own - exact_best, q).tolist()])
    print("   E        ", [round(v, 5) for v in torch.quantile(r["E"], q).tolist()])
    print("   lb-ub    ", [round(v, 5) for v in torch.quantile(lb - ub, q).tolist()], flush=True)

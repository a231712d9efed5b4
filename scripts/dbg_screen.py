"""Diagnostics of the screen certificate on config-2-shaped f32 data: rechecked rows per pass and the
distribution of (lb - ub) against 2·(err_x + err_c)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from bench import make_blobs  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine  # noqa: E402

n, d, k = 2_000_000, 128, 64
x = make_blobs(n, d, k, seed=1000, device=torch.device("cuda"), dtype=torch.float32)
eng = LloydEngine(x, d, k, precision="screen")
eng.track_prune = True
init = eng.init_kmeans_parallel(seed=42)
print("init rechecked per pass:", eng._scr.rechecked, flush=True)
eng._scr.rechecked = []
eng.set_centers(init)
eng.fit(3, 0.0)
st = eng._scr
print("lloyd rechecked per pass:", st.rechecked, flush=True)
gap = (st.lb[:n].double() - st.ub[:n].double())
print("ub quantiles", torch.quantile(st.ub[:n].double()[:100000], torch.tensor([0.01, 0.5, 0.99], device="cuda",
                                                                               dtype=torch.float64)).tolist())
print("lb quantiles", torch.quantile(st.lb[:n].double()[:100000], torch.tensor([0.01, 0.5, 0.99], device="cuda",
                                                                               dtype=torch.float64)).tolist())
print("gap quantiles", torch.quantile(gap[:100000], torch.tensor([0.01, 0.5, 0.99], device="cuda",
                                                                  dtype=torch.float64)).tolist())
print("err_x quantiles", torch.quantile(st.ex[:100000].double(), torch.tensor([0.01, 0.5, 0.99], device="cuda",
                                                                               dtype=torch.float64)).tolist())
print("xn", float(st.xn[:n].mean()), "tau", st.tau)

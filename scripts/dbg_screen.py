"""Diagnostics of the screen on config-2-shaped f32 data (2M x 128, k = 64): rows re-checked per screened
pass (split and plain screens), the init's candidate counts, and the certified steps' lists."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from bench import make_blobs  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.models import kmeans as KM  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine  # noqa: E402

n, d, k = 2_000_000, 128, 64
x = make_blobs(n, d, k, seed=1000, device=torch.device("cuda"), dtype=torch.float32)
orig = LloydEngine._screen_labels


def traced(self, C, lab, best=None):
    st = self._screen_state()
    orig(self, C, lab, best)
    cnt = int(st.cnt.item())
    u, l = st.ub[:self.n].double(), st.lb[:self.n].double()
    gap = (l - u)
    print(f"  screen pass kc={C.shape[0]} split={st.split} rechecked={cnt} "
          f"gap q01/q10/q50 = {[round(v, 4) for v in torch.quantile(gap[:200000], torch.tensor([0.01, 0.1, 0.5], device='cuda', dtype=torch.float64)).tolist()]}",
          flush=True)


LloydEngine._screen_labels = traced
for split in ("1", "0"):
    os.environ["CML_KMEANS_SCREEN_SPLIT"] = split
    if hasattr(x, "_cml_screen"):
        del x._cml_screen
    eng = LloydEngine(x, d, k, precision="screen")
    eng.track_prune = True
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    init = eng.init_kmeans_parallel(seed=42)
    torch.cuda.synchronize()
    print(f"split={split} init {1000 * (time.perf_counter() - t0):.1f} ms", flush=True)
    eng.set_centers(init)
    t0 = time.perf_counter()
    eng.fit(6, 0.0)
    torch.cuda.synchronize()
    print(f"split={split} 6 steps {1000 * (time.perf_counter() - t0):.1f} ms cert {eng._scr.cert.history}", flush=True)

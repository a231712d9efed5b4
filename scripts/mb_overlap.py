"""Does the sort-regime accumulate of one row chunk overlap with the assign of the next one when the
two run on separate HIP streams? Times each alone and both together for several assign variants.

    python scripts/mb_overlap.py [rows_per_chunk]
"""
import sys

import torch

from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import kmeans_ops as K


def timeit(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(reps):
        s, e = torch.cuda.Event(True), torch.cuda.Event(True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e))
    return best


n = int(sys.argv[1]) if len(sys.argv) > 1 else 25_000_000
d = k = 256
g = torch.Generator(device="cuda")
g.manual_seed(0)
cen = torch.randn(k, d, device="cuda", generator=g) * 4
xs = [(cen[torch.randint(0, k, (n,), device="cuda", generator=g)] +
       torch.randn(n, d, device="cuda", generator=g)).to(torch.bfloat16) for _ in range(2)]
init = xs[0][:k].double().cpu().numpy()
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

for v in (0, 2, 4, 1):
    K.set_assign_variant(v)
    engs = []
    for x in xs:
        e = LloydEngine(x, d, k, accum_mode="sort", use_graph=False)
        e.set_centers(init)
        e.step()
        engs.append(e)
    ea, eb = engs

    def assign(e, stream=None):
        K.assign_bf16(e.x, e.n, e.dp, e.cb, e.cnorm, e.aplan, e.labels, e._best(0, e.n), e.cost_part, e.hist,
                      e.rank, stream=stream, xnorm=e.xnorm)

    def accum(e, stream=None):
        K.accumulate_sort(e.x, e.n, e.dp, e.d, e.labels, e.rank, e.hist, e.aplan, e.k, e.cost_part, e.off, e.seg,
                          e.perm, e.cplan, e.msgs[0], e.slots, stream=stream)

    def both():
        cur = torch.cuda.current_stream()
        s1.wait_stream(cur)
        s2.wait_stream(cur)
        assign(eb, s1)
        accum(ea, s2)
        cur.wait_stream(s1)
        cur.wait_stream(s2)

    def serial():
        assign(eb)
        accum(ea)

    ta = timeit(lambda: assign(eb))
    tc = timeit(lambda: accum(ea))
    ts = timeit(serial)
    tb = timeit(both)
    print(f"variant {v} grid {eb.aplan.grid}: assign {ta:.3f} ms, accumulate {tc:.3f} ms, serial {ts:.3f} ms, "
          f"two streams {tb:.3f} ms (overlap saves {ts - tb:.3f} ms)", flush=True)
    del engs, ea, eb
    torch.cuda.empty_cache()

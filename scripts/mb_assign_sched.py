"""K9 assign pass time vs partner-wave scheduling (kmeans_ops.set_assign_sched), 20M x 256, k = 256."""
import sys
import torch
import bench
from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import kmeans_ops as K

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20_000_000
scheds = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0, 1, 18, 34, 66, 35, 0]
x = bench.make_blobs(n, 256, 256, seed=1000, device=torch.device("cuda"))
eng = LloydEngine(x, 256, 256, use_graph=False)
eng.set_centers(x[:256].double().cpu().numpy())
eng.step()


def run():
    K.assign_bf16(eng.x, n, eng.dp, eng.cb, eng.cnorm, eng.aplan, eng.labels, None, eng.cost_part, eng.hist,
                  eng.rank, xnorm=eng.xnorm)


for sc in scheds:
    K.set_assign_sched(sc)
    run()
    torch.cuda.synchronize()
    ts = []
    for _ in range(7):
        a, b = torch.cuda.Event(True), torch.cuda.Event(True)
        a.record()
        run()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    t = ts[len(ts) // 2]
    print(f"sched {sc:3d}: median {t:.3f} ms (min {ts[0]:.3f}) -> {2 * n * 256 * 256 / t / 1e9:.0f} TF/s, "
          f"{n * 512 / t / 1e9:.2f} TB/s", flush=True)

# bounds: compute only (every row aliases row 0: no HBM stream) and a 32-centre launch (memory only)
K.set_assign_sched(0)
x0 = torch.as_strided(eng.x, (n, eng.dp), (0, 1))
for name, fn in (("compute-only (ldx=0)", lambda: K.assign_bf16(x0, n, eng.dp, eng.cb, eng.cnorm, eng.aplan,
                                                                  eng.labels, None, eng.cost_part, eng.hist, eng.rank,
                                                                  xnorm=eng.xnorm)),):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(7):
        a, b = torch.cuda.Event(True), torch.cuda.Event(True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    t = ts[len(ts) // 2]
    print(f"{name}: median {t:.3f} ms -> {2 * n * 256 * 256 / t / 1e9:.0f} TF/s", flush=True)
e32 = LloydEngine(x, 256, 32, use_graph=False)
e32.set_centers(x[:32].double().cpu().numpy())
e32.step()
fn = lambda: K.assign_bf16(e32.x, n, e32.dp, e32.cb, e32.cnorm, e32.aplan, e32.labels, None, e32.cost_part,
                           None, None, xnorm=e32.xnorm)
fn()
torch.cuda.synchronize()
a, b = torch.cuda.Event(True), torch.cuda.Event(True)
a.record()
for _ in range(5):
    fn()
b.record()
torch.cuda.synchronize()
t = a.elapsed_time(b) / 5
print(f"k=32 (memory-bound): {t:.3f} ms -> {n * 512 / t / 1e9:.2f} TB/s", flush=True)

import sys, time, json
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/3d-genome-cycle_amd')
import bench
from gcs import synthetic
from gcs.config import InterphaseConfig
cfg = InterphaseConfig()
d = synthetic.make_c2(master_seed=1)
e = bench.make_engine(d, cfg, 0, 0)
t0 = time.perf_counter()
step = 0
for target in [1000, 10000, 50000, 100000, 200000, 300000, 302200]:
    e.run(target - step, first_step=step, seed=7)
    step = target
    e.synchronize()
    p = e.profile(10, first_step=step, seed=7); step += 10
    c = e.get_context()
    print(json.dumps({"step": step, "t": round(time.perf_counter() - t0, 2), "neighbors": p["mean_neighbors"],
                      "force_us": p["force_ms"] * 1e3, "cs": c["core_scale"], "wall": c["wall_semiaxes"]}), flush=True)

"""Which HIP runtime do torch and libgcs share in one process, for each import order (GPU box probe)."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "3d-genome-cycle_amd"))
order = sys.argv[1]


def hip_libs():
    return sorted({l.split()[-1] for l in open("/proc/self/maps") if "amdhip64" in l or "hsa-runtime" in l})


if order == "torch_first":
    import torch
    print("torch cuda", torch.cuda.is_available(), flush=True)
    x = torch.ones(4, device="cuda")
    from gcs import _abi as A
    A.load()
else:
    from gcs import _abi as A
    A.load()
    import torch
    print("torch cuda", torch.cuda.is_available(), flush=True)
print(hip_libs(), flush=True)
from gcs import synthetic, interphase
from gcs.config import InterphaseConfig
from gcs.engine import Engine
d = synthetic.make_c1()
e, _ = interphase.build_interphase(Engine, d, InterphaseConfig(), device=0)
e.run(10, seed=1)
print("engine ok", e.get_positions()[0], flush=True)
t = torch.zeros(8, dtype=torch.float64, device="cuda")
print("tensor ptr", hex(t.data_ptr()), flush=True)

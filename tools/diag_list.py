import sys, numpy as np
sys.path.insert(0, '3d-genome-cycle_amd'); sys.path.insert(0, 'tests'); sys.path.insert(0, '.')
from gcs import _abi as A, interphase, synthetic
from gcs.config import InterphaseConfig
from gcs.engine import Engine
import oracle
cfg = InterphaseConfig()
d = synthetic.make_c1() if hasattr(synthetic, 'make_c1') else None
print('design', d.n if d is not None else None)
for fmt in (0, 3):
    e, _ = interphase.build_interphase(Engine, d, cfg, precision=64)
    e.set_option(A.OPT_FUSED_STEP, 3); e.set_option(A.OPT_DENSE_NEIGHBORS, 0); e.set_option(A.OPT_LIST_FORMAT, fmt)
    o, _ = interphase.build_interphase(oracle.OracleSystem, d, cfg, precision=64)
    for s in (e, o):
        s.set_schedule(**interphase.interphase_schedule(cfg)); s.apply_schedule(0)
    for k in range(3):
        for s in (e, o):
            s.run(20, first_step=20 * k, temperature=cfg.temperature, timestep=cfg.timestep, seed=98)
        print('fmt', fmt, 'chunk', k, 'err', np.abs(e.get_positions() - o.get_positions()).max(), e.list_stats(), e.run_stats())

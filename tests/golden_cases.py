"""The golden cases (SURVEY.md §8c "golden vectors to generate here and commit"): small systems built the same way on
the fp64 oracle and on the HIP engine (both expose the micromd-named methods), their inputs and the quantities
recorded in tests/golden/oracle_golden.npz by tests/golden/gen_oracle_fixtures.py.

The reference itself cannot be built here (micromd is an un-vendored submodule), so these vectors are
the oracle's outputs: they pin the oracle against drift (tests/test_golden.py) and the engine against the same
numbers without re-running the oracle (tests/test_gpu_golden.py). Closed forms behind the KATs:
stage_interphase/simulation_driver_forcefield.cpp:21-53 (softcore A/B), :57-96 (semispring chain bonds), :164-185
(softwell droplet), common/potentials/force_flux_potential.hpp:24-37 (force flux), simulation_store.cpp:22-33
(quantize)."""
import numpy as np

KAT_R = np.linspace(0.0, 0.45, 16)  # radii of the two-particle KATs (both sides of every cutoff)
SEED_NOISE = 123                    # reference-order normals (mt19937_64 + libstdc++ normal_distribution)
TRAJ_STEPS = 10
PAIR_DISTANCES = (0.24, 0.3)
# fp32-representable inputs: the engine stores positions in fp32 and quantises those (the store's sampled values)
QUANTIZE_IN = np.concatenate([[0.0, 1.0, -1.0, 1.0 / 3.0, 1e-30, -2.5e7],
                              np.random.default_rng(2024).normal(size=58) * 3.0]).astype(np.float32).astype(np.float64)


def kat_softcore(cls):
    """U = a SC<2,3>(2.5, 0.30) + b SC<8,3>(2.5, 0.24), pair means of ab = (1, 0) and (0.5, 0.5)"""
    s = cls(2, ab_factors=[[1.0, 0.0], [0.5, 0.5]])
    s.add_neighbor_softcore(a_energy=2.5, a_diameter=0.3, b_energy=2.5, b_diameter=0.24, neighbor_distance=0.3,
                            mix=True, scaled=False)
    return s


def kat_semispring(cls):
    """chain-bond semispring K = 100, l = 0.1 (one-sided: zero force below l)"""
    from gcs import _abi as A
    s = cls(2)
    s.add_bonded_pairwise(A.POT_SEMISPRING, a_spring=100.0, a_length=0.1, pairs=[(0, 1)])
    return s


def kat_softwell(cls):
    """droplet softwell<6>(0.3, 0.2) cut off at 0.4 between two targets"""
    s = cls(2, ab_factors=[[0.0, 10.0]] * 2)
    s.add_neighbor_softwell(energy=0.3, decay_distance=0.2, cutoff=0.4, targets=[0, 1])
    return s


def kat_force_flux(cls):
    """force-flux point source f = 0.7, b = 0.4 at the origin (particle 0 pinned far away by nothing: it only
    contributes its own term, so the KAT reads particle 1)"""
    from gcs import _abi as A
    s = cls(2)
    s.add_point_source(A.POT_FORCE_FLUX, [0.0, 0.0, 0.0], force=0.7, reactive_distance=0.4)
    return s


KATS = {"softcore": kat_softcore, "semispring": kat_semispring, "softwell": kat_softwell,
        "force_flux": kat_force_flux}


def kat_eval(build, cls):
    """energy and the x force on particle 1 at each radius of KAT_R (particle 0 at the origin)"""
    s = build(cls)
    e = np.empty(KAT_R.size)
    f = np.empty(KAT_R.size)
    for k, r in enumerate(KAT_R):
        s.set_positions([[0.0, 0.0, 0.0], [r, 0.0, 0.0]])
        e[k] = s.compute_energy()[0]
        f[k] = s.compute_forces()[1, 0]
    return e, f


def c1_system(cls):
    """C1 (1,002 beads, the full interphase force field) at the step-0 schedule"""
    from gcs import interphase, synthetic
    from gcs.config import InterphaseConfig
    cfg = InterphaseConfig()
    design = synthetic.make_c1()
    s, _ = interphase.build_interphase(cls, design, cfg)
    s.set_schedule(**interphase.interphase_schedule(cfg))
    s.apply_schedule(0)
    return s, design, cfg


def c1_noise(n):
    import oracle
    return oracle.reference_normals(SEED_NOISE, TRAJ_STEPS * n * 3).reshape(TRAJ_STEPS, n, 3)


def c1_run(s, cfg, xi, steps):
    from gcs import _abi as A
    s.set_noise(xi)
    s.run(steps, temperature=cfg.temperature, timestep=cfg.timestep, noise=A.NOISE_INJECTED)
    return s.get_positions(), s.get_context()

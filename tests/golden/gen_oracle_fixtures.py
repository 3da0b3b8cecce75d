"""Writes tests/golden/oracle_golden.npz: the golden vectors of SURVEY.md §8c computed by the fp64 oracle
(oracle/, test infrastructure) on the cases of tests/golden_cases.py.

    python tests/golden/gen_oracle_fixtures.py        # from the repo root; builds the oracle if needed

Items: two-particle KATs (energy, x force) of softcore A/B, semispring, softwell and force flux at 16 radii; the C1
pair sets within 0.24 and 0.30 (strict fp32 predicate and strict fp64 predicate, i < j); the C1 interphase forces, energy per kind and
reactions at the step-0 schedule; C1 positions and context after 1 and 10 BD steps with injected reference-order
noise (seed 123); a quantize table."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "oracle"), str(ROOT / "3d-genome-cycle_amd"), str(ROOT / "tests")]

import golden_cases as G  # noqa: E402
import oracle  # noqa: E402


def main(out=ROOT / "tests" / "golden" / "oracle_golden.npz"):
    oracle.build()
    rec = {"kat_r": G.KAT_R}
    for name, build in G.KATS.items():
        rec[f"kat_{name}_e"], rec[f"kat_{name}_f"] = G.kat_eval(build, oracle.OracleSystem)
    s, design, cfg = G.c1_system(oracle.OracleSystem)
    x0 = np.asarray(design.positions, dtype=np.float64)
    rec["c1_x0"] = x0
    for d in G.PAIR_DISTANCES:
        rec[f"c1_pairs_{int(round(d * 100)):03d}"] = oracle.search_neighbors(x0, d, 32).astype(np.int32)
        rec[f"c1_pairs64_{int(round(d * 100)):03d}"] = oracle.search_neighbors(x0, d, 64).astype(np.int32)
    rec["c1_forces"] = s.compute_forces()
    tot, parts = s.compute_energy()
    rec["c1_energy"] = np.array([tot]) if np.isscalar(tot) else np.asarray(tot)
    rec["c1_energy_parts"] = np.asarray(parts, dtype=np.float64)
    c = s.get_context()
    rec["c1_inward_reaction"] = np.asarray(c["inward_reaction"], dtype=np.float64)
    rec["c1_outward_reaction"] = np.asarray(c["outward_reaction"], dtype=np.float64)
    xi = G.c1_noise(design.n)
    s1, _, _ = G.c1_system(oracle.OracleSystem)
    rec["c1_step1"], _ = G.c1_run(s1, cfg, xi[:1], 1)
    s10, _, _ = G.c1_system(oracle.OracleSystem)
    rec["c1_traj10"], c10 = G.c1_run(s10, cfg, xi, G.TRAJ_STEPS)
    rec["c1_traj10_wall"] = np.asarray(c10["wall_semiaxes"], dtype=np.float64)
    rec["c1_traj10_core_scale"] = np.array([c10["core_scale"]])
    rec["quantize_in"] = G.QUANTIZE_IN
    rec["quantize_out"] = np.array([oracle.quantize(v) for v in G.QUANTIZE_IN])
    np.savez_compressed(out, **rec)
    print(f"wrote {out} ({Path(out).stat().st_size} bytes): {', '.join(sorted(rec))}")


if __name__ == "__main__":
    main()

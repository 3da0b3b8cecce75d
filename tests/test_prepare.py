"""`prepare` from a config JSON + chain TSV (gcs/prepare.py; stage_prepare/*.cpp), checked against the designs the
synthetic generator builds for the same chains, and through the CLI into the store."""
import numpy as np
import pytest

from gcs import cli, mitotic, prepare, store, synthetic
from gcs.config import SimulationConfig, format_simulation_config

TYPE_TAGS = {1: "A", 2: "B", 3: "u", 4: "cen", 5: "anor,A", 6: "bnor", 0: ""}


def _tsv(design, header=True):
    rows = ["chain\tstart\tend\tA\tB\ttags"] if header else []
    for name, s, e in design.chains:
        for k, i in enumerate(range(s, e)):
            a, b = design.ab_factors[i]
            rows.append(f"{name}\t{k * 100000}\t{(k + 1) * 100000}\t{a}\t{b}\t{TYPE_TAGS[int(design.particle_types[i])]}")
    return "\n".join(rows) + "\n"


@pytest.mark.parametrize("header", [True, False])
def test_prepare_matches_the_synthetic_designs(header):
    cfg = SimulationConfig()
    d = synthetic.make_c2(3)
    chains = prepare.load_chain_tsv(_tsv(d, header))
    assert len(chains) == 46
    i, a, p = prepare.prepare_designs(cfg, chains, 3)
    assert i.n == d.n and np.array_equal(i.particle_types, d.particle_types)
    assert np.array_equal(i.ab_factors, d.ab_factors) and i.chains == d.chains
    assert np.array_equal(i.nucleolar_bonds, d.nucleolar_bonds) and i.seed == d.seed
    assert i.centromeres == d.centromeres
    a2 = mitotic.anatelophase_design(d, cfg.mitotic_phase, 3)
    assert a.chains == a2.chains and a.seed == a2.seed
    assert p.n == 2 * a.n


def test_tag_precedence():
    assert prepare._bead_type("A,anor") == 5 and prepare._bead_type("cen,B") == 4
    assert prepare._bead_type("B") == 2 and prepare._bead_type("x,y") == 0 and prepare._bead_type("") == 0
    assert prepare._bead_type("Anor") == 0  # whole comma fields only (prepare.cpp:145-162)


def test_prepare_cli_writes_the_store(tmp_path):
    cfg = SimulationConfig()
    d = synthetic.make_c1()
    (tmp_path / "config.json").write_text(format_simulation_config(cfg))
    (tmp_path / "chains.tsv").write_text(_tsv(d))
    out = tmp_path / "t.h5"
    cli.main(["prepare", "-s", "7", "-o", str(out), str(tmp_path / "config.json"), str(tmp_path / "chains.tsv")])
    with store.SimulationStore(out) as st:
        i = st.load_interphase_design()
        assert i.n == d.n and i.chains == d.chains
        assert st.f.read_string("/metadata/chains_source").startswith("chain\tstart")
        assert int(st.f.read_array("/metadata/master_seed", store.H5_U32)) == 7
        a = st.load_anatelophase_design()
        assert len(a.chains) == 1 and a.chains[0][2] == d.chains[0][2] // cfg.mitotic_phase.coarse_graining
        st.set_stage("relaxation")
        assert not st.check_positions(0)  # prepare writes no structure (the anatelophase stage starts from rods)


def test_prepare_launcher_at_the_reference_path(tmp_path):
    """<project>/src/simulation/prepare with scripts/simulate:44's argv (a CPU stage: no device needed)."""
    import os
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    d = synthetic.make_c1()
    (tmp_path / "config.json").write_text(format_simulation_config(SimulationConfig()))
    (tmp_path / "chains.tsv").write_text(_tsv(d))
    out = tmp_path / "out.h5"
    env = dict(os.environ, GCS_PYTHON=sys.executable)
    p = subprocess.run([str(root / "src" / "simulation" / "prepare"), "-s", "5", "-o", str(out),
                        str(tmp_path / "config.json"), str(tmp_path / "chains.tsv")],
                       capture_output=True, text=True, env=env, timeout=120)
    assert p.returncode == 0, p.stderr
    with store.SimulationStore(out) as st:
        assert int(st.f.read_array("/metadata/master_seed", store.H5_U32)) == 5
        assert st.load_interphase_design().n == d.n
    bad = subprocess.run([str(root / "src" / "simulation" / "transition"), "interphase"], capture_output=True,
                         text=True, env=env, timeout=120)
    assert bad.returncode != 0  # usage errors surface as a failing status, like the reference's main

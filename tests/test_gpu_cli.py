"""GPU: the whole cell-cycle pipeline (BASELINE configs[2], C3) through the stage entry points (gcs/cli.py,
mirroring scripts/simulate and the reference's stage executables) on the HIP engine, reading and writing the HDF5
store: prepare (config JSON + chain TSV) -> anatelophase -> transition interphase -> interphase (relaxation + simulation, contact map) ->
transition prometaphase -> prometaphase -> transition cycle -> the daughter's anatelophase."""
import dataclasses

import numpy as np
import pytest

from gcs import cli, mitotic, store, synthetic
from gcs.config import SimulationConfig

pytestmark = pytest.mark.gpu


def _inputs(path, master_seed, cfg):
    """config.json + chains.tsv (the synthetic C2 chains) next to `path`"""
    from gcs.config import format_simulation_config
    d = synthetic.make_c2(master_seed)
    tags = {1: "A", 2: "B", 3: "u", 4: "cen", 5: "anor", 6: "bnor", 0: ""}
    rows = []
    for name, s, e in d.chains:
        for k, i in enumerate(range(s, e)):
            a, b = d.ab_factors[i]
            rows.append(f"{name}\t{k * 100000}\t{(k + 1) * 100000}\t{a}\t{b}\t{tags[int(d.particle_types[i])]}")
    cj, ct = path.with_suffix(".json"), path.with_suffix(".tsv")
    cj.write_text(format_simulation_config(cfg))
    ct.write_text("\n".join(rows) + "\n")
    return d, cj, ct


def _prepare(path, master_seed, cfg):
    """`prepare -s seed -o path config.json chains.tsv` with the synthetic C2 chains written as a TSV"""
    d, cj, ct = _inputs(path, master_seed, cfg)
    cli.main(["prepare", "-s", str(master_seed), "-o", str(path), str(cj), str(ct)])
    a = mitotic.anatelophase_design(d, cfg.mitotic_phase)
    pm = mitotic.prometaphase_design(a, cfg.mitotic_phase, master_seed)
    return d, a, pm


def test_cell_cycle_through_the_store(tmp_path):
    cfg = SimulationConfig()
    cfg.interphase = dataclasses.replace(cfg.interphase, relaxation_sampling_interval=100,
                                         relaxation_logging_interval=100, sampling_interval=200, logging_interval=200,
                                         contactmap_output_window=2)
    cfg.mitotic_phase = dataclasses.replace(cfg.mitotic_phase, sampling_interval=50, logging_interval=50)
    p = tmp_path / "mother.h5"
    d, a, pm = _prepare(p, 1, cfg)

    cli.main(["anatelophase", str(p), "--anaphase-steps", "100", "--telophase-steps", "100", "--quiet"])
    cli.main(["transition", "interphase", str(p)])
    cli.main(["interphase", str(p), "--relaxation-steps", "200", "--steps", "400", "--quiet"])
    cli.main(["transition", "prometaphase", str(p)])
    cli.main(["prometaphase", str(p), "--steps", "100", "--quiet"])
    q = tmp_path / "daughter.h5"
    _prepare(q, 2, cfg)
    cli.main(["transition", "cycle", str(p), str(q)])
    cli.main(["anatelophase", str(q), "--anaphase-steps", "50", "--telophase-steps", "50", "--quiet"])

    with store.SimulationStore(p) as st:
        st.set_stage("anaphase")
        assert st.load_steps() == [0, 50, 100]
        st.set_stage("telophase")
        assert st.load_steps() == [0, 50, 100]
        st.set_stage("relaxation")
        assert st.load_steps() == [0, 100, 200]
        st.set_stage("interphase")
        assert st.load_steps() == [0, 200, 400]
        ctx = st.load_interphase_context(400)
        assert ctx["time"] == pytest.approx(400 * cfg.interphase.timestep) and ctx["mean_energy"] != 0
        c = st.load_contacts(400)
        assert c.shape[0] > d.n // 2 and (c[:, 0] < c[:, 1]).all() and c[:, 2].max() <= 20
        x = st.load_positions(400)
        assert np.isfinite(x).all()
        st.set_stage("prometaphase")
        assert st.load_steps() == [0, 50, 100] and np.isfinite(st.load_positions(100)).all()
    with store.SimulationStore(q) as st:
        st.set_stage("anaphase")
        x0 = st.load_positions(0)  # the transition's structure was used (no rods)
        assert x0.shape == (a.n, 3) and np.isfinite(st.load_positions(50)).all()


def test_scripts_simulate_argv(tmp_path):
    """The four stage calls of the reference's scripts/simulate:44-47, with its exact argv, at the paths it uses
    (<project>/src/simulation/<stage>): prepare -s seed -o out.h5 config.json chains.tsv; anatelophase out.h5;
    transition interphase out.h5; interphase out.h5.  Step counts come from the config, as in the reference."""
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    stage = root / "src" / "simulation"
    cfg = SimulationConfig()
    cfg.mitotic_phase = dataclasses.replace(cfg.mitotic_phase, anaphase_steps=60, telophase_steps=40,
                                            sampling_interval=20, logging_interval=20)
    cfg.interphase = dataclasses.replace(cfg.interphase, relaxation_steps=100, steps=200,
                                         relaxation_sampling_interval=50, relaxation_logging_interval=50,
                                         sampling_interval=100, logging_interval=100, contactmap_output_window=2)
    out = tmp_path / "out.h5"
    d, cj, ct = _inputs(out, 7, cfg)
    env = dict(__import__("os").environ, GCS_PYTHON=sys.executable)
    calls = [[str(stage / "prepare"), "-s", "7", "-o", str(out), str(cj), str(ct)],
             [str(stage / "anatelophase"), str(out)],
             [str(stage / "transition"), "interphase", str(out)],
             [str(stage / "interphase"), str(out)]]
    for argv in calls:
        p = subprocess.run(argv, capture_output=True, text=True, env=env, timeout=300)
        assert p.returncode == 0, (argv, p.stderr[-2000:])
    with store.SimulationStore(out) as st:
        st.set_stage("telophase")
        assert st.load_steps() == [0, 20, 40]
        st.set_stage("relaxation")
        assert st.load_steps() == [0, 50, 100]
        st.set_stage("interphase")
        assert st.load_steps() == [0, 100, 200]
        x = st.load_positions(200)
        assert x.shape == (d.n, 3) and np.isfinite(x).all()
        c = st.load_contacts(200)
        assert c.shape[0] > 0 and (c[:, 0] < c[:, 1]).all()

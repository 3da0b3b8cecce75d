"""Stage entry points over the HDF5 trajectory store, mirroring the reference's stage executables
(stage_interphase/main.cpp, stage_anatelophase/main.cpp, stage_prometaphase/main.cpp: `<stage> <trajectory.h5>`)
with the HIP engine underneath.  `prepare-synthetic` writes a prepared file from the synthetic generators (the
reference's `prepare` reads TSV inputs instead).

    python -m gcs.cli prepare [-s seed] -o out.h5 config.json chains.tsv
    python -m gcs.cli prepare-synthetic out.h5 --config c1 [--master-seed 1]
    python -m gcs.cli interphase out.h5 [--relaxation-steps N] [--steps N] [--device 0] [--precision 64|32]
    python -m gcs.cli anatelophase out.h5 [--anaphase-steps N] [--telophase-steps N]
    python -m gcs.cli prometaphase out.h5 [--steps N]   (needs /stages/prometaphase/0/positions)
    python -m gcs.cli transition interphase|prometaphase out.h5
    python -m gcs.cli transition cycle prev.h5 next.h5
"""
from __future__ import annotations

import argparse
import sys

from . import interphase, mitotic, prepare, store, synthetic, transition
from .config import SimulationConfig


def cmd_prepare_synthetic(a):
    cfg = SimulationConfig()
    design = {"c1": synthetic.make_c1, "c2": synthetic.make_c2, "c5": synthetic.make_c5}[a.config](a.master_seed)
    anat = mitotic.anatelophase_design(design, cfg.mitotic_phase, a.master_seed) if design.centromeres else None
    prom = mitotic.prometaphase_design(anat, cfg.mitotic_phase, a.master_seed) if anat is not None else None
    store.write_prepared(a.path, cfg, design, a.master_seed, anatelophase=anat, prometaphase=prom,
                         chains_source=f"synthetic:{a.config}")


def cmd_prepare(a):
    prepare.prepare(a.output, a.config, a.chains, a.seed)


def cmd_interphase(a):
    from .engine import Engine
    with store.SimulationStore(a.path) as st:
        cfg = st.load_config().interphase
        design = st.load_interphase_design()
        eng, _ = interphase.build_interphase(Engine, design, cfg, device=a.device, precision=a.precision)
        drv = interphase.InterphaseDriver(eng, design, cfg, store=st, log=None if a.quiet else sys.stderr)
        # run_relaxation (simulation_driver_relaxation.cpp:10-23): stage, clear, initial structure from step 0
        st.set_stage("relaxation")
        st.clear_frames()
        eng.set_positions(st.load_positions(0))
        drv.run_relaxation(a.relaxation_steps)
        # run_simulation (simulation_driver_interphase.cpp:11-12)
        st.set_stage("interphase")
        st.clear_frames()
        drv.run_simulation(a.steps)


def cmd_anatelophase(a):
    from .engine import Engine
    with store.SimulationStore(a.path) as st:
        cfg = st.load_config().mitotic_phase
        design = st.load_anatelophase_design()
        sys_, h = mitotic.build_anatelophase(Engine, design, cfg, device=a.device, precision=a.precision)
        drv = mitotic.AnatelophaseDriver(sys_, h, design, cfg, store=st, log=None if a.quiet else sys.stderr)
        st.set_stage("anaphase")  # run (stage_anatelophase/simulation_driver.cpp:193-203): clear_frames before set_stage
        st.clear_frames()
        st.set_stage("anaphase")
        init = st.load_positions(0) if st.check_positions(0) else None
        drv.run(init, a.anaphase_steps, a.telophase_steps)


def cmd_prometaphase(a):
    from .engine import Engine
    with store.SimulationStore(a.path) as st:
        cfg = st.load_config().mitotic_phase
        design = st.load_prometaphase_design()
        sys_, _ = mitotic.build_prometaphase(Engine, design, cfg, device=a.device, precision=a.precision)
        st.set_stage("prometaphase")
        st.clear_frames()
        if not st.check_positions(0):
            raise SystemExit("no initial structure is given")
        mitotic.PrometaphaseDriver(sys_, design, cfg, store=st, log=None if a.quiet else sys.stderr).run(
            st.load_positions(0), a.steps)


def cmd_transition(a):
    """stage_transition/main.cpp:43-81"""
    if a.mode == "cycle":
        if len(a.paths) != 2:
            raise SystemExit("prev and next trajectory files must be specified")
        with store.SimulationStore(a.paths[0]) as prev, store.SimulationStore(a.paths[1]) as nxt:
            transition.transition_cycle(prev, nxt)
        return
    if len(a.paths) != 1:
        raise SystemExit("single trajectory file must be specified")
    with store.SimulationStore(a.paths[0]) as st:
        (transition.transition_interphase if a.mode == "interphase" else transition.transition_prometaphase)(st)


def main(argv=None):
    ap = argparse.ArgumentParser(prog="gcs")
    sub = ap.add_subparsers(dest="cmd", required=True)
    p = sub.add_parser("prepare")  # stage_prepare/main.cpp: prepare [-s seed] -o out.h5 config.json chains.tsv
    p.add_argument("-s", "--seed", type=int, default=None)
    p.add_argument("-o", "--output", required=True)
    p.add_argument("config")
    p.add_argument("chains")
    p.set_defaults(fn=cmd_prepare)
    p = sub.add_parser("prepare-synthetic")
    p.add_argument("path")
    p.add_argument("--config", default="c1", choices=["c1", "c2", "c5"])
    p.add_argument("--master-seed", type=int, default=1)
    p.set_defaults(fn=cmd_prepare_synthetic)
    for name, fn in (("interphase", cmd_interphase), ("anatelophase", cmd_anatelophase),
                     ("prometaphase", cmd_prometaphase)):
        p = sub.add_parser(name)
        p.add_argument("path")
        p.add_argument("--device", type=int, default=0)
        # the engine's arithmetic: 64 (default) is the reference's double; 32 the fp32 engine
        p.add_argument("--precision", type=int, default=64, choices=[32, 64])
        p.add_argument("--quiet", action="store_true")
        if name == "interphase":
            p.add_argument("--relaxation-steps", type=int, default=None)
            p.add_argument("--steps", type=int, default=None)
        elif name == "anatelophase":
            p.add_argument("--anaphase-steps", type=int, default=None)
            p.add_argument("--telophase-steps", type=int, default=None)
        else:
            p.add_argument("--steps", type=int, default=None)
        p.set_defaults(fn=fn)
    p = sub.add_parser("transition")
    p.add_argument("mode", choices=["interphase", "prometaphase", "cycle"])
    p.add_argument("paths", nargs="+")
    p.set_defaults(fn=cmd_transition)
    a = ap.parse_args(argv)
    a.fn(a)


if __name__ == "__main__":
    main()

"""`prepare` (stage_prepare/main.cpp, chains.cpp:14-63, prepare.cpp:128-576): a config JSON and a
chain-definition TSV into a prepared trajectory file (the interphase, anatelophase and prometaphase designs,
their seeds and the inputs as text).

Chain TSV rows: chain, bin start, bin end, A factor, B factor, comma-separated tags; contiguous rows with the same
chain name form one chain (chains.cpp:37-60).  The TSV reader of the reference (snsinfu/cxx-tsv, an un-vendored
submodule) is restated leniently: a first row whose bin fields are not integers is taken as a header.
"""
from __future__ import annotations

import random

import numpy as np

from . import mitotic, store
from .config import SimulationConfig, parse_simulation_config
from .seeds import stage_seeds
from .synthetic import InterphaseDesign

# prepare.cpp:171-178 (first matching tag wins, in this order)
TAG_TYPES = (("anor", 5), ("bnor", 6), ("cen", 4), ("A", 1), ("B", 2), ("u", 3))


def load_chain_tsv(text: str):
    """[(name, [(bin_start, bin_end, a, b, tags)])]"""
    chains = []
    for k, line in enumerate(text.splitlines()):
        if not line.strip():
            continue
        f = line.split("\t")
        if len(f) < 5:
            raise ValueError(f"cannot load chain definitions: line {k + 1}: expected 6 fields")
        try:
            rec = (int(f[1]), int(f[2]), float(f[3]), float(f[4]), f[5] if len(f) > 5 else "")
        except ValueError:
            if k == 0:
                continue  # header row
            raise
        if not chains or chains[-1][0] != f[0]:
            chains.append((f[0], []))
        chains[-1][1].append(rec)
    return chains


def _bead_type(tags: str) -> int:
    fields = tags.split(",") if tags else []
    for tag, t in TAG_TYPES:
        if tag in fields:
            return t
    return 0


def prepare_designs(cfg: SimulationConfig, chains, master_seed: int):
    """define_chains / define_nucleolar_particles / define_anatelophase_chains / define_prometaphase_chains
    (prepare.cpp:166-372) -> (interphase design, anatelophase design, prometaphase design)."""
    ab, types, ranges, nors, cens = [], [], [], [], []
    for name, beads in chains:
        start = len(types)
        for _, _, a, b, tags in beads:
            t = _bead_type(tags)
            if t == 5:
                nors.append(len(types))
            types.append(t)
            ab.append((a, b))
        end = len(types)
        ranges.append((name, start, end))
        cidx = [i for i in range(start, end) if types[i] == 4]
        cens.append((cidx[0], cidx[-1] + 1) if cidx else (start, end))  # prepare.cpp:256-273
    bonds = []
    ic = cfg.interphase
    for nor in nors:
        for _ in range(ic.nucleolus_bead_count):
            bonds.append((nor, len(types)))
            types.append(7)
            ab.append((ic.nucleolus_ab_factor.a, ic.nucleolus_ab_factor.b))
    n = len(types)
    idesign = InterphaseDesign(seed=stage_seeds(master_seed)["interphase"], ab_factors=np.array(ab, dtype=np.float64),
                               particle_types=np.array(types, dtype=np.int32), chains=ranges,
                               nucleolar_bonds=np.array(bonds, dtype=np.int64).reshape(-1, 2),
                               positions=np.zeros((n, 3)), master_seed=master_seed, centromeres=cens)
    adesign = mitotic.anatelophase_design(idesign, cfg.mitotic_phase, master_seed)
    pdesign = mitotic.prometaphase_design(adesign, cfg.mitotic_phase, master_seed)
    return idesign, adesign, pdesign


def prepare(out_path, config_path, chains_path, master_seed=None):
    """stage_prepare/main.cpp:45-66: `prepare [-s seed] -o <trajectory.h5> <config.json> <chains.tsv>`"""
    config_text = open(config_path).read()
    chains_text = open(chains_path).read()
    cfg = parse_simulation_config(config_text)
    seed = master_seed if master_seed is not None else random.SystemRandom().getrandbits(32)
    i, a, p = prepare_designs(cfg, load_chain_tsv(chains_text), seed)
    store.write_prepared(out_path, cfg, i, seed, anatelophase=a, prometaphase=p, chains_source=chains_text,
                         initial_positions=False)
    return i, a, p

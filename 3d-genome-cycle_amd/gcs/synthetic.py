"""Synthetic inputs of the benchmark configurations.

There is no network, so no real chains TSV; these generators produce designs with the reference's
layout (stage_prepare/prepare.cpp:169-255: chains in order, nucleolar beads appended after all chains and
bonded to their active NOR, nucleolar beads placed on their NOR, transition_interphase.cpp:80-82).

  C1  one 1,000-bead chain, bead 500 an active NOR -> 1,002 particles
  C2  46 chains with hg38 lengths at 100 kb (chr1..22 x2, X x2) = 60,642 + 20 nucleolar = 60,662
  C5  the same at 10 kb = 606,228 + 20 = 606,248
A/B blocks have geometric lengths (mean 20 beads) and alternate; C2/C5 tag 5% of beads "u" = (0.5, 0.5).
Initial positions are confined random walks.  Everything is seeded (numpy PCG64).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

from .seeds import stage_seeds

# particle type codes (stage_prepare/prepare.cpp:14-25)
T_UNKNOWN, T_A, T_B, T_U, T_CENTROMERE, T_ACTIVE_NOR, T_SILENT_NOR, T_NUCLEOLUS = range(8)

HG38 = [  # (name, length bp, approximate centromere midpoint bp)
    ("chr1", 248956422, 123400000), ("chr2", 242193529, 93900000), ("chr3", 198295559, 90900000),
    ("chr4", 190214555, 50000000), ("chr5", 181538259, 48800000), ("chr6", 170805979, 59800000),
    ("chr7", 159345973, 60100000), ("chr8", 145138636, 45200000), ("chr9", 138394717, 43000000),
    ("chr10", 133797422, 39800000), ("chr11", 135086622, 53400000), ("chr12", 133275309, 35500000),
    ("chr13", 114364328, 17700000), ("chr14", 107043718, 17200000), ("chr15", 101991189, 19000000),
    ("chr16", 90338345, 36800000), ("chr17", 83257441, 25100000), ("chr18", 80373285, 18500000),
    ("chr19", 58617616, 26200000), ("chr20", 64444167, 28100000), ("chr21", 46709983, 12000000),
    ("chr22", 50818468, 15000000), ("chrX", 156040895, 60600000),
]
ACROCENTRIC = {"chr13", "chr14", "chr15", "chr21", "chr22"}


@dataclass
class InterphaseDesign:
    """interphase_design (common/simulation_store.hpp:47-53) + what prepare writes beside it."""
    seed: int
    ab_factors: np.ndarray                  # (N, 2)
    particle_types: np.ndarray              # (N,) int
    chains: list                            # [(name, start, end)]
    nucleolar_bonds: np.ndarray             # (M, 2) int (nor, nucleolus)
    positions: np.ndarray                   # (N, 3) initial positions
    master_seed: int = 0
    centromeres: list = field(default_factory=list)  # per chain (start, end) of the centromeric beads

    @property
    def n(self) -> int:
        return int(self.ab_factors.shape[0])


def _ab_blocks(rng, length, mean_block=20.0, u_fraction=0.0):
    ab = np.zeros((length, 2))
    types = np.zeros(length, dtype=np.int32)
    cur = int(rng.integers(0, 2))
    k = 0
    p = 1.0 / mean_block
    while k < length:
        blk = int(rng.geometric(p))
        end = min(length, k + blk)
        if cur == 0:
            ab[k:end] = (1.0, 0.0)
            types[k:end] = T_A
        else:
            ab[k:end] = (0.0, 1.0)
            types[k:end] = T_B
        cur ^= 1
        k = end
    if u_fraction > 0:
        u = rng.random(length) < u_fraction
        ab[u] = (0.5, 0.5)
        types[u] = T_U
    return ab, types


def _confined_walk(rng, length, step, radius, start):
    pts = np.empty((length, 3))
    x = np.array(start, dtype=np.float64)
    for k in range(length):
        pts[k] = x
        d = rng.normal(size=3)
        d *= step / np.linalg.norm(d)
        x = x + d
        r = np.linalg.norm(x)
        if r > radius:  # reflect back into the sphere
            x = x * ((2 * radius - r) / r)
    return pts


def _finish(chains_ab, chains_types, chains_pos, names, nor_offsets, centromeres, master_seed, nucleolus_count=2,
            nucleolus_ab=(0.0, 10.0)):
    ab = np.concatenate(chains_ab)
    types = np.concatenate(chains_types)
    pos = np.concatenate(chains_pos)
    chains = []
    start = 0
    nors = []
    cens = []
    for name, a, nor, cen in zip(names, chains_ab, nor_offsets, centromeres):
        end = start + len(a)
        chains.append((name, start, end))
        if nor is not None:
            types[start + nor] = T_ACTIVE_NOR
            nors.append(start + nor)
        if cen is not None:
            cb, ce = cen
            types[start + cb:start + ce] = np.where(types[start + cb:start + ce] == T_ACTIVE_NOR, T_ACTIVE_NOR,
                                                    T_CENTROMERE)
            cens.append((start + cb, start + ce))
        else:
            cens.append((start, end))
        start = end
    extra_ab, extra_pos, bonds = [], [], []
    idx = ab.shape[0]
    for nor in nors:  # prepare.cpp:232-255 (define_nucleolar_particles)
        for _ in range(nucleolus_count):
            extra_ab.append(nucleolus_ab)
            extra_pos.append(pos[nor])  # transition_interphase.cpp:80-82
            bonds.append((nor, idx))
            idx += 1
    if extra_ab:
        ab = np.concatenate([ab, np.array(extra_ab)])
        pos = np.concatenate([pos, np.array(extra_pos)])
        types = np.concatenate([types, np.full(len(extra_ab), T_NUCLEOLUS, dtype=np.int32)])
    seed = stage_seeds(master_seed)["interphase"]
    return InterphaseDesign(seed=seed, ab_factors=ab, particle_types=types, chains=chains,
                            nucleolar_bonds=np.array(bonds, dtype=np.int64).reshape(-1, 2), positions=pos,
                            master_seed=master_seed, centromeres=cens)


def make_c1(master_seed: int = 1, length: int = 1000) -> InterphaseDesign:
    """C1: one 1,000-bead chain; bead 500 an active NOR (+2 nucleolar beads); random walk of step 0.1 from
    the origin reflected into a sphere of radius 1.5."""
    rng = np.random.default_rng(np.random.PCG64(1000 + master_seed))
    ab, types = _ab_blocks(rng, length)
    pos = _confined_walk(rng, length, 0.1, 1.5, (0.0, 0.0, 0.0))
    return _finish([ab], [types], [pos], ["chr1"], [length // 2], [(length // 2 - 5, length // 2 + 5)],
                   master_seed)


def hg38_chain_lengths(bin_bp: int = 100_000):
    out = []
    for copy in ("a", "b"):
        for name, size, cen in HG38:
            out.append((f"{name}{copy}", math.ceil(size / bin_bp), cen // bin_bp, name))
    return out


def make_diploid(master_seed: int = 1, bin_bp: int = 100_000, radius: float = 1.9, step: float = 0.1
                 ) -> InterphaseDesign:
    """C2 (bin 100 kb) / C5 (bin 10 kb): female diploid hg38, 46 chains."""
    rng = np.random.default_rng(np.random.PCG64(2000 + master_seed + bin_bp))
    abs_, types_, poss, names, nors, cens = [], [], [], [], [], []
    for name, length, cen_bin, base in hg38_chain_lengths(bin_bp):
        ab, types = _ab_blocks(rng, length, u_fraction=0.05)
        d = rng.normal(size=3)
        start = d / np.linalg.norm(d) * radius * rng.random() ** (1 / 3) * 0.8
        pos = _confined_walk(rng, length, step, radius, start)
        abs_.append(ab)
        types_.append(types)
        poss.append(pos)
        names.append(name)
        nors.append(min(5, length - 1) if base in ACROCENTRIC else None)
        half = max(1, length // 200)
        c = min(max(cen_bin, half), length - half)
        cens.append((c - half, c + half))
    return _finish(abs_, types_, poss, names, nors, cens, master_seed)


def make_c2(master_seed: int = 1) -> InterphaseDesign:
    return make_diploid(master_seed, 100_000)


def make_c5(master_seed: int = 1) -> InterphaseDesign:
    return make_diploid(master_seed, 10_000, step=0.1 / math.sqrt(10.0))

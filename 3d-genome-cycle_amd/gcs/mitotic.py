"""Mitotic stages (C3): anaphase/telophase (stage_anatelophase) and prometaphase (stage_prometaphase).

`anatelophase_design` / `prometaphase_design` restate prepare's coarse-graining of the interphase chains
(stage_prepare/prepare.cpp:279-372).  `build_anatelophase` / `build_prometaphase` compose the force fields exactly as
the stage drivers do (stage_anatelophase/simulation_driver.cpp:56-189, stage_prometaphase/simulation_driver.cpp:
38-182) on any backend with the engine's method names (the HIP `Engine`, or the CPU oracle in tests), and the
drivers keep the reference's stage order, field swap and seed plumbing (anatelophase :192-310, prometaphase
:185-246).  The per-step callbacks only sample and log, so the host regains control at interval boundaries.
"""
from __future__ import annotations

import math
import sys
import time as _time
from dataclasses import dataclass, field

import numpy as np

from . import _abi as A
from .config import MitoticPhaseConfig
from .seeds import MT19937_64, stage_seeds

# mitotic_particle_type (prepare.cpp:14-25 mitotic enum)
T_UNKNOWN, T_ARM, T_KINETOCHORE = 0, 1, 2


@dataclass
class MitoticDesign:
    """anatelophase_design / prometaphase_design (common/simulation_store.hpp)."""
    seed: int
    particle_types: np.ndarray
    chains: list                      # [(name, start, end, kinetochore)]
    sister_chromatids: list = field(default_factory=list)  # [(target chain, sister chain)] (prometaphase)
    pole_positions: np.ndarray = None  # (2, 3) (prometaphase)

    @property
    def n(self) -> int:
        return int(self.particle_types.shape[0])


def anatelophase_design(idesign, cfg: MitoticPhaseConfig, master_seed=None) -> MitoticDesign:
    """prepare.cpp:279-313: each interphase chain coarse-grained by `coarse_graining` (floor), the kinetochore at
    the bin of the centromeric region's midpoint."""
    cg = cfg.coarse_graining
    types, chains = [], []
    for (name, start, end), (cs, ce) in zip(idesign.chains, idesign.centromeres):
        length = end - start
        coarse = length // cg
        c0 = len(types)
        koff = ((cs + ce) // 2 - start) // cg
        kin = None
        for b in range(coarse):
            if b == koff:
                kin = len(types)
                types.append(T_KINETOCHORE)
            else:
                types.append(T_ARM)
        chains.append((name, c0, c0 + coarse, kin))
    ms = idesign.master_seed if master_seed is None else master_seed
    return MitoticDesign(seed=stage_seeds(ms)["anaphase"], particle_types=np.array(types, dtype=np.int32),
                         chains=chains)


def prometaphase_design(adesign: MitoticDesign, cfg: MitoticPhaseConfig, master_seed: int) -> MitoticDesign:
    """prepare.cpp:319-372: every anatelophase chain doubled into target + sister ("-copy"), interleaved; poles at
    -/+ spindle_axis."""
    chains, sisters, types = [], [], []
    for k, (name, start, end, kin) in enumerate(adesign.chains):
        if kin is None:
            raise ValueError(f"chain {name} has no kinetochore bead (prepare.cpp:333 dereferences it)")
        length = end - start
        koff = kin - start
        ts = 2 * start
        chains.append((name, ts, ts + length, ts + koff))
        chains.append((name + "-copy", ts + length, ts + 2 * length, ts + length + koff))
        sisters.append((2 * k, 2 * k + 1))
        seg = adesign.particle_types[start:end]
        types.extend(seg.tolist())
        types.extend(seg.tolist())
    axis = np.asarray(cfg.spindle_axis, dtype=np.float64)
    return MitoticDesign(seed=stage_seeds(master_seed)["prometaphase"], particle_types=np.array(types, dtype=np.int32),
                         chains=chains, sister_chromatids=sisters, pole_positions=np.stack([np.zeros(3) - axis, np.zeros(3) + axis]))  # origin -/+ axis


class StdNormal:
    """std::normal_distribution<double> (libstdc++ Marsaglia polar, bits/random.tcc:1795-1830) over
    generate_canonical<double, 53>(mt19937_64): one object keeps its cached second value."""

    def __init__(self, rng: MT19937_64):
        self.rng = rng
        self.saved = None

    def _u(self):
        r = float(self.rng()) / 18446744073709551616.0
        return r if r < 1.0 else math.nextafter(1.0, 0.0)

    def __call__(self) -> float:
        if self.saved is not None:
            v, self.saved = self.saved, None
            return v
        while True:
            x = 2.0 * self._u() - 1.0
            y = 2.0 * self._u() - 1.0
            r2 = x * x + y * y
            if r2 <= 1.0 and r2 != 0.0:
                break
        mult = math.sqrt(-2.0 * math.log(r2) / r2)
        self.saved = x * mult
        return y * mult


def _writer(store):
    """the stage's sampling writes on a background thread (gcs.store.AsyncWriter), or None without a store"""
    if store is None:
        return None
    from .store import AsyncWriter
    return AsyncWriter(store)


def sampled_positions(system):
    from .store import sampled_positions as sp
    return sp(system)


def normal_vector(rng: MT19937_64) -> np.ndarray:
    """stage_anatelophase/simulation_driver.cpp:25-32: a FRESH normal_distribution per vector."""
    nd = StdNormal(rng)
    return np.array([nd(), nd(), nd()])


def _kfiber_specs(design, cfg, idx_chains, decay, length):
    """kinetochore_fiber_forcefield::add_kinetochore with mobility = core_mobility / chain length
    (anatelophase :160-172, prometaphase :138-157)."""
    specs = []
    for c in idx_chains:
        _, start, end, kin = design.chains[c]
        specs.append((kin, cfg.core_mobility / float(end - start), decay, length))
    return specs


def _bend_ranges(design, cfg):
    out = []
    for _, start, end, kin in design.chains:
        if cfg.penalize_centromere_bending:
            out.append((start, end))
        else:
            out.append((start, kin))
            out.append((kin + 1, end))
    return out


def build_anatelophase(backend_cls, design: MitoticDesign, cfg: MitoticPhaseConfig, **backend_kw):
    """setup_particles + setup_forcefield (stage_anatelophase/simulation_driver.cpp:56-189).  The anaphase bonds and
    bending are active; the kinetochore fibers, the packing well and the telophase bonds/bending are added by the
    driver's stages.  Returns (system, handles)."""
    sys_ = backend_cls(design.n, mobilities=np.full(design.n, cfg.core_mobility), **backend_kw)
    h = {}
    h["repulsion"] = sys_.add_neighbor_softcore(a_energy=cfg.core_repulsion, a_diameter=cfg.core_diameter,
                                                neighbor_distance=cfg.core_diameter, mix=False)
    ranges = [(s, e) for _, s, e, _ in design.chains]
    h["anaphase_bonds"] = sys_.add_bonded_pairwise(A.POT_SEMISPRING, a_spring=cfg.bond_spring,
                                                   a_length=cfg.bond_length, ranges=ranges)
    h["anaphase_bending"] = sys_.add_bonded_triplewise(cfg.bending_energy, ranges=_bend_ranges(design, cfg))
    return sys_, h


class AnatelophaseDriver:
    """run_initialization / run_dragging_stage / run_packing_stage (stage_anatelophase/simulation_driver.cpp:192-310)."""

    def __init__(self, system, handles, design: MitoticDesign, cfg: MitoticPhaseConfig, store=None, log=sys.stderr):
        self.sys, self.h, self.design, self.cfg = system, handles, design, cfg
        self.store, self.log = store, log
        self.random = MT19937_64(design.seed)  # _random(_design.seed) (:39)

    def initial_rods(self) -> np.ndarray:
        """run_initialization without a stored structure (:213-229): each chain a rod of bond_length steps around
        -spindle_axis + anaphase_start_stddev * N(0, 1)^3, direction normalize(N(0, 1)^3)."""
        cfg = self.cfg
        x = np.zeros((self.design.n, 3))
        start_center = np.zeros(3) - np.asarray(cfg.spindle_axis, dtype=np.float64)  # origin - spindle_axis
        for _, start, end, _ in self.design.chains:
            centroid = start_center + cfg.anaphase_start_stddev * normal_vector(self.random)
            d = normal_vector(self.random)
            step = cfg.bond_length * d / np.linalg.norm(d)
            pos = centroid - step * float(end - start) / 2
            for i in range(start, end):
                x[i] = pos
                pos = pos + step
        return x

    def run_initialization(self, positions=None):
        if positions is not None:  # "Initial structure may be given" (:203-211)
            x = np.asarray(positions, dtype=np.float64)
            if x.shape != (self.design.n, 3):
                raise RuntimeError("initial structure size mismatch")
        else:
            x = self.initial_rods()
        self.sys.set_positions(x)

    def _stage(self, name, steps, seed):
        cfg = self.cfg
        every = math.gcd(cfg.sampling_interval, cfg.logging_interval)
        self._writer = _writer(self.store)
        try:
            # a sample's frame is handed to the writer after the next run is enqueued (the device then computes
            # while the host queues the write; the frames and their order are unchanged)
            pending = self._callback(name, 0)
            done = 0
            while done < steps:
                k = min(every - done % every, steps - done)
                self.sys.run(k, first_step=done, temperature=cfg.temperature, timestep=cfg.timestep, seed=seed)
                if pending is not None:
                    pending()
                done += k
                pending = self._callback(name, done)
            if pending is not None:
                pending()
        except BaseException as exc:
            if self._writer is not None:
                self._writer.close(exc)
            raise
        else:
            if self._writer is not None:
                self._writer.close()

    def _callback(self, name, step):
        """the step's sample and log line; returns the frame write (or None), for the caller to hand over once the
        next run is enqueued"""
        cfg = self.cfg
        write = None
        if step % cfg.sampling_interval == 0 and self.store is not None:
            x, q = sampled_positions(self.sys)
            write = lambda: self._writer.save_frame(name, step, x, None, quantized=q)  # noqa: E731
        if step % cfg.logging_interval == 0 and self.log is not None:
            e, _ = self.sys.compute_energy()
            stamp = _time.strftime("%Y-%m-%d %H:%M:%S")
            print(f"[{name}] {stamp}\t{step}\tE: {e / self.design.n:g}", file=self.log)
        return write

    def run_dragging_stage(self, steps=None):
        """:232-262: kinetochore fibers to the pole at anaphase_spindle_shift"""
        cfg = self.cfg
        pole = np.asarray(cfg.anaphase_spindle_shift, dtype=np.float64)
        specs = _kfiber_specs(self.design, cfg, range(len(self.design.chains)), cfg.kfiber_decay_rate_anaphase,
                              cfg.kfiber_length_anaphase)
        self.h["dragging"] = self.sys.add_kinetochore_fiber(pole, specs)
        self._stage("anaphase", cfg.anaphase_steps if steps is None else steps, self.random())

    def run_packing_stage(self, steps=None):
        """:265-310: fibers off, packing well on, anaphase bonds/bending swapped for the telophase ones"""
        cfg = self.cfg
        s = self.sys
        s.remove_forcefield(self.h.pop("dragging"))
        self.h["packing"] = s.add_point_source(A.POT_SEMISPRING, [0.0, 0.0, 0.0], spring=cfg.telophase_packing_spring,
                                               length=cfg.telophase_packing_radius)
        s.remove_forcefield(self.h.pop("anaphase_bonds"))
        s.remove_forcefield(self.h.pop("anaphase_bending"))
        ranges = [(a, b) for _, a, b, _ in self.design.chains]
        self.h["telophase_bonds"] = s.add_bonded_pairwise(
            A.POT_SEMISPRING, a_spring=cfg.bond_spring * cfg.telophase_bond_spring_multiplier,
            a_length=cfg.bond_length, ranges=ranges)
        self.h["telophase_bending"] = s.add_bonded_triplewise(
            cfg.bending_energy * cfg.telophase_bending_energy_multiplier, ranges=_bend_ranges(self.design, cfg))
        self._stage("telophase", cfg.telophase_steps if steps is None else steps, self.random())

    def run(self, positions=None, anaphase_steps=None, telophase_steps=None):
        self.run_initialization(positions)
        self.run_dragging_stage(anaphase_steps)
        self.run_packing_stage(telophase_steps)


def build_prometaphase(backend_cls, design: MitoticDesign, cfg: MitoticPhaseConfig, **backend_kw):
    """stage_prometaphase/simulation_driver.cpp:24-182: repulsion, chain bonds + bending, sister bonds (spring
    constant bond_spring, length sister_separation: the driver does not use sister_spring), kinetochore fibers to
    both poles, polar-ejection force-flux point sources at both poles."""
    sys_ = backend_cls(design.n, mobilities=np.full(design.n, cfg.core_mobility), **backend_kw)
    h = {}
    h["repulsion"] = sys_.add_neighbor_softcore(a_energy=cfg.core_repulsion, a_diameter=cfg.core_diameter,
                                                neighbor_distance=cfg.core_diameter, mix=False)
    ranges = [(s, e) for _, s, e, _ in design.chains]
    h["bonds"] = sys_.add_bonded_pairwise(A.POT_SEMISPRING, a_spring=cfg.bond_spring, a_length=cfg.bond_length,
                                          ranges=ranges)
    h["bending"] = sys_.add_bonded_triplewise(cfg.bending_energy, ranges=_bend_ranges(design, cfg))
    pairs = [(design.chains[t][3], design.chains[s][3]) for t, s in design.sister_chromatids]
    h["sisters"] = sys_.add_bonded_pairwise(A.POT_SEMISPRING, a_spring=cfg.bond_spring,
                                            a_length=cfg.sister_separation, pairs=pairs)
    tp, sp = design.pole_positions
    targets = [t for t, _ in design.sister_chromatids]
    sisters = [s for _, s in design.sister_chromatids]
    dec, ln = cfg.kfiber_decay_rate_prometaphase, cfg.kfiber_length_prometaphase
    h["kfiber_target"] = sys_.add_kinetochore_fiber(tp, _kfiber_specs(design, cfg, targets, dec, ln))
    h["kfiber_sister"] = sys_.add_kinetochore_fiber(sp, _kfiber_specs(design, cfg, sisters, dec, ln))
    rd = math.sqrt(cfg.polar_ejection_cross_section)
    for k, pole in enumerate((tp, sp)):
        h[f"ejection{k}"] = sys_.add_point_source(A.POT_FORCE_FLUX, list(pole), force=cfg.polar_ejection_force,
                                                  reactive_distance=rd)
    return sys_, h


class PrometaphaseDriver:
    """run_initialization (a stored structure is required, :196-210) + run_sampling (:213-236)."""

    def __init__(self, system, design: MitoticDesign, cfg: MitoticPhaseConfig, store=None, log=sys.stderr):
        self.sys, self.design, self.cfg, self.store, self.log = system, design, cfg, store, log
        self.random = MT19937_64(design.seed)  # _random.seed(_design.seed) (:18)
        self.time = 0.0

    def run(self, positions, steps=None):
        x = np.asarray(positions, dtype=np.float64)
        if x.shape != (self.design.n, 3):
            raise RuntimeError("initial structure size mismatch")
        self.sys.set_positions(x)
        cfg = self.cfg
        steps = cfg.prometaphase_steps if steps is None else steps
        every = math.gcd(cfg.sampling_interval, cfg.logging_interval)
        self._writer = _writer(self.store)
        try:
            pending = self._callback(0)  # (frame writes handed over after the next run is enqueued, as above)
            seed = self.random()  # .seed = _random() (:230; callback(0) draws nothing)
            done = 0
            while done < steps:
                k = min(every - done % every, steps - done)
                self.sys.run(k, first_step=done, temperature=cfg.temperature, timestep=cfg.timestep, seed=seed)
                if pending is not None:
                    pending()
                done += k
                pending = self._callback(done)
            if pending is not None:
                pending()
        except BaseException as exc:
            if self._writer is not None:
                self._writer.close(exc)
            raise
        else:
            if self._writer is not None:
                self._writer.close()

    def _callback(self, step):
        cfg = self.cfg
        self.time = step * cfg.timestep  # update_context (:239-243)
        if step % cfg.logging_interval == 0 and self.log is not None:
            e, _ = self.sys.compute_energy()
            stamp = _time.strftime("%Y-%m-%d %H:%M:%S")
            print(f"[prometaphase] {stamp}\t{step}\tE: {e:g}", file=self.log)
        if step % cfg.sampling_interval == 0 and self.store is not None:
            x, q = sampled_positions(self.sys)
            return lambda: self._writer.save_frame("prometaphase", step, x, None, quantized=q)
        return None

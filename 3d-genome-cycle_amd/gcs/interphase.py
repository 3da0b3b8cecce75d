"""Interphase stage: force-field composition and the host driver loop.

`build_interphase` mirrors simulation_driver::setup_particles / setup_forcefield / setup_context
(stage_interphase/simulation_driver_particles.cpp:9-35, simulation_driver_forcefield.cpp:9-244,
stage_interphase/simulation_driver.cpp:35-43) on any backend with the engine's method names: the HIP `Engine` (product)
or the CPU oracle (tests only).  `InterphaseDriver` mirrors run_relaxation / run_simulation
(simulation_driver_relaxation.cpp:8-56, simulation_driver_interphase.cpp:9-90): the per-step callback's
state updates live on the device; the host regains control at interval boundaries only.
"""
from __future__ import annotations

import sys
import time as _time

import numpy as np

from . import _abi as A
from .config import InterphaseConfig
from .seeds import interphase_bd_seeds


def interphase_mobilities(design, cfg: InterphaseConfig) -> np.ndarray:
    """simulation_driver_particles.cpp:19-34"""
    mu = np.ones(design.n)
    for _, start, end in design.chains:
        ab = design.ab_factors[start:end]
        mu[start:end] = np.where(ab[:, 0] >= ab[:, 1], cfg.a_core_mobility, cfg.b_core_mobility)
    for nor, nuc in design.nucleolar_bonds:
        mu[nuc] = cfg.nucleolus_mobility
    return mu


def add_interphase_forcefields(sys_, design, cfg: InterphaseConfig) -> dict:
    """simulation_driver_forcefield.cpp:9-244, in the reference's add_forcefield order."""
    h = {}
    # setup_repulsive_forcefield (:20-53)
    h["repulsion"] = sys_.add_neighbor_softcore(
        a_energy=cfg.a_core_repulsion, a_diameter=cfg.a_core_diameter, b_energy=cfg.b_core_repulsion,
        b_diameter=cfg.b_core_diameter, neighbor_distance=max(cfg.a_core_diameter, cfg.b_core_diameter),
        mix=True, scaled=True)
    ranges = [(s, e) for _, s, e in design.chains]
    # setup_connectivity_forcefield (:56-96): semispring, K = a*100 + b*50, l = a*0 + b*0, scaled
    h["chain_bonds"] = sys_.add_bonded_pairwise(
        A.POT_SEMISPRING, a_spring=cfg.a_core_bond_spring, b_spring=cfg.b_core_bond_spring,
        a_length=cfg.a_core_bond_length, b_length=cfg.b_core_bond_length, mix=True, scaled=True,
        ranges=ranges, stride=1)
    # setup_loop_forcefield (:99-136): harmonic i,i+2, K = (a*K2a + b*K2b)/s^2
    h["loop_bonds"] = sys_.add_bonded_pairwise(
        A.POT_HARMONIC, a_spring=cfg.a_core_2nd_bond_spring, b_spring=cfg.b_core_2nd_bond_spring, mix=True,
        scaled=True, ranges=ranges, stride=2)
    # setup_nucleolus_forcefield (:139-186)
    bonds = np.asarray(design.nucleolar_bonds, dtype=np.int64).reshape(-1, 2)
    h["nucleolar_bonds"] = sys_.add_bonded_pairwise(
        A.POT_SEMISPRING, a_spring=cfg.nucleolus_bond_spring, a_length=cfg.nucleolus_bond_length, mix=False,
        scaled=True, pairs=bonds)
    if cfg.nucleolus_droplet_energy != 0:
        h["droplet"] = sys_.add_neighbor_softwell(
            energy=cfg.nucleolus_droplet_energy, decay_distance=cfg.nucleolus_droplet_decay,
            cutoff=cfg.nucleolus_droplet_cutoff, targets=bonds[:, 1] if bonds.size else [])
    # setup_membrane_forcefield (:189-244)
    h["wall_in"] = sys_.add_ellipsoid_inward(
        a_energy=cfg.a_core_repulsion, a_diameter=cfg.a_core_diameter / 2, b_energy=cfg.b_core_repulsion,
        b_diameter=cfg.b_core_diameter / 2, wall_a=cfg.wall_ab_factor.a, wall_b=cfg.wall_ab_factor.b,
        center=(0.0, 0.0, 0.0), mix=True, scaled=True)
    h["wall_out"] = sys_.add_ellipsoid_outward(spring=cfg.wall_packing_spring, center=(0.0, 0.0, 0.0))
    return h


def interphase_schedule(cfg: InterphaseConfig) -> dict:
    """The callback's update_core_scale + update_wall_semiaxes (simulation_driver_interphase.cpp:67-90)."""
    return dict(update_time=1, update_scales=1, update_wall=1, timestep=cfg.timestep,
                core_scale_init=cfg.core_scale_init, core_scale_tau=cfg.core_scale_tau,
                bond_scale_init=cfg.bond_scale_init, bond_scale_tau=cfg.bond_scale_tau,
                wall_semiaxes_spring=cfg.wall_semiaxes_spring, wall_mobility=cfg.wall_mobility)


def initial_context(cfg: InterphaseConfig) -> dict:
    """stage_interphase/simulation_driver.cpp:35-43"""
    return {"step": 0, "time": 0.0, "wall_semiaxes": list(cfg.wall_semiaxes_init), "core_scale": cfg.core_scale_init,
            "bond_scale": cfg.bond_scale_init}


def build_interphase(backend_cls, design, cfg: InterphaseConfig, **backend_kw):
    """Construct a backend system carrying the interphase model; returns (system, handles)."""
    mu = interphase_mobilities(design, cfg)
    sys_ = backend_cls(design.n, mobilities=mu, ab_factors=design.ab_factors, **backend_kw)
    handles = add_interphase_forcefields(sys_, design, cfg)
    sys_.set_context(initial_context(cfg))
    sys_.set_positions(design.positions)
    return sys_, handles


SINGLE_SKIN_BASE_F64 = 400  # GCS_OPT_LIST_SKIN_BASE of a stage's one trajectory (per mille of the pair cutoff)


class InterphaseDriver:
    """run_relaxation + run_simulation with the reference callback order, chunked at interval boundaries.  On an fp64
    engine it sets GCS_OPT_LIST_SKIN_BASE to SINGLE_SKIN_BASE_F64 (the stage's one trajectory; set the option again
    after construction to override)."""

    def __init__(self, system, design, cfg: InterphaseConfig, store=None, log=sys.stderr):
        self.sys = system
        self.design = design
        self.cfg = cfg
        self.store = store
        self.log = log
        self.relaxation_seed, self.interphase_seed = interphase_bd_seeds(design.seed)
        self.context = initial_context(cfg)
        self.mean_energy = 0.0
        self._writer = None
        # one trajectory alone on its GPU is latency-bound: at fp64 it takes longer lists and fewer rebuilds than the
        # engine's default, which suits several trajectories per GPU (the 700k-step stage 1.1 % faster at s1 = 400
        # than at 350 per mille, profiles/r06h2_skin_base.txt; trajectories stay bitwise reproducible for a given s1)
        if getattr(system, "precision", None) == 64 and hasattr(system, "set_option"):
            from . import _abi
            system.set_option(_abi.OPT_LIST_SKIN_BASE, SINGLE_SKIN_BASE_F64)

    def _out(self):
        """the store's sampling writes, on a background writer for the length of a stage (gcs.store.AsyncWriter)"""
        if self._writer is None:
            from .store import AsyncWriter
            self._writer = AsyncWriter(self.store)
        return self._writer

    def _close_out(self, propagating=None):
        if self._writer is not None:
            w, self._writer = self._writer, None
            w.close(propagating)

    def _progress(self, phase, step):
        if self.log is None:
            return
        c = self.sys.get_context()
        r = float(np.cbrt(np.prod(c["wall_semiaxes"])))
        stamp = _time.strftime("%Y-%m-%d %H:%M:%S")
        print(f"[{phase}] {stamp}\t{step}\tt: {c['time']:g}\tR: {r:g}\tE: {self.mean_energy:g}", file=self.log)

    def _energy(self):
        tot, _ = self.sys.compute_energy()
        self.mean_energy = tot / self.design.n

    def run_relaxation(self, steps=None):
        """simulation_driver_relaxation.cpp:8-56 (no schedule updates; spacestep-limited)"""
        cfg = self.cfg
        steps = cfg.relaxation_steps if steps is None else steps
        self.sys.set_schedule(update_time=0, update_scales=0, update_wall=0, timestep=cfg.timestep)
        every = np.gcd(cfg.relaxation_logging_interval, cfg.relaxation_sampling_interval)
        try:
            self._callback_relax(0)
            done = 0
            while done < steps:
                k = min(every - done % every, steps - done)
                self.sys.run(k, first_step=done, temperature=cfg.temperature, timestep=cfg.timestep,
                             spacestep=cfg.relaxation_spacestep, seed=self.relaxation_seed)
                done += k
                self._callback_relax(done)
        except BaseException as exc:
            self._close_out(exc)
            raise
        else:
            self._close_out()

    def _callback_relax(self, step):
        cfg = self.cfg
        log = step % cfg.relaxation_logging_interval == 0
        sample = step % cfg.relaxation_sampling_interval == 0
        if log or sample:
            self._energy()
        if log:
            self._progress("relaxation", step)
        if sample and self.store is not None:
            from .store import sampled_positions
            x, q = sampled_positions(self.sys)
            self._out().save_frame("relaxation", step, x, self._context_record(), quantized=q)

    def _context_record(self):
        c = self.sys.get_context()
        return {"time": c["time"], "wall_semiaxes": c["wall_semiaxes"], "core_scale": c["core_scale"],
                "bond_scale": c["bond_scale"], "mean_energy": self.mean_energy, "wall_energy": 0.0}

    def contact_distance(self, step):
        """The distance contact_map::update uses in callback(step): the one update_core_scale set in callback(step - 1)
        (simulation_driver_interphase.cpp:38-39, 68-76), i.e. contactmap_distance x core_scale(time (step - 1) dt).
        callback(0) runs before any update_core_scale: the map's initial distance 0 (contact_map.hpp:65) -> no pairs."""
        cfg = self.cfg
        if step <= 0:
            return 0.0
        t = (step - 1) * cfg.timestep
        cs = 1 - (1 - cfg.core_scale_init) * np.exp(-t / cfg.core_scale_tau)
        return cfg.contactmap_distance * cs

    def run_simulation(self, steps=None, contacts=True):
        """simulation_driver_interphase.cpp:9-64"""
        cfg = self.cfg
        steps = cfg.steps if steps is None else steps
        self.sys.set_schedule(**interphase_schedule(cfg))
        intervals = [cfg.logging_interval, cfg.sampling_interval]
        if contacts:
            intervals.append(cfg.contactmap_update_interval)
            self.sys.contacts_clear()
        every = int(np.gcd.reduce(intervals))
        if hasattr(self.sys, "set_option"):  # replay whole callback intervals from one captured graph
            self.sys.set_option(A.OPT_GRAPH_STEPS, every)
        # callback(0): time 0, energy, log/sample, then update_core_scale + update_wall_semiaxes
        try:
            self._callback_sim(0, contacts)
            self.sys.apply_schedule(0)
            done = 0
            while done < steps:
                k = min(every - done % every, steps - done)
                self.sys.run(k, first_step=done, temperature=cfg.temperature, timestep=cfg.timestep,
                             seed=self.interphase_seed)
                done += k
                self._callback_sim(done, contacts)
        except BaseException as exc:
            self._close_out(exc)
            raise
        else:
            self._close_out()

    def _callback_sim(self, step, contacts=True):
        cfg = self.cfg
        log = step % cfg.logging_interval == 0
        sample = step % cfg.sampling_interval == 0
        if log or sample:
            self._energy()
        if log:
            self._progress("interphase", step)
        if sample and self.store is not None:
            from .store import sampled_positions
            x, q = sampled_positions(self.sys)
            self._out().save_frame("interphase", step, x, self._context_record(), quantized=q)
        if contacts and step % cfg.contactmap_update_interval == 0:
            d = self.contact_distance(step)
            if d > 0:  # distance 0 finds no pair (callback(0))
                self.sys.contacts_update(d)
        if contacts and sample and (step // cfg.sampling_interval) % cfg.contactmap_output_window == 0:
            table = self.sys.contacts_accumulate()
            if self.store is not None:
                self._out().save_contacts(step, table)
            self.last_contacts = table
            self.sys.contacts_clear()

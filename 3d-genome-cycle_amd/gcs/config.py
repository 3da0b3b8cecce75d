"""Simulation configuration with the reference's field names, defaults and JSON rules.

Mirrors common/simulation_config.hpp:8-130 and the JSON traits of common/simulation_config.cpp:42-164:
every field inside "mitotic_phase" / "interphase" is optional (the struct default applies), both sections
are required, and ``a_core_2nd_bond_spring`` / ``b_core_2nd_bond_spring`` are NOT read from JSON (they are
absent from JSONCONS_N_MEMBER_TRAITS at simulation_config.cpp:109-118), so the i,i+2 loop field always has
K = 0 unless set programmatically.
"""
from __future__ import annotations

import dataclasses
import json
from dataclasses import dataclass, field


@dataclass
class ABFactor:
    a: float = 0.0
    b: float = 0.0


@dataclass
class MitoticPhaseConfig:  # simulation_config.hpp:15-58
    temperature: float = 1.0
    timestep: float = 1e-4
    anaphase_steps: int = 200000
    telophase_steps: int = 50000
    prometaphase_steps: int = 400000
    sampling_interval: int = 1000
    logging_interval: int = 10000
    anaphase_start_stddev: float = 1.0
    coarse_graining: int = 100
    core_diameter: float = 0.3
    core_repulsion: float = 2.0
    bond_length: float = 0.3
    bond_spring: float = 1000.0
    bending_energy: float = 1.0
    penalize_centromere_bending: bool = False
    core_mobility: float = 0.1
    sister_separation: float = 0.3
    sister_spring: float = 1000.0
    spindle_axis: tuple = (0.0, 5.0, 0.0)
    kfiber_decay_rate_prometaphase: float = 1.0
    kfiber_decay_rate_anaphase: float = 1.0
    kfiber_length_prometaphase: float = 0.0
    kfiber_length_anaphase: float = 0.0
    polar_ejection_force: float = 0.0
    polar_ejection_cross_section: float = 0.0
    anaphase_spindle_shift: tuple = (0.0, 2.0, 0.0)
    telophase_packing_radius: float = 1.5
    telophase_packing_spring: float = 100.0
    telophase_bond_spring_multiplier: float = 1.0
    telophase_bending_energy_multiplier: float = 1.0


@dataclass
class InterphaseConfig:  # simulation_config.hpp:61-115
    temperature: float = 1.0
    timestep: float = 1e-5
    steps: int = 700000
    sampling_interval: int = 1000
    logging_interval: int = 1000
    relaxation_spacestep: float = 0.001
    relaxation_steps: int = 10000
    relaxation_sampling_interval: int = 1000
    relaxation_logging_interval: int = 100
    contactmap_distance: float = 0.24
    contactmap_update_interval: int = 20
    contactmap_output_window: int = 10
    a_core_diameter: float = 0.30
    b_core_diameter: float = 0.24
    a_core_repulsion: float = 2.5
    b_core_repulsion: float = 2.5
    a_core_bond_spring: float = 100.0
    b_core_bond_spring: float = 50.0
    a_core_bond_length: float = 0.0
    b_core_bond_length: float = 0.0
    a_core_2nd_bond_spring: float = 0.0
    b_core_2nd_bond_spring: float = 0.0
    a_core_mobility: float = 1.0
    b_core_mobility: float = 1.0
    core_scale_init: float = 0.5
    core_scale_tau: float = 0.5
    bond_scale_init: float = 0.5
    bond_scale_tau: float = 0.5
    nucleolus_bead_count: int = 2
    nucleolus_ab_factor: ABFactor = field(default_factory=lambda: ABFactor(0.0, 10.0))
    nucleolus_bond_spring: float = 10.0
    nucleolus_bond_length: float = 0.0
    nucleolus_droplet_energy: float = 0.3
    nucleolus_droplet_decay: float = 0.2
    nucleolus_droplet_cutoff: float = 0.4
    nucleolus_mobility: float = 1.0
    wall_semiaxes_init: tuple = (2.0, 2.0, 2.0)
    wall_semiaxes_spring: tuple = (3e4, 3e4, 3e4)
    wall_packing_spring: float = 1000.0
    wall_ab_factor: ABFactor = field(default_factory=lambda: ABFactor(0.0, 10.0))
    wall_mobility: float = 2e-4


def resolution_scaled(cfg: "InterphaseConfig", bin_ratio: float) -> "InterphaseConfig":
    """The interphase force field for beads `bin_ratio` times finer than the 100 kb default (C5: 10 kb, ratio 10),
    rescaled so a bead's neighbourhood looks the same: every bead-scale length (core and droplet diameters, bond
    lengths, contact distance) x f, every bead-scale spring x f^-2, f = bin_ratio^(-1/3) (the bead volume is
    bin_ratio times smaller).  The timestep x f^2: with springs x f^-2 the explicit Euler-Maruyama update keeps
    the same k mu dt (the 10 kb soft core's stiffest pairs reach k mu dt ~ 1.6 at the 100 kb timestep, where
    the fp64 reference itself amplifies a 1-ulp perturbation of the start to 3e-2 in 10 steps -- DESIGN.md §6);
    the Brownian time sigma^2 / D of a bead scales the same way.  Energies, mobilities, the wall and the schedule
    (in time units) are unchanged.  The reference has no 10 kb configuration of its own
    (common/simulation_config.hpp:61-115 are the 100 kb defaults); this is the benchmark's stated choice
    (DESIGN.md "Measurement")."""
    import dataclasses
    f = bin_ratio ** (-1.0 / 3.0)
    k = f ** -2
    return dataclasses.replace(
        cfg,
        timestep=cfg.timestep * f * f,
        a_core_diameter=cfg.a_core_diameter * f, b_core_diameter=cfg.b_core_diameter * f,
        a_core_bond_length=cfg.a_core_bond_length * f, b_core_bond_length=cfg.b_core_bond_length * f,
        a_core_bond_spring=cfg.a_core_bond_spring * k, b_core_bond_spring=cfg.b_core_bond_spring * k,
        a_core_2nd_bond_spring=cfg.a_core_2nd_bond_spring * k, b_core_2nd_bond_spring=cfg.b_core_2nd_bond_spring * k,
        nucleolus_bond_spring=cfg.nucleolus_bond_spring * k, nucleolus_bond_length=cfg.nucleolus_bond_length * f,
        nucleolus_droplet_decay=cfg.nucleolus_droplet_decay * f,
        nucleolus_droplet_cutoff=cfg.nucleolus_droplet_cutoff * f,
        contactmap_distance=cfg.contactmap_distance * f)


# fields the reference's JSON traits do not list (common/simulation_config.cpp:88-118)
NOT_IN_JSON = {"a_core_2nd_bond_spring", "b_core_2nd_bond_spring"}


@dataclass
class SimulationConfig:
    mitotic_phase: MitoticPhaseConfig = field(default_factory=MitoticPhaseConfig)
    interphase: InterphaseConfig = field(default_factory=InterphaseConfig)
    source: str = ""


def _apply(obj, section: dict, skip=frozenset()):
    for f in dataclasses.fields(obj):
        if f.name in skip or f.name not in section:
            continue
        v = section[f.name]
        cur = getattr(obj, f.name)
        if isinstance(cur, ABFactor):
            if not (isinstance(v, list) and len(v) == 2):
                raise ValueError(f"{f.name}: expected [a, b]")
            v = ABFactor(float(v[0]), float(v[1]))
        elif isinstance(cur, tuple):
            if not (isinstance(v, list) and len(v) == 3):
                raise ValueError(f"{f.name}: expected [x, y, z]")
            v = tuple(float(x) for x in v)
        elif isinstance(cur, bool):
            v = bool(v)
        elif isinstance(cur, int):
            v = int(v)
        else:
            v = float(v)
        setattr(obj, f.name, v)


def parse_simulation_config(text: str) -> SimulationConfig:
    """simulation_config.cpp:151-156 (decode_json with the member traits above)."""
    doc = json.loads(text)
    if "mitotic_phase" not in doc or "interphase" not in doc:
        raise ValueError("config must contain both 'mitotic_phase' and 'interphase' objects")
    cfg = SimulationConfig()
    _apply(cfg.mitotic_phase, doc["mitotic_phase"])
    _apply(cfg.interphase, doc["interphase"], NOT_IN_JSON)
    cfg.source = text
    return cfg


def format_simulation_config(cfg: SimulationConfig) -> str:
    """simulation_config.cpp:159-164: canonical JSON of every traited member."""
    def enc(obj, skip=frozenset()):
        out = {}
        for f in dataclasses.fields(obj):
            if f.name in skip:
                continue
            v = getattr(obj, f.name)
            if isinstance(v, ABFactor):
                v = [v.a, v.b]
            elif isinstance(v, tuple):
                v = list(v)
            out[f.name] = v
        return out
    return json.dumps({"mitotic_phase": enc(cfg.mitotic_phase), "interphase": enc(cfg.interphase, NOT_IN_JSON)})

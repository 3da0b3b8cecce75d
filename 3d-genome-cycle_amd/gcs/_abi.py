"""ctypes mirror of include/gcs.h (the engine's C ABI).

The structures below are field-for-field copies of the C declarations; ``tests/test_abi.py`` checks
their sizes against the header and that every declared symbol is exported by ``libgcs.so``.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

GCS_OK = 0
GCS_EINVAL = 1
GCS_EHIP = 2
GCS_ESTATE = 3
GCS_ENOMEM = 4
GCS_ECAPACITY = 5

POT_SEMISPRING = 0
POT_HARMONIC = 1
POT_SPRING = 2
POT_FORCE_FLUX = 3

NOISE_PHILOX = 0
NOISE_INJECTED = 1
NOISE_NONE = 2

PRECISION_DEFAULT = 0  # = PRECISION_F64
PRECISION_F32 = 32
PRECISION_F64 = 64

OPT_GRAPH_STEPS = 1
OPT_WAVES_PER_TILE = 2
OPT_CHUNK_ORDER = 3
OPT_FUSED_STEP = 4
OPT_SPLIT_TILES = 5
OPT_TILE_PRIORITY = 6
OPT_SUBTILES = 7
OPT_SCAN_BLOCKS = 8
OPT_CONTACT_BITS = 9
OPT_LIST_SKIN = 10
OPT_LIST_EVERY = 11
OPT_LIST_CAP = 12
OPT_LIST_WAVES = 13
OPT_DENSE_NEIGHBORS = 15
OPT_LIST_DEAL = 16
OPT_LIST_FORMAT = 17  # 0 default (16-bit slots, plane-relative beyond 65,536), 1 plane-relative, 2 32-bit
OPT_SMALL_STEP = 18  # 1 default: the persistent all-pairs step for <= 1,536 particles; 0 off
OPT_LIST_PHASE = 19  # list step: rebuild steps s with (s + phase) % period == 0 (staggered replicas)
OPT_LIST_SKIN_BASE = 20  # list step: s1 of the core-scale-following default skin (0 = the precision's default)


def list_deal(pattern: str) -> int:
    """GCS_OPT_LIST_DEAL value of a chunk deal pattern: "0120123" = chunk p of every period of 7 goes to wave
    pattern[p] (include/gcs.h); "" = round robin (0)."""
    if not pattern:
        return 0
    if len(pattern) > 15:
        raise ValueError("a deal pattern has at most 15 chunks")
    v = len(pattern) << 60
    for p, c in enumerate(pattern):
        v |= int(c) << (4 * p)
    return v - (1 << 64) if v >= 1 << 63 else v  # as the int64 the ABI takes

ENERGY_KINDS = ("pair", "softwell", "bonds", "bending", "wall_in", "wall_out", "point_source", "kinetochore_fiber")

_d = C.c_double
_i32 = C.c_int32
_i64 = C.c_int64
_u64 = C.c_uint64
_pd = C.POINTER(C.c_double)
_pi64 = C.POINTER(C.c_int64)


class SystemDesc(C.Structure):
    _fields_ = [("particle_count", _i64), ("mobilities", _pd), ("ab_factors", _pd), ("device", _i32),
                ("precision", _i32)]


class SoftcoreParams(C.Structure):
    _fields_ = [("a_energy", _d), ("a_diameter", _d), ("b_energy", _d), ("b_diameter", _d),
                ("neighbor_distance", _d), ("mix", _i32), ("scaled", _i32)]


class BondParams(C.Structure):
    _fields_ = [("potential", _i32), ("mix", _i32), ("scaled", _i32), ("reserved", _i32), ("a_spring", _d),
                ("b_spring", _d), ("a_length", _d), ("b_length", _d)]


class SoftwellParams(C.Structure):
    _fields_ = [("energy", _d), ("decay_distance", _d), ("cutoff", _d), ("exponent", _i32), ("reserved", _i32)]


class WallParams(C.Structure):
    _fields_ = [("a_energy", _d), ("a_diameter", _d), ("b_energy", _d), ("b_diameter", _d), ("wall_a", _d),
                ("wall_b", _d), ("center", _d * 3), ("mix", _i32), ("scaled", _i32)]


class PointSourceParams(C.Structure):
    _fields_ = [("potential", _i32), ("reserved", _i32), ("point", _d * 3), ("spring", _d), ("length", _d),
                ("force", _d), ("reactive_distance", _d)]


class KinetochoreSpec(C.Structure):
    _fields_ = [("particle_index", _i64), ("mobility", _d), ("decay_rate", _d), ("stationary_length", _d)]


class Context(C.Structure):
    _fields_ = [("step", _i64), ("time", _d), ("core_scale", _d), ("bond_scale", _d), ("wall_semiaxes", _d * 3),
                ("inward_reaction", _d * 3), ("outward_reaction", _d * 3), ("last_timestep", _d)]


class Schedule(C.Structure):
    _fields_ = [("update_time", _i32), ("update_scales", _i32), ("update_wall", _i32), ("reserved", _i32),
                ("timestep", _d), ("core_scale_init", _d), ("core_scale_tau", _d), ("bond_scale_init", _d),
                ("bond_scale_tau", _d), ("wall_semiaxes_spring", _d * 3), ("wall_mobility", _d)]


class BDConfig(C.Structure):
    _fields_ = [("temperature", _d), ("timestep", _d), ("spacestep", _d), ("seed", _u64), ("noise", _i32),
                ("reserved", _i32)]


class Profile(C.Structure):
    _fields_ = [("steps", _i64), ("total_ms", _d), ("force_ms", _d), ("cell_ms", _d), ("tail_ms", _d),
                ("mean_neighbors", _d)]


class ListStats(C.Structure):
    _fields_ = [("active", _i32), ("rebuild_every", _i32), ("builds", _i64), ("fallback_particle_steps", _i64),
                ("skin", _d), ("max_displacement", _d), ("pair_classes", _i32), ("capacity", _i32),
                ("sync_stalls", _i64), ("deal", _i64)]


class RunStats(C.Structure):
    _fields_ = [("graph_launches", _i64), ("graph_steps", _i64), ("eager_steps", _i64), ("graphs_captured", _i64),
                ("graphs_cached", _i64), ("fused_contact_steps", _i64), ("density_probes", _i64)]


# name -> (restype, argtypes); the exported surface of include/gcs.h
PROTOTYPES = {
    "gcs_last_error": (C.c_char_p, []),
    "gcs_abi_version": (C.c_int, []),
    "gcs_device_count": (C.c_int, [C.POINTER(_i32)]),
    "gcs_engine_create": (C.c_int, [C.POINTER(SystemDesc), C.POINTER(C.c_void_p)]),
    "gcs_engine_destroy": (C.c_int, [C.c_void_p]),
    "gcs_engine_particle_count": (C.c_int, [C.c_void_p, C.POINTER(_i64)]),
    "gcs_engine_precision": (C.c_int, [C.c_void_p, C.POINTER(_i32)]),
    "gcs_add_neighbor_softcore": (C.c_int, [C.c_void_p, C.POINTER(SoftcoreParams), C.POINTER(_i32)]),
    "gcs_add_neighbor_softwell": (C.c_int, [C.c_void_p, C.POINTER(SoftwellParams), _pi64, _i64, C.POINTER(_i32)]),
    "gcs_add_bonded_pairwise": (C.c_int, [C.c_void_p, C.POINTER(BondParams), _pi64, _i64, _i32, _pi64, _i64,
                                          C.POINTER(_i32)]),
    "gcs_add_bonded_triplewise": (C.c_int, [C.c_void_p, _d, _pi64, _i64, C.POINTER(_i32)]),
    "gcs_add_ellipsoid_inward": (C.c_int, [C.c_void_p, C.POINTER(WallParams), C.POINTER(_i32)]),
    "gcs_add_ellipsoid_outward": (C.c_int, [C.c_void_p, _d, _pd, C.POINTER(_i32)]),
    "gcs_add_point_source": (C.c_int, [C.c_void_p, C.POINTER(PointSourceParams), C.POINTER(_i32)]),
    "gcs_add_kinetochore_fiber": (C.c_int, [C.c_void_p, _pd, C.POINTER(KinetochoreSpec), _i64, C.POINTER(_i32)]),
    "gcs_remove_forcefield": (C.c_int, [C.c_void_p, _i32]),
    "gcs_engine_set_positions": (C.c_int, [C.c_void_p, _pd, _i64]),
    "gcs_engine_get_positions": (C.c_int, [C.c_void_p, _pd, _i64]),
    "gcs_engine_set_context": (C.c_int, [C.c_void_p, C.POINTER(Context)]),
    "gcs_engine_get_context": (C.c_int, [C.c_void_p, C.POINTER(Context)]),
    "gcs_engine_set_schedule": (C.c_int, [C.c_void_p, C.POINTER(Schedule)]),
    "gcs_engine_apply_schedule": (C.c_int, [C.c_void_p, _i64]),
    "gcs_engine_set_noise": (C.c_int, [C.c_void_p, _pd, _i64]),
    "gcs_engine_run": (C.c_int, [C.c_void_p, C.POINTER(BDConfig), _i64, _i64]),
    "gcs_engine_synchronize": (C.c_int, [C.c_void_p]),
    "gcs_engine_compute_energy": (C.c_int, [C.c_void_p, _pd, _pd]),
    "gcs_engine_compute_forces": (C.c_int, [C.c_void_p, _pd, _i64]),
    "gcs_engine_search_neighbors": (C.c_int, [C.c_void_p, _pd, _i64, _d, C.POINTER(C.c_uint32), _i64,
                                              C.POINTER(_i64)]),
    "gcs_engine_profile": (C.c_int, [C.c_void_p, C.POINTER(BDConfig), _i64, _i64, C.POINTER(Profile)]),
    "gcs_engine_set_option": (C.c_int, [C.c_void_p, _i32, _i64]),
    "gcs_engine_get_list_stats": (C.c_int, [C.c_void_p, C.POINTER(ListStats)]),
    "gcs_engine_get_run_stats": (C.c_int, [C.c_void_p, C.POINTER(RunStats)]),
    "gcs_engine_set_cu_mask": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint32), _i32]),
    "gcs_engine_contacts_update": (C.c_int, [C.c_void_p, _d]),
    "gcs_engine_contacts_read": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint32), _i64, C.POINTER(_i64)]),
    "gcs_engine_contacts_clear": (C.c_int, [C.c_void_p]),
    "gcs_engine_sample_positions": (C.c_int, [C.c_void_p, C.POINTER(C.c_float), _i64, _i32]),
    "gcs_engine_set_domain": (C.c_int, [C.c_void_p, _pd, _d, _pd, _i32, _i32, _i32]),
    "gcs_engine_stream": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p)]),
    "gcs_engine_set_domain_shared": (C.c_int, [C.c_void_p, C.POINTER(_i64), _i32]),
    "gcs_engine_domain_step": (C.c_int, [C.c_void_p, C.POINTER(BDConfig), _i64, C.c_void_p]),
    "gcs_engine_domain_finish": (C.c_int, [C.c_void_p, C.c_void_p]),
    "gcs_engine_domain_pack": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, _i32, C.c_void_p]),
    "gcs_engine_domain_unpack": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, _i32, _i32]),
    "gcs_engine_domain_buffers": (C.c_int, [C.c_void_p, _i32, C.POINTER(_i32)]),
    "gcs_rccl_unique_id": (C.c_int, [C.POINTER(C.c_uint8)]),
    "gcs_engine_domain_rccl": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint8), _i32, _i32, C.POINTER(_i32)]),
    "gcs_engine_domain_run": (C.c_int, [C.c_void_p, C.POINTER(BDConfig), _i64, _i64]),
    "gcs_engine_domain_step_host": (C.c_int, [C.c_void_p, C.POINTER(BDConfig), _i64, _pd, _i32]),
    "gcs_engine_domain_finish_host": (C.c_int, [C.c_void_p, _pd, _i32]),
    "gcs_engine_domain_pack_host": (C.c_int, [C.c_void_p, C.c_void_p]),
    "gcs_engine_domain_unpack_host": (C.c_int, [C.c_void_p, C.c_void_p]),
    "gcs_engine_domain_receive": (C.c_int, [C.c_void_p, _i32, C.c_void_p, _i32]),
    "gcs_engine_domain_unpack_received": (C.c_int, [C.c_void_p]),
    "gcs_engine_domain_flags": (C.c_int, [C.c_void_p, C.POINTER(_i32)]),
}

LIB_PATH = Path(__file__).resolve().parent / "libgcs.so"

_lib = None


class GcsError(RuntimeError):
    def __init__(self, code: int, message: str):
        super().__init__(f"gcs error {code}: {message}")
        self.code = code


def load(path: os.PathLike | str | None = None):
    """Load libgcs.so.  Raises loudly when the HIP library is missing: there is no CPU fallback."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    # GCS_LIB: an alternative build of the same library (kernel-variant experiments, tools/)
    p = Path(path) if path else Path(os.environ.get("GCS_LIB", LIB_PATH))
    if not p.exists():
        raise FileNotFoundError(
            f"{p} not found: build it with `make -C 3d-genome-cycle_amd/csrc` (or __graft_entry__.build()); "
            "the gcs engine has no CPU fallback")
    lib = C.CDLL(str(p))
    for name, (res, args) in PROTOTYPES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def check(code: int):
    if code != GCS_OK:
        msg = load().gcs_last_error()
        raise GcsError(code, msg.decode() if msg else "")

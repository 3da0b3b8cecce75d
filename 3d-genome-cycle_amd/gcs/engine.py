"""Python handle on the HIP engine (libgcs.so) through its C ABI.

`Engine` exposes the md::system-like surface of include/gcs.h with numpy arrays.  The CPU oracle binding
(oracle/oracle.py, test infrastructure) implements the same method names so parity tests drive both
through one force-field composition (gcs.interphase / gcs.mitotic).
"""
from __future__ import annotations

import atexit
import ctypes as C
import weakref

import numpy as np

from . import _abi as A


def _f64(a, shape=None):
    arr = np.ascontiguousarray(a, dtype=np.float64)
    if shape is not None:
        arr = arr.reshape(shape)
    return arr


def _i64(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.int64).reshape(-1))


def _pd(arr):
    return arr.ctypes.data_as(C.POINTER(C.c_double)) if arr is not None else None


def _pi(arr):
    return arr.ctypes.data_as(C.POINTER(C.c_int64)) if arr is not None and arr.size else None


def context_to_dict(c: A.Context) -> dict:
    return {
        "step": int(c.step),
        "time": c.time,
        "core_scale": c.core_scale,
        "bond_scale": c.bond_scale,
        "wall_semiaxes": list(c.wall_semiaxes),
        "inward_reaction": list(c.inward_reaction),
        "outward_reaction": list(c.outward_reaction),
        "last_timestep": c.last_timestep,
    }


def dict_to_context(d: dict) -> A.Context:
    c = A.Context()
    c.step = int(d.get("step", 0))
    c.time = float(d.get("time", 0.0))
    c.core_scale = float(d.get("core_scale", 1.0))
    c.bond_scale = float(d.get("bond_scale", 1.0))
    for k in range(3):
        c.wall_semiaxes[k] = float(d.get("wall_semiaxes", (0, 0, 0))[k])
        c.inward_reaction[k] = float(d.get("inward_reaction", (0, 0, 0))[k])
        c.outward_reaction[k] = float(d.get("outward_reaction", (0, 0, 0))[k])
    c.last_timestep = float(d.get("last_timestep", 0.0))
    return c


def make_schedule(**kw) -> A.Schedule:
    s = A.Schedule()
    s.update_time = int(kw.get("update_time", 0))
    s.update_scales = int(kw.get("update_scales", 0))
    s.update_wall = int(kw.get("update_wall", 0))
    s.timestep = float(kw.get("timestep", 0.0))
    s.core_scale_init = float(kw.get("core_scale_init", 1.0))
    s.core_scale_tau = float(kw.get("core_scale_tau", 1.0))
    s.bond_scale_init = float(kw.get("bond_scale_init", 1.0))
    s.bond_scale_tau = float(kw.get("bond_scale_tau", 1.0))
    spring = kw.get("wall_semiaxes_spring", (0.0, 0.0, 0.0))
    for k in range(3):
        s.wall_semiaxes_spring[k] = float(spring[k])
    s.wall_mobility = float(kw.get("wall_mobility", 0.0))
    return s


def make_bd(temperature=1.0, timestep=1e-5, spacestep=0.0, seed=0, noise=A.NOISE_PHILOX) -> A.BDConfig:
    c = A.BDConfig()
    c.temperature = temperature
    c.timestep = timestep
    c.spacestep = spacestep
    c.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    c.noise = noise
    return c


_live = weakref.WeakSet()


@atexit.register
def _close_live_engines():
    # engines still alive at interpreter exit are destroyed here, while the HIP runtime (and RCCL) are intact:
    # a destructor run from the C library's own exit handlers would free device memory of a torn-down runtime
    for e in list(_live):
        e.close()


def precision_bits(precision) -> int:
    """GCS_PRECISION_* of a precision given as 32 / 64 / "f32" / "f64" / "fp32" / "fp64" (None: the default, fp64)"""
    if precision is None:
        return A.PRECISION_F64
    p = str(precision).lower().lstrip("f").lstrip("p")
    if p in ("32", "64"):
        return int(p)
    raise ValueError(f"precision must be 32 or 64 (or 'f32' / 'f64'), not {precision!r}")


class Engine:
    """One simulated system on one HIP device (md::system + md::simulate_brownian_dynamics).

    precision: 64 (default; md::scalar is double) or 32 (the fp32 engine: the tile-step shapes and the spatial
    decomposition are fp32 only)."""

    def __init__(self, n: int, mobilities=None, ab_factors=None, device: int = 0, precision=None):
        self._lib = A.load()
        self.n = int(n)
        self.precision = precision_bits(precision)
        self._mu = _f64(mobilities, (self.n,)) if mobilities is not None else None
        self._ab = _f64(ab_factors, (self.n, 2)) if ab_factors is not None else None
        d = A.SystemDesc()
        d.particle_count = self.n
        d.mobilities = _pd(self._mu)
        d.ab_factors = _pd(self._ab)
        d.device = device
        d.precision = self.precision
        h = C.c_void_p()
        A.check(self._lib.gcs_engine_create(C.byref(d), C.byref(h)))
        self._h = h
        _live.add(self)

    def close(self):
        if getattr(self, "_h", None):
            self._lib.gcs_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # ---- force fields ----
    def _handle(self, fn, *args):
        h = C.c_int32()
        A.check(fn(self._h, *args, C.byref(h)))
        return int(h.value)

    def add_neighbor_softcore(self, a_energy, a_diameter, b_energy=0.0, b_diameter=1.0, neighbor_distance=None,
                              mix=True, scaled=False):
        p = A.SoftcoreParams(a_energy, a_diameter, b_energy, b_diameter,
                             neighbor_distance if neighbor_distance is not None else max(a_diameter, b_diameter),
                             int(mix), int(scaled))
        return self._handle(self._lib.gcs_add_neighbor_softcore, C.byref(p))

    def add_neighbor_softwell(self, energy, decay_distance, cutoff, targets, exponent=6):
        t = _i64(targets)
        p = A.SoftwellParams(energy, decay_distance, cutoff, exponent, 0)
        return self._handle(self._lib.gcs_add_neighbor_softwell, C.byref(p), _pi(t), t.size)

    def add_bonded_pairwise(self, potential, a_spring, a_length=0.0, b_spring=0.0, b_length=0.0, mix=False,
                            scaled=False, ranges=None, stride=1, pairs=None):
        r = _i64(ranges if ranges is not None else [])
        q = _i64(pairs if pairs is not None else [])
        p = A.BondParams(potential, int(mix), int(scaled), 0, a_spring, b_spring, a_length, b_length)
        return self._handle(self._lib.gcs_add_bonded_pairwise, C.byref(p), _pi(r), r.size // 2, stride, _pi(q),
                            q.size // 2)

    def add_bonded_triplewise(self, bending_energy, ranges):
        r = _i64(ranges)
        return self._handle(self._lib.gcs_add_bonded_triplewise, bending_energy, _pi(r), r.size // 2)

    def add_ellipsoid_inward(self, a_energy, a_diameter, b_energy=0.0, b_diameter=1.0, wall_a=0.0, wall_b=0.0,
                             center=(0.0, 0.0, 0.0), mix=True, scaled=False):
        p = A.WallParams(a_energy, a_diameter, b_energy, b_diameter, wall_a, wall_b, (C.c_double * 3)(*center),
                         int(mix), int(scaled))
        return self._handle(self._lib.gcs_add_ellipsoid_inward, C.byref(p))

    def add_ellipsoid_outward(self, spring, center=(0.0, 0.0, 0.0)):
        c = _f64(center, (3,))
        return self._handle(self._lib.gcs_add_ellipsoid_outward, spring, _pd(c))

    def add_point_source(self, potential, point, spring=0.0, length=0.0, force=0.0, reactive_distance=1.0):
        p = A.PointSourceParams(potential, 0, (C.c_double * 3)(*point), spring, length, force, reactive_distance)
        return self._handle(self._lib.gcs_add_point_source, C.byref(p))

    def add_kinetochore_fiber(self, pole, specs):
        arr = (A.KinetochoreSpec * max(1, len(specs)))()
        for k, (idx, mob, decay, length) in enumerate(specs):
            arr[k] = A.KinetochoreSpec(int(idx), mob, decay, length)
        pl = _f64(pole, (3,))
        return self._handle(self._lib.gcs_add_kinetochore_fiber, _pd(pl), arr, len(specs))

    def remove_forcefield(self, handle):
        A.check(self._lib.gcs_remove_forcefield(self._h, int(handle)))

    # ---- state ----
    def set_positions(self, xyz):
        x = _f64(xyz, (self.n, 3))
        A.check(self._lib.gcs_engine_set_positions(self._h, _pd(x), self.n))

    def get_positions(self):
        out = np.empty((self.n, 3), dtype=np.float64)
        A.check(self._lib.gcs_engine_get_positions(self._h, _pd(out), self.n))
        return out

    def set_context(self, ctx: dict):
        c = dict_to_context(ctx)
        A.check(self._lib.gcs_engine_set_context(self._h, C.byref(c)))

    def get_context(self) -> dict:
        c = A.Context()
        A.check(self._lib.gcs_engine_get_context(self._h, C.byref(c)))
        return context_to_dict(c)

    def set_schedule(self, **kw):
        s = make_schedule(**kw)
        A.check(self._lib.gcs_engine_set_schedule(self._h, C.byref(s)))

    def apply_schedule(self, step):
        A.check(self._lib.gcs_engine_apply_schedule(self._h, int(step)))

    def set_noise(self, normals):
        x = _f64(normals)
        steps = x.size // (3 * self.n)
        A.check(self._lib.gcs_engine_set_noise(self._h, _pd(x), steps))

    # ---- dynamics ----
    def run(self, steps, first_step=0, temperature=1.0, timestep=1e-5, spacestep=0.0, seed=0,
            noise=A.NOISE_PHILOX):
        cfg = make_bd(temperature, timestep, spacestep, seed, noise)
        A.check(self._lib.gcs_engine_run(self._h, C.byref(cfg), int(first_step), int(steps)))

    def synchronize(self):
        A.check(self._lib.gcs_engine_synchronize(self._h))

    def compute_energy(self):
        tot = C.c_double()
        per = np.zeros(8, dtype=np.float64)
        A.check(self._lib.gcs_engine_compute_energy(self._h, C.byref(tot), _pd(per)))
        return tot.value, per

    def compute_forces(self):
        out = np.empty((self.n, 3), dtype=np.float64)
        A.check(self._lib.gcs_engine_compute_forces(self._h, _pd(out), self.n))
        return out

    def search_neighbors(self, distance, points=None):
        pts = _f64(points, (-1, 3)) if points is not None else None
        npts = pts.shape[0] if pts is not None else self.n
        cnt = C.c_int64()
        cap = max(16, npts * 8)
        while True:
            buf = np.empty((cap, 2), dtype=np.uint32)
            rc = self._lib.gcs_engine_search_neighbors(self._h, _pd(pts), npts, float(distance),
                                                       buf.ctypes.data_as(C.POINTER(C.c_uint32)), cap,
                                                       C.byref(cnt))
            if rc == A.GCS_ECAPACITY:
                cap = int(cnt.value)
                continue
            A.check(rc)
            self._last_contacts = int(cnt.value)
            return buf[: cnt.value].copy()

    # ---- contact map (stage_interphase/contact_map.cpp:28-85) and sampled positions (simulation_store.cpp:192-216)

    def contacts_update(self, distance):
        """contact_map::update: count every pair i < j of the current positions closer than `distance` (device)."""
        A.check(self._lib.gcs_engine_contacts_update(self._h, float(distance)))

    def contacts_accumulate(self):
        """contact_map::accumulate: (K, 3) uint32 rows (i, j, count) sorted by (i, j)."""
        cnt = C.c_int64()
        # one read in the common case: room for the last table's size (+25 %) or 16 pairs per particle
        cap = max(int(1.25 * getattr(self, "_last_contacts", 0)), 16 * self.n)
        while True:
            buf = np.empty((max(cap, 1), 3), dtype=np.uint32)
            rc = self._lib.gcs_engine_contacts_read(self._h, buf.ctypes.data_as(C.POINTER(C.c_uint32)), cap,
                                                    C.byref(cnt))
            if rc == A.GCS_ECAPACITY and cnt.value > cap:
                cap = int(cnt.value)
                continue
            A.check(rc)
            self._last_contacts = int(cnt.value)
            return buf[: cnt.value]  # a view (no copy of a ~50 MB table); the rows past it are never read

    def contacts_clear(self):
        """contact_map::clear"""
        A.check(self._lib.gcs_engine_contacts_clear(self._h))

    def sample_positions(self, fraction_bits=16):
        """Positions as simulation_store::save_positions stores them: quantised, f32 (N, 3)."""
        out = np.empty((self.n, 3), dtype=np.float32)
        A.check(self._lib.gcs_engine_sample_positions(self._h, out.ctypes.data_as(C.POINTER(C.c_float)), self.n,
                                                      int(fraction_bits)))
        return out

    # ---- spatial domain decomposition (gcs.domain drives these; device pointers are plain ints) ----

    def set_domain(self, box, halo, peer_boxes=(), index=0, ndomains=1):
        """box: (lo[3], hi[3]) of this domain (+-inf: an open face); peer_boxes: [(lo[3], hi[3])] of the domains whose
        regions overlap this one's (the engine extends them by the halo); index / ndomains: this domain's number and
        the domain count."""
        b = np.ascontiguousarray(np.clip(np.asarray(box, dtype=np.float64).reshape(6), -3e38, 3e38))
        reg = np.ascontiguousarray(np.clip(np.asarray(peer_boxes, dtype=np.float64).reshape(-1, 6), -3e38, 3e38))
        A.check(self._lib.gcs_engine_set_domain(self._h, _pd(b), float(halo), _pd(reg) if reg.size else None,
                                                reg.shape[0], int(index), int(ndomains)))

    def set_domain_shared(self, idx):
        a = np.ascontiguousarray(np.asarray(idx, dtype=np.int64).reshape(-1))
        A.check(self._lib.gcs_engine_set_domain_shared(self._h, a.ctypes.data_as(C.POINTER(C.c_int64)) if a.size
                                                       else None, a.size))

    def stream_handle(self) -> int:
        p = C.c_void_p()
        A.check(self._lib.gcs_engine_stream(self._h, C.byref(p)))
        return int(p.value or 0)

    def domain_step(self, step, reaction_ptr, temperature=1.0, timestep=1e-5, seed=0):
        cfg = make_bd(temperature, timestep, 0.0, seed, A.NOISE_PHILOX)
        A.check(self._lib.gcs_engine_domain_step(self._h, C.byref(cfg), int(step), C.c_void_p(reaction_ptr)))

    def domain_finish(self, reaction_ptr):
        A.check(self._lib.gcs_engine_domain_finish(self._h, C.c_void_p(reaction_ptr)))

    def domain_pack(self, out_ptr, counts_ptr, cap, flags_ptr):
        A.check(self._lib.gcs_engine_domain_pack(self._h, C.c_void_p(out_ptr), C.c_void_p(counts_ptr), int(cap),
                                                 C.c_void_p(flags_ptr)))

    def domain_unpack(self, in_ptr, counts_ptr, nbuf, cap):
        A.check(self._lib.gcs_engine_domain_unpack(self._h, C.c_void_p(in_ptr), C.c_void_p(counts_ptr), int(nbuf),
                                                   int(cap)))

    # engine-owned exchange of a decomposed run (include/gcs.h "Engine-owned exchange")
    def domain_buffers(self, cap) -> int:
        nred = C.c_int32()
        A.check(self._lib.gcs_engine_domain_buffers(self._h, int(cap), C.byref(nred)))
        return int(nred.value)

    def domain_rccl(self, uid: bytes, nranks, rank, peer_ranks):
        buf = (C.c_uint8 * 128).from_buffer_copy(bytes(uid))
        pr = (C.c_int32 * max(1, len(peer_ranks)))(*[int(p) for p in peer_ranks])
        A.check(self._lib.gcs_engine_domain_rccl(self._h, buf, int(nranks), int(rank), pr))

    def domain_run(self, steps, first_step=0, temperature=1.0, timestep=1e-5, seed=0):
        cfg = make_bd(temperature, timestep, 0.0, seed, A.NOISE_PHILOX)
        A.check(self._lib.gcs_engine_domain_run(self._h, C.byref(cfg), int(first_step), int(steps)))

    def domain_step_host(self, step, red, temperature=1.0, timestep=1e-5, seed=0):
        cfg = make_bd(temperature, timestep, 0.0, seed, A.NOISE_PHILOX)
        A.check(self._lib.gcs_engine_domain_step_host(self._h, C.byref(cfg), int(step), _pd(red), red.size))

    def domain_finish_host(self, glob):
        A.check(self._lib.gcs_engine_domain_finish_host(self._h, _pd(glob), glob.size))

    def domain_pack_host(self, bands):
        A.check(self._lib.gcs_engine_domain_pack_host(
            self._h, C.c_void_p(bands.ctypes.data) if bands is not None else None))

    def domain_unpack_host(self, bands):
        A.check(self._lib.gcs_engine_domain_unpack_host(self._h, C.c_void_p(bands.ctypes.data)))

    def domain_receive(self, slot, src, src_slot):
        A.check(self._lib.gcs_engine_domain_receive(self._h, int(slot), src._h, int(src_slot)))

    def domain_unpack_received(self):
        A.check(self._lib.gcs_engine_domain_unpack_received(self._h))

    def domain_flags(self) -> int:
        f = C.c_int32()
        A.check(self._lib.gcs_engine_domain_flags(self._h, C.byref(f)))
        return int(f.value)

    def profile(self, steps, first_step=0, temperature=1.0, timestep=1e-5, seed=0, noise=A.NOISE_PHILOX) -> dict:
        cfg = make_bd(temperature, timestep, 0.0, seed, noise)
        p = A.Profile()
        A.check(self._lib.gcs_engine_profile(self._h, C.byref(cfg), int(first_step), int(steps), C.byref(p)))
        return {"steps": p.steps, "total_ms": p.total_ms, "force_ms": p.force_ms, "cell_ms": p.cell_ms,
                "tail_ms": p.tail_ms, "mean_neighbors": p.mean_neighbors}

    def set_option(self, option, value):
        A.check(self._lib.gcs_engine_set_option(self._h, int(option), int(value)))

    def set_cu_mask(self, cus):
        """Run this engine's kernels on the compute units `cus` only (None or empty: all)."""
        cus = sorted(int(c) for c in (cus or []))
        words = (max(cus) // 32 + 1) if cus else 0
        m = (C.c_uint32 * max(1, words))()
        for c in cus:
            m[c // 32] |= 1 << (c % 32)
        A.check(self._lib.gcs_engine_set_cu_mask(self._h, m, words))

    def list_stats(self) -> dict:
        s = A.ListStats()
        A.check(self._lib.gcs_engine_get_list_stats(self._h, C.byref(s)))
        return {k: getattr(s, k) for k, _ in A.ListStats._fields_}

    def run_stats(self) -> dict:
        """graph replays vs eager steps of every run so far (gcs_engine_get_run_stats)"""
        s = A.RunStats()
        A.check(self._lib.gcs_engine_get_run_stats(self._h, C.byref(s)))
        return {k: getattr(s, k) for k, _ in A.RunStats._fields_}


def rccl_unique_id() -> bytes:
    """An RCCL communicator id (rank 0 draws it; every rank passes it to Engine.domain_rccl)."""
    lib = A.load()
    buf = (C.c_uint8 * 128)()
    A.check(lib.gcs_rccl_unique_id(buf))
    return bytes(buf)


def device_count() -> int:
    lib = A.load()
    c = C.c_int32()
    rc = lib.gcs_device_count(C.byref(c))
    return int(c.value) if rc == A.GCS_OK else 0

"""The HDF5 trajectory store: the reference's simulation_store
(src/simulation/common/simulation_store.{hpp,cpp}) over libgcs_store.so (include/gcs_store.h, HDF5 C library).

`SimulationStore` keeps the reference's method names, dataset paths, types and filters, so the files it writes are
read unchanged by the reference's Python tools (dumpgsd.py, cool.py) and by the stage drivers here.
`write_prepared` writes what `prepare` leaves for the stages (prepare.cpp:374-562) from a design object (the
synthetic generators, or any caller-built design): metadata, per-stage designs and seeds, soft links, and the
relaxation stage's initial structure.
"""
from __future__ import annotations

import ctypes as C
import json
import os
import sys
from pathlib import Path

import zlib

import numpy as np

from .config import SimulationConfig, format_simulation_config, parse_simulation_config

LIB_PATH = Path(__file__).resolve().parent / "libgcs_store.so"

H5_F32, H5_F64, H5_I32, H5_U32, H5_U64 = 1, 2, 3, 4, 5
CONTACT_CHUNK_ROWS = 1 << 16  # rows per chunk of a contact table (each chunk encoded on its own host thread)
_NP = {H5_F32: np.float32, H5_F64: np.float64, H5_I32: np.int32, H5_U32: np.uint32, H5_U64: np.uint64}

# interphase_particle_type / mitotic_particle_type (stage_prepare/prepare.cpp:14-25)
INTERPHASE_TYPES = {"unknown": 0, "a": 1, "b": 2, "u": 3, "centromere": 4, "active_nor": 5, "silent_nor": 6,
                    "nucleolus": 7}
MITOTIC_TYPES = {"unknown": 0, "arm": 1, "kinetochore": 2}

_lib = None


class StoreError(RuntimeError):
    pass


def load_lib():
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise FileNotFoundError(f"{LIB_PATH} not found: build it with `make -C 3d-genome-cycle_amd/csrc`")
        lib = C.CDLL(str(LIB_PATH))
        vp, cp, i32, i64 = C.c_void_p, C.c_char_p, C.c_int32, C.c_int64
        pi64 = C.POINTER(i64)
        sig = {
            "gcs_store_last_error": (cp, []),
            "gcs_store_open": (C.c_int, [cp, i32, C.POINTER(vp)]),
            "gcs_store_close": (C.c_int, [vp]),
            "gcs_store_flush": (C.c_int, [vp]),
            "gcs_store_exists": (C.c_int, [vp, cp, C.POINTER(i32)]),
            "gcs_store_remove": (C.c_int, [vp, cp]),
            "gcs_store_soft_link": (C.c_int, [vp, cp, cp]),
            "gcs_store_write_string": (C.c_int, [vp, cp, cp]),
            "gcs_store_read_string": (C.c_int, [vp, cp, C.c_char_p, i64, pi64]),
            "gcs_store_write_strings": (C.c_int, [vp, cp, C.POINTER(C.c_char_p), i64]),
            "gcs_store_read_strings": (C.c_int, [vp, cp, vp, i64, pi64, pi64]),
            "gcs_store_write_array": (C.c_int, [vp, cp, i32, i32, pi64, vp, i32, i32]),
            "gcs_store_write_deflated": (C.c_int, [vp, cp, i32, i32, pi64, vp, i64, i32]),
            "gcs_store_write_scaleoffset_i32": (C.c_int, [vp, cp, vp, i64, i32, i32, i64, i32]),
            "gcs_store_read_array": (C.c_int, [vp, cp, i32, vp, i64, C.POINTER(i32), pi64]),
            "gcs_store_write_enum": (C.c_int, [vp, cp, C.POINTER(i32), i64, C.POINTER(C.c_char_p), C.POINTER(i32),
                                               i32]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def _b(s: str) -> bytes:
    return s.encode()


class H5File:
    """The primitives of include/gcs_store.h."""

    def __init__(self, path, create=False):
        self.lib = load_lib()
        h = C.c_void_p()
        self._check(self.lib.gcs_store_open(_b(os.fspath(path)), 1 if create else 0, C.byref(h)))
        self.h = h

    def _check(self, rc):
        if rc != 0:
            raise StoreError(self.lib.gcs_store_last_error().decode())

    def close(self):
        if getattr(self, "h", None):
            self._check(self.lib.gcs_store_close(self.h))
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def exists(self, path) -> bool:
        e = C.c_int32()
        self._check(self.lib.gcs_store_exists(self.h, _b(path), C.byref(e)))
        return bool(e.value)

    def remove(self, path):
        self._check(self.lib.gcs_store_remove(self.h, _b(path)))

    def soft_link(self, target, link):
        self._check(self.lib.gcs_store_soft_link(self.h, _b(target), _b(link)))

    def write_string(self, path, text: str):
        self._check(self.lib.gcs_store_write_string(self.h, _b(path), _b(text)))

    def read_string(self, path) -> str:
        n = C.c_int64()
        self._check(self.lib.gcs_store_read_string(self.h, _b(path), None, 0, C.byref(n)))
        buf = C.create_string_buffer(n.value + 1)
        self._check(self.lib.gcs_store_read_string(self.h, _b(path), buf, n.value + 1, C.byref(n)))
        return buf.raw[: n.value].decode()

    def write_strings(self, path, items):
        arr = (C.c_char_p * max(1, len(items)))(*[_b(s) for s in items])
        self._check(self.lib.gcs_store_write_strings(self.h, _b(path), arr, len(items)))

    def read_strings(self, path) -> list:
        cnt, nb = C.c_int64(), C.c_int64()
        self._check(self.lib.gcs_store_read_strings(self.h, _b(path), None, 0, C.byref(cnt), C.byref(nb)))
        buf = C.create_string_buffer(max(1, nb.value))
        self._check(self.lib.gcs_store_read_strings(self.h, _b(path), buf, nb.value, C.byref(cnt), C.byref(nb)))
        return [s.decode() for s in buf.raw[: nb.value].split(b"\0")[: cnt.value]]

    def write_array(self, path, data, dtype, deflate=0, scaleoffset_int=False):
        a = np.array(data, dtype=_NP[dtype], order="C")  # (keeps 0-d arrays scalar datasets)
        dims = (C.c_int64 * max(1, a.ndim))(*a.shape)
        self._check(self.lib.gcs_store_write_array(self.h, _b(path), dtype, a.ndim, dims, a.ctypes.data_as(C.c_void_p),
                                                   int(deflate), 1 if scaleoffset_int else 0))

    def write_deflated(self, path, shape, dtype, zdata: bytes, deflate):
        """an array already deflated (zlib.compress(array bytes, deflate), deflated_frame) as its one chunk"""
        dims = (C.c_int64 * len(shape))(*shape)
        buf = C.create_string_buffer(zdata, len(zdata))
        self._check(self.lib.gcs_store_write_deflated(self.h, _b(path), dtype, len(shape), dims, buf, len(zdata),
                                                      int(deflate)))

    def write_scaleoffset_i32(self, path, data, deflate, chunk_rows=CONTACT_CHUNK_ROWS, threads=None):
        """i32 (rows, cols) with integer scale-offset + deflate, chunks encoded on host threads"""
        a = np.ascontiguousarray(data, dtype=np.int32)
        threads = threads or min(16, os.cpu_count() or 1)
        self._check(self.lib.gcs_store_write_scaleoffset_i32(self.h, _b(path), a.ctypes.data_as(C.c_void_p),
                                                             a.shape[0], a.shape[1], int(deflate), int(chunk_rows),
                                                             int(threads)))

    def read_array(self, path, dtype) -> np.ndarray:
        rank = C.c_int32()
        dims = (C.c_int64 * 2)()
        self._check(self.lib.gcs_store_read_array(self.h, _b(path), dtype, None, 0, C.byref(rank), dims))
        shape = tuple(dims[k] for k in range(rank.value))
        out = np.empty(shape, dtype=_NP[dtype])
        cap = max(1, out.size)
        self._check(self.lib.gcs_store_read_array(self.h, _b(path), dtype, out.ctypes.data_as(C.c_void_p), cap,
                                                  C.byref(rank), dims))
        return out

    def write_enum(self, path, values, members: dict):
        v = np.ascontiguousarray(values, dtype=np.int32)
        names = (C.c_char_p * len(members))(*[_b(k) for k in members])
        codes = (C.c_int32 * len(members))(*members.values())
        self._check(self.lib.gcs_store_write_enum(self.h, _b(path), v.ctypes.data_as(C.POINTER(C.c_int32)), v.size,
                                                  names, codes, len(members)))


def quantize_positions(x, fraction_bits=16) -> np.ndarray:
    """simulation_store.cpp:22-33 on fp64 coordinates (frexp, nearbyint of the scaled mantissa, ldexp), as f32."""
    x = np.asarray(x, dtype=np.float64)
    m, e = np.frexp(x)
    return np.ldexp(np.rint(np.ldexp(m, fraction_bits)), e - fraction_bits).astype(np.float32)


class SimulationStore:
    """simulation_store (common/simulation_store.hpp:60-118) with the same method names."""

    def __init__(self, path, create=False):
        self.f = H5File(path, create=create)
        self.stage = ""

    def close(self):
        self.f.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # ---- paths (simulation_store.cpp:377-394) ----
    def locate_metadata_in(self, stage, key):
        return f"/stages/{stage}/metadata/{key}"

    def locate_data(self, key, step=None):
        return f"/stages/{self.stage}/{key}" if step is None else f"/stages/{self.stage}/{step}/{key}"

    def set_stage(self, name):
        self.stage = name

    # ---- config / designs (simulation_store.cpp:69-112, 270-374) ----
    def load_config(self) -> SimulationConfig:
        return parse_simulation_config(self.f.read_string("/metadata/config"))

    def load_seed(self, stage) -> int:
        return int(self.f.read_array(self.locate_metadata_in(stage, "seed"), H5_U64))

    def load_chains(self, stage) -> list:
        names = self.f.read_strings(self.locate_metadata_in(stage, "chain_names"))
        ranges = self.f.read_array(self.locate_metadata_in(stage, "chain_ranges"), H5_U32).reshape(-1, 2)
        kpath = self.locate_metadata_in(stage, "kinetochore_beads")
        if self.f.exists(kpath):
            kin = self.f.read_array(kpath, H5_U32).reshape(-1)
            if kin.size != len(names):
                raise StoreError("chains and kinetochore_beads datasets mismatch")
            return [(n, int(r[0]), int(r[1]), int(k)) for n, r, k in zip(names, ranges, kin)]
        return [(n, int(r[0]), int(r[1])) for n, r in zip(names, ranges)]

    def load_interphase_design(self):
        from .synthetic import InterphaseDesign
        st = "interphase"
        ab = self.f.read_array(self.locate_metadata_in(st, "ab_factors"), H5_F32).astype(np.float64)
        types = self.f.read_array(self.locate_metadata_in(st, "particle_types"), H5_I32)
        bonds = self.f.read_array(self.locate_metadata_in(st, "nucleolar_bonds"), H5_U32).astype(np.int64)
        return InterphaseDesign(seed=self.load_seed(st), ab_factors=ab.reshape(-1, 2), particle_types=types,
                                chains=self.load_chains(st), nucleolar_bonds=bonds.reshape(-1, 2),
                                positions=np.zeros((ab.shape[0], 3)))

    def load_anatelophase_design(self):
        from .mitotic import MitoticDesign
        st = "anaphase"
        types = self.f.read_array(self.locate_metadata_in(st, "particle_types"), H5_I32)
        return MitoticDesign(seed=self.load_seed(st), particle_types=types, chains=self.load_chains(st))

    def load_prometaphase_design(self):
        from .mitotic import MitoticDesign
        st = "prometaphase"
        types = self.f.read_array(self.locate_metadata_in(st, "particle_types"), H5_I32)
        sis = self.f.read_array(self.locate_metadata_in(st, "sister_chromatids"), H5_U32).reshape(-1, 2)
        poles = self.f.read_array(self.locate_metadata_in(st, "pole_positions"), H5_F32).astype(np.float64)
        if poles.shape != (2, 3):
            raise StoreError("unexpected pole_positions shape")
        return MitoticDesign(seed=self.load_seed(st), particle_types=types, chains=self.load_chains(st),
                             sister_chromatids=[tuple(int(v) for v in r) for r in sis], pole_positions=poles)

    # ---- frames (simulation_store.cpp:114-267) ----
    def save_interphase_context(self, step, context: dict):
        keys = ("time", "wall_semiaxes", "core_scale", "bond_scale", "mean_energy", "wall_energy")
        doc = {k: (list(map(float, context[k])) if k == "wall_semiaxes" else float(context.get(k, 0.0)))
               for k in keys}
        self.f.write_string(self.locate_data("context", step), json.dumps(doc, separators=(",", ":")))

    def load_interphase_context(self, step) -> dict:
        return json.loads(self.f.read_string(self.locate_data("context", step)))

    def check_positions(self, step) -> bool:
        return self.f.exists(self.locate_data("positions", step))

    def clear_frames(self):
        p = self.locate_data(".steps")
        if self.f.exists(p):
            self.f.write_strings(p, [])

    def append_frame(self, step):
        p = self.locate_data(".steps")
        steps = self.f.read_strings(p) if self.f.exists(p) else []
        steps.append(str(int(step)))
        self.f.write_strings(p, steps)

    def load_steps(self) -> list:
        p = self.locate_data(".steps")
        return [int(s) for s in self.f.read_strings(p)] if self.f.exists(p) else []

    def save_positions(self, step, positions, quantized=False, zdata=None):
        """f32 (N, 3) with 16 fraction bits and deflate 6.  `quantized`: the caller already quantised them (the
        engine's gcs_engine_sample_positions does it on the device, bit-exactly).  `zdata`: those positions already
        deflated (deflated_frame, e.g. on another thread): written as the dataset's chunk, the same file."""
        q = np.asarray(positions, dtype=np.float32) if quantized else quantize_positions(positions)
        path = self.locate_data("positions", step)
        if zdata is not None and q.size > 0 and len(zdata) < q.nbytes:
            self.f.write_deflated(path, q.shape, H5_F32, zdata, POSITIONS_DEFLATE)
        else:  # (a chunk deflate cannot shrink: the library stores it raw, as it would here)
            self.f.write_array(path, q, H5_F32, deflate=POSITIONS_DEFLATE)

    def load_positions(self, step) -> np.ndarray:
        return self.f.read_array(self.locate_data("positions", step), H5_F32).astype(np.float64).reshape(-1, 3)

    def save_contacts(self, step, contacts):
        """i32 (K, 3) (i, j, count) sorted by (i, j), deflate 4 + integer scale-offset; nothing when empty"""
        c = np.asarray(contacts)
        if c.size == 0:
            return
        # chunks of CONTACT_CHUNK_ROWS rows encoded on host threads (a C2 window's ~4 M rows took ~1.4 s of one core
        # through the library's filters, more than the window's device time)
        self.f.write_scaleoffset_i32(self.locate_data("contacts", step), c.astype(np.int32), 4)

    def load_contacts(self, step) -> np.ndarray:
        return self.f.read_array(self.locate_data("contacts", step), H5_I32).reshape(-1, 3)

    # ---- the drivers' sampling hook: positions (+ context) + the frame index, under `stage` ----
    def save_frame(self, stage, step, positions, context=None, quantized=False, zdata=None):
        self.set_stage(stage)
        self.save_positions(step, positions, quantized=quantized, zdata=zdata)
        if context is not None:
            self.save_interphase_context(step, context)
        self.append_frame(step)


POSITIONS_DEFLATE = 6  # simulation_store.cpp: positions f32 with deflate 6


def deflated_frame(q) -> bytes:
    """the chunk HDF5's deflate filter stores for f32 positions `q`: zlib format, compress2 at level 6 (zlib.compress
    uses the same defaults: 15 window bits, memory level 8)"""
    return zlib.compress(np.ascontiguousarray(q, dtype="<f4").tobytes(), POSITIONS_DEFLATE)


class AsyncWriter:
    """The drivers' sampling writes (save_frame / save_contacts) on a background thread, so the device keeps stepping
    while a frame is deflated and written (deflate 6 of a C2 frame takes ~0.1 s of one host core: at the reference's
    cadence of one frame per 1,000 steps that is several times the steps' own device time).  The HDF5 library is not
    thread-safe: while a writer is open only its thread touches the store; `flush()` waits for every queued write
    (the drivers flush at the end of each stage, before any other store call).  Writes keep their order, so the
    file is the one the synchronous calls would write.  ctypes releases the GIL inside the HDF5 calls.  The frames'
    deflate runs on a pool of `deflaters` threads (zlib releases the GIL) and the writer thread stores each chunk as
    it is (gcs_store_write_deflated): at one frame per 1,000 C2 steps a single deflating thread was the stage's
    bound (~0.1 s per frame against ~0.02 s of device time)."""

    def __init__(self, store, depth=16, deflaters=8):
        import queue
        import threading
        from concurrent.futures import ThreadPoolExecutor
        self.store = store
        self.q = queue.Queue(maxsize=depth)
        self.err = None
        self.pool = ThreadPoolExecutor(max_workers=deflaters, thread_name_prefix="gcs-deflate")
        self.t = threading.Thread(target=self._loop, name="gcs-store-writer", daemon=True)
        self.t.start()

    def _loop(self):
        while True:
            item = self.q.get()
            try:
                if item is None:
                    return
                if self.err is None:
                    fn, args, kw = item
                    if "zdata" in kw:
                        kw = dict(kw, zdata=kw["zdata"].result())
                    fn(*args, **kw)
            except BaseException as exc:  # re-raised on the caller's thread at the next put / flush
                self.err = exc
            finally:
                self.q.task_done()

    def _put(self, fn, *args, **kw):
        if self.err is not None:
            raise self.err
        self.q.put((fn, args, kw))

    def save_frame(self, stage, step, positions, context=None, quantized=False):
        q = np.asarray(positions, dtype=np.float32) if quantized else quantize_positions(positions)
        self._put(self.store.save_frame, stage, step, q, context, quantized=True,
                  zdata=self.pool.submit(deflated_frame, q))

    def save_contacts(self, *args, **kw):
        self._put(self.store.save_contacts, *args, **kw)

    def flush(self):
        self.q.join()
        if self.err is not None:
            err, self.err = self.err, None
            raise err

    def close(self, propagating=None):
        """Flush and stop.  A deferred write error is raised -- unless the caller passes the exception it is already
        propagating (`propagating`: close() on an unwind, as __exit__ does): then the write error is added to that
        exception as a note and the original exception survives.  A plain close() always raises it."""
        try:
            self.flush()
        except BaseException as err:
            if propagating is None:
                raise
            if hasattr(propagating, "add_note"):
                propagating.add_note(f"gcs.store.AsyncWriter: a deferred write also failed: {err!r}")
            else:
                print(f"gcs.store.AsyncWriter: a deferred write also failed: {err!r}", file=sys.stderr)
        finally:
            self.q.put(None)
            self.t.join()
            self.pool.shutdown(wait=True)

    def __enter__(self):
        return self

    def __exit__(self, exc_type, exc, tb):
        self.close(propagating=exc)
        return False


def sampled_positions(system):
    """Positions as save_positions stores them, and whether they are already quantised: the engine quantises on the
    device (gcs_engine_sample_positions, bit-exact with quantize_positions), other backends return raw positions."""
    if hasattr(system, "sample_positions"):
        return system.sample_positions(16), True
    return system.get_positions(), False


def write_prepared(path, cfg: SimulationConfig, design, master_seed: int, anatelophase=None, prometaphase=None,
                   chains_source="", create=True, initial_positions=True):
    """What `prepare` writes (prepare.cpp:374-562) for a given interphase design (+ optional mitotic designs):
    /metadata/{master_seed, config, config_source, chains_source}; /stages/interphase/metadata/* with soft links
    from /stages/relaxation/metadata/*; per-stage seeds; the relaxation stage's initial structure at step 0 (the
    position transition_interphase would write)."""
    from .seeds import stage_seeds
    seeds = stage_seeds(master_seed)
    with H5File(path, create=create) as f:
        f.write_array("/metadata/master_seed", np.uint32(master_seed), H5_U32)
        f.write_string("/metadata/config", format_simulation_config(cfg))
        f.write_string("/metadata/config_source", cfg.source)
        f.write_string("/metadata/chains_source", chains_source)
        ip = "/stages/interphase/metadata/"
        f.write_enum(ip + "particle_types", design.particle_types, INTERPHASE_TYPES)
        f.write_array(ip + "ab_factors", np.asarray(design.ab_factors, dtype=np.float32), H5_F32)
        f.write_strings(ip + "chain_names", [c[0] for c in design.chains])
        f.write_array(ip + "chain_ranges", np.array([[c[1], c[2]] for c in design.chains], dtype=np.int32), H5_I32)
        f.write_array(ip + "nucleolar_bonds", np.asarray(design.nucleolar_bonds, dtype=np.int32).reshape(-1, 2),
                      H5_I32)
        for key in ("particle_types", "ab_factors", "chain_names", "chain_ranges", "nucleolar_bonds"):
            f.soft_link(ip + key, "/stages/relaxation/metadata/" + key)
        if anatelophase is not None:
            ap = "/stages/anaphase/metadata/"
            f.write_enum(ap + "particle_types", anatelophase.particle_types, MITOTIC_TYPES)
            f.write_strings(ap + "chain_names", [c[0] for c in anatelophase.chains])
            f.write_array(ap + "chain_ranges", np.array([[c[1], c[2]] for c in anatelophase.chains], dtype=np.int32),
                          H5_I32)
            f.write_array(ap + "kinetochore_beads", np.array([-1 if c[3] is None else c[3]  # value_or(-1) (:470)
                                                              for c in anatelophase.chains], dtype=np.int32), H5_I32)
            for key in ("particle_types", "chain_names", "chain_ranges"):
                f.soft_link(ap + key, "/stages/telophase/metadata/" + key)
        if prometaphase is not None:
            pp = "/stages/prometaphase/metadata/"
            f.write_enum(pp + "particle_types", prometaphase.particle_types, MITOTIC_TYPES)
            f.write_strings(pp + "chain_names", [c[0] for c in prometaphase.chains])
            f.write_array(pp + "chain_ranges", np.array([[c[1], c[2]] for c in prometaphase.chains], dtype=np.int32),
                          H5_I32)
            f.write_array(pp + "kinetochore_beads", np.array([c[3] for c in prometaphase.chains], dtype=np.int32),
                          H5_I32)
            f.write_array(pp + "sister_chromatids", np.array(prometaphase.sister_chromatids, dtype=np.int32), H5_I32)
            f.write_array(pp + "pole_positions", np.asarray(prometaphase.pole_positions, dtype=np.float32), H5_F32)
        for stage in ("anaphase", "interphase", "prometaphase"):  # prepare.cpp:559-561
            f.write_array(f"/stages/{stage}/metadata/seed", np.uint32(seeds[stage]), H5_U32)
        if initial_positions:  # (synthetic designs carry a structure; prepare itself writes none)
            f.write_array("/stages/relaxation/0/positions", quantize_positions(design.positions), H5_F32, deflate=6)

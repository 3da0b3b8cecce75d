"""The HDF5 trajectory store (gcs/store.py over libgcs_store.so): round trips, the
reference's dataset contract as the reference's own readers see it (h5py, run with the image's conda Python when
present), and the drivers writing through it."""
import shutil
import subprocess

import numpy as np
import pytest

from gcs import interphase, mitotic, store, synthetic
from gcs.config import InterphaseConfig, SimulationConfig, format_simulation_config

import oracle

PY39 = shutil.which("/opt/conda/bin/python3.9")


@pytest.fixture
def prepared(tmp_path, c1_design):
    cfg = SimulationConfig()
    p = tmp_path / "traj.h5"
    store.write_prepared(p, cfg, c1_design, 1)
    return p, cfg


def test_quantize_matches_the_oracle(c1_design):
    x = c1_design.positions * 1.7 + 0.123
    q = store.quantize_positions(x)
    exp = np.vectorize(lambda v: oracle.quantize(v, 16))(x).astype(np.float32)
    assert np.array_equal(q.view(np.uint32), exp.view(np.uint32))


def test_prepared_round_trip(prepared, c1_design):
    p, cfg = prepared
    with store.SimulationStore(p) as s:
        assert format_simulation_config(s.load_config()) == format_simulation_config(cfg)
        d = s.load_interphase_design()
        assert d.seed == c1_design.seed and d.chains == [(n, a, b) for n, a, b in c1_design.chains]
        assert np.array_equal(d.particle_types, c1_design.particle_types)
        assert np.array_equal(d.nucleolar_bonds, c1_design.nucleolar_bonds)
        assert np.array_equal(d.ab_factors, c1_design.ab_factors.astype(np.float32).astype(np.float64))
        s.set_stage("relaxation")
        assert s.check_positions(0) and not s.check_positions(1)
        assert np.array_equal(s.load_positions(0), store.quantize_positions(c1_design.positions).astype(np.float64))


def test_frames_contacts_context(prepared):
    p, _ = prepared
    with store.SimulationStore(p) as s:
        s.set_stage("interphase")
        assert s.load_steps() == []
        s.clear_frames()  # nothing to clear: no dataset is created
        for st in (0, 1000, 2000):
            s.append_frame(st)
        assert s.load_steps() == [0, 1000, 2000]
        s.clear_frames()
        assert s.load_steps() == []
        t = np.array([[0, 1, 7], [0, 5, 1], [3, 4, 2]], dtype=np.uint32)
        s.save_contacts(1000, t)
        s.save_contacts(2000, np.zeros((0, 3), dtype=np.uint32))  # empty: not written (simulation_store.cpp:257)
        assert np.array_equal(s.load_contacts(1000), t) and not s.f.exists("/stages/interphase/2000/contacts")
        ctx = dict(time=0.01, wall_semiaxes=[2.0, 2.1, 2.2], core_scale=0.6, bond_scale=0.6, mean_energy=1.5)
        s.save_interphase_context(1000, ctx)
        assert s.load_interphase_context(1000) == dict(ctx, wall_energy=0.0)


def test_mitotic_designs_round_trip(tmp_path):
    cfg = SimulationConfig()
    i = synthetic.make_c2()
    a = mitotic.anatelophase_design(i, cfg.mitotic_phase)
    pm = mitotic.prometaphase_design(a, cfg.mitotic_phase, i.master_seed)
    p = tmp_path / "m.h5"
    store.write_prepared(p, cfg, i, i.master_seed, anatelophase=a, prometaphase=pm)
    with store.SimulationStore(p) as s:
        a2 = s.load_anatelophase_design()
        p2 = s.load_prometaphase_design()
    assert a2.seed == a.seed and a2.chains == a.chains and np.array_equal(a2.particle_types, a.particle_types)
    assert p2.chains == pm.chains and p2.sister_chromatids == pm.sister_chromatids
    assert np.array_equal(p2.pole_positions, pm.pole_positions)


@pytest.mark.skipif(PY39 is None, reason="no conda python with h5py in this image")
def test_reader_contract_with_h5py(prepared):
    """What dumpgsd.py / cool.py rely on: particle_types an HDF5 enum, strings that .decode(),
    relaxation metadata linked to interphase, positions f32 deflate 6, contacts i32 deflate 4 + scale-offset."""
    p, _ = prepared
    with store.SimulationStore(p) as s:
        s.set_stage("interphase")
        s.save_positions(1000, np.zeros((1002, 3)))
        s.save_contacts(1000, np.array([[0, 1, 3]], dtype=np.uint32))
        s.append_frame(1000)
    code = f"""
import h5py, numpy as np
f = h5py.File({str(p)!r}, "r")
m = f["stages/interphase/metadata"]
assert h5py.check_enum_dtype(m["particle_types"].dtype)["nucleolus"] == 7
assert [n.decode() for n in m["chain_names"]] == ["chr1"]
assert f["stages/relaxation/metadata/ab_factors"].shape == (1002, 2)
assert f["stages/relaxation/metadata/particle_types"].dtype.metadata["enum"]["a"] == 1
assert isinstance(f["metadata/config"][()], bytes) and f["metadata/master_seed"][()] == 1
pos = f["stages/interphase/1000/positions"]
assert pos.dtype == np.float32 and pos.shape == (1002, 3) and pos.compression == "gzip" and pos.compression_opts == 6
c = f["stages/interphase/1000/contacts"]
assert c.dtype == np.int32 and c.compression == "gzip" and c.compression_opts == 4 and c.scaleoffset == 0
assert [s.decode() for s in f["stages/interphase/.steps"]] == ["1000"]
print("ok")
"""
    out = subprocess.run([PY39, "-c", code], capture_output=True, text=True)
    assert out.returncode == 0 and out.stdout.strip() == "ok", out.stderr


def test_interphase_driver_writes_the_store(prepared, c1_design):
    p, cfg = prepared
    icfg = InterphaseConfig()
    icfg.relaxation_steps = 20
    icfg.relaxation_sampling_interval = 10
    icfg.relaxation_logging_interval = 10
    icfg.sampling_interval = 20
    icfg.logging_interval = 20
    icfg.contactmap_output_window = 2
    with store.SimulationStore(p) as st:
        o, _ = interphase.build_interphase(oracle.OracleSystem, c1_design, icfg)
        drv = interphase.InterphaseDriver(o, c1_design, icfg, store=st, log=None)
        st.set_stage("relaxation")
        st.clear_frames()
        o.set_positions(st.load_positions(0))
        drv.run_relaxation()
        st.set_stage("interphase")
        st.clear_frames()
        drv.run_simulation(steps=40)
        st.set_stage("relaxation")
        assert st.load_steps() == [0, 10, 20]
        st.set_stage("interphase")
        assert st.load_steps() == [0, 20, 40]
        assert np.isfinite(st.load_positions(40)).all()
        assert st.load_interphase_context(40)["time"] == pytest.approx(40 * icfg.timestep)
        # contacts at the window ends (sample frames 0 and 2): frame 0 has none (distance 0), frame 2 (step 40) has
        c = st.load_contacts(40)
        assert c.shape[1] == 3 and (c[:, 0] < c[:, 1]).all() and not st.f.exists("/stages/interphase/0/contacts")


def test_store_library_exports_every_declared_symbol():
    import ctypes
    import re
    from pathlib import Path
    hdr = (Path(__file__).resolve().parents[1] / "include" / "gcs_store.h").read_text()
    names = re.findall(r"^(?:int|const char\*) (gcs_store_\w+)\(", hdr, flags=re.M)
    assert len(names) >= 14
    lib = ctypes.CDLL(str(store.LIB_PATH))
    for n in names:
        assert hasattr(lib, n), n


def test_async_writer_keeps_order_and_raises(prepared):
    """gcs.store.AsyncWriter: the drivers' sampling writes on a background thread land exactly as the synchronous
    calls would write them (same frames, same .steps order), and a failing write re-raises on the caller's thread"""
    p, _ = prepared
    rng = np.random.default_rng(3)
    frames = [rng.normal(size=(50, 3)) for _ in range(6)]
    with store.SimulationStore(p) as s:
        s.set_stage("interphase")
        s.clear_frames()
        w = store.AsyncWriter(s, depth=2)
        for k, x in enumerate(frames):
            w.save_frame("interphase", 10 * (k + 1), x)
        w.save_contacts(60, np.array([[0, 1, 2], [0, 3, 1]], dtype=np.uint32))
        w.flush()
        assert s.load_steps() == [10, 20, 30, 40, 50, 60]
        for k, x in enumerate(frames):
            got = s.load_positions(10 * (k + 1))
            assert np.array_equal(got.astype(np.float32), store.quantize_positions(x))
        assert np.array_equal(s.load_contacts(60), [[0, 1, 2], [0, 3, 1]])
        def bad():
            raise store.StoreError("write failed")
        w._put(bad)  # a failing write: raised on this thread at close, not lost
        with pytest.raises(store.StoreError):
            w.close()


def test_async_writer_close_inside_a_handler_still_raises(prepared):
    """a plain close() raises a failed deferred write even when it runs inside an unrelated, handled `except` block
    (sys.exc_info() is set there); only close(propagating=exc) / the context manager's unwind adds it as a note"""
    p, _ = prepared

    def bad():
        raise store.StoreError("write failed")
    with store.SimulationStore(p) as s:
        w = store.AsyncWriter(s, depth=2)
        w._put(bad)
        try:
            raise KeyError("handled elsewhere")
        except KeyError:
            with pytest.raises(store.StoreError):
                w.close()
        w = store.AsyncWriter(s, depth=2)
        with pytest.raises(ValueError) as info:
            with w:
                w._put(bad)
                w.q.join()
                raise ValueError("the stage failed")
        notes = getattr(info.value, "__notes__", [])
        assert any("deferred write also failed" in n for n in notes) or not hasattr(info.value, "add_note")


def test_deflated_frames_equal_the_filter_path(prepared):
    """gcs_store_write_deflated (the async writer's frames, deflated on a thread pool): the chunk stored is byte for
    byte the one HDF5's deflate-6 filter stores for the same positions, and the dataset reads back the same"""
    p, _ = prepared
    x = store.quantize_positions(np.random.default_rng(5).normal(size=(3000, 3)))
    with store.SimulationStore(p) as s:
        s.set_stage("interphase")
        s.save_positions(1000, x, quantized=True)
        s.save_positions(2000, x, quantized=True, zdata=store.deflated_frame(x))
        assert np.array_equal(s.load_positions(1000), s.load_positions(2000))
        assert np.array_equal(s.load_positions(2000).astype(np.float32), x)
    if PY39 is None:
        pytest.skip("no h5py interpreter for the raw-chunk comparison")
    code = f"""
import h5py
f = h5py.File({str(p)!r}, "r")
a, b = f["stages/interphase/1000/positions"], f["stages/interphase/2000/positions"]
assert b.compression == "gzip" and b.compression_opts == 6 and b.chunks == (3000, 3)
ma, ca = a.id.read_direct_chunk((0, 0))
mb, cb = b.id.read_direct_chunk((0, 0))
assert ma == mb == 0 and ca == cb, (ma, mb, len(ca), len(cb))
print("ok")
"""
    out = subprocess.run([PY39, "-c", code], capture_output=True, text=True)
    assert out.returncode == 0 and out.stdout.strip() == "ok", out.stderr


@pytest.mark.parametrize("rows,chunk", [(1, 8), (7, 8), (16, 8), (1000, 64), (5000, 1 << 16)])
def test_scaleoffset_contacts_equal_the_library_chunks(tmp_path, rows, chunk):
    """gcs_store_write_scaleoffset_i32 (contact tables encoded on host threads): every stored chunk is byte for byte
    the one HDF5's scale-offset + deflate-4 filters store for the same chunking (h5py writes the reference), and the
    array reads back exactly; the tables hold index 0 (the fill value, coded apart by the filter)"""
    rng = np.random.default_rng(rows)
    i = np.sort(rng.integers(0, 50, rows))
    t = np.stack([i, i + rng.integers(1, 40, rows), rng.integers(1, 9, rows)], axis=1).astype(np.int32)
    t[0, 0] = 0
    p = tmp_path / "c.h5"
    with store.H5File(p, create=True) as h:
        h.write_scaleoffset_i32("/ours", t, 4, chunk_rows=chunk, threads=4)
        assert np.array_equal(h.read_array("/ours", store.H5_I32).reshape(-1, 3), t)
    if PY39 is None:
        pytest.skip("no h5py interpreter for the raw-chunk comparison")
    np.save(tmp_path / "t.npy", t)
    code = f"""
import h5py, numpy as np
t = np.load({str(tmp_path / "t.npy")!r})
cr = min({chunk}, t.shape[0])
with h5py.File({str(p)!r}, "a") as f:
    f.create_dataset("lib", data=t, chunks=(cr, 3), scaleoffset=0, compression="gzip", compression_opts=4)
with h5py.File({str(p)!r}, "r") as f:
    a, b = f["lib"], f["ours"]
    assert b.chunks == a.chunks and b.scaleoffset == 0 and b.compression == "gzip" and b.compression_opts == 4
    assert a.id.get_create_plist().get_filter(0)[0] == b.id.get_create_plist().get_filter(0)[0]
    for r0 in range(0, t.shape[0], cr):
        ma, ca = a.id.read_direct_chunk((r0, 0))
        mb, cb = b.id.read_direct_chunk((r0, 0))
        assert ma == mb == 0 and ca == cb, (r0, len(ca), len(cb))
print("ok")
"""
    out = subprocess.run([PY39, "-c", code], capture_output=True, text=True)
    assert out.returncode == 0 and out.stdout.strip() == "ok", out.stderr

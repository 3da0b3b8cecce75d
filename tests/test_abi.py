"""CPU tests of the C-ABI boundary: libgcs.so loads, exports every symbol include/gcs.h declares, and the
ctypes mirror agrees with the C layout.  No compute call is made without a GPU."""
import re
import subprocess
import ctypes as C
from pathlib import Path

import pytest

from gcs import _abi as A

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "gcs.h"


def declared_functions():
    text = HEADER.read_text()
    return sorted(set(re.findall(r"^(?:const\s+char\s*\*|int)\s+(gcs_\w+)\s*\(", text, flags=re.M)))


def test_header_declares_the_boundary():
    names = declared_functions()
    assert len(names) >= 29
    assert set(names) == set(A.PROTOTYPES), set(names) ^ set(A.PROTOTYPES)


def test_library_exports_every_symbol():
    lib = A.load()
    for name in declared_functions():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", str(A.LIB_PATH)], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (gcs_\w+)", out))
    assert set(declared_functions()) <= exported


def test_abi_version():
    assert A.load().gcs_abi_version() == 3


STRUCTS = {
    "gcs_system_desc": A.SystemDesc, "gcs_softcore_params": A.SoftcoreParams, "gcs_bond_params": A.BondParams,
    "gcs_softwell_params": A.SoftwellParams, "gcs_wall_params": A.WallParams,
    "gcs_point_source_params": A.PointSourceParams, "gcs_kinetochore_spec": A.KinetochoreSpec,
    "gcs_context": A.Context, "gcs_schedule": A.Schedule, "gcs_bd_config": A.BDConfig, "gcs_profile": A.Profile, "gcs_list_stats": A.ListStats, "gcs_run_stats": A.RunStats,
}


def test_ctypes_layout_matches_header(tmp_path):
    src = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void) {"]
    for cname, py in STRUCTS.items():
        src.append(f'printf("{cname} %zu\\n", sizeof({cname}));')
        for fname, _ in py._fields_:
            src.append(f'printf("{cname}.{fname} %zu\\n", offsetof({cname}, {fname}));')
    src.append("return 0; }")
    (tmp_path / "l.c").write_text("\n".join(src))
    subprocess.run(["gcc", "-o", str(tmp_path / "l"), str(tmp_path / "l.c")], check=True)
    lines = subprocess.run([str(tmp_path / "l")], capture_output=True, text=True, check=True).stdout.split("\n")
    got = dict(line.rsplit(" ", 1) for line in lines if line)
    for cname, py in STRUCTS.items():
        assert int(got[cname]) == C.sizeof(py), cname
        for fname, _ in py._fields_:
            assert int(got[f"{cname}.{fname}"]) == getattr(py, fname).offset, f"{cname}.{fname}"


def test_errors_are_reported_not_crashed():
    lib = A.load()
    h = C.c_void_p()
    d = A.SystemDesc()
    d.particle_count = 0
    assert lib.gcs_engine_create(C.byref(d), C.byref(h)) == A.GCS_EINVAL
    assert b"particle_count" in lib.gcs_last_error()
    assert lib.gcs_engine_create(None, C.byref(h)) == A.GCS_EINVAL
    d.particle_count = 10
    d.precision = 16  # neither 0, 32 nor 64
    assert lib.gcs_engine_create(C.byref(d), C.byref(h)) == A.GCS_EINVAL
    assert b"precision" in lib.gcs_last_error()


def test_precision_names():
    from gcs.engine import precision_bits
    assert precision_bits(None) == 64 and precision_bits("f64") == 64 and precision_bits("fp32") == 32
    assert precision_bits(32) == 32
    with pytest.raises(ValueError):
        precision_bits(16)


def test_no_cpu_fallback_without_device():
    from gcs.engine import Engine, device_count
    if device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(A.GcsError):
        Engine(10)


def test_option_numbers_match_header():
    """every GCS_OPT_* the header defines has the same number in the ctypes mirror (gcs._abi.OPT_*)"""
    opts = dict((k, int(v)) for k, v in re.findall(r"^#define GCS_OPT_(\w+)\s+(\d+)", HEADER.read_text(), flags=re.M))
    assert "LIST_FORMAT" in opts and len(opts) >= 15
    for name, num in opts.items():
        assert getattr(A, "OPT_" + name) == num, name

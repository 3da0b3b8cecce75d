"""CPU: the reference-side C++ binding that INTEGRATION.md §3 documents compiles against include/gcs.h and links
libgcs.so, so the snippet cannot rot silently.  The three code blocks of §3 are taken from the
document as they stand: the `gcs_backend` header (with a stub `md::point` of 3 doubles, the micromd type it binds,
common/simulation_store.hpp-style exceptions), and the two driver fragments -- setup_repulsive_forcefield
(stage_interphase/simulation_driver_forcefield.cpp:21-53) and run_simulation's loop
(stage_interphase/simulation_driver_interphase.cpp:9-64) -- compiled inside a stub driver whose `_config` carries the
simulation_config.hpp fields they read.  The program then checks gcs_abi_version() == 3 and that constructing the
backend without a device throws std::runtime_error carrying gcs_last_error() (no CPU fallback)."""
import re
import shutil
import subprocess
from pathlib import Path

import pytest

from gcs import _abi as A

ROOT = Path(__file__).resolve().parents[1]
DOC = ROOT / "INTEGRATION.md"

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")

STUB_PRE = r"""
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <numeric>
#include <random>
#include <stdexcept>
#include <string>
#include <vector>
namespace md {
struct point { double x, y, z; };  // micromd's point: three doubles, contiguous
using step = long;
}
"""

DRIVER = r"""
struct stub_config {
    double a_core_repulsion = 2.5, a_core_diameter = 0.3, b_core_repulsion = 2.5, b_core_diameter = 0.24;
    double timestep = 1e-4, temperature = 1.0;
    double core_scale_init = 0.5, core_scale_tau = 1.0, bond_scale_init = 0.5, bond_scale_tau = 1.0;
    double wall_semiaxes_spring[3] = {1, 1, 1};
    double wall_mobility = 1.0;
    double contactmap_distance = 0.3;
    md::step steps = 10, logging_interval = 5, sampling_interval = 5, contactmap_update_interval = 5;
};

struct stub_driver {
    stub_config _config;
    gcs_backend& _gcs;
    std::mt19937_64 _random{42};
    explicit stub_driver(gcs_backend& g) : _gcs(g) {}
    double core_scale_at(md::step) const { return 1.0; }
    void callback(md::step) {}
    void host_callback(md::step) {}

    void setup_repulsive_forcefield()
    {
@@REPULSIVE@@
    }

    void run_simulation()
    {
@@RUN@@
    }
};

int main()
{
    if (gcs_abi_version() != 3) {
        std::printf("abi %d\n", gcs_abi_version());
        return 2;
    }
    std::vector<double> mu(10, 1.0), ab(20, 0.5);
    try {
        gcs_backend b(mu, ab, 0);
        stub_driver d(b);
        (void)d;
        std::printf("no exception without a device\n");
        return 3;
    } catch (std::runtime_error const& err) {
        std::string const what = err.what(), last = gcs_last_error();
        if (last.empty() || what.find(last) == std::string::npos) {
            std::printf("message '%s' does not carry gcs_last_error '%s'\n", what.c_str(), last.c_str());
            return 4;
        }
        std::printf("ok: %s\n", what.c_str());
        return 0;
    }
}
"""


def cpp_blocks():
    text = DOC.read_text()
    sec = text[text.index("## 3. The binding a maintainer would add"):text.index("## 4.")]
    return re.findall(r"```cpp\n(.*?)```", sec, flags=re.S)


def test_section_3_has_the_three_blocks():
    blocks = cpp_blocks()
    assert len(blocks) == 3
    assert "class gcs_backend" in blocks[0]
    assert "gcs_add_neighbor_softcore" in blocks[1]
    assert "gcs_engine_run" in blocks[2]


def test_reference_binding_compiles_links_and_fails_without_device(tmp_path):
    backend, repulsive, run = cpp_blocks()
    (tmp_path / "gcs_backend.hpp").write_text(STUB_PRE + backend)
    indent = lambda s: "\n".join("        " + ln for ln in s.splitlines())
    src = '#include "gcs_backend.hpp"\n' + DRIVER.replace("@@REPULSIVE@@", indent(repulsive)).replace(
        "@@RUN@@", indent(run))
    (tmp_path / "main.cpp").write_text(src)
    libdir = A.LIB_PATH.parent
    exe = tmp_path / "binding"
    cc = subprocess.run(["g++", "-std=c++17", "-Wall", "-Werror", "-Wno-unused-variable", "-I", str(ROOT / "include"),
                         str(tmp_path / "main.cpp"), "-o", str(exe), f"-L{libdir}", "-lgcs",
                         f"-Wl,-rpath,{libdir}", "-Wl,--allow-shlib-undefined"],
                        capture_output=True, text=True)
    assert cc.returncode == 0, cc.stderr
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    assert r.stdout.startswith("ok: gcs: "), r.stdout

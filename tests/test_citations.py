"""Every reference citation `path.ext:lines` in the boundary headers (include/*.h), the oracle, the package sources,
the docs and the tests points at lines
that exist in /root/reference (paths relative to src/simulation/ or the reference root, or a unique file name).
A bare `:lines` continues the file cited last in the same comment.  Skipped where the reference is absent (the GPU
box)."""
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
REF = Path("/root/reference")
BASES = [REF / "src" / "simulation", REF / "src", REF]

_TOKEN = re.compile(r"(?P<file>[A-Za-z_][\w./-]*\.(?:cpp|hpp|py|h))?:(?P<lines>\d+(?:-\d+)?)")
_CONT = re.compile(r",\s*(\d+)(?:-(\d+))?(?![\d.:\w])")


def citations(text: str):
    """(file, first, last) for every citation; bare `:a-b` refers to the previous file token"""
    out, last = [], None
    for m in _TOKEN.finditer(text):
        f = m.group("file")
        if f is None:
            # only a continuation like ", :81-83" or ", 49-51" directly after a citation counts
            prefix = text[max(0, m.start() - 3):m.start()]
            if last is None or not re.search(r"[,;(]\s*$", prefix):
                continue
            f = last
        last = f
        a, _, b = m.group("lines").partition("-")
        out.append((f, int(a), int(b or a)))
        # comma-continued plain ranges: "cpp:16-17, 51-52, 67-90"
        pos = m.end()
        while (mm := _CONT.match(text, pos)) is not None:
            out.append((f, int(mm.group(1)), int(mm.group(2) or mm.group(1))))
            pos = mm.end()
    return out


def resolve(name: str):
    for b in BASES:
        p = b / name
        if p.is_file():
            return p
    hits = [p for p in REF.rglob(Path(name).name) if str(p).endswith(name) and p.is_file()]
    if len(hits) == 1:
        return hits[0]
    return None if not hits else "ambiguous"


PKG = ROOT / "3d-genome-cycle_amd"
FILES = (sorted((ROOT / "include").glob("*.h")) + [ROOT / "oracle" / "gcs_oracle.c", ROOT / "oracle" / "gcs_oracle.h"]
         + sorted((PKG / "gcs").glob("*.py")) + sorted(p for p in (PKG / "csrc").glob("*") if p.suffix in (".hip", ".hpp", ".cpp"))
         + [ROOT / "DESIGN.md", ROOT / "INTEGRATION.md", ROOT / "bench.py"]
         + sorted(p for p in (ROOT / "tests").glob("*.py") if p.name != "test_citations.py"))


@pytest.mark.skipif(not REF.is_dir(), reason="reference checkout not present")
@pytest.mark.parametrize("path", FILES, ids=lambda p: p.name)
def test_cited_lines_exist(path):
    cites = citations(path.read_text())
    assert cites or path.suffix != ".c", f"no citations found in {path.name}"
    bad = []
    for f, a, b in cites:
        p = resolve(f)
        if p is None or p == "ambiguous":
            bad.append(f"{f}:{a}-{b} ({'ambiguous' if p else 'no such file'})")
            continue
        n = len(p.read_text(errors="replace").splitlines())
        if not (1 <= a <= b <= n):
            bad.append(f"{f}:{a}-{b} (file has {n} lines)")
    assert not bad, bad


def test_parser_reads_continuations():
    c = citations("x (stage_interphase/simulation_driver_interphase.cpp:16-17, 51-52, 67-90) y (:81-83, :147-149)")
    assert c[:3] == [("stage_interphase/simulation_driver_interphase.cpp", 16, 17),
                     ("stage_interphase/simulation_driver_interphase.cpp", 51, 52),
                     ("stage_interphase/simulation_driver_interphase.cpp", 67, 90)]
    assert c[3:] == [("stage_interphase/simulation_driver_interphase.cpp", 81, 83),
                     ("stage_interphase/simulation_driver_interphase.cpp", 147, 149)]

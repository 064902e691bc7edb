"""The render kernel's f32 candidate filters may keep a primitive the exact f64 test rejects, never
reject one it accepts. Both fuzzers run the filters' exact f32 sequences (the quad one compiles the
kernel's own header, crt_quad_filter.h) against the reference-order exact tests; CPU only."""
import shutil
import subprocess

import pytest

from conftest import ROOT

pytestmark = pytest.mark.skipif(shutil.which("g++") is None or shutil.which("gcc") is None,
                                reason="needs gcc/g++")


def _run(tmp_path, compiler, src, std, millions):
    exe = tmp_path / src.stem
    subprocess.run([compiler, std, "-O2", "-ffp-contract=off", "-o", str(exe), str(src), "-lm"], check=True)
    r = subprocess.run([str(exe), str(millions)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def test_quad_filter_never_rejects_a_hit(tmp_path):
    # both the generic filter and the flat-box filter of axis-aligned parallelograms
    out = _run(tmp_path, "g++", ROOT / "tools" / "fuzz_quad_filter.cpp", "-std=c++20", 1)
    lines = [l for l in out.splitlines() if "violations" in l]
    assert len(lines) == 2 and all("violations 0;" in l for l in lines), out
    # the kernel's per-axis form of the flat-box filter gives the same bit on every flat case
    axis = [l for l in out.splitlines() if l.startswith("per-axis flat filter")]
    assert len(axis) == 1 and axis[0].rstrip().endswith(" 0 differ from the flat-box filter"), out


def test_sphere_filter_never_rejects_a_hit(tmp_path):
    out = _run(tmp_path, "gcc", ROOT / "tools" / "fuzz_sphere_filter.c", "-std=c11", 1)
    lines = [l for l in out.splitlines() if "violations" in l]
    assert len(lines) == 2 and all(l.rstrip().endswith("violations 0") for l in lines), out

"""div_rn (csrc/cwq_refmath.h, the device fitter's KL-term divisions: a reciprocal and two
Markstein corrections) against IEEE float division -- every float dividend (both signs) for
a set of divisors (counts and variance-like values, incl. an all-ones significand), plus
random and near-midpoint pairs over the guarded exponent range and beyond it (the IEEE
fallback).  The host build of the function the GPU fitter inlines (scripts/check_div_rn.hip).
CPU only: hipcc compiles the host program."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("hipcc") is None, reason="hipcc not on PATH")
def test_div_rn_equals_ieee_division(tmp_path):
    exe = tmp_path / "check_div_rn"
    subprocess.run(["hipcc", "-O2", "-std=c++17", os.path.join(ROOT, "scripts", "check_div_rn.hip"),
                    "-o", str(exe), "-lpthread"], check=True, timeout=300)
    out = subprocess.run([str(exe), "40000000"], capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stdout + out.stderr
    assert " 0 mismatches" in out.stdout

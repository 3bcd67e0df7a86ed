"""ref_logf (csrc/cwq_refmath.h, the fitters' float32 log) against the double log rounded
once, on every positive float bit pattern -- the host build of the same function the GPU
fitters inline (scripts/check_ref_logf.hip).  CPU only: hipcc compiles the host program."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("hipcc") is None, reason="hipcc not on PATH")
def test_ref_logf_exhaustive(tmp_path):
    exe = tmp_path / "check_ref_logf"
    subprocess.run(["hipcc", "-O2", "-std=c++17", os.path.join(ROOT, "scripts", "check_ref_logf.hip"),
                    "-o", str(exe), "-lpthread"], check=True, timeout=300)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "0 mismatches" in out.stdout

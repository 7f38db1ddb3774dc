"""Host-side equivalence of the product's lean arithmetic (lazy Montgomery, 64-bit
M_EXT + Barrett Poseidon2, lazy extension multiply) with step-by-step restatements.
Builds tests/native/field_equiv.cpp with g++ against risc0_amd/csrc headers."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_field_and_poseidon2_equivalence(tmp_path):
    exe = tmp_path / "field_equiv"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "risc0_amd", "csrc"), "-o", str(exe),
                    os.path.join(ROOT, "tests", "native", "field_equiv.cpp")], check=True)
    out = subprocess.run([str(exe), "50000"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.startswith("OK")

"""GPU: the reference's GoogleTest cases restated against the C++ façade (tests/cpp/test_facade.cpp)."""
import os
import subprocess

import pytest

from cpp_build import ROOT, build

pytestmark = pytest.mark.gpu


def test_cpp_facade_reference_cases(tmp_path):
    exe = build(os.path.join(ROOT, "tests", "cpp", "test_facade.cpp"), str(tmp_path / "test_facade"))
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0 and "ALL PASSED" in r.stdout, r.stdout[-3000:] + r.stderr[-2000:]


def test_demo_cli_reference_data(tmp_path):
    """The demo on the reference's data files: the answers of SURVEY App. A (A.txt complex: power
    -> 5-i, shifted at 3.1 -> 5-i, QR converges; B.txt complex: shifted at 2.3 -> 3+2i, QR refuses
    the sparse matrix like the reference; A.txt as double: 1 + sqrt(15))."""
    exe = build(os.path.join(ROOT, "examples", "eigsol_demo.cpp"), str(tmp_path / "eigsol_demo"))
    data = os.path.join(ROOT, "tests", "golden")
    r = subprocess.run([exe, os.path.join(data, "A.txt"), os.path.join(data, "B.txt")], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    out = r.stdout
    assert out.count("Converged : true") >= 1
    assert "Eigenvalue near the shift: (5,-1)" in out or "Eigenvalue near the shift: (5," in out
    assert "Eigenvalue near the shift: (3,2)" in out or "Eigenvalue near the shift: (3," in out
    assert "QR eigenvalues for Matrix A" in out
    assert "only dense matrices" in r.stderr
    r = subprocess.run([exe, "--real", os.path.join(data, "A.txt")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "Eigenvalue: 4.87298" in r.stdout

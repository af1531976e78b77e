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


def test_reference_shaped_caller(tmp_path):
    """examples/main_dropin.cpp: the reference demo's code shape (includes "src/...", helpers
    constrained on EigSol::ScalarConcept, v.transpose() printing, structured bindings of
    qr_decompose) compiled with -std=c++20 against the compat include tree, run on the reference
    data: A.txt complex is upper triangular with eigenvalues {1+3i, 2+4i, 5-i}; the reference-
    signature qr_eigenvalues runs the default (Francis) path, which reports them like the
    reference's converged diag(H) (compared as a set, as the reference's tests sort them)."""
    exe = build(os.path.join(ROOT, "examples", "main_dropin.cpp"), str(tmp_path / "main_dropin"),
                extra_includes=(os.path.join(ROOT, "include", "eigsol", "compat"),))
    data = os.path.join(ROOT, "tests", "golden")
    r = subprocess.run([exe, os.path.join(data, "A.txt"), os.path.join(data, "B.txt")], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    out = r.stdout
    shifted = out.split("===== Shifted inverse power method =====")[1].split("===== QR")[0]
    assert "Eigenvalue: (5,-1)" in shifted or "Eigenvalue: (5," in shifted        # A, shift 3.1
    assert "Eigenvalue: (3,2)" in shifted or "Eigenvalue: (3," in shifted         # B, shift 2.3
    assert "H(A) = " in out and "Q_A * R_A (should approximate A) = " in out
    qa = out.split("QR eigenvalues for Matrix A")[1]
    assert "Converged              : true" in qa.splitlines()[1]
    # the three eigenvalues, compared as a set
    diag = qa.split("Eigenvalues (diag of H): \n")[1].splitlines()[0]
    got = [complex(t.replace(",", "+").replace("+-", "-").strip("()") + "j") for t in diag.split()]
    want = sorted([1 + 3j, 2 + 4j, 5 - 1j], key=lambda z: (z.real, z.imag))
    got = sorted(got, key=lambda z: (z.real, z.imag))
    assert all(abs(g - w) < 1e-8 for g, w in zip(got, want)), diag
    assert "only dense matrices" in r.stderr

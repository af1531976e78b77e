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

"""CPU: the C++ drop-in façade (include/eigsol/*.hpp) compiles with -Wall -Wextra -Werror and
links against libeigsol_hip.so; the reference-style test program builds (it runs under -m gpu)."""
import os

import pytest

from cpp_build import ROOT, build


@pytest.mark.skipif(not os.path.exists(os.path.join(ROOT, "pcsc_eigenvalue_solver_project_amd", "libeigsol_hip.so")),
                    reason="library not built")
def test_facade_compiles_and_links(tmp_path):
    out = build(os.path.join(ROOT, "tests", "cpp", "test_facade.cpp"), str(tmp_path / "test_facade"))
    assert os.path.getsize(out) > 0


@pytest.mark.skipif(not os.path.exists(os.path.join(ROOT, "pcsc_eigenvalue_solver_project_amd", "libeigsol_hip.so")),
                    reason="library not built")
def test_demo_cli_compiles(tmp_path):
    """examples/eigsol_demo.cpp (the reference main.cpp's counterpart) builds with -Werror."""
    out = build(os.path.join(ROOT, "examples", "eigsol_demo.cpp"), str(tmp_path / "eigsol_demo"))
    assert os.path.getsize(out) > 0


@pytest.mark.skipif(not os.path.exists(os.path.join(ROOT, "pcsc_eigenvalue_solver_project_amd", "libeigsol_hip.so")),
                    reason="library not built")
def test_reference_shaped_caller_compiles(tmp_path):
    """examples/main_dropin.cpp keeps the reference demo's #include "src/..." lines and its
    `template <EigSol::ScalarConcept S>` helpers; it builds with -std=c++20 -Werror."""
    out = build(os.path.join(ROOT, "examples", "main_dropin.cpp"), str(tmp_path / "main_dropin"),
                extra_includes=(os.path.join(ROOT, "include", "eigsol", "compat"),))
    assert os.path.getsize(out) > 0

"""General (non-triangular) sparse shifted inverse iteration and solve_shifted on the RCM-banded
direct LU (band_lu.hip), against the committed fixture of the reference loop.

Fixture (tests/golden/convdiff141.json + convdiff141_eigvec.npy, made by
tests/golden/make_golden.py convdiff with scipy's SuperLU, a direct sparse LU like the reference's
SparseLU): shiftedInversePowerImpl (shifted_inverse_power_solver.hpp:21-79) on the randomly
permuted complex 2-D convection-diffusion matrix of synthetic.convdiff_complex (n = 19881, LU with
real fill, ILU(0) drops it), sigma at 0.1 of the nearest-neighbour gap from an interior eigenvalue,
x0 = synthetic.start_vector(n, complex, seed 7), tol 1e-12.

Tolerances (SURVEY §8d parity): lambda within 1e-10 (1 + |lambda|); iteration count equal, +-1 only
when the last step sits at the tolerance; |x^H x_ref| >= 1 - 1e-10; solve residuals
||(A - sigma I) y - b|| <= 1e-11 ||b|| for the direct factor.  Failure semantics: ILU(0)-GMRES
forced on the same system stagnates and, with the densified-LU fallback disabled, raises
EIGSOL_E_SOLVER "SparseLU solve failed" (solve_shifted.hpp:112-114); with the fallback (default) it
finishes on the densified LU and matches the fixture; a structurally singular A - sigma I raises
"SparseLU factorization failed" (:108-110)."""
import json
import os

import numpy as np
import pytest
import scipy.sparse as sp

import pcsc_eigenvalue_solver_project_amd as E
from oracle import oracle as O
from pcsc_eigenvalue_solver_project_amd import synthetic as S

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def ctx():
    c = E.Context(0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def convdiff():
    fx = json.load(open(os.path.join(GOLD, "convdiff141.json")))
    rp, ci, v = S.convdiff_complex(fx["nx"], seed=fx["seed"])
    assert len(v) == fx["nnz"] and int(ci.astype(np.int64).sum()) == fx["colidx_sum"]
    assert abs(np.abs(v).sum() - fx["values_abs_sum"]) <= 1e-9 * fx["values_abs_sum"]
    xref = np.load(os.path.join(GOLD, "convdiff141_eigvec.npy"))
    return fx, rp, ci, v, xref


@pytest.fixture
def env():
    saved = {}

    def set_(k, val):
        saved.setdefault(k, os.environ.get(k))
        os.environ[k] = val

    yield set_
    for k, val in saved.items():
        if val is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = val


def _check_fixture(r, fx, xref):
    lam = complex(*fx["lambda"])
    assert r.converged and fx["converged"]
    assert abs(r.eigenvalue - lam) <= 1e-10 * (1 + abs(lam)), (r.eigenvalue, lam)
    if r.iterations != fx["iterations"]:
        tr = fx["trace"]
        last = abs(complex(*tr[-1]) - complex(*tr[-2])) / (1 + abs(complex(*tr[-1])))
        assert abs(r.iterations - fx["iterations"]) == 1 and 1e-13 <= last <= 1e-11, (r.iterations, last)
    assert abs(abs(np.vdot(r.eigenvector, xref)) - 1) <= 1e-10


def test_band_lu_convdiff_fixture(ctx, convdiff, env):
    fx, rp, ci, v, xref = convdiff
    env("EIGSOL_SPARSE_SOLVER", "band")   # n = 19881 > 16384 defaults to the multifrontal LU (test_gpu_multifrontal.py)
    n = fx["n"]
    A = E.CsrMatrix(ctx, rp, ci, v, (n, n))
    sigma = complex(*fx["sigma"])
    sess = E.ShiftedSession(A, sigma)
    info = sess.kernel_info()
    sess.close()
    assert info["variant"] == 8, info                 # the banded LU, not a fallback
    assert info["tiles"] <= 2 * 141 + 8               # kl + ku of the RCM order (~ 2 nx)
    r = E.shifted_inverse_power_method(A, E.ShiftedSolverOptions(fx["max_iter"], fx["tol"], sigma),
                                       S.start_vector(n, np.complex128))
    _check_fixture(r, fx, xref)
    M = sp.csr_matrix((v, ci, rp), shape=(n, n))
    assert np.linalg.norm(M @ r.eigenvector - r.eigenvalue * r.eigenvector) <= 1e-9
    A.close()


def test_band_lu_solve_shifted_residual(ctx, convdiff, env):
    fx, rp, ci, v, _ = convdiff
    env("EIGSOL_SPARSE_SOLVER", "band")
    n = fx["n"]
    A = E.CsrMatrix(ctx, rp, ci, v, (n, n))
    M = sp.csr_matrix((v, ci, rp), shape=(n, n))
    for sigma in (complex(*fx["sigma"]), 0.5 - 0.25j, 7.9 + 0.0j):
        b = S.start_vector(n, np.complex128, seed=11)
        y = E.solve_shifted(A, sigma, b)
        assert np.linalg.norm(M @ y - sigma * y - b) <= 1e-11 * np.linalg.norm(b) * max(1.0, np.linalg.norm(y) / np.linalg.norm(b) * 1e-3)
    A.close()


def test_band_lu_real_parity_with_reference_loop(ctx, env):
    """f64: a real nonsymmetric permuted stencil (real part of the generator, n = 900) against the
    oracle's restatement of the reference loop with a direct LU solve per iteration."""
    env("EIGSOL_SPARSE_SOLVER", "band")
    rp, ci, v = S.convdiff_complex(30, seed=5)
    v = np.ascontiguousarray(v.real)
    n = 900
    D = sp.csr_matrix((v, ci, rp), shape=(n, n)).toarray()
    ev = np.linalg.eigvals(D)
    re = np.sort(ev.real[np.abs(ev.imag) < 1e-12])
    i = len(re) // 3
    sigma = re[i] + 0.1 * min(re[i + 1] - re[i], re[i] - re[i - 1])
    A = E.CsrMatrix(ctx, rp, ci, v, (n, n))
    x0 = S.start_vector(n)
    r = E.shifted_inverse_power_method(A, E.ShiftedSolverOptions(500, 1e-12, sigma), x0)
    ref = O.shifted_dense(D, sigma, x0, 500, 1e-12)
    assert r.converged and ref["converged"]
    lam = ref["eigenvalue"]
    assert abs(r.eigenvalue - lam) <= 1e-10 * (1 + abs(lam)), (r.eigenvalue, lam)
    assert abs(r.iterations - ref["iterations"]) <= 1
    assert abs(abs(np.vdot(r.eigenvector, ref["eigenvector"])) - 1) <= 1e-10
    b = S.start_vector(n, seed=3)
    y = E.solve_shifted(A, sigma, b)
    assert np.linalg.norm(D @ y - sigma * y - b) <= 1e-10 * np.linalg.norm(b) * np.linalg.norm(y)
    A.close()


def test_band_lu_components_and_missing_diagonal(ctx, env):
    """Two disconnected stencils plus isolated rows without a stored diagonal (coeffRef inserts
    0 - sigma, solve_shifted.hpp:100-102): solve against a dense solve."""
    env("EIGSOL_SPARSE_SOLVER", "band")
    rp1, ci1, v1 = S.convdiff_complex(20, seed=1)
    rp2, ci2, v2 = S.convdiff_complex(15, seed=2)
    M1 = sp.csr_matrix((v1, ci1, rp1), shape=(400, 400))
    M2 = sp.csr_matrix((v2, ci2, rp2), shape=(225, 225))
    Z = sp.csr_matrix((5, 5), dtype=np.complex128)
    M = sp.block_diag([M1, Z, M2], format="csr")
    M.sort_indices()
    n = M.shape[0]
    A = E.CsrMatrix.from_scipy(ctx, M)
    sigma = 0.3 + 0.2j
    b = S.start_vector(n, np.complex128, seed=4)
    y = E.solve_shifted(A, sigma, b)
    ref = np.linalg.solve(M.toarray() - sigma * np.eye(n), b)
    assert np.linalg.norm(y - ref) <= 1e-11 * np.linalg.norm(ref)
    A.close()


def test_band_lu_singular_reports_factorization_failure(ctx, env):
    env("EIGSOL_SPARSE_SOLVER", "band")
    rp, ci, v = S.convdiff_complex(20, seed=3)
    M = sp.csr_matrix((v, ci, rp), shape=(400, 400)).tolil()
    sigma = 2.0 + 0.0j
    M[17, :] = 0                      # row 17 of A - sigma I vanishes: a zero pivot
    M[17, 17] = sigma
    M = sp.csr_matrix(M)
    M.eliminate_zeros()
    M.sort_indices()
    A = E.CsrMatrix.from_scipy(ctx, M)
    with pytest.raises(E.EigSolError) as ei:
        E.solve_shifted(A, sigma, np.ones(400, np.complex128))
    assert ei.value.status == 6 and "SparseLU factorization failed" in str(ei.value)
    A.close()


def test_gmres_stagnation_reports_solve_failure(ctx, convdiff, env):
    fx, rp, ci, v, _ = convdiff
    env("EIGSOL_SPARSE_SOLVER", "gmres")
    env("EIGSOL_GMRES_FALLBACK", "0")
    env("EIGSOL_LU_FILL_CAP", "0")       # ILU(0): the incomplete factor is what stagnates
    n = fx["n"]
    A = E.CsrMatrix(ctx, rp, ci, v, (n, n))
    with pytest.raises(E.EigSolError) as ei:
        E.solve_shifted(A, complex(*fx["sigma"]), S.start_vector(n, np.complex128, seed=11))
    assert ei.value.status == 6 and "SparseLU solve failed" in str(ei.value), str(ei.value)
    A.close()


def test_gmres_stagnation_falls_back_to_dense_lu(ctx, convdiff, env):
    fx, rp, ci, v, xref = convdiff
    env("EIGSOL_SPARSE_SOLVER", "gmres")
    env("EIGSOL_LU_FILL_CAP", "0")
    n = fx["n"]
    A = E.CsrMatrix(ctx, rp, ci, v, (n, n))
    sigma = complex(*fx["sigma"])
    r = E.shifted_inverse_power_method(A, E.ShiftedSolverOptions(fx["max_iter"], fx["tol"], sigma),
                                       S.start_vector(n, np.complex128))
    _check_fixture(r, fx, xref)
    A.close()


def test_mid_size_general_sparse_defaults_to_the_direct_family(ctx, env):
    """From n = 2048 (EIGSOL_SPARSE_FAMILY_MIN_N) a general sparse shifted factor takes the GMRES family's
    direct factors (here the nested-dissection multifrontal LU, variant 19) instead of the RCM band LU,
    whose one-workgroup solve was 15-40x slower per iteration at n = 4096-16384: the solution agrees with
    the band LU's (EIGSOL_SPARSE_SOLVER=band) and is backward stable (solve_shifted.hpp:96-115)."""
    rp, ci, v = S.convdiff_complex(64, seed=7)
    n = 4096
    M = sp.csr_matrix((v, ci, rp), shape=(n, n))
    A = E.CsrMatrix(ctx, rp, ci, v, (n, n))
    sigma = 3.0 - 0.2j
    b = S.start_vector(n, np.complex128, seed=5)
    s = E.ShiftedSession(A, sigma)
    assert s.kernel_info()["variant"] == 19, s.kernel_info()
    s.close()
    y = E.solve_shifted(A, sigma, b)
    env("EIGSOL_SPARSE_SOLVER", "band")
    yb = E.solve_shifted(A, sigma, b)
    assert np.linalg.norm(M @ y - sigma * y - b) <= 1e-11 * np.linalg.norm(b) * max(1.0, np.linalg.norm(y))
    assert np.linalg.norm(y - yb) <= 1e-10 * np.linalg.norm(yb)
    A.close()

"""GPU: the triangular factor of shiftedInversePowerMethod / solve_shifted
(shifted_inverse_power_solver.hpp:21-79, solve_shifted.hpp:48-118) analysed and laid out on the device
(round 5, shifted.hip factor_tri_device) against the host build (EIGSOL_TRSV_HOST=1).

The device build produces the host build's layout bit for bit (same dependency levels, positions
sorted by level with ascending rows inside a level, same padding, chunk CSR and one-wave head), so
every solve must agree BITWISE: solve_shifted's solution, the shifted inverse iteration's lambda
trace, iteration count and eigenvector, and kernel_info.  Cases: config-5-class complex upper
triangular (planted eigenvalue), real upper and lower, single precision, rows without a stored
diagonal (pivot 0 - sigma), a diagonal matrix, rows longer than 16 entries (two entries per lane),
an empty head (wide first level), and the zero-pivot error."""
import numpy as np
import pytest
import scipy.sparse as sp

import pcsc_eigenvalue_solver_project_amd as E
from pcsc_eigenvalue_solver_project_amd import synthetic as S

pytestmark = pytest.mark.gpu
TARGET = 1.5 * np.exp(0.7j)


@pytest.fixture(scope="module")
def ctx():
    c = E.Context(0)
    yield c
    c.close()


def _run(ctx, M, sigma, x0, b, host, monkeypatch, K=None):
    if host:
        monkeypatch.setenv("EIGSOL_TRSV_HOST", "1")
    else:
        monkeypatch.delenv("EIGSOL_TRSV_HOST", raising=False)
    if K is not None:
        monkeypatch.setenv("EIGSOL_TRSV_MULTI", str(K))
    A = E.CsrMatrix.from_scipy(ctx, M)
    y = E.solve_shifted(A, sigma, b)
    s = E.ShiftedSession(A, sigma, trace_capacity=256)
    info = s.kernel_info()
    s.begin(E.ShiftedSolverOptions(200, 1e-12 if M.dtype.itemsize >= 16 or M.dtype == np.float64 else 1e-5,
                                   sigma), x0)
    s.step(300)
    assert s.query()[0]
    r = s.finish()
    tr = s.trace(256)
    s.close()
    A.close()
    return y, r, tr, info


def _same(ctx, M, sigma, monkeypatch, K=None):
    n = M.shape[0]
    dt = M.dtype
    x0 = S.start_vector(n, dt, seed=5)
    b = S.start_vector(n, dt, seed=6)
    yh, rh, th, ih = _run(ctx, M, sigma, x0, b, True, monkeypatch, K)
    yd, rd, td, idv = _run(ctx, M, sigma, x0, b, False, monkeypatch, K)
    assert ih == idv, (ih, idv)
    assert np.array_equal(yh, yd)
    assert rh.iterations == rd.iterations and rh.converged == rd.converged
    assert np.array_equal(th, td)
    assert np.array_equal(np.asarray(rh.eigenvalue), np.asarray(rd.eigenvalue))
    assert np.array_equal(rh.eigenvector, rd.eigenvector)
    return yd, rd


def _csr(rp, ci, v, n):
    M = sp.csr_matrix((v, ci, rp), shape=(n, n))
    M.sort_indices()
    return M


@pytest.mark.parametrize("K", [1, 4])
def test_config5_class_complex_upper(ctx, monkeypatch, K):
    n = 200_000
    rp, ci, v, _ = S.triu_complex(n, 16)
    M = _csr(rp, ci, v, n)
    y, r = _same(ctx, M, TARGET + 1e-3, monkeypatch, K)
    assert r.converged and abs(r.eigenvalue - TARGET) <= 1e-10
    b = S.start_vector(n, np.complex128, seed=6)
    assert np.linalg.norm(M @ y - (TARGET + 1e-3) * y - b) <= 1e-10 * np.linalg.norm(b)


@pytest.mark.parametrize("dtype", [np.float64, np.float32, np.complex64])
def test_real_and_single_upper_and_lower(ctx, monkeypatch, dtype):
    n = 30_000
    rp, ci, v, d = S.triu_complex(n, 12, seed=3)
    M = _csr(rp, ci, v, n)
    if not np.issubdtype(dtype, np.complexfloating):
        M = _csr(rp, ci, v.real + 0.0, n)
        M.setdiag(1.0 + np.arange(n) % 97 / 50.0)   # real spectrum, distinct near the shift
    M = M.astype(dtype)
    sigma = 1.303 + (0.05j if np.issubdtype(dtype, np.complexfloating) else 0.0)   # next to 1.30, not on it
    _same(ctx, M, sigma, monkeypatch, K=1)
    L = sp.csr_matrix(M.T)
    L.sort_indices()
    _same(ctx, L, sigma, monkeypatch, K=1)


def test_missing_diagonal_diag_only_and_long_rows(ctx, monkeypatch):
    n = 20_000
    rp, ci, v, _ = S.triu_complex(n, 28, seed=8)       # 27 off-diagonal entries: two per lane
    M = _csr(rp, ci, v, n).tolil()
    for i in range(5, n, 997):
        M[i, i] = 0.0                                   # no stored diagonal: pivot 0 - sigma
    M = sp.csr_matrix(M)
    M.eliminate_zeros()
    M.sort_indices()
    sigma = TARGET + 1e-3
    _same(ctx, M, sigma, monkeypatch, K=1)
    _same(ctx, M, sigma, monkeypatch, K=3)
    D = sp.diags(np.linspace(1.0, 2.0, 5000) + 0j, format="csr")
    _same(ctx, D, 1.2501 + 0j, monkeypatch, K=1)


def test_empty_head_wide_first_level(ctx, monkeypatch):
    """A first level wider than the head allows (every row of the upper half independent): the
    head is empty and the whole solve is the chunk tail."""
    n = 40_000
    rng = np.random.default_rng(4)
    rows, cols, vals = [np.arange(n)], [np.arange(n)], [1.0 + rng.random(n)]
    top = np.arange(n // 2)
    for k in range(6):                                  # the top half reads the bottom half only
        rows.append(top)
        cols.append(n // 2 + (top * 7 + k * 131) % (n // 2))
        vals.append(0.1 * rng.standard_normal(n // 2))
    M = sp.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))), shape=(n, n))
    M.sum_duplicates()
    M.sort_indices()
    _same(ctx, M, 1.5, monkeypatch, K=1)


def test_zero_pivot_reported(ctx, monkeypatch):
    """A - sigma I with a zero pivot: the reference's SparseLU failure (solve_shifted.hpp:112-114),
    raised by both builds."""
    n = 5000
    rp, ci, v, d = S.triu_complex(n, 8)
    for host in (True, False):
        if host:
            monkeypatch.setenv("EIGSOL_TRSV_HOST", "1")
        else:
            monkeypatch.delenv("EIGSOL_TRSV_HOST", raising=False)
        A = E.CsrMatrix(ctx, rp, ci, v, (n, n))
        with pytest.raises(E.EigSolError, match="SparseLU"):
            E.solve_shifted(A, d[123], S.start_vector(n, np.complex128))
        A.close()

"""Triplets straight to the device CSR (the reader's sparse path,
file_matrix_reader.hpp:84-132): eigsol_csr_create_from_coo orders by (row, column) and sums repeated
positions in input order, which is what Matrix::Sparse's compression does with repeated insert()s.
Checked bitwise against a numpy restatement, and the resulting matrix runs the power method exactly
like one created from the equivalent CSR (same λ bits, same iteration count)."""
import numpy as np
import pytest

import pcsc_eigenvalue_solver_project_amd as E
from pcsc_eigenvalue_solver_project_amd import synthetic as S
from pcsc_eigenvalue_solver_project_amd._capi import EIGSOL_E_INVALID, EIGSOL_E_SIZE_MISMATCH

pytestmark = pytest.mark.gpu


def _expected_csr(r, c, v, nrows):
    order = np.lexsort((np.arange(len(r)), c, r))   # (row, col), ties in input order
    r, c, v = r[order], c[order], v[order]
    keep_r, keep_c, keep_v = [], [], []
    for i in range(len(r)):
        if keep_r and keep_r[-1] == r[i] and keep_c[-1] == c[i]:
            keep_v[-1] = keep_v[-1] + v[i]
        else:
            keep_r.append(r[i]); keep_c.append(c[i]); keep_v.append(v[i])
    rp = np.zeros(nrows + 1, np.int32)
    np.add.at(rp, np.asarray(keep_r, np.int64) + 1, 1)
    return np.cumsum(rp).astype(np.int32), np.asarray(keep_c, np.int32), np.asarray(keep_v, v.dtype)


@pytest.fixture(scope="module")
def ctx():
    c = E.Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("dtype", [np.float64, np.complex128, np.float32])
def test_coo_to_device_csr_bitwise(ctx, dtype):
    rng = np.random.default_rng(3)
    n, m = 500, 6000
    r = rng.integers(0, n, m).astype(np.int32)
    c = rng.integers(0, n, m).astype(np.int32)
    r[-300:], c[-300:] = r[:300], c[:300]            # repeated positions, some three times
    r[-50:], c[-50:] = r[:50], c[:50]
    v = rng.standard_normal(m)
    if np.issubdtype(dtype, np.complexfloating):
        v = v + 1j * rng.standard_normal(m)
    v = v.astype(dtype)
    A = E.CsrMatrix.from_coo(ctx, r, c, v, (n, n))
    rp, ci, vv = A.download()
    erp, eci, ev = _expected_csr(r, c, v, n)
    assert A.nnz == len(eci)
    assert np.array_equal(rp, erp) and np.array_equal(ci, eci)
    assert np.array_equal(vv.view(np.uint8), ev.view(np.uint8))
    A.close()


def test_coo_power_matches_csr(ctx):
    n, k = 50_000, 10
    rp, ci, v = S.band(n, k)
    rows = np.repeat(np.arange(n, dtype=np.int32), np.diff(rp))
    perm = np.random.default_rng(1).permutation(len(ci))        # file order: shuffled
    A = E.CsrMatrix.from_coo(ctx, rows[perm], ci[perm], v[perm], (n, n))
    B = E.CsrMatrix(ctx, rp, ci, v, (n, n))
    x0 = S.start_vector(n)
    opts = E.SolverOptions(500, 1e-12)
    ra, rb = E.power_method(A, opts, x0), E.power_method(B, opts, x0)
    assert ra.iterations == rb.iterations and ra.eigenvalue == rb.eigenvalue
    assert np.array_equal(ra.eigenvector, rb.eigenvector)
    A.close(); B.close()


def test_coo_rejects_bad_input(ctx):
    with pytest.raises(E.EigSolError) as ei:
        E.CsrMatrix.from_coo(ctx, [0, 5], [0, 1], np.ones(2), (3, 3))
    assert ei.value.status == EIGSOL_E_INVALID
    with pytest.raises(E.EigSolError) as ei:
        E.CsrMatrix.from_coo(ctx, [0, 1], [0], np.ones(2), (3, 3))
    assert ei.value.status == EIGSOL_E_SIZE_MISMATCH

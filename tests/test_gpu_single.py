"""GPU: native single precision (float / std::complex<float>, ScalarConcept types.hpp:28-30).

The reference instantiates every solver for float and std::complex<float>.  The device stores and
multiplies these in single precision (4 / 8 bytes per value: the f32 sliced SpMV moves 4 + 1 bytes
per nonzero instead of 8 + 1); norm and Rayleigh partial sums accumulate in double.  The oracle's
single-precision restatement (oracle/eigsol_oracle.cpp ORC_SINGLE: float products and row sums,
norm/dot accumulated in double and rounded to the scalar type, x = y / (float)normY,
power_method.hpp:47-99) runs from the same x0.

Tolerances (fp32):
  * SpMV (sliced layout and the row-per-lane fallback): bitwise equal to the CSC scatter in float;
  * dense GEMV: |y - y_ref| <= 1e-5 * (|A| |x|) (chunked column order);
  * power iteration at tol 1e-5: |dlambda| <= 1e-5 (1 + |lambda|), iterations +-1 (borderline
    stopping test only), |x^H x_ref| >= 1 - 1e-5;
  * triangular shifted inverse (config-5 class, complex<float>): the planted eigenvalue within
    1e-5, and the oracle's result within 1e-5;
  * dense and general-sparse (RCM band LU) shifted inverse in float: planted / numpy eigenvalues
    within 1e-4, solve backward errors at single precision (1e-4 ||M|| ||y||).
"""
import os

import numpy as np
import pytest
import scipy.sparse as sp
import scipy.sparse.linalg as spla

import pcsc_eigenvalue_solver_project_amd as E
from pcsc_eigenvalue_solver_project_amd import synthetic as S
from oracle import oracle as O

pytestmark = pytest.mark.gpu

SINGLE = [np.float32, np.complex64]


def _with_imag(v, dtype, seed=1):
    v = v.astype(dtype)
    if np.issubdtype(dtype, np.complexfloating):
        v = (v + 1j * np.random.default_rng(seed).uniform(-1, 1, len(v))).astype(dtype)
    return v


def _spmv_gpu(ctx, A, x):
    xd = ctx.malloc(x.nbytes)
    yd = ctx.malloc(A.shape[0] * x.itemsize)
    try:
        ctx.h2d(xd, x)
        A.spmv(xd, yd)
        y = np.empty(A.shape[0], dtype=x.dtype)
        ctx.d2h(y, yd)
        return y
    finally:
        ctx.free(xd)
        ctx.free(yd)


def _ragged(n, seed, dtype, max_len=40, long_rows=()):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, max_len, n)
    lens[rng.integers(0, n, 5)] = 0
    for r, L in long_rows:
        lens[r] = L
    rows, cols = [], []
    for i, L in enumerate(lens):
        c = np.sort(rng.choice(n, size=min(L, n), replace=False))
        rows.append(np.full(len(c), i))
        cols.append(c)
    rows, cols = np.concatenate(rows), np.concatenate(cols)
    vals = _with_imag(rng.uniform(-1, 1, len(rows)), dtype, seed + 1)
    return sp.csr_matrix((vals, (rows, cols)), shape=(n, n))


@pytest.mark.parametrize("dtype", SINGLE)
@pytest.mark.parametrize("kind", ["band", "uniform", "ragged", "long_rows"])
def test_single_spmv_bitwise(ctx, dtype, kind):
    n = 20000
    if kind == "band":
        rp, ci, v = S.band(n, 10)
        v = _with_imag(v, dtype)
    elif kind == "uniform":
        rp, ci, v = S.uniform(n, 16)
        v = _with_imag(v, dtype)
    else:
        lr = [(7, 3000), (n // 2, 9000)] if kind == "long_rows" else []
        M = _ragged(n, 3, dtype, long_rows=lr)
        rp, ci, v = M.indptr, M.indices, M.data
    A = E.CsrMatrix(ctx, rp, ci, v, (n, n))
    assert A.dtype == dtype
    x = S.start_vector(n, dtype)
    y = _spmv_gpu(ctx, A, x)
    cp, ri, vv = O.csr_to_csc(rp, ci, v, n)
    y_ref = O.spmv_csc(cp, ri, vv, x, n)
    assert y.dtype == dtype and y_ref.dtype == dtype
    assert np.array_equal(y, y_ref), np.max(np.abs(y - y_ref))


@pytest.mark.parametrize("dtype", SINGLE)
def test_single_spmv_rectangular(ctx, dtype):
    m, n = 3000, 5000
    M = sp.random(m, n, density=4e-3, random_state=np.random.default_rng(4), format="csr")
    M.data = _with_imag(M.data * 2 - 1, dtype)
    M.sort_indices()
    A = E.CsrMatrix(ctx, M.indptr, M.indices, M.data, (m, n))
    x = S.start_vector(n, dtype)
    y = _spmv_gpu(ctx, A, x)
    y_ref = O.spmv_csr(M.indptr, M.indices, M.data, x)
    assert np.array_equal(y, y_ref)


def _assert_single_parity(res, ref, tol):
    lam, lam_ref = res.eigenvalue, ref["eigenvalue"]
    assert abs(lam - lam_ref) <= 1e-5 * (1 + abs(lam_ref)), (lam, lam_ref)
    assert res.converged == ref["converged"]
    if res.iterations != ref["iterations"]:
        assert abs(res.iterations - ref["iterations"]) == 1
        tr = ref["trace"]
        k = min(res.iterations, ref["iterations"]) - 1
        assert abs(tr[k] - tr[k - 1]) <= 10 * tol * (1 + abs(tr[k]))
    x, xr = res.eigenvector, ref["eigenvector"]
    assert x.dtype == xr.dtype
    assert abs(np.vdot(x.astype(np.complex128), xr.astype(np.complex128))) >= 1 - 1e-5


@pytest.mark.parametrize("dtype", SINGLE)
@pytest.mark.parametrize("kind", ["band", "uniform", "long_rows"])
def test_single_power_csr_parity(ctx, dtype, kind):
    n = 40000
    if kind == "long_rows":
        M = _ragged(n, 9, dtype, max_len=20, long_rows=[(11, 5000)])
        M = M + sp.diags(np.full(n, 3.0, dtype=dtype))   # a dominant real part
        M = sp.csr_matrix(M, dtype=dtype)
        M.sort_indices()
        rp, ci, v = M.indptr, M.indices, M.data
    else:
        rp, ci, v = S.band(n, 10) if kind == "band" else S.uniform(n, 16)
        v = v.astype(dtype)
    A = E.CsrMatrix(ctx, rp, ci, v, (n, n))
    x0 = S.start_vector(n, dtype)
    tol = 1e-5
    res = E.power_method(A, E.SolverOptions(500, tol), x0)
    cp, ri, vv = O.csr_to_csc(rp, ci, v, n)
    ref = O.power_csc(cp, ri, vv, x0, 500, tol, want_trace=True)
    assert np.asarray(res.eigenvector).dtype == dtype
    _assert_single_parity(res, ref, tol)


@pytest.mark.parametrize("dtype", SINGLE)
def test_single_gemv_and_dense_power(ctx, dtype):
    n = 1536
    rng = np.random.default_rng(12)
    A = rng.uniform(0, 1, (n, n))
    if np.issubdtype(dtype, np.complexfloating):
        A = A + 0.1j * rng.uniform(-1, 1, (n, n))
    A = A.astype(dtype)
    D = E.DenseMatrix(ctx, A)
    x = S.start_vector(n, dtype)
    xd, yd = ctx.malloc(x.nbytes), ctx.malloc(x.nbytes)
    ctx.h2d(xd, x)
    D.gemv(xd, yd)
    y = np.empty(n, dtype=dtype)
    ctx.d2h(y, yd)
    ctx.free(xd)
    ctx.free(yd)
    y_ref = O.gemv(A, x)
    scale = np.abs(A).astype(np.float64) @ np.abs(x).astype(np.float64)
    assert np.all(np.abs(y - y_ref) <= 1e-5 * scale)
    tol = 1e-5
    res = E.power_method(D, E.SolverOptions(300, tol), x)
    ref = O.power_dense(A, x, 300, tol, want_trace=True)
    assert abs(res.eigenvalue - ref["eigenvalue"]) <= 1e-5 * (1 + abs(ref["eigenvalue"]))
    assert abs(abs(np.vdot(res.eigenvector.astype(np.complex128), ref["eigenvector"].astype(np.complex128))) - 1) <= 1e-5


def test_single_shifted_inverse_triangular(ctx):
    n = 100_000
    rp, ci, v, d = S.triu_complex(n, 16)
    v = v.astype(np.complex64)
    target = 1.5 * np.exp(0.7j)
    sigma = np.complex64(target + 1e-3)
    T = E.CsrMatrix(ctx, rp, ci, v, (n, n))
    x0 = S.start_vector(n, np.complex64)
    tol = 1e-6
    res = E.shifted_inverse_power_method(T, E.ShiftedSolverOptions(100, tol, sigma), x0)
    assert res.converged
    assert abs(res.eigenvalue - target) <= 1e-5, res.eigenvalue
    ref = O.shifted_triu_csr(rp, ci, v, sigma, x0, 100, tol)
    assert abs(res.eigenvalue - ref["eigenvalue"]) <= 1e-5
    assert abs(abs(np.vdot(res.eigenvector.astype(np.complex128), ref["eigenvector"].astype(np.complex128))) - 1) <= 1e-4
    # solve_shifted on the same triangular matrix: residual in single precision
    b = S.start_vector(n, np.complex64, seed=9)
    xs = E.solve_shifted(T, sigma, b)
    assert xs.dtype == np.complex64
    M = sp.csr_matrix((v.astype(np.complex128), ci, rp), shape=(n, n))
    r = M @ xs.astype(np.complex128) - complex(sigma) * xs.astype(np.complex128) - b
    assert np.linalg.norm(r) <= 1e-4 * np.linalg.norm(b)


def test_single_algorithmic_bytes_and_band_solve(ctx):
    n = 50000
    rp, ci, v = S.band(n, 10)
    A = E.CsrMatrix(ctx, rp, ci, v.astype(np.float32), (n, n))
    s = E.PowerSession(A)
    info = s.kernel_info()
    nnz = len(ci)
    # SURVEY §8d accounting with 4-byte values: (4 + 4) nnz + 4 (n + 1) + 2 * 4 n
    assert info["bytes_per_iteration"] == 8 * nnz + 4 * (n + 1) + 8 * n
    s.close()
    # a general (non-triangular) single-precision sparse shifted solve past n = 16384: the GMRES family
    # (here the exact no-pivot LU) on the values widened to double, the solution rounded to float
    # (solve_shifted.hpp:85-117's SparseLU branch); backward error at single precision
    b = S.start_vector(n, np.float32, seed=3)
    y = E.solve_shifted(A, np.float32(0.5), b)
    assert y.dtype == np.float32
    M = sp.csr_matrix((v.astype(np.float64), ci, rp), shape=(n, n)) - 0.5 * sp.identity(n)
    r = M @ y.astype(np.float64) - b
    assert np.linalg.norm(r) <= 1e-4 * spla.norm(M) * np.linalg.norm(y)


def _planted_dense(n, dtype, seed):
    rng = np.random.default_rng(seed)
    Q, _ = np.linalg.qr(rng.standard_normal((n, n)))
    d = np.linspace(1.0, 4.0, n)
    d[np.abs(d - 2.5) < 0.05] = 1.0
    d[0] = 2.5
    return ((Q * d) @ Q.T).astype(dtype)


@pytest.mark.parametrize("dtype", SINGLE)
@pytest.mark.parametrize("n", [700, 1536])
def test_single_dense_shifted_native(ctx, dtype, n):
    """Dense shifted inverse and solve_shifted in single precision: the LU factor and the solves in
    float (rank-64 / rank-32 trailing updates on v_mfma_f32_16x16x4_f32), n = 700 on the
    one-workgroup substitution, 1536 on the multi-CU one; planted eigenvalue 2.5 (isolated by 0.05)
    within 1e-4, x in the scalar's own type, solve backward error at single precision."""
    A = _planted_dense(n, dtype, n)
    sigma = dtype(2.5 + 1e-2)
    D = E.DenseMatrix(ctx, A)
    r = E.shifted_inverse_power_method(D, E.ShiftedSolverOptions(200, 1e-6, sigma))
    assert r.converged and abs(r.eigenvalue - 2.5) <= 1e-4, r.eigenvalue
    assert np.asarray(r.eigenvector).dtype == dtype
    b = S.start_vector(n, dtype, seed=4)
    y = E.solve_shifted(D, sigma, b)
    D.close()
    assert y.dtype == dtype
    M = A.astype(np.complex128) - complex(sigma) * np.eye(n)
    res = M @ y.astype(np.complex128) - b.astype(np.complex128)
    assert np.linalg.norm(res) <= 1e-4 * np.linalg.norm(M, 2) * np.linalg.norm(y)


def test_single_general_sparse_shifted_band(ctx):
    """complex<float> general sparse shifted inverse on the permuted convection-diffusion matrix
    (nx = 40, n = 1600): the direct GMRES family on the values widened to double (the default from
    n = 1024; the RCM band LU in single precision with EIGSOL_SPARSE_SOLVER=band, the second run), the
    eigenvalue nearest the shift (numpy, fp64) within 1e-4 relative."""
    rp, ci, v = S.convdiff_complex(40)
    n = len(rp) - 1
    Md = sp.csr_matrix((v, ci, rp), shape=(n, n)).toarray()
    ev = np.linalg.eigvals(Md)
    k = n // 3
    order = np.argsort(ev.real)
    lam = ev[order[k]]
    gap = np.min(np.abs(np.delete(ev, order[k]) - lam))
    sigma = np.complex64(lam + 0.1 * gap)
    A = E.CsrMatrix(ctx, rp, ci, v.astype(np.complex64), (n, n))
    for band in (False, True):
        if band:
            os.environ["EIGSOL_SPARSE_SOLVER"] = "band"
        try:
            r = E.shifted_inverse_power_method(A, E.ShiftedSolverOptions(300, 1e-6, sigma),
                                               S.start_vector(n, np.complex64))
        finally:
            os.environ.pop("EIGSOL_SPARSE_SOLVER", None)
        assert r.converged and abs(r.eigenvalue - lam) <= 1e-4 * (1 + abs(lam)), (band, r.eigenvalue, lam)
        assert np.asarray(r.eigenvector).dtype == np.complex64


@pytest.mark.parametrize("dtype", SINGLE)
def test_single_hessenberg_and_qr_decompose_native(ctx, dtype):
    """to_hessenberg / qr_decompose in the scalar's own precision (the blocked compact-WY kernels
    instantiated for float and complex<float>: f32 panels, VALU panel GEMMs, rank-2nb updates on
    v_mfma_f32_16x16x4_f32) against the fp64 restatement of the reference's loops
    (to_hessenberg.hpp:38-77, qr_decompose.hpp:46-85): |H| within 2e-5 ||A||, zero below the
    subdiagonal; Q R = A and Q^H Q = I at single precision.  The reference's reflector takes its
    sign / phase from x0, and where |x0| / ||x|| is below the single-precision rounding (column 89
    of this matrix: 3.4e-7) float and double legitimately choose opposite reflectors, so H is
    checked as H_f32 = D H_f64 D^H entrywise, with the diagonal unitary D (D_0 = 1, +-1 for real
    matrices) recovered from the subdiagonal phases."""
    rng = np.random.default_rng(77)
    n = 200
    A = rng.standard_normal((n, n))
    if np.issubdtype(dtype, np.complexfloating):
        A = A + 1j * rng.standard_normal((n, n))
    A = A.astype(dtype)
    H = E.to_hessenberg(ctx, A)
    assert H.dtype == dtype
    sc = np.linalg.norm(A.astype(np.complex128))
    Hr = O.hessenberg(A.astype(np.complex128 if np.iscomplexobj(A) else np.float64))
    Hd, Hrc = H.astype(np.complex128), Hr.astype(np.complex128)
    d = np.ones(n, np.complex128)
    for i in range(n - 1):   # h(i+1, i) = d(i+1) h_ref(i+1, i) conj(d(i))
        a, b = Hd[i + 1, i], Hrc[i + 1, i]
        d[i + 1] = d[i] * (a / abs(a)) / (b / abs(b))
    if not np.iscomplexobj(A):
        assert np.all(np.abs(np.abs(d.real) - 1) <= 1e-6) and np.all(np.abs(d.imag) <= 1e-6)
        d = np.sign(d.real)
    assert np.abs(d[:, None] * Hrc * np.conj(d)[None, :] - Hd).max() <= 2e-5 * sc
    assert np.abs(np.tril(H, -2)).max() == 0.0
    B = A[:, :150]
    Q, R = E.qr_decompose(ctx, B)
    assert Q.dtype == dtype and R.dtype == dtype
    Qd, Rd = Q.astype(np.complex128), R.astype(np.complex128)
    assert np.abs(Qd @ Rd - B).max() <= 2e-5 * sc
    assert np.abs(Qd.conj().T @ Qd - np.eye(n)).max() <= 2e-5 * n
    assert np.abs(np.tril(R, -1)).max() == 0.0


@pytest.mark.parametrize("dtype", SINGLE)
def test_single_qr_eigenvalues(ctx, dtype):
    """qr_eigenvalues<float / complex<float>>: the reference's unshifted iteration natively in float
    (qr_eigenvalues.hpp:62-105) on the reference test's 2 x 2 (eigenvalues 3 and 1), and the default
    Francis path (fp64 sweeps on the promoted matrix, eigenvalues rounded to the scalar type) on a
    120 x 120 matrix, matched to LAPACK within 1e-5 ||A||."""
    A = np.array([[2.0, 1.0], [1.0, 2.0]], dtype=dtype)
    r = E.qr_eigenvalues(ctx, A, E.SolverOptions(1000, 1e-6), variant="unshifted")
    assert r.converged and 1 <= r.iterations <= 1000
    assert r.eigenvalues.dtype == dtype
    ev = np.sort(np.asarray(r.eigenvalues).real)
    assert abs(ev[0] - 1) <= 1e-5 and abs(ev[1] - 3) <= 1e-5
    rng = np.random.default_rng(8)
    B = rng.standard_normal((120, 120))
    if np.issubdtype(dtype, np.complexfloating):
        B = B + 1j * rng.standard_normal((120, 120))
    B = B.astype(dtype)
    r = E.qr_eigenvalues(ctx, B, E.SolverOptions(1000, 1e-6))
    assert r.converged and r.eigenvalues.dtype == dtype
    ref = np.linalg.eigvals(B.astype(np.complex128))
    got = np.asarray(r.eigenvalues_complex, np.complex128)
    d = np.abs(got[:, None] - ref[None, :]).min(axis=1)
    assert d.max() <= 1e-5 * np.linalg.norm(B.astype(np.complex128))


@pytest.mark.parametrize("dtype", SINGLE)
@pytest.mark.parametrize("kind", ["band", "uniform"])
def test_single_power_distance_to_both_float_semantics(ctx, dtype, kind):
    """The device's float / complex<float> power method against BOTH oracle variants: the default
    (norm and dot accumulated in double, rounded) and O.single_accumulation() (one sequential sum in
    the scalar type: the reference's float Eigen instantiation, power_method.hpp:72,81; pinned
    bitwise to a numpy float32 restatement in tests/test_oracle_golden.py).  The two variants differ
    by ~1e-6 relative here; the device must be within 1e-5 (1 + |lambda|) of each with the same
    iteration count (+-1), |x^H x_ref| >= 1 - 1e-5.  The distances are appended to
    gpurun_out/single_accum_distances.jsonl as evidence."""
    import json
    import os
    n = 40000
    rp, ci, v = S.band(n, 10) if kind == "band" else S.uniform(n, 16)
    v = _with_imag(v, dtype)
    A = E.CsrMatrix(ctx, rp, ci, v, (n, n))
    x0 = S.start_vector(n, dtype)
    tol = 1e-5
    res = E.power_method(A, E.SolverOptions(500, tol), x0)
    A.close()
    cp, ri, vv = O.csr_to_csc(rp, ci, v, n)
    ref_d = O.power_csc(cp, ri, vv, x0, 500, tol)
    with O.single_accumulation():
        ref_f = O.power_csc(cp, ri, vv, x0, 500, tol)
    lam = complex(res.eigenvalue)
    rec = {"kind": kind, "dtype": np.dtype(dtype).name, "device": [lam.real, lam.imag], "iterations": res.iterations}
    xd = res.eigenvector.astype(np.complex128)
    for name, ref in (("double_acc", ref_d), ("float_acc", ref_f)):
        lr = complex(ref["eigenvalue"])
        dist = abs(lam - lr) / (1 + abs(lr))
        rec[name] = {"rel_dist": dist, "iterations": ref["iterations"]}
        assert dist <= 1e-5, (name, lam, lr)
        assert abs(res.iterations - ref["iterations"]) <= 1, (name, res.iterations, ref["iterations"])
        assert abs(abs(np.vdot(xd, ref["eigenvector"].astype(np.complex128))) - 1) <= 1e-5
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
    if os.path.isdir(out):
        with open(os.path.join(out, "single_accum_distances.jsonl"), "a") as f:
            f.write(json.dumps(rec) + "\n")

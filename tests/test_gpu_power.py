"""GPU parity of the fused power iteration (C ABI -> gfx950 kernels) against the CPU oracle.

Reference: powerMethod<S> / powerMethodImpl (src/power_method/power_method.hpp:47-148) and the
known-answer tests of test/power_method_test.cpp.  The oracle (oracle/eigsol_oracle.cpp) runs the
reference's algorithm (two products per iteration, CSC scatter) from the SAME x0.

Tolerances:
  * SpMV rows of at most one LDS tile: bitwise equal to the reference's CSC scatter;
  * eigenvalue: |lam_gpu - lam_cpu| <= 1e-10 * (1 + |lam_cpu|) (north_star: within 1e-10);
  * iterations equal (±1 only if the stopping test is borderline: |dlam| within 10x tol);
  * eigenvector phase-invariant: |x_gpu^H x_cpu| >= 1 - 1e-10.
"""
import numpy as np
import pytest
import scipy.sparse as sp

import pcsc_eigenvalue_solver_project_amd as E
from pcsc_eigenvalue_solver_project_amd import synthetic as S
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _dev_vec(ctx, x):
    p = ctx.malloc(x.nbytes)
    ctx.h2d(p, x)
    return p


def _spmv_gpu(ctx, A, x):
    xd = _dev_vec(ctx, x)
    yd = ctx.malloc(A.shape[0] * x.itemsize)
    try:
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
    lens[rng.integers(0, n, 5)] = 0          # empty rows
    for r, L in long_rows:
        lens[r] = L
    rows, cols = [], []
    for i, L in enumerate(lens):
        c = np.sort(rng.choice(n, size=min(L, n), replace=False))
        rows.append(np.full(len(c), i))
        cols.append(c)
    rows = np.concatenate(rows)
    cols = np.concatenate(cols)
    vals = rng.uniform(-1, 1, len(rows))
    if dtype == np.complex128:
        vals = vals + 1j * rng.uniform(-1, 1, len(rows))
    return sp.csr_matrix((vals, (rows, cols)), shape=(n, n))


@pytest.mark.parametrize("dtype", [np.float64, np.complex128])
@pytest.mark.parametrize("kind", ["band", "uniform", "ragged"])
def test_spmv_bitwise_vs_reference_scatter(ctx, dtype, kind):
    n = 20000
    if kind == "band":
        rp, ci, v = S.band(n, 10)
    elif kind == "uniform":
        rp, ci, v = S.uniform(n, 16)
    else:
        M = _ragged(n, 3, dtype)
        rp, ci, v = M.indptr, M.indices, M.data
    v = v.astype(dtype)
    if dtype == np.complex128 and kind != "ragged":
        v = v + 1j * np.random.default_rng(1).uniform(-1, 1, len(v))
    A = E.CsrMatrix(ctx, rp, ci, v, (n, n))
    x = S.start_vector(n, dtype)
    y = _spmv_gpu(ctx, A, x)
    cp, ri, vv = O.csr_to_csc(rp, ci, v, n)
    y_ref = O.spmv_csc(cp, ri, vv, x, n)
    assert np.array_equal(y, y_ref), np.max(np.abs(y - y_ref))


@pytest.mark.parametrize("dtype", [np.float64, np.complex128])
def test_spmv_long_rows_and_csc_input(ctx, dtype):
    n = 30000
    M = _ragged(n, 5, dtype, max_len=12, long_rows=[(7, 9000), (n // 2, 25000), (n - 1, 4097)])
    Acsc = M.tocsc()
    Acsc.sort_indices()
    A = E.CsrMatrix.from_scipy(ctx, Acsc)          # Eigen canonical CSC layout in
    x = S.start_vector(n, dtype)
    y = _spmv_gpu(ctx, A, x)
    y_ref = O.spmv_csc(Acsc.indptr, Acsc.indices, Acsc.data, x, n)
    short = np.diff(M.indptr) <= 1024        # rows inside one LDS tile (both dtypes)
    assert np.array_equal(y[short], y_ref[short])
    scale = np.abs(M).dot(np.abs(x))
    assert np.all(np.abs(y - y_ref) <= 1e-13 * (scale + 1e-300))


def _assert_power_parity(res, ref, tol):
    lam, lam_ref = res.eigenvalue, ref["eigenvalue"]
    assert abs(lam - lam_ref) <= 1e-10 * (1 + abs(lam_ref)), (lam, lam_ref)
    assert res.converged == ref["converged"]
    if res.iterations != ref["iterations"]:
        assert abs(res.iterations - ref["iterations"]) == 1
        tr = ref["trace"]
        k = min(res.iterations, ref["iterations"]) - 1
        assert abs(tr[k] - tr[k - 1]) <= 10 * tol * (1 + abs(tr[k]))
    x, xr = res.eigenvector, ref["eigenvector"]
    assert abs(np.vdot(x, xr)) >= 1 - 1e-10
    assert abs(np.linalg.norm(x) - 1) <= 1e-12


@pytest.mark.parametrize("dtype", [np.float64, np.complex128])
@pytest.mark.parametrize("kind", ["band", "uniform"])
def test_power_csr_parity(ctx, dtype, kind):
    n = 50000
    rp, ci, v = S.band(n, 10) if kind == "band" else S.uniform(n, 16)
    v = v.astype(dtype)
    A = E.CsrMatrix(ctx, rp, ci, v, (n, n))
    x0 = S.start_vector(n, dtype)
    tol = 1e-12
    res = E.power_method(A, E.SolverOptions(1000, tol), x0)
    cp, ri, vv = O.csr_to_csc(rp, ci, v, n)
    ref = O.power_csc(cp, ri, vv, x0, 1000, tol, want_trace=True)
    assert ref["converged"]
    _assert_power_parity(res, ref, tol)


def test_power_trace_matches_reference_sequence(ctx):
    n = 20000
    rp, ci, v = S.band(n, 10)
    A = E.CsrMatrix(ctx, rp, ci, v, (n, n))
    x0 = S.start_vector(n)
    s = E.PowerSession(A, trace_capacity=64)
    s.begin(E.SolverOptions(30, -1.0), x0)      # tol < 0: never converges -> exactly 30 iterations
    s.step(40)
    done, launches = s.query()
    assert done and launches == 32
    res = s.finish()
    assert res.iterations == 30 and not res.converged
    tr = s.trace(64)
    cp, ri, vv = O.csr_to_csc(rp, ci, v, n)
    ref = O.power_csc(cp, ri, vv, x0, 30, -1.0, want_trace=True)
    assert len(tr) == 30
    # early Rayleigh quotients are tiny (cancellation): scale the bound by the converged value
    np.testing.assert_allclose(tr, ref["trace"], rtol=1e-13, atol=1e-13 * np.max(np.abs(ref["trace"])))
    assert abs(res.eigenvalue - ref["eigenvalue"]) <= 1e-13 * abs(ref["eigenvalue"])


@pytest.mark.parametrize("dtype", [np.float64, np.complex128])
def test_power_dense_parity(ctx, dtype):
    rng = np.random.default_rng(11)
    n = 700
    Amat = rng.uniform(0, 1, (n, n))
    if dtype == np.complex128:
        Amat = Amat + 0.1j * rng.uniform(-1, 1, (n, n))
    A = E.DenseMatrix(ctx, Amat)
    x0 = S.start_vector(n, dtype)
    res = E.power_method(A, E.SolverOptions(1000, 1e-12), x0)
    ref = O.power_dense(Amat, x0, 1000, 1e-12, want_trace=True)
    _assert_power_parity(res, ref, 1e-12)


def test_dense_gemv_vs_oracle(ctx):
    rng = np.random.default_rng(2)
    for (m, n) in [(1000, 1000), (257, 63), (1, 5), (3001, 17)]:
        Amat = rng.standard_normal((m, n))
        A = E.DenseMatrix(ctx, Amat)
        x = rng.standard_normal(n)
        xd = _dev_vec(ctx, x)
        yd = ctx.malloc(m * 8)
        A.gemv(xd, yd)
        y = ctx.d2h(np.empty(m), yd)
        ctx.free(xd); ctx.free(yd)
        ref = O.gemv(Amat, x)
        assert np.all(np.abs(y - ref) <= 1e-13 * (np.abs(Amat) @ np.abs(x)))


# --------------------------------------------------------- reference known-answer tests (C ABI)
def test_kat_dense_simple_matrix(ctx):
    # power_method_test.cpp:38-57  diag(2,1) -> 2, converged, eigenpair residual 1e-5
    Amat = np.array([[2.0, 0.0], [0.0, 1.0]])
    res = E.power_method(E.DenseMatrix(ctx, Amat), E.SolverOptions(1000, 1e-10), np.array([0.3, 0.7]))
    assert res.converged and res.iterations > 0
    assert abs(res.eigenvalue - 2.0) <= 1e-5 * (1 + 2.0)
    lhs, rhs = Amat @ res.eigenvector, res.eigenvalue * res.eigenvector
    assert np.all(np.abs(lhs - rhs) <= 1e-5 * (1 + np.abs(rhs)))


def test_kat_sparse_matrix(ctx):
    # power_method_test.cpp:62-83  [[3,1],[0,2]] sparse -> 3 (rel 1e-6, tol 1e-8)
    Ad = np.array([[3.0, 1.0], [0.0, 2.0]])
    A = E.CsrMatrix.from_scipy(ctx, sp.csc_matrix(Ad))
    res = E.power_method(A, E.SolverOptions(1000, 1e-8), np.array([0.5, -0.25]))
    assert res.converged and res.iterations > 0
    assert abs(res.eigenvalue - 3.0) <= 1e-6 * (1 + 3.0)


def test_kat_few_iterations(ctx):
    # power_method_test.cpp:103-119  maxIterations = 1 -> iterations == 1
    Amat = np.array([[5.0, 1.0], [1.0, 4.0]])
    res = E.power_method(E.DenseMatrix(ctx, Amat), E.SolverOptions(1, 1e-12), np.array([1.0, 0.2]))
    assert res.iterations == 1 and not res.converged
    ref = O.power_dense(Amat, np.array([1.0, 0.2]), 1, 1e-12)
    assert abs(res.eigenvalue - ref["eigenvalue"]) <= 1e-14 * abs(ref["eigenvalue"])


def test_kat_errors(ctx):
    # power_method_test.cpp:88-98 (non-square) and :124-134 (zero size)
    with pytest.raises(E.EigSolError) as e:
        E.PowerSession(E.DenseMatrix(ctx, np.zeros((2, 3))))
    assert e.value.status == 1 and "must be square" in str(e.value)
    with pytest.raises(E.EigSolError) as e:
        E.PowerSession(E.DenseMatrix(ctx, np.zeros((0, 0))))
    assert e.value.status == 2 and "zero size" in str(e.value)


def test_edge_zero_matrix_and_zero_start(ctx):
    # normY == 0 at k = 0 -> iterations = 1, lambda = 0, x = normalised x0 (power_method.hpp:73-76)
    n = 300
    A = E.CsrMatrix(ctx, np.zeros(n + 1, np.int32), np.zeros(0, np.int32), np.zeros(0), (n, n))
    x0 = S.start_vector(n)
    res = E.power_method(A, E.SolverOptions(100, 1e-10), x0)
    assert res.iterations == 1 and not res.converged and res.eigenvalue == 0.0
    np.testing.assert_allclose(res.eigenvector, x0 / np.sqrt(np.sum(x0 * x0)), rtol=1e-15, atol=0)
    # x0 == 0 is kept unnormalised by Eigen's normalize(); y = 0 -> same exit
    rp, ci, v = S.band(n, 5)
    B = E.CsrMatrix(ctx, rp, ci, v, (n, n))
    res = E.power_method(B, E.SolverOptions(100, 1e-10), np.zeros(n))
    assert res.iterations == 1 and res.eigenvalue == 0.0 and not np.any(res.eigenvector)


def test_edge_max_iterations_zero(ctx):
    n = 300
    rp, ci, v = S.band(n, 5)
    A = E.CsrMatrix(ctx, rp, ci, v, (n, n))
    x0 = S.start_vector(n)
    res = E.power_method(A, E.SolverOptions(0, 1e-10), x0)
    assert res.iterations == 0 and not res.converged and res.eigenvalue == 0.0
    np.testing.assert_allclose(res.eigenvector, x0 / np.sqrt(np.sum(x0 * x0)), rtol=1e-15, atol=0)


def test_data_A_txt_as_double(ctx):
    # config 1: data/A.txt read as double -> [[1,3,3],[5,1,4],[0,0,2]], lambda = 1 + sqrt(15)
    Amat = np.array([[1.0, 3.0, 3.0], [5.0, 1.0, 4.0], [0.0, 0.0, 2.0]])
    x0 = np.array([0.25, -0.5, 0.75])
    res = E.power_method(E.DenseMatrix(ctx, Amat), E.SolverOptions(1000, 1e-10), x0)
    ref = O.power_dense(Amat, x0, 1000, 1e-10, want_trace=True)
    _assert_power_parity(res, ref, 1e-10)
    assert abs(res.eigenvalue - (1 + np.sqrt(15))) < 1e-8


def _slice_mix(n, dtype, seed=21):
    """Rows shaped to exercise every case of the sliced layout: uniform band slices (8-bit window
    offsets), a slice of empty rows, a slice with columns spread over the whole matrix (gather
    slice), ragged slices with a few short rows, and one slice holding a 60-entry row (row
    longer than the entries a lane keeps in registers)."""
    rng = np.random.default_rng(seed)
    rows, cols = [], []
    for i in range(n):
        s = i // 64
        if s == 10:
            continue                                          # an all-empty slice
        if s == 20:
            c = np.sort(rng.choice(n, size=10, replace=False))  # wide window: gather slice
        elif s == 30 and i % 64 == 5:
            lo = max(0, min(i - 100, n - 200))
            c = np.sort(rng.choice(np.arange(lo, lo + 200), size=60, replace=False))
        else:
            k = 10 if (s % 7 != 3 or i % 5) else 7               # ragged slices: some 7-entry rows
            lo = max(0, min(i - 40, n - 81))
            c = np.sort(rng.choice(np.arange(lo, lo + 81), size=k, replace=False))
        rows.append(np.full(len(c), i))
        cols.append(c)
    rows = np.concatenate(rows)
    cols = np.concatenate(cols)
    vals = rng.uniform(-1, 1, len(rows))
    if dtype == np.complex128:
        vals = vals + 1j * rng.uniform(-1, 1, len(rows))
    M = sp.csr_matrix((vals, (rows, cols)), shape=(n, n)).tolil()
    M[n // 2, n // 2] = 10.0                                  # a dominant eigenvalue near 10
    M = M.tocsr()
    M.sort_indices()
    return M


@pytest.mark.parametrize("dtype", [np.float64, np.complex128])
def test_slice_layout_mix_bitwise_and_power(ctx, dtype):
    n = 64 * 40 + 17                                          # a partial last slice
    M = _slice_mix(n, dtype)
    A = E.CsrMatrix.from_scipy(ctx, M)
    x = S.start_vector(n, dtype)
    y = _spmv_gpu(ctx, A, x)
    cp, ri, vv = O.csr_to_csc(M.indptr, M.indices, M.data, n)
    y_ref = O.spmv_csc(cp, ri, vv, x, n)
    assert np.array_equal(y, y_ref), np.max(np.abs(y - y_ref))
    sess = E.PowerSession(A)
    assert sess.kernel_info()["variant"] == 5                # the sliced kernel ran
    sess.close()
    tol = 1e-12
    res = E.power_method(A, E.SolverOptions(3000, tol), x)
    ref = O.power_csc(cp, ri, vv, x, 3000, tol, want_trace=True)
    _assert_power_parity(res, ref, tol)


@pytest.mark.parametrize("shape", [(300, 200), (200, 301)])
def test_spmv_rectangular_sliced(ctx, shape):
    """Plain SpMV of a rectangular matrix (x shorter or longer than y) in the sliced layout: row
    sums in ascending column order, bitwise."""
    m, n = shape
    rng = np.random.default_rng(8)
    rows, cols = [], []
    for i in range(m):
        lo = min(max(0, i * n // m - 20), n - 41)
        c = np.sort(rng.choice(np.arange(lo, lo + 41), size=8, replace=False))
        rows.append(np.full(8, i))
        cols.append(c)
    M = sp.csr_matrix((rng.uniform(-1, 1, 8 * m), (np.concatenate(rows), np.concatenate(cols))), shape=(m, n))
    M.sort_indices()
    A = E.CsrMatrix.from_scipy(ctx, M)
    x = S.start_vector(n)
    y = _spmv_gpu(ctx, A, x)
    y_ref = np.zeros(m)
    for i in range(m):
        acc = 0.0
        for e in range(M.indptr[i], M.indptr[i + 1]):
            acc += M.data[e] * x[M.indices[e]]
        y_ref[i] = acc
    assert np.array_equal(y, y_ref)


@pytest.mark.parametrize("dtype", [np.float64, np.complex128])
def test_slice_stream_segments_bitwise_and_power(ctx, dtype, monkeypatch):
    """Slice streams cut into several segments (EIGSOL_SLICE_SEG_BYTES forces 4 MiB segments: 4 to 13 of them here; the
    default limit is 4 GiB): every product bitwise equal to the CSC scatter, and the power
    iteration identical to the one-segment layout (same λ bits, same iterate)."""
    n = 200_000
    rp, ci, v = S.band(n, 10)
    rp2, ci2, v2 = S.uniform(n, 16, seed=5)
    v, v2 = v.astype(dtype), v2.astype(dtype)
    x0 = S.start_vector(n, dtype)
    opts = E.SolverOptions(300, 1e-12)
    ref = {}
    for key, (a, b, c) in {"band": (rp, ci, v), "uniform": (rp2, ci2, v2)}.items():
        A = E.CsrMatrix(ctx, a, b, c, (n, n))
        ref[key] = E.power_method(A, opts, x0)
        A.close()
    monkeypatch.setenv("EIGSOL_SLICE_SEG_BYTES", str(1 << 22))
    for key, (a, b, c) in {"band": (rp, ci, v), "uniform": (rp2, ci2, v2)}.items():
        A = E.CsrMatrix(ctx, a, b, c, (n, n))
        s = E.PowerSession(A)
        assert s.kernel_info()["variant"] == 5
        s.close()
        y = _spmv_gpu(ctx, A, x0)
        cp, ri, vv = O.csr_to_csc(a, b, c, n)
        assert np.array_equal(y, O.spmv_csc(cp, ri, vv, x0, n))
        r = E.power_method(A, opts, x0)
        assert r.iterations == ref[key].iterations and r.eigenvalue == ref[key].eigenvalue
        assert np.array_equal(r.eigenvector, ref[key].eigenvector)
        A.close()


@pytest.mark.parametrize("dtype", [np.float64, np.complex128])
def test_column_blocked_gather_bitwise_and_power(ctx, dtype, monkeypatch):
    """Column-blocked gathers (uniform columns, x larger than an XCD's L2: csr_kernel passes over
    column blocks, each continuing the previous block's row partials): the product is bitwise the
    reference's CSC scatter (power_method.hpp:69, every row still summed in ascending column
    order), and the power iteration keeps the oracle parity of test_power_csr_parity.  Blocks are
    forced on a small matrix (x = 1.6 MB, 512 KB blocks: 4 passes; ~1 % of the rows have no entry
    in a given block)."""
    monkeypatch.setenv("EIGSOL_CSR_CBLK_MIN", "0")
    monkeypatch.setenv("EIGSOL_CSR_CBLK", "2")
    monkeypatch.setenv("EIGSOL_CSR_CBLK_BYTES", str(512 * 1024))
    n = 200_000
    rp, ci, v = S.uniform(n, 16)
    v = v.astype(dtype)
    if dtype == np.complex128:
        v = v + 1j * np.random.default_rng(1).uniform(-1, 1, len(v))
    A = E.CsrMatrix(ctx, rp, ci, v, (n, n))
    s = E.PowerSession(A)
    info = s.kernel_info()
    s.close()
    assert info["variant"] == 9 and info["tiles"] >= 2, info
    x = S.start_vector(n, dtype)
    y = _spmv_gpu(ctx, A, x)
    cp, ri, vv = O.csr_to_csc(rp, ci, v, n)
    assert np.array_equal(y, O.spmv_csc(cp, ri, vv, x, n))
    tol = 1e-12
    res = E.power_method(A, E.SolverOptions(1000, tol), x)
    ref = O.power_csc(cp, ri, vv, x, 1000, tol, want_trace=True)
    assert ref["converged"]
    _assert_power_parity(res, ref, tol)
    A.close()


@pytest.mark.parametrize("dtype", [np.float64, np.complex128, np.float32, np.complex64])
def test_column_binned_gather_bitwise_and_power(ctx, dtype, monkeypatch):
    """Column-binned gathers (csr_bin_kernel: row chunks whose sums live in LDS, entries ordered by
    column block, then level, then row): the product is bitwise the reference's CSC scatter
    (power_method.hpp:69; every row summed in ascending column order across levels and blocks)
    and the power iteration keeps the oracle parity of test_power_csr_parity.  Forced on a small
    matrix with 64 KB blocks (many blocks, several levels per block), plus a dense row (2000
    entries: thousands of one-entry levels) and empty rows."""
    monkeypatch.setenv("EIGSOL_CSR_BIN", "2")
    monkeypatch.setenv("EIGSOL_CSR_BIN_BYTES", str(64 * 1024))
    n = 150_000
    rp, ci, v = S.uniform(n, 16)
    # row 7: 2000 ascending columns; rows 100..199: empty
    lens = np.diff(rp).astype(np.int64)
    rows = [ci[rp[i]:rp[i + 1]] for i in range(n)]
    vals = [v[rp[i]:rp[i + 1]] for i in range(n)]
    rng = np.random.default_rng(11)
    rows[7] = np.sort(rng.choice(n, 2000, replace=False)).astype(np.int32)
    vals[7] = rng.uniform(-1, 1, 2000)
    for i in range(100, 200):
        rows[i] = rows[i][:0]
        vals[i] = vals[i][:0]
    lens = np.array([len(r) for r in rows], dtype=np.int64)
    rp = np.zeros(n + 1, dtype=np.int32)
    np.cumsum(lens, out=rp[1:])
    ci = np.concatenate(rows).astype(np.int32)
    v = np.concatenate(vals).astype(dtype)
    if np.issubdtype(dtype, np.complexfloating):
        v = (v + 1j * np.random.default_rng(1).uniform(-1, 1, len(v))).astype(dtype)
    A = E.CsrMatrix(ctx, rp, ci, v, (n, n))
    s = E.PowerSession(A)
    info = s.kernel_info()
    s.close()
    assert info["variant"] == 10 and info["tiles"] >= 2, info
    x = S.start_vector(n, dtype)
    y = _spmv_gpu(ctx, A, x)
    cp, ri, vv = O.csr_to_csc(rp, ci, v, n)
    assert np.array_equal(y, O.spmv_csc(cp, ri, vv, x, n))
    single = dtype in (np.float32, np.complex64)
    tol = 1e-5 if single else 1e-12
    res = E.power_method(A, E.SolverOptions(1000, tol), x)
    ref = O.power_csc(cp, ri, vv, x, 1000, tol, want_trace=True)
    assert ref["converged"]
    if single:
        assert abs(res.eigenvalue - ref["eigenvalue"]) <= 1e-5 * (1 + abs(ref["eigenvalue"]))
        assert abs(res.iterations - ref["iterations"]) <= 1
    else:
        _assert_power_parity(res, ref, tol)
    A.close()
    # rectangular product (2n columns): rows chunked by n, columns blocked over 2n
    _rect_binned(ctx, dtype, n)


@pytest.mark.parametrize("lds", [64, 128, 153])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_column_binned_lds_instantiations(ctx, dtype, lds, monkeypatch):
    """The large-LDS instantiations of csr_bin_kernel (64 / 128 / 153 KB of row sums per workgroup,
    the last one the default for matrices whose row sums exceed 64 MB, i.e. config 4's
    uniform10m) forced on a small matrix with balanced chunks (chunk rows chosen so the chunk
    count is a multiple of the grid), an empty row range, a 3000-entry row and a row longer than
    one x block: bitwise the reference's CSC scatter (power_method.hpp:69,81) and power parity."""
    monkeypatch.setenv("EIGSOL_CSR_BIN", "2")
    monkeypatch.setenv("EIGSOL_CSR_BIN_LDS", str(lds))
    monkeypatch.setenv("EIGSOL_CSR_BIN_BALANCE", "1")
    monkeypatch.setenv("EIGSOL_CSR_BIN_BYTES", str(256 * 1024))
    n = 400_000
    rp, ci, v = S.uniform(n, 10, seed=5)
    rows = [ci[rp[i]:rp[i + 1]] for i in range(n)]
    vals = [v[rp[i]:rp[i + 1]] for i in range(n)]
    rng = np.random.default_rng(17)
    rows[3] = np.sort(rng.choice(n, 3000, replace=False)).astype(np.int32)
    vals[3] = rng.uniform(0, 1, 3000)
    rows[n - 1] = np.arange(0, n, 40, dtype=np.int32)         # spans every x block
    vals[n - 1] = rng.uniform(0, 1, len(rows[n - 1]))
    for i in range(5000, 5100):
        rows[i] = rows[i][:0]
        vals[i] = vals[i][:0]
    lens = np.array([len(r) for r in rows], dtype=np.int64)
    rp = np.zeros(n + 1, dtype=np.int32)
    np.cumsum(lens, out=rp[1:])
    ci = np.concatenate(rows).astype(np.int32)
    v = np.concatenate(vals).astype(dtype)
    A = E.CsrMatrix(ctx, rp, ci, v, (n, n))
    s = E.PowerSession(A)
    info = s.kernel_info()
    kname = s.kernel_name()
    s.close()
    assert info["variant"] == 10, info
    assert f", {lds}, " in kname, kname
    x = S.start_vector(n, dtype)
    y = _spmv_gpu(ctx, A, x)
    cp, ri, vv = O.csr_to_csc(rp, ci, v, n)
    assert np.array_equal(y, O.spmv_csc(cp, ri, vv, x, n))
    single = dtype == np.float32
    tol = 1e-5 if single else 1e-12
    res = E.power_method(A, E.SolverOptions(1000, tol), x)
    ref = O.power_csc(cp, ri, vv, x, 1000, tol, want_trace=True)
    assert ref["converged"]
    if single:
        assert abs(res.eigenvalue - ref["eigenvalue"]) <= 1e-5 * (1 + abs(ref["eigenvalue"]))
        assert abs(res.iterations - ref["iterations"]) <= 1
    else:
        _assert_power_parity(res, ref, tol)
    A.close()


def _rect_binned(ctx, dtype, n):
    rp2, ci2, v2 = S.uniform(n, 12, seed=3)
    ci2 = (ci2.astype(np.int64) * 2 + (np.arange(len(ci2)) & 1)).astype(np.int32)
    v2 = v2.astype(dtype)
    B = E.CsrMatrix(ctx, rp2, ci2, v2, (n, 2 * n))
    xb = S.start_vector(2 * n, dtype)
    cp2, ri2, vv2 = O.csr_to_csc(rp2, ci2, v2, 2 * n)
    assert np.array_equal(_spmv_gpu(ctx, B, xb), O.spmv_csc(cp2, ri2, vv2, xb, n))
    B.close()

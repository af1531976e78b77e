"""Host-only plan of the multifrontal general-sparse solve (multifrontal.hip, C ABI eigsol_mf_analyze):
the nested-dissection ordering of the pattern of A + A^T and its supernodal tree.

Checked on the CPU, no device:
* the ordering is a permutation, the fronts own contiguous column ranges in postorder (every child
  numbered before its parent) and cover all columns;
* the dissection property the multifrontal structure rests on: for every edge (u, v) of A + A^T the
  supernode of one endpoint is the other's or one of its ancestors (so each front's struct lies in
  its ancestors and the children's Schur blocks extend-add into their parents);
* the stored factor holds the exact no-pivot fill of the permuted matrix (eigsol_sparse_lu_fill on
  P (A + A^T) P^T counts no more entries than the fronts' pivot rows and columns store);
* determinism, disconnected pieces and isolated rows, a dense row, argument errors."""
import ctypes as C

import numpy as np
import pytest
import scipy.sparse as sp

from pcsc_eigenvalue_solver_project_amd import synthetic as S
from pcsc_eigenvalue_solver_project_amd._capi import lib


def analyze(rp, ci, n, leaf=16, cx=1):
    rp = np.ascontiguousarray(rp, dtype=np.int32)
    ci = np.ascontiguousarray(ci, dtype=np.int32)
    st = (C.c_double * 8)()
    perm = np.empty(max(n, 1), np.int32)
    assert lib().eigsol_mf_analyze(n, rp.ctypes.data, ci.ctypes.data, leaf, cx, perm.ctypes.data, None, 0, st) == 0
    nf = int(st[0])
    fr = np.empty((max(nf, 1), 4), np.int32)
    assert lib().eigsol_mf_analyze(n, rp.ctypes.data, ci.ctypes.data, leaf, cx, None, fr.ctypes.data, nf, st) == 0
    return list(st), perm[:n], fr[:nf]


def check_plan(rp, ci, n, leaf):
    st, perm, fr = analyze(rp, ci, n, leaf)
    assert st[7] == 1.0
    assert np.array_equal(np.sort(perm), np.arange(n))
    nf = len(fr)
    # contiguous column ranges in front order, covering [0, n)
    assert fr[0, 0] == 0 and np.all(fr[1:, 0] == fr[:-1, 0] + fr[:-1, 1]) and fr[-1, 0] + fr[-1, 1] == n
    assert np.all(fr[:, 1] >= 1)
    par = fr[:, 3]
    assert np.all((par == -1) | (par > np.arange(nf)))      # postorder: parents after children
    assert np.all(fr[par == -1, 2] == 0)                     # a root's struct is empty
    snode = np.repeat(np.arange(nf), fr[:, 1])
    iperm = np.empty(n, np.int64)
    iperm[perm] = np.arange(n)
    # ancestor test by depth-first intervals of the tree
    kids = [[] for _ in range(nf)]
    for s in range(nf):
        if par[s] >= 0:
            kids[par[s]].append(s)
    lo = np.empty(nf, np.int64)
    for s in range(nf):              # postorder: a subtree is the contiguous front range [lo, s]
        lo[s] = min([lo[c] for c in kids[s]], default=s)
    A = sp.csr_matrix((np.ones(len(ci)), ci, rp), shape=(n, n))
    G = (A + A.T).tocoo()
    a, b = snode[iperm[G.row]], snode[iperm[G.col]]
    lo_a, hi_a = np.minimum(a, b), np.maximum(a, b)
    assert np.all(lo[hi_a] <= lo_a), "an edge joins two supernodes neither of which is the other's ancestor"
    # exact no-pivot fill of the permuted symmetric pattern fits the stored factor
    P = sp.csr_matrix((np.ones(n), (np.arange(n), perm)), shape=(n, n))
    B = (P @ ((A + A.T) + sp.identity(n)) @ P.T).tocsr()
    B.sort_indices()
    nnz = C.c_int64(0)
    brp, bci = B.indptr.astype(np.int32), B.indices.astype(np.int32)
    assert lib().eigsol_sparse_lu_fill(n, brp.ctypes.data, bci.ctypes.data, 2**40, C.byref(nnz), None) == 0
    assert nnz.value <= st[4]
    return st, perm, fr


@pytest.mark.parametrize("nx,leaf", [(30, 16), (45, 64), (20, 4), (12, 500)])
def test_convdiff_plan(nx, leaf):
    rp, ci, _ = S.convdiff_complex(nx, seed=3)
    st, perm, fr = check_plan(rp, ci, nx * nx, leaf)
    if leaf >= nx * nx:
        assert st[0] == 1 and st[2] == nx * nx                  # one leaf: one dense front
    else:
        assert st[3] <= 2 * nx + leaf                           # separators ~ the grid side


def test_plan_is_deterministic():
    rp, ci, _ = S.convdiff_complex(40, seed=7)
    a = analyze(rp, ci, 1600)
    b = analyze(rp, ci, 1600)
    assert a[0] == b[0] and np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2])


def test_components_isolated_rows_and_dense_row():
    rp1, ci1, v1 = S.convdiff_complex(20, seed=1)
    rp2, ci2, v2 = S.convdiff_complex(15, seed=2)
    M1 = sp.csr_matrix((v1, ci1, rp1), shape=(400, 400))
    M2 = sp.csr_matrix((v2, ci2, rp2), shape=(225, 225))
    M = sp.block_diag([M1, sp.csr_matrix((7, 7)), M2], format="lil")
    n = M.shape[0]
    rng = np.random.default_rng(5)
    for j in rng.choice(n, 80, replace=False):
        M[3, j] = 1.0
    M = sp.csr_matrix(M)
    M.sort_indices()
    check_plan(M.indptr, M.indices, n, 16)


def test_nonsymmetric_pattern_and_triangular():
    rng = np.random.default_rng(11)
    n = 500
    rows = rng.integers(0, n, 3000)
    cols = np.clip(rows + rng.integers(-30, 5, 3000), 0, n - 1)
    M = sp.csr_matrix((np.ones(3000), (rows, cols)), shape=(n, n))
    M.sum_duplicates()
    M.sort_indices()
    check_plan(M.indptr, M.indices, n, 16)


def test_argument_errors():
    st = (C.c_double * 8)()
    assert lib().eigsol_mf_analyze(-1, None, None, 16, 1, None, None, 0, st) == 9
    rp = np.array([0, 1], np.int32)
    ci = np.array([5], np.int32)
    assert lib().eigsol_mf_analyze(1, rp.ctypes.data, ci.ctypes.data, 16, 1, None, None, 0, st) == 9
    rp2, ci2, _ = S.convdiff_complex(10)
    assert lib().eigsol_mf_analyze(100, rp2.ctypes.data, ci2.ctypes.data, 0, 1, None, None, 0, st) == 9
    fr = np.empty((1, 4), np.int32)
    assert lib().eigsol_mf_analyze(100, rp2.ctypes.data, ci2.ctypes.data, 4, 1, None, fr.ctypes.data, 1, st) == 9


def test_plan_independent_of_host_threads(monkeypatch):
    """The dissection runs on a pool of host threads past n = 20000; the tree is put in a canonical
    order, so the plan is identical for any thread count."""
    rp, ci, _ = S.convdiff_complex(160, seed=9)
    n = 160 * 160
    out = []
    for t in ("1", "3", "8"):
        monkeypatch.setenv("EIGSOL_MF_THREADS", t)
        out.append(analyze(rp, ci, n, leaf=64))
    for st, perm, fr in out[1:]:
        assert st == out[0][0] and np.array_equal(perm, out[0][1]) and np.array_equal(fr, out[0][2])
    check_plan(rp, ci, n, 64)

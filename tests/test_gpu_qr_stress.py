"""GPU: the multishift Francis QR (francis.hip, zfrancis.hip) on matrices that stress its shift
strategy — after round 4's changes to it (the shifts' QR split at 1e-4, LAPACK's KEXSH trigger for
exceptional shifts, 32 bulges per sweep).

Reference semantics: qr_eigenvalues.hpp:40-108 (eigenvalues of a dense matrix; the reference's own
unshifted loop is only the oracle of the small KATs in test_gpu_qr.py).  Ill-conditioned spectra
(Grcar, Frank, companion, perturbed Jordan) cannot be compared entrywise against LAPACK, since
any backward-stable method may move them by cond(λ)·eps·||A||; they are checked through
size-independent properties instead:
  * convergence within the reference's iteration budget;
  * backward error: every computed λ is an eigenvalue of a nearby matrix,
    σ_min(A − λI) <= 1e-11 ||A||_F (a sample of up to 48 eigenvalues);
  * trace: |Σλ − tr A| <= 1e-9 n ||A||_F;
  * real input: the spectrum is closed under conjugation (pairs come out as exact conjugates).
Well-conditioned spectra (random seeds, graded and block-split matrices) are matched one-to-one
against LAPACK (numpy.linalg.eigvals) at 1e-9 ||A||_F as in test_gpu_qr.py.
"""
import numpy as np
import pytest

import pcsc_eigenvalue_solver_project_amd as E

pytestmark = pytest.mark.gpu

OPTS = E.SolverOptions(1000, 1e-10)


def _match(ev, ref, tol):
    ev, ref = np.asarray(ev, complex), np.asarray(ref, complex)
    assert len(ev) == len(ref)
    used = np.zeros(len(ref), bool)
    worst = 0.0
    for z in ev[np.argsort(-np.abs(ev))]:
        d = np.abs(ref - z)
        d[used] = np.inf
        j = int(np.argmin(d))
        used[j] = True
        worst = max(worst, d[j])
    assert worst <= tol, worst


def check_properties(A, ev, real_input, sample=48, seed=0):
    """Backward error, trace and conjugate closure of a computed spectrum (see module docstring)."""
    n = A.shape[0]
    ev = np.asarray(ev, complex)
    assert ev.shape == (n,) and np.all(np.isfinite(ev))
    nf = np.linalg.norm(A)
    assert abs(ev.sum() - np.trace(A)) <= 1e-9 * n * nf, (ev.sum(), np.trace(A))
    pick = np.random.default_rng(seed).choice(n, size=min(sample, n), replace=False)
    I = np.eye(n)
    worst = max(np.linalg.svd(A - z * I, compute_uv=False)[-1] for z in ev[pick])
    assert worst <= 1e-11 * nf, worst / nf
    if real_input:
        cpx = ev[ev.imag != 0]
        assert np.array_equal(np.sort_complex(cpx), np.sort_complex(cpx.conj()))


def grcar(n, k=3):
    return np.eye(n, k=-1) * -1.0 + sum(np.eye(n, k=j) for j in range(k + 1))


def frank(n):
    F = np.zeros((n, n))
    for i in range(n):
        for j in range(n):
            if j >= i - 1:
                F[i, j] = n - max(i, j)
    return F


def companion(c):
    c = np.asarray(c)
    n = len(c)
    C = np.zeros((n, n), dtype=np.result_type(c.dtype, np.float64))
    C[0, :] = -c
    C[1:, :-1] += np.eye(n - 1)
    return C


def graded(n, seed):
    rng = np.random.default_rng(seed)
    d = 2.0 ** (-np.arange(n) / (n / 40))   # 40 binades from the first row to the last
    return (d[:, None] * rng.standard_normal((n, n))) * (1.0 / d[None, :])


@pytest.fixture(scope="module")
def ctx():
    c = E.Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("n", [300, 700])
def test_grcar(ctx, n):
    A = grcar(n)
    r = E.qr_eigenvalues(ctx, A, OPTS)
    assert r.converged
    check_properties(A, r.eigenvalues_complex, True)


def test_frank(ctx):
    A = frank(300)
    r = E.qr_eigenvalues(ctx, A, OPTS)
    assert r.converged
    check_properties(A, r.eigenvalues_complex, True)


@pytest.mark.parametrize("n", [200, 600])
def test_companion_of_random_polynomial(ctx, n):
    c = np.random.default_rng(n).standard_normal(n)
    A = companion(c)
    r = E.qr_eigenvalues(ctx, A, OPTS)
    assert r.converged
    check_properties(A, r.eigenvalues_complex, True)


def test_perturbed_jordan_blocks(ctx):
    """Eight 64-order Jordan blocks (eigenvalues 1..8) under 1e-10 noise: each block's eigenvalues
    spread on a circle of radius ~(1e-10)^(1/64) ≈ 0.7 — defective-limit clustering."""
    n, m = 512, 64
    J = np.zeros((n, n))
    for b in range(n // m):
        s = b * m
        J[s:s + m, s:s + m] = np.eye(m) * (b + 1) + np.eye(m, k=1)
    A = J + 1e-10 * np.random.default_rng(5).standard_normal((n, n))
    r = E.qr_eigenvalues(ctx, A, OPTS)
    assert r.converged
    check_properties(A, r.eigenvalues_complex, True)


def test_integer_zero_one(ctx):
    """0/1 entries: an exactly singular matrix with a large null space (eigenvalue 0 many times)."""
    rng = np.random.default_rng(9)
    B = (rng.random((400, 40)) < 0.5).astype(float)
    A = B @ (rng.random((40, 400)) < 0.5).astype(float)    # rank <= 40
    r = E.qr_eigenvalues(ctx, A, OPTS)
    assert r.converged
    check_properties(A, r.eigenvalues_complex, True)
    ev = r.eigenvalues_complex
    assert np.sum(np.abs(ev) <= 1e-6 * np.linalg.norm(A)) >= 360


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_graded(ctx, seed):
    A = graded(500, seed)
    r = E.qr_eigenvalues(ctx, A, OPTS)
    assert r.converged
    check_properties(A, r.eigenvalues_complex, True)


@pytest.mark.parametrize("n,seed", [(640, 11), (900, 12), (1200, 13), (1536, 14)])
def test_random_seeds_against_lapack(ctx, n, seed):
    rng = np.random.default_rng(seed)
    A = rng.standard_normal((n, n)) if seed % 2 else rng.uniform(-1, 1, (n, n))
    r = E.qr_eigenvalues(ctx, A, OPTS)
    assert r.converged
    _match(r.eigenvalues_complex, np.linalg.eigvals(A), 1e-9 * np.linalg.norm(A))


def test_many_splits(ctx):
    """A Hessenberg matrix whose subdiagonal is zero at 40 random places: many independent
    active blocks, some of order 1 or 2."""
    n = 800
    rng = np.random.default_rng(21)
    H = np.triu(rng.standard_normal((n, n)), -1)
    cut = np.sort(rng.choice(np.arange(1, n), 40, replace=False))
    for c in cut:
        H[c, c - 1] = 0.0
    r = E.qr_eigenvalues(ctx, H, OPTS)
    assert r.converged
    _match(r.eigenvalues_complex, np.linalg.eigvals(H), 1e-9 * np.linalg.norm(H))


@pytest.mark.parametrize("case", ["grcar", "companion", "graded"])
def test_complex_stress(ctx, case):
    rng = np.random.default_rng(77)
    if case == "grcar":
        A = grcar(400).astype(complex) * np.exp(0.3j)
    elif case == "companion":
        A = companion(rng.standard_normal(400) + 1j * rng.standard_normal(400))
    else:
        A = graded(400, 4) + 1j * graded(400, 5)
    r = E.qr_eigenvalues(ctx, A, E.SolverOptions(1000, 1e-12))
    assert r.converged
    check_properties(A, r.eigenvalues_complex, False)

"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes view of ``oracle/build/liboracle.so`` (the CPU restatement of the reference algorithms in
``oracle/eigsol_oracle.cpp``).  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg import this module, and only as the checker / the timed CPU baseline.  The
product path (``pcsc_eigenvalue_solver_project_amd``) never imports it.

Dense matrices cross the boundary column-major (the reference's ``Matrix::Dense`` is an Eigen
column-major matrix, ``matrix.hpp:39-40``); complex values are interleaved (re, im) pairs.
"""
from __future__ import annotations

import contextlib
import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.environ.get("EIGSOL_ORACLE_LIB") or os.path.join(_HERE, "build", "liboracle.so")   # override: sanitizer builds
_lib = None

_i64 = C.c_int64
_int = C.c_int
_dbl = C.c_double
_p = C.c_void_p


def build(force: bool = False) -> str:
    if force or not os.path.exists(_LIB_PATH):
        subprocess.run(["make", "-C", _HERE], check=True, stdout=subprocess.DEVNULL)
    return _LIB_PATH


_AS_SHIPPED_PATH = os.path.join(_HERE, "build", "liboracle_O0.so")


@contextlib.contextmanager
def as_shipped():
    """Inside the block, every oracle call runs the same restatement compiled at -O0 without -march
    (the reference's CMake sets no build type, so it ships unoptimised) - the
    secondary CPU baseline; never a checker."""
    global _lib
    if not os.path.exists(_AS_SHIPPED_PATH):
        subprocess.run(["make", "-C", _HERE, "O0"], check=True, stdout=subprocess.DEVNULL)
    saved = lib()
    _lib = _configure(C.CDLL(_AS_SHIPPED_PATH))
    try:
        yield
    finally:
        _lib = saved


@contextlib.contextmanager
def single_accumulation():
    """Inside the block, float / complex<float> norms and dots accumulate in the scalar type itself,
    one sequential single-precision sum (a scalar Eigen reduction over Vector<float>,
    power_method.hpp:72,81) instead of in double then rounded (the default)."""
    L = lib()
    old = L.orc_set_single_accum(1)
    try:
        yield
    finally:
        L.orc_set_single_accum(old)


def lib():
    global _lib
    if _lib is None:
        build()
        _lib = _configure(C.CDLL(_LIB_PATH))
    return _lib


def _configure(L):
    if True:
        for name in ("spmv_csc_f64", "spmv_csc_c128", "spmv_csc_f32", "spmv_csc_c64"):
            getattr(L, "orc_" + name).argtypes = [_i64, _i64, _p, _p, _p, _p, _p]
        for name in ("spmv_csr_f64", "spmv_csr_c128", "spmv_csr_f32", "spmv_csr_c64"):
            getattr(L, "orc_" + name).argtypes = [_i64, _p, _p, _p, _p, _p]
        for name in ("gemv_f64", "gemv_c128", "gemv_f32", "gemv_c64"):
            getattr(L, "orc_" + name).argtypes = [_i64, _i64, _p, _p, _p]
        for name in ("power_csc_f64", "power_csc_c128", "power_csc_f32", "power_csc_c64"):
            f = getattr(L, "orc_" + name)
            f.argtypes = [_i64, _p, _p, _p, _p, _int, _dbl, _p, _p, _p, _p]
            f.restype = _int
        for name in ("power_dense_f64", "power_dense_c128", "power_dense_f32", "power_dense_c64"):
            f = getattr(L, "orc_" + name)
            f.argtypes = [_i64, _p, _p, _int, _dbl, _p, _p, _p, _p]
            f.restype = _int
        L.orc_set_single_accum.argtypes = [_int]
        L.orc_set_single_accum.restype = _int
        L.orc_power_csr_omp_f64.argtypes = [_i64, _p, _p, _p, _p, _int, _int]
        L.orc_power_csr_omp_f64.restype = _dbl
        L.orc_solve_shifted_dense_f64.argtypes = [_i64, _p, _dbl, _p, _p]
        L.orc_solve_shifted_dense_c128.argtypes = [_i64, _p, _p, _p, _p]
        L.orc_shifted_dense_f64.argtypes = [_i64, _p, _dbl, _p, _int, _dbl, _p, _p, _p, _p]
        L.orc_shifted_dense_f64.restype = _int
        L.orc_shifted_dense_c128.argtypes = [_i64, _p, _p, _p, _int, _dbl, _p, _p, _p, _p]
        L.orc_shifted_dense_c128.restype = _int
        L.orc_shifted_triu_csr_c128.argtypes = [_i64, _p, _p, _p, _p, _p, _int, _dbl, _p, _p, _p, _p]
        L.orc_shifted_triu_csr_c128.restype = _int
        L.orc_shifted_triu_csr_f64.argtypes = [_i64, _p, _p, _p, _dbl, _p, _int, _dbl, _p, _p, _p, _p]
        L.orc_shifted_triu_csr_f64.restype = _int
        L.orc_triu_shifted_solve_csr_c128.argtypes = [_i64, _p, _p, _p, _p, _p, _p]
        for name in ("shifted_triu_csr_f32", "shifted_triu_csr_c64"):
            f = getattr(L, "orc_" + name)
            f.argtypes = [_i64, _p, _p, _p, _p, _p, _int, _dbl, _p, _p, _p, _p]
            f.restype = _int
        for name in ("hessenberg_f64", "hessenberg_c128"):
            getattr(L, "orc_" + name).argtypes = [_i64, _p, _p]
        for name in ("qr_decompose_f64", "qr_decompose_c128"):
            getattr(L, "orc_" + name).argtypes = [_i64, _i64, _p, _p, _p]
        for name in ("qr_eigenvalues_f64", "qr_eigenvalues_c128"):
            f = getattr(L, "orc_" + name)
            f.argtypes = [_i64, _p, _int, _dbl, _p, _p]
            f.restype = _int
        L.orc_hqr_francis_f64.argtypes = [_i64, _p, _p, _p]
        L.orc_hqr_francis_f64.restype = _int
        L.orc_hqr_francis_f80.argtypes = [_i64, _p, _p, _p]
        L.orc_hqr_francis_f80.restype = _int
        # long double / std::complex<long double> (x87): the same restatements at extended precision
        for sfx in ("f80", "c80"):
            getattr(L, "orc_spmv_csc_" + sfx).argtypes = [_i64, _i64, _p, _p, _p, _p, _p]
            getattr(L, "orc_spmv_csr_" + sfx).argtypes = [_i64, _p, _p, _p, _p, _p]
            getattr(L, "orc_gemv_" + sfx).argtypes = [_i64, _i64, _p, _p, _p]
            for name, args in (("power_csc_", [_i64, _p, _p, _p, _p, _int, _dbl, _p, _p, _p, _p]),
                               ("power_dense_", [_i64, _p, _p, _int, _dbl, _p, _p, _p, _p]),
                               ("shifted_triu_csr_", [_i64, _p, _p, _p, _p, _p, _int, _dbl, _p, _p, _p, _p]),
                               ("shifted_dense_", [_i64, _p, _p, _p, _int, _dbl, _p, _p, _p, _p]),
                               ("qr_eigenvalues_", [_i64, _p, _int, _dbl, _p, _p])):
                f = getattr(L, "orc_" + name + sfx)
                f.argtypes = args
                f.restype = _int
            getattr(L, "orc_solve_shifted_dense_" + sfx).argtypes = [_i64, _p, _p, _p, _p]
            getattr(L, "orc_hessenberg_" + sfx).argtypes = [_i64, _p, _p]
            getattr(L, "orc_qr_decompose_" + sfx).argtypes = [_i64, _i64, _p, _p, _p]
    return L


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def _is_c(dt) -> bool:
    return np.dtype(dt) == np.complex128


def _wide(dt) -> bool:
    """long double / std::complex<long double> (numpy longdouble is the x87 80-bit format here)."""
    return np.dtype(dt) in (np.dtype(np.longdouble), np.dtype(np.clongdouble))


_SFX = {np.dtype(np.float64): "f64", np.dtype(np.complex128): "c128", np.dtype(np.float32): "f32",
        np.dtype(np.complex64): "c64", np.dtype(np.longdouble): "f80", np.dtype(np.clongdouble): "c80"}


def _sfx(dt) -> str:
    return _SFX[np.dtype(dt)]


def _single(dt) -> bool:
    return np.dtype(dt) in (np.dtype(np.float32), np.dtype(np.complex64))


def _vec(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


def _fortran(A, dt):
    return np.asfortranarray(A, dtype=dt)


# --------------------------------------------------------------------------- products
def spmv_csc(colptr, rowidx, vals, x, nrows):
    dt = vals.dtype
    cp, ri = _vec(colptr, np.int32), _vec(rowidx, np.int32)
    v, xx = _vec(vals, dt), _vec(x, dt)
    y = np.empty(nrows, dtype=dt)
    getattr(lib(), "orc_spmv_csc_" + _sfx(dt))(nrows, len(cp) - 1, _ptr(cp), _ptr(ri), _ptr(v), _ptr(xx), _ptr(y))
    return y


def spmv_csr(rowptr, colidx, vals, x):
    dt = vals.dtype
    rp, ci = _vec(rowptr, np.int32), _vec(colidx, np.int32)
    v, xx = _vec(vals, dt), _vec(x, dt)
    y = np.empty(len(rp) - 1, dtype=dt)
    getattr(lib(), "orc_spmv_csr_" + _sfx(dt))(len(rp) - 1, _ptr(rp), _ptr(ci), _ptr(v), _ptr(xx), _ptr(y))
    return y


def gemv(A, x):
    dt = A.dtype if _single(A.dtype) else np.result_type(A.dtype, np.float64)
    Af, xx = _fortran(A, dt), _vec(x, dt)
    y = np.empty(A.shape[0], dtype=dt)
    getattr(lib(), "orc_gemv_" + _sfx(dt))(A.shape[0], A.shape[1], _ptr(Af), _ptr(xx), _ptr(y))
    return y


# --------------------------------------------------------------------------- solvers
def _result(lam, x, iters, conv, trace):
    it = int(iters.value)
    return {
        "eigenvalue": lam[0] if (np.iscomplexobj(lam) or _wide(lam.dtype)) else float(lam[0]),
        "eigenvector": x,
        "iterations": it,
        "converged": bool(conv),
        "trace": None if trace is None else trace[: max(it, 0)],
    }


def power_csc(colptr, rowidx, vals, x0, max_iterations=1000, tolerance=1e-10, want_trace=False):
    """powerMethod<S> on the reference's canonical CSC storage (power_method.hpp:47-99)."""
    dt = vals.dtype
    n = len(colptr) - 1
    cp, ri, v, xx = _vec(colptr, np.int32), _vec(rowidx, np.int32), _vec(vals, dt), _vec(x0, dt)
    lam = np.zeros(1, dtype=dt)
    x = np.empty(n, dtype=dt)
    it = C.c_int(0)
    tr = np.zeros(max(max_iterations, 1), dtype=dt) if want_trace else None
    conv = getattr(lib(), "orc_power_csc_" + _sfx(dt))(
        n, _ptr(cp), _ptr(ri), _ptr(v), _ptr(xx), int(max_iterations), float(tolerance),
        _ptr(lam), _ptr(x), C.byref(it), None if tr is None else _ptr(tr))
    return _result(lam, x, it, conv, tr)


def power_csr_omp(rowptr, colidx, vals, x0, iterations, threads):
    """bench.py's all-cores CPU figure: fused CSR power iteration, OpenMP rows, fixed iteration
    count; returns the last Rayleigh quotient."""
    n = len(rowptr) - 1
    rp, ci, v, xx = _vec(rowptr, np.int32), _vec(colidx, np.int32), _vec(vals, np.float64), _vec(x0, np.float64)
    return float(lib().orc_power_csr_omp_f64(n, _ptr(rp), _ptr(ci), _ptr(v), _ptr(xx), int(iterations),
                                             int(threads)))


def power_dense(A, x0, max_iterations=1000, tolerance=1e-10, want_trace=False):
    dt = A.dtype if _single(A.dtype) else np.result_type(A.dtype, np.float64)
    n = A.shape[0]
    Af, xx = _fortran(A, dt), _vec(x0, dt)
    lam = np.zeros(1, dtype=dt)
    x = np.empty(n, dtype=dt)
    it = C.c_int(0)
    tr = np.zeros(max(max_iterations, 1), dtype=dt) if want_trace else None
    conv = getattr(lib(), "orc_power_dense_" + _sfx(dt))(
        n, _ptr(Af), _ptr(xx), int(max_iterations), float(tolerance), _ptr(lam), _ptr(x),
        C.byref(it), None if tr is None else _ptr(tr))
    return _result(lam, x, it, conv, tr)


def solve_shifted_dense(A, shift, b):
    dt = np.result_type(A.dtype, np.asarray(shift).dtype, np.float64)
    n = A.shape[0]
    Af, bb = _fortran(A, dt), _vec(b, dt)
    x = np.empty(n, dtype=dt)
    if _wide(dt):
        s = np.array([shift], dtype=dt)
        getattr(lib(), "orc_solve_shifted_dense_" + _sfx(dt))(n, _ptr(Af), _ptr(s), _ptr(bb), _ptr(x))
    elif _is_c(dt):
        s = np.array([complex(shift).real, complex(shift).imag])
        lib().orc_solve_shifted_dense_c128(n, _ptr(Af), _ptr(s), _ptr(bb), _ptr(x))
    else:
        lib().orc_solve_shifted_dense_f64(n, _ptr(Af), float(shift), _ptr(bb), _ptr(x))
    return x


def shifted_dense(A, shift, x0, max_iterations=1000, tolerance=1e-10, want_trace=False):
    """shiftedInversePowerMethod<S>, dense branch (refactor per iteration)."""
    dt = np.result_type(A.dtype, np.asarray(shift).dtype, np.float64)
    n = A.shape[0]
    Af, xx = _fortran(A, dt), _vec(x0, dt)
    lam = np.zeros(1, dtype=dt)
    x = np.empty(n, dtype=dt)
    it = C.c_int(0)
    tr = np.zeros(max(max_iterations, 1), dtype=dt) if want_trace else None
    trp = None if tr is None else _ptr(tr)
    if _wide(dt):
        s = np.array([shift], dtype=dt)
        conv = getattr(lib(), "orc_shifted_dense_" + _sfx(dt))(n, _ptr(Af), _ptr(s), _ptr(xx), int(max_iterations),
                                                              float(tolerance), _ptr(lam), _ptr(x), C.byref(it), trp)
    elif _is_c(dt):
        s = np.array([complex(shift).real, complex(shift).imag])
        conv = lib().orc_shifted_dense_c128(n, _ptr(Af), _ptr(s), _ptr(xx), int(max_iterations),
                                            float(tolerance), _ptr(lam), _ptr(x), C.byref(it), trp)
    else:
        conv = lib().orc_shifted_dense_f64(n, _ptr(Af), float(shift), _ptr(xx), int(max_iterations),
                                           float(tolerance), _ptr(lam), _ptr(x), C.byref(it), trp)
    return _result(lam, x, it, conv, tr)


def shifted_triu_csr(rowptr, colidx, vals, shift, x0, max_iterations=1000, tolerance=1e-10,
                     want_trace=False):
    """shiftedInversePowerMethod<S> on an upper-triangular CSR (config-5 class)."""
    dt = vals.dtype
    n = len(rowptr) - 1
    rp, ci, v, xx = _vec(rowptr, np.int32), _vec(colidx, np.int32), _vec(vals, dt), _vec(x0, dt)
    lam = np.zeros(1, dtype=dt)
    x = np.empty(n, dtype=dt)
    it = C.c_int(0)
    tr = np.zeros(max(max_iterations, 1), dtype=dt) if want_trace else None
    trp = None if tr is None else _ptr(tr)
    if _single(dt) or _wide(dt):
        s = np.array([shift], dtype=dt)
        conv = getattr(lib(), "orc_shifted_triu_csr_" + _sfx(dt))(
            n, _ptr(rp), _ptr(ci), _ptr(v), _ptr(s), _ptr(xx), int(max_iterations), float(tolerance), _ptr(lam),
            _ptr(x), C.byref(it), trp)
    elif _is_c(dt):
        s = np.array([complex(shift).real, complex(shift).imag])
        conv = lib().orc_shifted_triu_csr_c128(n, _ptr(rp), _ptr(ci), _ptr(v), _ptr(s), _ptr(xx),
                                               int(max_iterations), float(tolerance), _ptr(lam),
                                               _ptr(x), C.byref(it), trp)
    else:
        conv = lib().orc_shifted_triu_csr_f64(n, _ptr(rp), _ptr(ci), _ptr(v), float(shift), _ptr(xx),
                                              int(max_iterations), float(tolerance), _ptr(lam),
                                              _ptr(x), C.byref(it), trp)
    return _result(lam, x, it, conv, tr)


def triu_shifted_solve_csr(rowptr, colidx, vals, shift, b):
    n = len(rowptr) - 1
    rp, ci = _vec(rowptr, np.int32), _vec(colidx, np.int32)
    v, bb = _vec(vals, np.complex128), _vec(b, np.complex128)
    s = np.array([complex(shift).real, complex(shift).imag])
    x = np.empty(n, dtype=np.complex128)
    lib().orc_triu_shifted_solve_csr_c128(n, _ptr(rp), _ptr(ci), _ptr(v), _ptr(s), _ptr(bb), _ptr(x))
    return x


def hessenberg(A):
    dt = np.result_type(A.dtype, np.float64)
    n = A.shape[0]
    Af = _fortran(A, dt)
    H = np.empty((n, n), dtype=dt, order="F")
    getattr(lib(), "orc_hessenberg_" + _sfx(dt))(n, _ptr(Af), _ptr(H))
    return H


def qr_decompose(A):
    dt = np.result_type(A.dtype, np.float64)
    m, n = A.shape
    Af = _fortran(A, dt)
    Q = np.empty((m, m), dtype=dt, order="F")
    R = np.empty((m, n), dtype=dt, order="F")
    getattr(lib(), "orc_qr_decompose_" + _sfx(dt))(m, n, _ptr(Af), _ptr(Q), _ptr(R))
    return Q, R


def qr_eigenvalues(A, max_iterations=1000, tolerance=1e-10):
    dt = np.result_type(A.dtype, np.float64)
    n = A.shape[0]
    Af = _fortran(A, dt)
    eig = np.zeros(n, dtype=dt)
    it = C.c_int(0)
    conv = getattr(lib(), "orc_qr_eigenvalues_" + _sfx(dt))(n, _ptr(Af), int(max_iterations),
                                                           float(tolerance), _ptr(eig), C.byref(it))
    return {"eigenvalues": eig, "iterations": int(it.value), "converged": bool(conv)}


def hqr_francis(H):
    """Francis double-shift QR on an upper Hessenberg matrix; returns complex eigenvalues.  A long
    double H runs the same restatement in x87 long double (clongdouble eigenvalues)."""
    n = H.shape[0]
    if _wide(np.asarray(H).dtype):
        Hf = np.array(H, dtype=np.longdouble, order="F", copy=True)
        wr = np.zeros(n, dtype=np.longdouble)
        wi = np.zeros(n, dtype=np.longdouble)
        if lib().orc_hqr_francis_f80(n, _ptr(Hf), _ptr(wr), _ptr(wi)) != 0:
            raise RuntimeError("hqr_francis: no convergence")
        return wr + np.clongdouble(1j) * wi
    Hf = np.array(H, dtype=np.float64, order="F", copy=True)
    wr = np.zeros(n)
    wi = np.zeros(n)
    rc = lib().orc_hqr_francis_f64(n, _ptr(Hf), _ptr(wr), _ptr(wi))
    if rc != 0:
        raise RuntimeError("hqr_francis: no convergence")
    return wr + 1j * wi


# --------------------------------------------------------------------------- helpers
def csr_to_csc(rowptr, colidx, vals, ncols):
    """Transpose CSR -> CSC with ascending row indices per column (Eigen's compressed CSC)."""
    rowptr = np.asarray(rowptr, dtype=np.int64)
    nrows = len(rowptr) - 1
    rows = np.repeat(np.arange(nrows, dtype=np.int32), np.diff(rowptr))
    order = np.lexsort((rows, np.asarray(colidx)))
    ri = rows[order].astype(np.int32)
    v = np.asarray(vals)[order]
    counts = np.bincount(np.asarray(colidx), minlength=ncols)
    cp = np.zeros(ncols + 1, dtype=np.int32)
    np.cumsum(counts, out=cp[1:])
    return cp, ri, v

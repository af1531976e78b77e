"""MI355X-native eigenvalue-solver hot path (Python view of the C ABI).

The product is ``libeigsol_hip.so`` (hand-written HIP kernels for gfx950, ``csrc/``) behind the
C ABI in ``include/eigsol_hip.h`` and the C++ drop-in façade in ``include/eigsol/``.  This package
is the thin Python view used by the tests and the benchmark; its names follow the reference's
C++ API (``SolverOptions``, ``EigenResult``, ``power_method`` ≙ ``EigSol::powerMethod``).
No CPU fallback exists: without the library or a gfx950 device every call raises ``EigSolError``.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Optional

import numpy as np

from ._capi import (EIGSOL_C64, EIGSOL_C128, EIGSOL_CDD, EIGSOL_DD, EIGSOL_E_INVALID, EIGSOL_E_SIZE_MISMATCH, EIGSOL_E_UNSUPPORTED, EIGSOL_F32,
                    EIGSOL_F64, EigSolError, SolverOptionsC, call, check, last_error, lib)

__all__ = [
    "EigSolError", "SolverOptions", "EigenResult", "Context", "CsrMatrix", "DenseMatrix",
    "PowerSession", "power_method", "device_count", "lib", "last_error",
]


@dataclass
class SolverOptions:
    """``EigSol::SolverOptions`` (src/option/solver_option.hpp:14-20)."""

    maxIterations: int = 1000
    tolerance: float = 1e-10

    def to_c(self) -> SolverOptionsC:
        return SolverOptionsC(int(self.maxIterations), float(self.tolerance))


@dataclass
class EigenResult:
    """``EigSol::EigenResult<S>`` (src/result/eigen_result.hpp:22-52)."""

    eigenvalue: complex | float
    eigenvector: np.ndarray
    iterations: int
    converged: bool


def _dtype_code(dt) -> int:
    dt = np.dtype(dt)
    if dt == np.float64:
        return EIGSOL_F64
    if dt == np.complex128:
        return EIGSOL_C128
    if dt == np.float32:
        return EIGSOL_F32
    if dt == np.complex64:
        return EIGSOL_C64
    if dt == np.longdouble:
        return EIGSOL_DD
    if dt == np.clongdouble:
        return EIGSOL_CDD
    raise EigSolError(3, f"scalar type mismatch: {dt} (supported: float64, complex128, float32, complex64, "
                         "longdouble, clongdouble)")


def _np_dtype(code: int):
    return {EIGSOL_C128: np.complex128, EIGSOL_F32: np.float32, EIGSOL_C64: np.complex64,
            EIGSOL_DD: np.longdouble, EIGSOL_CDD: np.clongdouble}.get(code, np.float64)


def _ptr(a: np.ndarray) -> C.c_void_p:
    return a.ctypes.data_as(C.c_void_p)


def is_wide(dtype) -> bool:
    """long double / std::complex<long double>: crosses the C ABI as double-double pairs."""
    return np.dtype(dtype) in (np.dtype(np.longdouble), np.dtype(np.clongdouble))


def to_wire(a, dtype) -> np.ndarray:
    """Host scalars of ``dtype`` in the C ABI's layout (a contiguous buffer, flattened in C order).
    long double values become double-double pairs {hi = (double) v, lo = (double)(v - hi)}.  Exact
    for the x87 format (64-bit significand: 53 bits in hi, 11 in lo) while lo is a normal double,
    i.e. |v| >= ~2^-1010 (1e-304); below that lo falls under the subnormal grid, the pair is the nearest double-double and a
    RuntimeWarning says so.  A long double with another significand (IEEE binary128 on aarch64)
    is refused: its values do not fit {hi, lo}."""
    a = np.ascontiguousarray(a, dtype=dtype)
    if not is_wide(dtype):
        return a
    if np.finfo(np.longdouble).nmant != 63:
        raise EigSolError(EIGSOL_E_UNSUPPORTED, "long double is not the x87 80-bit format on this platform; "
                                                "the double-double wire format cannot carry it exactly")
    flat = a.reshape(-1)
    parts = [flat.real, flat.imag] if np.iscomplexobj(flat) else [flat]
    cols = []
    for p in parts:
        with np.errstate(over="ignore"):
            hi = p.astype(np.float64)
        if np.any(np.isinf(hi) & np.isfinite(p)):
            raise EigSolError(EIGSOL_E_INVALID, "long double value outside the double exponent range "
                                                "(double-double carries |v| < 1.8e308)")
        fin = np.isfinite(p)
        with np.errstate(invalid="ignore"):
            lo = np.where(fin, (p - hi.astype(np.longdouble)), 0).astype(np.float64)   # inf / NaN: lo = 0
        if np.any(fin & (hi.astype(np.longdouble) + lo.astype(np.longdouble) != p)):
            import warnings
            warnings.warn("long double values below ~2^-1010 (1e-304) lose low bits in the double-double wire format "
                          "(the low part falls under the subnormal grid)", RuntimeWarning, stacklevel=2)
        cols += [hi, lo]
    return np.ascontiguousarray(np.stack(cols, axis=-1))


def wire_buffer(dtype, n: int) -> np.ndarray:
    """Output buffer for n scalars of ``dtype`` in the C ABI's layout."""
    if not is_wide(dtype):
        return np.empty(max(n, 0), dtype=dtype)
    return np.zeros((max(n, 0), 4 if np.dtype(dtype) == np.clongdouble else 2), dtype=np.float64)


def from_wire(w: np.ndarray, dtype) -> np.ndarray:
    """Inverse of to_wire (double-double hi + lo rounded to the nearest long double)."""
    if not is_wide(dtype):
        return w
    w = np.asarray(w, dtype=np.float64).reshape(-1, 4 if np.dtype(dtype) == np.clongdouble else 2)
    re = w[:, 0].astype(np.longdouble) + w[:, 1].astype(np.longdouble)
    if np.dtype(dtype) == np.longdouble:
        return re
    z = np.empty(len(w), dtype=np.clongdouble)
    z.real = re
    z.imag = w[:, 2].astype(np.longdouble) + w[:, 3].astype(np.longdouble)
    return z


def _scalar(v, dtype):
    """eigenvalue as a Python / numpy scalar (long double kept at its precision)."""
    if is_wide(dtype):
        return v
    return complex(v) if np.iscomplexobj(v) else float(v)


def _vector(v, dtype, n: int, what: str) -> np.ndarray:
    """Host vector of exactly n entries (the C ABI copies n scalars from the pointer)."""
    v = np.ascontiguousarray(v, dtype=dtype).reshape(-1)
    if len(v) != n:
        raise EigSolError(EIGSOL_E_SIZE_MISMATCH, f"{what} has {len(v)} entries, the matrix has {n} rows")
    return to_wire(v, dtype)


def device_count() -> int:
    n = C.c_int(0)
    st = lib().eigsol_device_count(C.byref(n))
    return int(n.value) if st == 0 else 0


class Context:
    """One gfx950 device + one stream (``eigsol_ctx``)."""

    def __init__(self, device: int = 0, stream: Optional[int] = None):
        h = C.c_void_p()
        call("eigsol_ctx_create", int(device), C.byref(h))
        self.handle = h
        self.device = device
        if stream is not None:
            self.set_stream(stream)

    def set_stream(self, stream_ptr: Optional[int]) -> None:
        call("eigsol_ctx_set_stream", self.handle, C.c_void_p(stream_ptr or 0))

    def synchronize(self) -> None:
        call("eigsol_ctx_synchronize", self.handle)

    def malloc(self, nbytes: int) -> int:
        p = C.c_void_p()
        call("eigsol_malloc", self.handle, C.c_size_t(nbytes), C.byref(p))
        return int(p.value or 0)

    def free(self, ptr: int) -> None:
        call("eigsol_free", self.handle, C.c_void_p(ptr))

    def h2d(self, dptr: int, host: np.ndarray) -> None:
        host = np.ascontiguousarray(host)
        call("eigsol_memcpy_h2d", self.handle, C.c_void_p(dptr), _ptr(host), C.c_size_t(host.nbytes))

    def d2h(self, host: np.ndarray, dptr: int) -> np.ndarray:
        call("eigsol_memcpy_d2h", self.handle, _ptr(host), C.c_void_p(dptr), C.c_size_t(host.nbytes))
        return host

    def close(self) -> None:
        if getattr(self, "handle", None):
            lib().eigsol_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class CsrMatrix:
    """Device-resident CSR matrix (``eigsol_csr``)."""

    def __init__(self, ctx: Context, rowptr, colidx, values, shape, layout: str = "csr"):
        values = np.ascontiguousarray(values)
        code = _dtype_code(values.dtype)
        ptr = np.ascontiguousarray(rowptr, dtype=np.int32)
        idx = np.ascontiguousarray(colidx, dtype=np.int32)
        nrows, ncols = int(shape[0]), int(shape[1])
        nouter = nrows if layout == "csr" else ncols
        if len(ptr) != nouter + 1:
            raise EigSolError(EIGSOL_E_SIZE_MISMATCH,
                              f"{layout} pointer array has {len(ptr)} entries, expected {nouter + 1}")
        if len(values) != len(idx):
            raise EigSolError(EIGSOL_E_SIZE_MISMATCH,
                              f"values ({len(values)}) and index array ({len(idx)}) lengths differ")
        h = C.c_void_p()
        fn = "eigsol_csr_create" if layout == "csr" else "eigsol_csr_create_from_csc"
        vw = to_wire(values, values.dtype)
        call(fn, ctx.handle, code, nrows, ncols, len(idx), _ptr(ptr), _ptr(idx), _ptr(vw), C.byref(h))
        self.ctx, self.handle = ctx, h
        self.shape = (nrows, ncols)
        self.nnz = len(idx)
        self.dtype = _np_dtype(code)

    @classmethod
    def from_scipy(cls, ctx: Context, M):
        import scipy.sparse as sp
        if sp.isspmatrix_csc(M) or isinstance(M, sp.csc_array):
            M = M.copy()
            M.sort_indices()
            return cls(ctx, M.indptr, M.indices, M.data, M.shape, layout="csc")
        M = sp.csr_matrix(M)
        M.sort_indices()
        return cls(ctx, M.indptr, M.indices, M.data, M.shape)

    @classmethod
    def from_coo(cls, ctx: Context, rows, cols, values, shape):
        """Triplets in any order straight to the device CSR (``eigsol_csr_create_from_coo``):
        repeated positions are summed in input order, as the reader's Matrix::Sparse does."""
        values = np.ascontiguousarray(values)
        code = _dtype_code(values.dtype)
        r = np.ascontiguousarray(rows, dtype=np.int32)
        c = np.ascontiguousarray(cols, dtype=np.int32)
        if not (len(r) == len(c) == len(values)):
            raise EigSolError(EIGSOL_E_SIZE_MISMATCH,
                              f"triplet arrays differ in length ({len(r)}, {len(c)}, {len(values)})")
        h = C.c_void_p()
        vw = to_wire(values, values.dtype)
        call("eigsol_csr_create_from_coo", ctx.handle, code, int(shape[0]), int(shape[1]), len(r), _ptr(r),
             _ptr(c), _ptr(vw), C.byref(h))
        self = cls.__new__(cls)
        self.ctx, self.handle = ctx, h
        self.shape = (int(shape[0]), int(shape[1]))
        nnz = C.c_int64()
        call("eigsol_csr_info", h, None, None, C.byref(nnz), None)
        self.nnz = nnz.value
        self.dtype = _np_dtype(code)
        return self

    def download(self):
        """(rowptr, colidx, values) of the device CSR (``eigsol_csr_download``)."""
        rp = np.empty(self.shape[0] + 1, np.int32)
        ci = np.empty(self.nnz, np.int32)
        v = wire_buffer(self.dtype, self.nnz)
        call("eigsol_csr_download", self.handle, _ptr(rp), _ptr(ci), _ptr(v))
        return rp, ci, from_wire(v, self.dtype)

    def spmv(self, x_dev: int, y_dev: int) -> None:
        call("eigsol_csr_spmv", self.handle, C.c_void_p(x_dev), C.c_void_p(y_dev))

    def close(self) -> None:
        if getattr(self, "handle", None):
            lib().eigsol_csr_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DenseMatrix:
    """Device-resident column-major dense matrix (``eigsol_dense``; ``Matrix::Dense<S>``)."""

    def __init__(self, ctx: Context, A: np.ndarray):
        A = np.asarray(A)
        code = _dtype_code(A.dtype)
        Af = to_wire(np.asfortranarray(A).ravel(order="F"), A.dtype)   # column-major
        h = C.c_void_p()
        call("eigsol_dense_create", ctx.handle, code, A.shape[0], A.shape[1], _ptr(Af), C.byref(h))
        self.ctx, self.handle = ctx, h
        self.shape = A.shape
        self.dtype = _np_dtype(code)

    def gemv(self, x_dev: int, y_dev: int) -> None:
        call("eigsol_dense_gemv", self.handle, C.c_void_p(x_dev), C.c_void_p(y_dev))

    def close(self) -> None:
        if getattr(self, "handle", None):
            lib().eigsol_dense_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class PowerSession:
    """Device-resident power iteration (``eigsol_power``): begin / step / query / finish."""

    def __init__(self, matrix, trace_capacity: int = 0):
        h = C.c_void_p()
        if isinstance(matrix, CsrMatrix):
            call("eigsol_power_create_csr", matrix.handle, int(trace_capacity), C.byref(h))
        else:
            call("eigsol_power_create_dense", matrix.handle, int(trace_capacity), C.byref(h))
        self.matrix, self.handle = matrix, h
        self.n = matrix.shape[0]
        self.dtype = matrix.dtype

    def begin(self, opts: SolverOptions, x0=None, x0_dev: Optional[int] = None) -> None:
        o = opts.to_c()
        if x0_dev is not None:
            call("eigsol_power_begin", self.handle, C.byref(o), C.c_void_p(x0_dev), 1)
        else:
            x = _vector(x0, self.dtype, self.n, "x0")
            self._x0 = x
            call("eigsol_power_begin", self.handle, C.byref(o), _ptr(x), 0)

    def step(self, n: int) -> None:
        call("eigsol_power_step", self.handle, int(n))

    def query(self):
        done, launches = C.c_int32(0), C.c_int32(0)
        call("eigsol_power_query", self.handle, C.byref(done), C.byref(launches))
        return bool(done.value), int(launches.value)

    def finish(self, want_vector: bool = True) -> EigenResult:
        lam = wire_buffer(self.dtype, 1)
        x = wire_buffer(self.dtype, self.n) if want_vector else None
        it, conv = C.c_int32(0), C.c_int32(0)
        call("eigsol_power_finish", self.handle, _ptr(lam), None if x is None else _ptr(x), 0,
             C.byref(it), C.byref(conv))
        ev = _scalar(from_wire(lam, self.dtype)[0], self.dtype)
        return EigenResult(ev, None if x is None else from_wire(x, self.dtype), int(it.value), bool(conv.value))

    def trace(self, capacity: int) -> np.ndarray:
        buf = wire_buffer(self.dtype, max(capacity, 1))
        cnt = C.c_int32(0)
        call("eigsol_power_trace", self.handle, _ptr(buf), int(capacity), C.byref(cnt))
        return from_wire(buf, self.dtype)[: cnt.value]

    def transport(self) -> int:
        """EIGSOL_TRANSPORT_LOCAL / _COLLECTIVE / _PEER (per-iteration exchange of this session)."""
        t = C.c_int(0)
        call("eigsol_power_transport", self.handle, C.byref(t))
        return t.value

    def kernel_info(self):
        b, g, t, v = C.c_double(0), C.c_int32(0), C.c_int32(0), C.c_int32(0)
        call("eigsol_power_kernel_info", self.handle, C.byref(b), C.byref(g), C.byref(t), C.byref(v))
        names = {0: "csr_kernel (x gathered from HBM)", 1: "csr_win_kernel (x window staged in LDS)",
                 2: "dense_kernel (GEMV)", 3: "sptrsv_kernel (sync-free triangular solve)",
                 4: "dense LU substitution (dense_lu_solve_kernel on one CU up to n = 64, else "
                    "dense_trsv2_kernel: 64-row block rows, inverted diagonal blocks, value flags)",
                 5: "csr_slice_kernel (64-row slices, one row per lane)",
                 6: "csr_row_kernel (one row per lane, single-precision fallback layout)",
                 7: "ILU(0)-preconditioned GMRES (tiles = Arnoldi steps of the last solve)",
                 8: "band_solve_kernel (RCM-banded LU; tiles = kl + ku)",
                 9: "csr_kernel column-block passes (x blocks L2-resident; tiles = blocks)",
                 10: "csr_bin_kernel (column-binned row chunks, row sums in LDS; tiles = chunks)",
                 11: "csr_bin_kernel in two row halves per iteration, the first half's all-gather "
                     "overlapped with the second half (row-sharded; tiles = chunks)",
                 12: "sptrsv multi-solve kernel (sync-free triangular solves, 2 iterations per launch, "
                     "solve j one dependency round behind solve j-1)",
                 13: "sptrsv multi-solve kernel (sync-free triangular solves, 3 iterations per launch, "
                     "solve j one dependency round behind solve j-1)",
                 14: "sptrsv multi-solve kernel (sync-free triangular solves, 4 iterations per launch, "
                     "solve j one dependency round behind solve j-1)",
                 15: "wide power_fused2_kernel (double-double: x = y / normY, A x and the norm / Rayleigh partials in one pass; a tile's row sums by 2-32 lanes per row into LDS, then one row's epilogue per thread)",
                 16: "wide gemv kernels (double-double dense product)",
                 17: "wide shifted inverse (fp64 factor + double-double residual refinement; "
                     "tiles = refinement steps of the last solve)",
                 18: "GMRES over the exact sparse LU (complete fill, no pivoting; tiles = Arnoldi "
                     "steps of the last solve)",
                 19: "GMRES over the nested-dissection multifrontal LU (dense fronts, pivoting inside each "
                     "front; tiles = Arnoldi steps of the last solve)"}
        return {"bytes_per_iteration": b.value, "grid": g.value, "tiles": t.value,
                "variant": v.value, "kernel": names.get(v.value, "?"),
                "iterations_per_launch": v.value - 10 if 12 <= v.value <= 14 else 1}

    def kernel_name(self) -> str:
        """Demangled name of the per-iteration kernel (CSR power sessions), as rocprofv3 reports it."""
        buf = C.create_string_buffer(512)
        call("eigsol_power_kernel_name", self.handle, buf, 512)
        return buf.value.decode()

    def close(self) -> None:
        if getattr(self, "handle", None):
            lib().eigsol_power_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def power_method(matrix, opts: SolverOptions = SolverOptions(), x0=None) -> EigenResult:
    """``EigSol::powerMethod<S>`` on a device-resident matrix, with an explicit start vector."""
    if x0 is None:
        rng = np.random.default_rng(0)
        x0 = rng.uniform(-1, 1, matrix.shape[0])
        if np.issubdtype(matrix.dtype, np.complexfloating):
            x0 = x0 + 1j * rng.uniform(-1, 1, matrix.shape[0])
    x0 = _vector(x0, matrix.dtype, matrix.shape[0], "x0")
    lam = wire_buffer(matrix.dtype, 1)
    x = wire_buffer(matrix.dtype, matrix.shape[0])
    it, conv = C.c_int32(0), C.c_int32(0)
    o = opts.to_c()
    fn = "eigsol_power_csr" if isinstance(matrix, CsrMatrix) else "eigsol_power_dense"
    call(fn, matrix.handle, C.byref(o), _ptr(x0), _ptr(lam), _ptr(x), C.byref(it), C.byref(conv))
    ev = _scalar(from_wire(lam, matrix.dtype)[0], matrix.dtype)
    return EigenResult(ev, from_wire(x, matrix.dtype), int(it.value), bool(conv.value))


@dataclass
class ShiftedSolverOptions(SolverOptions):
    """``EigSol::ShiftedSolverOptions<S>`` (src/option/shifted_solver_option.hpp:24-68)."""

    shift: complex | float = 0.0


def _sigma(shift, dtype) -> np.ndarray:
    if not np.issubdtype(dtype, np.complexfloating) and np.iscomplexobj(shift) and complex(shift).imag != 0:
        raise EigSolError(3, "scalar type mismatch: complex shift for a real matrix")
    return to_wire(np.array([shift], dtype=dtype), dtype)


class ShiftedSession(PowerSession):
    """Shifted inverse iteration session: A - sigma I factored once on the device
    (``eigsol_shifted_create_*``); driven with the PowerSession methods."""

    def __init__(self, matrix, shift, trace_capacity: int = 0):
        h = C.c_void_p()
        sig = _sigma(shift, matrix.dtype)
        fn = "eigsol_shifted_create_csr" if isinstance(matrix, CsrMatrix) else "eigsol_shifted_create_dense"
        call(fn, matrix.handle, _ptr(sig), int(trace_capacity), C.byref(h))
        self.matrix, self.handle = matrix, h
        self.n = matrix.shape[0]
        self.dtype = matrix.dtype
        self.shift = from_wire(sig, matrix.dtype)[0]


def shifted_inverse_power_method(matrix, opts: ShiftedSolverOptions = ShiftedSolverOptions(),
                                  x0=None) -> EigenResult:
    """``EigSol::shiftedInversePowerMethod<S>`` with an explicit start vector."""
    if x0 is None:
        rng = np.random.default_rng(0)
        x0 = rng.uniform(-1, 1, matrix.shape[0])
        if np.issubdtype(matrix.dtype, np.complexfloating):
            x0 = x0 + 1j * rng.uniform(-1, 1, matrix.shape[0])
    x0 = _vector(x0, matrix.dtype, matrix.shape[0], "x0")
    sig = _sigma(opts.shift, matrix.dtype)
    lam = wire_buffer(matrix.dtype, 1)
    x = wire_buffer(matrix.dtype, matrix.shape[0])
    it, conv = C.c_int32(0), C.c_int32(0)
    o = opts.to_c()
    fn = "eigsol_shifted_inverse_csr" if isinstance(matrix, CsrMatrix) else "eigsol_shifted_inverse_dense"
    call(fn, matrix.handle, _ptr(sig), C.byref(o), _ptr(x0), _ptr(lam), _ptr(x), C.byref(it), C.byref(conv))
    ev = _scalar(from_wire(lam, matrix.dtype)[0], matrix.dtype)
    return EigenResult(ev, from_wire(x, matrix.dtype), int(it.value), bool(conv.value))


def solve_shifted(matrix, shift, b) -> np.ndarray:
    """``EigSol::solve_shifted<S>``: x = (A - shift I)^{-1} b on the device."""
    b = np.ascontiguousarray(b, dtype=matrix.dtype).reshape(-1)
    nb = len(b)
    sig = _sigma(shift, matrix.dtype)
    x = wire_buffer(matrix.dtype, nb)
    bw = to_wire(b, matrix.dtype)
    fn = "eigsol_solve_shifted_csr" if isinstance(matrix, CsrMatrix) else "eigsol_solve_shifted_dense"
    call(fn, matrix.handle, _ptr(sig), _ptr(bw), nb, _ptr(x))
    return from_wire(x, matrix.dtype)


# ------------------------------------------------------------------------------------ QR method
@dataclass
class QRResult:
    """``EigSol::QRResult<S>`` (src/result/qr_result.hpp:25-43).  For the Francis variant on a
    real matrix, ``eigenvalues`` holds the real parts (the diagonal of the standardised real Schur
    form) and ``eigenvalues_complex`` the full complex eigenvalues."""

    eigenvalues: np.ndarray
    iterations: int
    converged: bool
    eigenvalues_complex: Optional[np.ndarray] = None


def _square_dense(A, who: str) -> np.ndarray:
    A = np.asarray(A)
    if A.ndim != 2 or A.shape[0] != A.shape[1]:
        raise EigSolError(1, f"{who}: A must be square")
    return A


def to_hessenberg(ctx: Context, A) -> np.ndarray:
    """``EigSol::to_hessenberg_dense<S>`` (to_hessenberg.hpp:23-80) on the device."""
    A = _square_dense(A, "to_hessenberg_dense")
    code = _dtype_code(A.dtype)
    n = A.shape[0]
    if is_wide(A.dtype):
        Hw = wire_buffer(A.dtype, n * n)
        call("eigsol_hessenberg_dense", ctx.handle, code, n, _ptr(to_wire(A.ravel(order="F"), A.dtype)), _ptr(Hw))
        return from_wire(Hw, A.dtype).reshape((n, n), order="F")
    Af = np.asfortranarray(A)
    H = np.empty_like(Af, order="F")
    call("eigsol_hessenberg_dense", ctx.handle, code, n, _ptr(Af), _ptr(H))
    return H


def qr_decompose(ctx: Context, A):
    """``EigSol::qr_decompose_dense<S>`` (qr_decompose.hpp:25-86): returns (Q, R)."""
    A = np.asarray(A)
    code = _dtype_code(A.dtype)
    m, n = A.shape
    if is_wide(A.dtype):
        Qw, Rw = wire_buffer(A.dtype, m * m), wire_buffer(A.dtype, m * n)
        call("eigsol_qr_decompose_dense", ctx.handle, code, m, n, _ptr(to_wire(A.ravel(order="F"), A.dtype)),
             _ptr(Qw), _ptr(Rw))
        return (from_wire(Qw, A.dtype).reshape((m, m), order="F"), from_wire(Rw, A.dtype).reshape((m, n), order="F"))
    Af = np.asfortranarray(A)
    Q = np.empty((m, m), dtype=A.dtype, order="F")
    R = np.empty((m, n), dtype=A.dtype, order="F")
    call("eigsol_qr_decompose_dense", ctx.handle, code, m, n, _ptr(Af), _ptr(Q), _ptr(R))
    return Q, R


def qr_eigenvalues(ctx: Context, A, opts: SolverOptions = SolverOptions(), variant: str = "francis") -> QRResult:
    """``EigSol::qr_eigenvalues<S>``.  variant "unshifted" = the reference algorithm
    (qr_eigenvalues.hpp:40-108); "francis" = implicit multishift sweeps (real: double-shift
    bulges, francis.hip; complex: complex two-shift bulges, zfrancis.hip)."""
    A = _square_dense(A, "qr_eigenvalues_dense")
    code = _dtype_code(A.dtype)
    n = A.shape[0]
    v = 1 if variant == "unshifted" else 0
    if is_wide(A.dtype):
        # long double: "unshifted" = the reference's iteration in double-double; "francis" = the fp64
        # multishift sweeps on the rounded double-double Hessenberg matrix, every eigenvalue then
        # refined in double-double by Newton's method on det(H - mu I) (wide.hip)
        eig = wire_buffer(A.dtype, max(n, 1))
        eim = np.zeros((max(n, 1), 2)) if (v == 0 and A.dtype == np.longdouble) else None
        it, conv = C.c_int32(0), C.c_int32(0)
        o = opts.to_c()
        call("eigsol_qr_eigenvalues_dense", ctx.handle, code, n, _ptr(to_wire(A.ravel(order="F"), A.dtype)),
             C.byref(o), v, _ptr(eig), None if eim is None else _ptr(eim), C.byref(it), C.byref(conv))
        ev = from_wire(eig, A.dtype)[:n]
        full = None
        if v == 0:
            full = ev.astype(np.clongdouble)
            if eim is not None:
                full = full + np.clongdouble(1j) * from_wire(eim, np.longdouble)[:n]
        return QRResult(ev, int(it.value), bool(conv.value), full)
    if v == 0 and A.dtype in (np.float32, np.complex64):
        # single precision: the multishift sweeps are double kernels (as in the C++ facade, the
        # matrix is promoted and the eigenvalues rounded back); "unshifted" runs natively in float
        wide = np.float64 if A.dtype == np.float32 else np.complex128
        r = qr_eigenvalues(ctx, A.astype(wide), opts, variant)
        return QRResult(r.eigenvalues.astype(A.dtype), r.iterations, r.converged,
                        None if r.eigenvalues_complex is None else r.eigenvalues_complex.astype(np.complex64))
    Af = np.asfortranarray(A)
    eig = np.zeros(max(n, 1), dtype=A.dtype)
    wi = np.zeros(max(n, 1))
    it, conv = C.c_int32(0), C.c_int32(0)
    o = opts.to_c()
    call("eigsol_qr_eigenvalues_dense", ctx.handle, code, n, _ptr(Af), C.byref(o), v, _ptr(eig),
         _ptr(wi), C.byref(it), C.byref(conv))
    eig = eig[:n]
    full = None
    if v == 0 and A.dtype == np.float64:
        full = eig + 1j * wi[:n]
    elif v == 0 and A.dtype == np.complex128:
        full = eig.copy()
    return QRResult(eig, int(it.value), bool(conv.value), full)

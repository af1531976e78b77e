"""ctypes binding of ``libeigsol_hip.so`` (the C ABI declared in ``include/eigsol_hip.h``).

This module is plumbing: it loads the in-tree gfx950 library and declares every exported symbol.
It never falls back to a CPU implementation — if the library is missing or no gfx950 device is
visible, the calls raise :class:`EigSolError`.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("EIGSOL_LIB_PATH") or os.path.join(_HERE, "libeigsol_hip.so")   # override: A/B builds

EIGSOL_OK = 0
EIGSOL_E_NOT_SQUARE = 1
EIGSOL_E_ZERO_SIZE = 2
EIGSOL_E_SCALAR_MISMATCH = 3
EIGSOL_E_SIZE_MISMATCH = 4
EIGSOL_E_NOT_DENSE = 5
EIGSOL_E_SOLVER = 6
EIGSOL_E_HIP = 7
EIGSOL_E_RCCL = 8
EIGSOL_E_INVALID = 9
EIGSOL_E_NO_DEVICE = 10
EIGSOL_E_EMPTY = 11
EIGSOL_E_UNSUPPORTED = 12

EIGSOL_F64 = 0
EIGSOL_C128 = 1
EIGSOL_F32 = 2   # float (single-precision power / SpMV / triangular shifted inverse)
EIGSOL_C64 = 3   # std::complex<float>
EIGSOL_DD = 4    # long double, carried as double-double {hi, lo} (numpy longdouble: x87 80-bit)
EIGSOL_CDD = 5   # std::complex<long double>: {re.hi, re.lo, im.hi, im.lo}

EIGSOL_TRANSPORT_LOCAL = 0
EIGSOL_TRANSPORT_COLLECTIVE = 1
EIGSOL_TRANSPORT_PEER = 2

# int (*)(const void* send, void* recv, size_t bytes_per_rank, void* user)
ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p)

EIGSOL_QR_FRANCIS = 0
EIGSOL_QR_UNSHIFTED = 1


class EigSolError(RuntimeError):
    """A failing C-ABI call; ``status`` is the eigsol_status code."""

    def __init__(self, status: int, message: str):
        super().__init__(message)
        self.status = status


class SolverOptionsC(C.Structure):
    _fields_ = [("max_iterations", C.c_int32), ("tolerance", C.c_double)]


_vp = C.c_void_p
_i32 = C.c_int32
_i64 = C.c_int64
_pi32 = C.POINTER(C.c_int32)
_pi64 = C.POINTER(C.c_int64)
_pint = C.POINTER(C.c_int)
_pd = C.POINTER(C.c_double)
_ppv = C.POINTER(C.c_void_p)

# name -> argtypes (restype int unless listed in _RESTYPES)
SIGNATURES = {
    "eigsol_abi_version": [],
    "eigsol_status_string": [C.c_int],
    "eigsol_last_error": [],
    "eigsol_device_count": [_pint],
    "eigsol_ctx_create": [C.c_int, _ppv],
    "eigsol_ctx_destroy": [_vp],
    "eigsol_ctx_set_stream": [_vp, _vp],
    "eigsol_ctx_get_stream": [_vp, _ppv],
    "eigsol_ctx_synchronize": [_vp],
    "eigsol_malloc": [_vp, C.c_size_t, _ppv],
    "eigsol_free": [_vp, _vp],
    "eigsol_memcpy_h2d": [_vp, _vp, _vp, C.c_size_t],
    "eigsol_memcpy_d2h": [_vp, _vp, _vp, C.c_size_t],
    "eigsol_csr_create": [_vp, C.c_int, _i64, _i64, _i64, _vp, _vp, _vp, _ppv],
    "eigsol_csr_create_from_csc": [_vp, C.c_int, _i64, _i64, _i64, _vp, _vp, _vp, _ppv],
    "eigsol_csr_create_from_coo": [_vp, C.c_int, _i64, _i64, _i64, _vp, _vp, _vp, _ppv],
    "eigsol_csr_download": [_vp, _vp, _vp, _vp],
    "eigsol_csr_destroy": [_vp],
    "eigsol_csr_info": [_vp, _pi64, _pi64, _pi64, _pint],
    "eigsol_csr_spmv": [_vp, _vp, _vp],
    "eigsol_dense_create": [_vp, C.c_int, _i64, _i64, _vp, _ppv],
    "eigsol_dense_destroy": [_vp],
    "eigsol_dense_gemv": [_vp, _vp, _vp],
    "eigsol_power_csr": [_vp, C.POINTER(SolverOptionsC), _vp, _vp, _vp, _pi32, _pi32],
    "eigsol_power_dense": [_vp, C.POINTER(SolverOptionsC), _vp, _vp, _vp, _pi32, _pi32],
    "eigsol_power_create_csr": [_vp, _i32, _ppv],
    "eigsol_power_create_dense": [_vp, _i32, _ppv],
    "eigsol_power_destroy": [_vp],
    "eigsol_power_begin": [_vp, C.POINTER(SolverOptionsC), _vp, C.c_int],
    "eigsol_power_step": [_vp, _i32],
    "eigsol_power_query": [_vp, _pi32, _pi32],
    "eigsol_power_finish": [_vp, _vp, _vp, C.c_int, _pi32, _pi32],
    "eigsol_power_trace": [_vp, _vp, _i32, _pi32],
    "eigsol_power_kernel_info": [_vp, _pd, _pi32, _pi32, _pi32],
    "eigsol_power_kernel_name": [_vp, C.c_char_p, C.c_size_t],
    "eigsol_dist_unique_id_bytes": [],
    "eigsol_dist_get_unique_id": [_vp],
    "eigsol_dist_loopback_id": [C.c_int, _vp],
    "eigsol_ctx_create_dist": [C.c_int, C.c_int, C.c_int, _vp, _ppv],
    "eigsol_csr_create_dist": [_vp, C.c_int, _vp, _i64, _vp, _vp, _vp, _ppv],
    "eigsol_ghost_plan": [C.c_int, _vp, C.c_int, _i64, _vp, _vp, _pi64, _vp, _vp],
    "eigsol_exchange_mode": [C.c_int, _vp, _vp, C.POINTER(C.c_int)],
    "eigsol_csr_dist_info": [_vp, C.POINTER(C.c_int), _pi64],
    "eigsol_ctx_create_dist_host": [C.c_int, C.c_int, C.c_int, _vp, _vp, _ppv],
    "eigsol_power_transport": [_vp, C.POINTER(C.c_int)],
    "eigsol_peer_plan": [C.c_int, C.c_int, _vp, _vp, _vp, _i64, _vp],
    "eigsol_shifted_create_csr": [_vp, _vp, _i32, _ppv],
    "eigsol_shifted_create_dense": [_vp, _vp, _i32, _ppv],
    "eigsol_shifted_inverse_csr": [_vp, _vp, C.POINTER(SolverOptionsC), _vp, _vp, _vp, _pi32, _pi32],
    "eigsol_shifted_inverse_dense": [_vp, _vp, C.POINTER(SolverOptionsC), _vp, _vp, _vp, _pi32, _pi32],
    "eigsol_solve_shifted_csr": [_vp, _vp, _vp, _i64, _vp],
    "eigsol_solve_shifted_dense": [_vp, _vp, _vp, _i64, _vp],
    "eigsol_hessenberg_dense": [_vp, C.c_int, _i64, _vp, _vp],
    "eigsol_qr_decompose_dense": [_vp, C.c_int, _i64, _i64, _vp, _vp, _vp],
    "eigsol_qr_eigenvalues_dense": [_vp, C.c_int, _i64, _vp, C.POINTER(SolverOptionsC), C.c_int, _vp,
                                    _vp, _pi32, _pi32],
    "eigsol_hbm_probe": [_vp, C.c_size_t, C.c_int, _pd, _pd, _pd, _pint],
    "eigsol_hbm_probe_mix": [_vp, C.c_size_t, C.c_int, _pd, _pint],
    "eigsol_ctx_info": [_vp, _pint, _pint, _pint, _pint],
    "eigsol_sparse_lu_fill": [_i64, _vp, _vp, _i64, _pi64, _pi32],
    "eigsol_mf_analyze": [_i64, _vp, _vp, _i32, _i32, _vp, _vp, _i64, _pd],
}
_RESTYPES = {"eigsol_status_string": C.c_char_p, "eigsol_last_error": C.c_char_p}

_lib = None


def lib():
    """Load the gfx950 library (raises loudly if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise EigSolError(EIGSOL_E_NO_DEVICE,
                              f"{LIB_PATH} is missing: run __graft_entry__.build() (hipcc gfx950)")
        L = C.CDLL(LIB_PATH)
        for name, args in SIGNATURES.items():
            f = getattr(L, name)
            f.argtypes = args
            f.restype = _RESTYPES.get(name, C.c_int)
        _lib = L
    return _lib


def last_error() -> str:
    return lib().eigsol_last_error().decode(errors="replace")


def check(status: int, what: str = "") -> None:
    if status != EIGSOL_OK:
        raise EigSolError(status, f"{what}: {last_error()}" if what else last_error())


def call(name: str, *args) -> None:
    check(getattr(lib(), name)(*args), name)

"""The measurement entry points bench.py reports beside the roofline (include/eigsol_hip.h):
eigsol_hbm_probe (hand-written streaming kernels, probe.hip) and eigsol_ctx_info (the ranks the
library itself exchanges with)."""
import ctypes as C

import pytest

import pcsc_eigenvalue_solver_project_amd as E
from pcsc_eigenvalue_solver_project_amd import lib

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = E.Context(0)
    yield c
    c.close()


def test_hbm_probe_reports_rates(ctx):
    rd, cp, wr, b = C.c_double(), C.c_double(), C.c_double(), C.c_int()
    st = lib().eigsol_hbm_probe(ctx.handle, C.c_size_t(256 << 20), 2, C.byref(rd), C.byref(cp), C.byref(wr),
                                C.byref(b))
    assert st == 0
    # 256 MB fits the Infinity Cache, so only sanity bounds: positive, below any plausible cache rate
    for v in (rd.value, cp.value, wr.value):
        assert 100.0 < v < 60000.0, (rd.value, cp.value, wr.value)
    assert b.value in (1, 2, 4, 8)


def test_hbm_probe_rejects_bad_arguments(ctx):
    rd = C.c_double()
    assert lib().eigsol_hbm_probe(None, C.c_size_t(1 << 20), 1, C.byref(rd), None, None, None) == 9
    assert lib().eigsol_hbm_probe(ctx.handle, C.c_size_t(8), 1, C.byref(rd), None, None, None) == 9


def test_ctx_info_single_gpu(ctx):
    dev, rank, nranks, kind = C.c_int(-1), C.c_int(-1), C.c_int(-1), C.c_int(-1)
    assert lib().eigsol_ctx_info(ctx.handle, C.byref(dev), C.byref(rank), C.byref(nranks), C.byref(kind)) == 0
    assert (dev.value, rank.value, nranks.value, kind.value) == (0, 0, 1, 0)
    assert lib().eigsol_ctx_info(None, None, None, None, None) == 9

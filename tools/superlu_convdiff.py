"""CPU context figure for config5_convdiff_1M: scipy's SuperLU (supernodal LU with COLAMD column
ordering and threshold partial pivoting, the algorithm family of the reference's Eigen SparseLU,
solve_shifted.hpp:104-115) on the same permuted complex convection-diffusion matrix, one core:
factor time, one solve, and the factor's size.  Usage: python tools/superlu_convdiff.py [nx ...]"""
import os
import sys
import time

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as sla

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pcsc_eigenvalue_solver_project_amd import synthetic as S  # noqa: E402

for nx in [int(a) for a in sys.argv[1:]] or [300, 1000]:
    rp, ci, v = S.convdiff_complex(nx)
    n = nx * nx
    M = (sp.csr_matrix((v, ci, rp), shape=(n, n)) - (4.0 + 0.5j) * sp.identity(n, format="csr")).tocsc()
    t = time.perf_counter()
    lu = sla.splu(M, permc_spec="COLAMD")
    tf = time.perf_counter() - t
    b = S.start_vector(n, np.complex128)
    t = time.perf_counter()
    y = lu.solve(b)
    ts = time.perf_counter() - t
    res = np.linalg.norm(M @ y - b) / np.linalg.norm(b)
    print(f"nx={nx} n={n} superlu_factor_s={tf:.2f} solve_ms={ts * 1e3:.1f} fill={lu.L.nnz + lu.U.nnz} "
          f"relres={res:.1e} threads=1", flush=True)

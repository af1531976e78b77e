"""A/B of the GMRES family's host build of M = A - sigma I (gmres.hip): solutions of the general-sparse
1M matrix (exact LU) and the 300^2 convection-diffusion stencil (multifrontal LU) with the library
given by EIGSOL_LIB_PATH, saved for a bitwise comparison.  Usage: python tools/r06_buildM_ab.py OUT.npz"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pcsc_eigenvalue_solver_project_amd as E  # noqa: E402
from pcsc_eigenvalue_solver_project_amd import synthetic as S  # noqa: E402

ctx = E.Context(0)
out = {}
rp, ci, v, _ = S.general_complex(1_000_000, 16)
A = E.CsrMatrix(ctx, rp, ci, v, (len(rp) - 1, len(rp) - 1))
b = S.start_vector(len(rp) - 1, np.complex128, seed=3)
t = time.perf_counter()
out["general"] = E.solve_shifted(A, 1.5 * np.exp(0.7j) + 1e-3, b)
print("general solve_shifted %.3f s" % (time.perf_counter() - t), flush=True)
A.close()
rp, ci, v = S.convdiff_complex(300, seed=4)
n = 90000
A = E.CsrMatrix(ctx, rp, ci, v, (n, n))
out["convdiff"] = E.solve_shifted(A, 4.0 + 0.5j, S.start_vector(n, np.complex128, seed=11))
A.close()
np.savez(sys.argv[1], **out)
print("saved", flush=True)

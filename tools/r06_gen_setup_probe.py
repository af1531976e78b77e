"""Set-up laps of the 1M general-sparse (config 5 made non-triangular) shifted factor: EIGSOL_MF_DEBUG=1 python tools/r06_gen_setup_probe.py"""
import sys, time, os
import numpy as np
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import pcsc_eigenvalue_solver_project_amd as E
from pcsc_eigenvalue_solver_project_amd import synthetic as S
n = 1_000_000
rp, ci, v, _ = S.general_complex(n, 16)
ctx = E.Context(0)
A = E.CsrMatrix(ctx, rp, ci, v, (n, n))
sigma = 1.5 * np.exp(0.7j) + 1e-3
for rep in range(2):
    t = time.perf_counter(); s = E.ShiftedSession(A, sigma); print("factor", round(time.perf_counter() - t, 3), s.kernel_info()["variant"], flush=True); s.close()

"""Config 5's matrix made non-triangular (general sparse, ILU(0)-GMRES): ms per shifted-inverse
iteration, Arnoldi steps of the last solve, eigenvalue error, with and without the warm start."""
import json, os, sys, time
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np
import pcsc_eigenvalue_solver_project_amd as E
from pcsc_eigenvalue_solver_project_amd import synthetic as S
ctx = E.Context(0)
n = 1_000_000
rp, ci, v, _ = S.general_complex(n, 16)
target = 1.5 * np.exp(0.7j)
sigma = target + 1e-3
x0 = S.start_vector(n, np.complex128)
A = E.CsrMatrix(ctx, rp, ci, v, (n, n))
warm = os.environ.get("EIGSOL_GMRES_WARM", "default")   # read once per process: set it outside
for rep in range(2):   # the first session pays first-launch costs
    sess = E.ShiftedSession(A, sigma, trace_capacity=64)
    sess.begin(E.ShiftedSolverOptions(1000, 1e-12, sigma), x0)
    t = time.perf_counter()
    done = False
    steps = []
    while not done:
        sess.step(1)
        done, _ = sess.query()
        steps.append(sess.kernel_info()["tiles"])
    res = sess.finish()
    dt = time.perf_counter() - t
    print(json.dumps({"warm_env": warm, "iterations": res.iterations, "ms_per_iteration": round(1e3 * dt / res.iterations, 3),
                      "arnoldi_steps_per_solve": steps, "err": float(abs(res.eigenvalue - target))}), flush=True)
    sess.close()

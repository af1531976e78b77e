"""Dense solve_shifted timing (blocked LU on the device + one substitution): n, seconds, TF/s of the LU."""
import json, sys, time
import numpy as np
ROOT = __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))
sys.path.insert(0, ROOT)
import pcsc_eigenvalue_solver_project_amd as E

ctx = E.Context(0)
for spec in sys.argv[1:] or ["4096:f64", "8192:f64", "16384:f64", "8192:c128"]:
    n, dt = spec.split(":")
    n = int(n)
    dtype = np.float64 if dt == "f64" else np.complex128
    rng = np.random.default_rng(1)
    A = rng.standard_normal((n, n)).astype(dtype)
    b = rng.standard_normal(n).astype(dtype)
    D = E.DenseMatrix(ctx, A)
    E.solve_shifted(E.DenseMatrix(ctx, A[:256, :256].copy()), 0.5, b[:256])   # warm-up
    t = time.perf_counter()
    x = E.solve_shifted(D, 0.5, b)
    dtm = time.perf_counter() - t
    fl = (2 / 3) * n ** 3 * (4 if dtype == np.complex128 else 1)
    r = float(np.linalg.norm(A @ x - 0.5 * x - b) / (np.linalg.norm(A, 1) * np.linalg.norm(x)))
    print(json.dumps({"n": n, "dtype": dt, "seconds": round(dtm, 4), "lu_TFLOPs_incl_solve": round(fl / dtm / 1e12, 2),
                      "rel_residual": r}), flush=True)
    D.close()
ctx.close()

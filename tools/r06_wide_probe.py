"""Timing of the double-double (long double) solvers at moderate sizes, host in/out:
to_hessenberg, qr_decompose, qr_eigenvalues (Francis + Newton refinement) on N(0,1) matrices."""
import json, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import pcsc_eigenvalue_solver_project_amd as E

ctx = E.Context(0)
for n in [int(a) for a in sys.argv[1:]] or [256, 1024]:
    A = np.random.default_rng(n).standard_normal((n, n)).astype(np.longdouble)
    out = {"n": n}
    t = time.perf_counter(); E.to_hessenberg(ctx, A); out["to_hessenberg_s"] = round(time.perf_counter() - t, 3)
    t = time.perf_counter(); E.qr_decompose(ctx, A); out["qr_decompose_s"] = round(time.perf_counter() - t, 3)
    t = time.perf_counter(); r = E.qr_eigenvalues(ctx, A, E.SolverOptions(1000, 1e-12)); out["qr_eigenvalues_s"] = round(time.perf_counter() - t, 3)
    out["converged"] = bool(r.converged)
    print(json.dumps(out), flush=True)
ctx.close()

"""A/B for the QR eigenvalue path: eigenvalues (bitwise) and wall time with the library at
EIGSOL_LIB_PATH (default: the in-tree build).  usage: python tools/qr_ab.py OUT.npz"""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import pcsc_eigenvalue_solver_project_amd as E
from pcsc_eigenvalue_solver_project_amd import synthetic as S

ctx = E.Context(0)
out = {}
sizes = [int(v) for v in os.environ.get("QR_AB_SIZES", "60,128,512,4096,-200,-1024").split(",")]
for n in sizes:     # negative: complex N(0,1)
    rng = np.random.default_rng(abs(n))
    A = rng.standard_normal((n, n)) if n > 0 else rng.standard_normal((-n, -n)) + 1j * rng.standard_normal((-n, -n))
    best = 1e9
    for rep in range(2 if abs(n) >= 1024 else 3):
        t = time.perf_counter()
        r = E.qr_eigenvalues(ctx, A, E.SolverOptions(1000, 1e-10))
        best = min(best, time.perf_counter() - t)
    out[f"ev{n}"] = np.asarray(r.eigenvalues_complex)
    out[f"t{n}"] = best
    print(n, f"{best:.4f}s", r.iterations, r.converged, flush=True)
np.savez(sys.argv[1], **out)

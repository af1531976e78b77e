"""Time the blocked Hessenberg reduction alone (host in/out)."""
import json, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import pcsc_eigenvalue_solver_project_amd as E
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
ctx = E.Context(0)
A = np.asfortranarray(np.random.default_rng(20251226).standard_normal((n, n)))   # column-major, like Matrix::Dense
E.to_hessenberg(ctx, A[:300, :300].copy())
for rep in range(2):
    t = time.perf_counter()
    H = E.to_hessenberg(ctx, A)
    print(json.dumps({"n": n, "rep": rep, "seconds": time.perf_counter() - t}), flush=True)
ctx.close()

"""to_hessenberg past the cooperative panel's size limit (real > 8192, complex > 4096): host in/out seconds.
Usage: python tools/r06_hess_large_probe.py f64:12288 c128:6144 ..."""
import json, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import pcsc_eigenvalue_solver_project_amd as E

ctx = E.Context(0)
for spec in sys.argv[1:]:
    dt, n = spec.split(":")
    n = int(n)
    rng = np.random.default_rng(n)
    A = rng.standard_normal((n, n))
    if dt == "c128":
        A = A + 1j * rng.standard_normal((n, n))
    A = np.asfortranarray(A)
    t = time.perf_counter()
    H = E.to_hessenberg(ctx, A)
    print(json.dumps({"dtype": dt, "n": n, "seconds": round(time.perf_counter() - t, 3),
                      "below_subdiag_max": float(np.abs(np.tril(H, -2)).max())}), flush=True)
ctx.close()

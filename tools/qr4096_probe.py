"""bench.py's config-2 QR (4096^2 N(0,1), seed 20251226, column-major) timed REPS times in one
process: python tools/qr4096_probe.py [reps]; knobs come from the environment."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import pcsc_eigenvalue_solver_project_amd as E

ctx = E.Context(0)
n = int(os.environ.get("QR_N", 4096))
A = np.asfortranarray(np.random.default_rng(20251226).standard_normal((n, n)))
E.qr_eigenvalues(ctx, A[:256, :256].copy())
ts = []
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    t = time.perf_counter()
    r = E.qr_eigenvalues(ctx, A)
    ts.append(time.perf_counter() - t)
ev = np.sort_complex(np.asarray(r.eigenvalues_complex))
print({k: v for k, v in os.environ.items() if k.startswith("EIGSOL_")}, "n", n, "times", [round(t, 3) for t in ts],
      "iters", r.iterations, "evsum", complex(ev.sum()), flush=True)

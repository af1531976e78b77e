"""Complex QR tuning grid: bulges per sweep x concurrent chains (EIGSOL_ZQR_NB / EIGSOL_ZQR_GROUPS are read
once per process, so each point runs in its own process).  usage: python tools/zqr_grid.py [n]"""
import os, subprocess, sys
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
code = f"""
import sys, time, numpy as np
sys.path.insert(0, {os.path.dirname(os.path.dirname(os.path.abspath(__file__)))!r})
import pcsc_eigenvalue_solver_project_amd as E
rng = np.random.default_rng({n}); A = rng.standard_normal(({n}, {n})) + 1j * rng.standard_normal(({n}, {n}))
ref = np.load(sys.argv[1]) if len(sys.argv) > 1 else None
ctx = E.Context(0); best = 1e9
for _ in range(2):
    t = time.perf_counter(); r = E.qr_eigenvalues(ctx, A, E.SolverOptions(1000, 1e-10)); best = min(best, time.perf_counter() - t)
ev = np.asarray(r.eigenvalues_complex)
print(f"{{best:.4f}} s iters={{r.iterations}} conv={{r.converged}}", flush=True)
"""
for nb in (16, 24, 32):
    for g in (2, 3, 4):
        env = dict(os.environ, EIGSOL_ZQR_NB=str(nb), EIGSOL_ZQR_GROUPS=str(g))
        out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
        print(f"nb={nb} groups={g}: {out.stdout.strip()} {out.stderr.strip()[-200:]}", flush=True)

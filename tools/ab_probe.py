"""A/B probe: fused band10m power iteration (f64 and f32) with the library at EIGSOL_LIB_PATH."""
import sys, os, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import pcsc_eigenvalue_solver_project_amd as E
from pcsc_eigenvalue_solver_project_amd import synthetic as S
st = torch.cuda.Stream(); torch.cuda.set_stream(st)
ctx = E.Context(0, stream=st.cuda_stream)
n, k = 10_000_000, 10
rp, ci, v = S.band(n, k)
for dt in (np.float64, np.float32):
    A = E.CsrMatrix(ctx, rp, ci, v.astype(dt), (n, n))
    s = E.PowerSession(A); s.begin(E.SolverOptions(2**31-1, -1.0), S.start_vector(n, dt)); s.step(10)
    best = 1e9
    for rep in range(3):
        torch.cuda.synchronize(); e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st); s.step(200); e1.record(st); torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / 200)
    print(json.dumps({"lib": os.environ.get("EIGSOL_LIB_PATH", "tree"), "dtype": np.dtype(dt).name, "us": round(best * 1e3, 1)}), flush=True)
    s.close(); A.close()

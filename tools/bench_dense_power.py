"""Dense power iteration (column-major fp64 / c128 GEMV fused with the norm and Rayleigh partials):
per-iteration time and algorithmic GB/s (8 n^2 + 16 n bytes) at the given sizes."""
import json, sys
import numpy as np
ROOT = __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
import pcsc_eigenvalue_solver_project_amd as E
from pcsc_eigenvalue_solver_project_amd import synthetic as S

st = torch.cuda.Stream()
torch.cuda.set_stream(st)
ctx = E.Context(0, stream=st.cuda_stream)
for spec in sys.argv[1:] or ["16384:f64", "32768:f64", "16384:c128"]:
    n, dt = spec.split(":")
    n = int(n)
    dtype = np.float64 if dt == "f64" else np.complex128
    A = np.random.default_rng(1).standard_normal((n, n)).astype(dtype)
    D = E.DenseMatrix(ctx, A)
    del A
    s = E.PowerSession(D)
    s.begin(E.SolverOptions(2**31 - 1, -1.0), S.start_vector(n, dtype))
    s.step(5)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    s.step(50)
    e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 50
    info = s.kernel_info()
    print(json.dumps({"n": n, "dtype": dt, "ms_per_iteration": round(ms, 4),
                      "GBps": round(info["bytes_per_iteration"] / ms / 1e6, 1), "kernel": info["kernel"]}), flush=True)
    s.close()
    D.close()
ctx.close()

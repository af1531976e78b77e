"""A/B of the headline slice kernel's workgroups per CU (EIGSOL_CSR_BLOCKS_PER_CU; default cap 2 for
the sliced layout) on band10m (10M x 10M, 10 nnz/row): ms per fused iteration and algorithmic GB/s."""
import json, os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch
import pcsc_eigenvalue_solver_project_amd as E
from pcsc_eigenvalue_solver_project_amd import synthetic as S
st = torch.cuda.Stream(); torch.cuda.set_stream(st)
ctx = E.Context(0, stream=st.cuda_stream)
import numpy as np
n, k = 10_000_000, 10
dt = np.float32 if (len(sys.argv) > 1 and sys.argv[1] == "f32") else np.float64
rp, ci, v = S.band(n, k)
v = v.astype(dt)
x = S.start_vector(n).astype(dt)
A = E.CsrMatrix(ctx, rp, ci, v, (n, n))
for bpc in ("2", "3", "4", "6", "2"):
    os.environ["EIGSOL_CSR_BLOCKS_PER_CU"] = bpc
    s = E.PowerSession(A); s.begin(E.SolverOptions(2**31 - 1, -1.0), x); s.step(10)
    torch.cuda.synchronize()
    best = 1e9
    for rep in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st); s.step(100); e1.record(st); torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / 100)
    info = s.kernel_info()
    print(json.dumps({"dtype": np.dtype(dt).name, "blocks_per_cu": bpc, "ms": round(best, 5), "GBps": round(info["bytes_per_iteration"] / best / 1e6, 1),
                      "grid": info["grid"]}), flush=True)
    s.close()
A.close()

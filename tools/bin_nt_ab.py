"""A/B of the column-binned kernel's workgroup size at 153 KB row-sum chunks (uniform10m, 10M x 10
uniform columns): EIGSOL_CSR_BIN_NT = 1024 / 512 / 256 -> ms per fused iteration, algorithmic GB/s,
bitwise product against the first variant."""
import json, os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np, torch
import pcsc_eigenvalue_solver_project_amd as E
from pcsc_eigenvalue_solver_project_amd import synthetic as S
st = torch.cuda.Stream(); torch.cuda.set_stream(st)
ctx = E.Context(0, stream=st.cuda_stream)
n, k = 10_000_000, 10
rp, ci, v = S.uniform(n, k)
x = S.start_vector(n)
ref = None
for nt, xb in (("1024", "1048576"), ("1024", "524288"), ("1024", "2097152"), ("1024", "4194304"), ("1024", "1048576")):
    os.environ["EIGSOL_CSR_BIN_LDS"] = "153"
    os.environ["EIGSOL_CSR_BIN_NT"] = nt
    os.environ["EIGSOL_CSR_BIN_BYTES"] = xb
    A = E.CsrMatrix(ctx, rp, ci, v, (n, n))
    xd, yd = ctx.malloc(8 * n), ctx.malloc(8 * n)
    ctx.h2d(xd, x)
    A.spmv(xd, yd)
    y = np.empty(n)
    ctx.d2h(y, yd)
    ctx.free(xd); ctx.free(yd)
    same = None if ref is None else bool(np.array_equal(y, ref))
    if ref is None:
        ref = y
    s = E.PowerSession(A); s.begin(E.SolverOptions(2**31 - 1, -1.0), x); s.step(5)
    torch.cuda.synchronize()
    best = 1e9
    for rep in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st); s.step(40); e1.record(st); torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / 40)
    info = s.kernel_info()
    print(json.dumps({"nt": nt, "x_block_bytes": xb, "ms": round(best, 4), "GBps": round(info["bytes_per_iteration"] / best / 1e6, 1),
                      "chunks": info["tiles"], "grid": info["grid"], "bitwise_same_as_first": same}), flush=True)
    s.close(); A.close()

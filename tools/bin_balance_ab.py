"""A/B of the column-binned chunk schedules on uniform-column matrices (config 3 1M x 16, config 4's
uniform10m): (LDS KB of row sums, balanced chunk count) -> ms per fused iteration, algorithmic
GB/s, and the bitwise product against the first variant's (the row sums' order is the same)."""
import json, os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np, torch
import pcsc_eigenvalue_solver_project_amd as E
from pcsc_eigenvalue_solver_project_amd import synthetic as S
st = torch.cuda.Stream(); torch.cuda.set_stream(st)
ctx = E.Context(0, stream=st.cuda_stream)
variants = [("64", "0"), ("64", "1"), ("128", "1"), ("153", "1"), ("16", "1")]
for n, k in [(1_000_000, 16), (10_000_000, 10)]:
    rp, ci, v = S.uniform(n, k)
    x = S.start_vector(n)
    ref = None
    for lds, bal in variants:
        os.environ["EIGSOL_CSR_BIN_LDS"] = lds
        os.environ["EIGSOL_CSR_BIN_BALANCE"] = bal
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
        print(json.dumps({"n": n, "k": k, "lds_kb": lds, "balanced": bal, "ms": round(best, 4),
                          "GBps": round(info["bytes_per_iteration"] / best / 1e6, 1), "chunks": info["tiles"],
                          "grid": info["grid"], "bitwise_same_as_first": same}), flush=True)
        s.close(); A.close()

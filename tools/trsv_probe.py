"""Sync-free triangular solve probe: per-row throughput vs dependency-chain latency."""
import json, sys, time
import numpy as np
ROOT = __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
import pcsc_eigenvalue_solver_project_amd as E
from pcsc_eigenvalue_solver_project_amd import synthetic as S

st = torch.cuda.Stream()
torch.cuda.set_stream(st)
ctx = E.Context(0, stream=st.cuda_stream)
rng = np.random.default_rng(1)


def csr_from_rows(n, cols_per_row, vals=None):
    lens = np.array([len(c) for c in cols_per_row])
    rp = np.zeros(n + 1, dtype=np.int32)
    rp[1:] = np.cumsum(lens)
    ci = np.concatenate(cols_per_row).astype(np.int32)
    v = (rng.uniform(-1, 1, len(ci)) + 1j * rng.uniform(-1, 1, len(ci))) * 0.05
    v[rp[:-1]] = 2.0 + 0.5j
    return rp, ci, v


def run(name, rp, ci, v, n, steps=20):
    M = E.CsrMatrix(ctx, rp, ci, v, (n, n))
    s = E.ShiftedSession(M, 0.1 + 0.1j)
    s.begin(E.ShiftedSolverOptions(2**31 - 1, -1.0, 0.1 + 0.1j), S.start_vector(n, np.complex128))
    s.step(3)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    s.step(steps)
    e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    info = s.kernel_info()
    print(json.dumps({"case": name, "n": n, "ms": round(ms, 4), "levels": info["tiles"],
                      "GBps": round(info["bytes_per_iteration"] / ms / 1e6, 1)}), flush=True)
    s.close(); M.close()


n = 1_000_000
# (a) diagonal only: one level, no waits
rp = np.arange(n + 1, dtype=np.int32); ci = np.arange(n, dtype=np.int32)
v = np.full(n, 2.0 + 0.5j)
run("diag", rp, ci, v, n)
# (b) two levels: rows < n/2 read 15 rows of [n/2, n); the rest diagonal
h = n // 2
off = np.sort(rng.integers(h, n, (h, 15)), axis=1)
rows = [np.concatenate([[i], np.unique(off[i])]) for i in range(h)] + [np.array([i]) for i in range(h, n)]
rp, ci, v = csr_from_rows(n, rows)
run("two_levels", rp, ci, v, n)
# (c) chain of L levels at the bottom: rows n-L..n-1 bidiagonal, others diagonal
for L in (64, 256):
    rows = [np.array([i]) for i in range(n - L)] + [np.array([i, i + 1]) if i + 1 < n else np.array([i]) for i in range(n - L, n)]
    rp, ci, v = csr_from_rows(n, rows)
    run(f"chain{L}", rp, ci, v, n)
# (d) config 5
rp, ci, v, _ = S.triu_complex(n, 16)
run("config5", rp, ci, v, n)
ctx.close()

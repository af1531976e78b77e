"""Gather-bound SpMV probe: uniform-column CSR at several sizes, and the same 1M matrix split into
column blocks (each block's slice of x fits one XCD's L2).  Prints us per product."""
import sys
import time
import numpy as np
import torch
import pcsc_eigenvalue_solver_project_amd as E
from pcsc_eigenvalue_solver_project_amd import synthetic as S


def timed(torch, fn, reps=200):
    fn(); ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    ctx.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


ctx = E.Context(0)
for n in (250_000, 500_000, 1_000_000, 2_000_000, 4_000_000):
    rp, ci, v = S.uniform(n, 16)
    A = E.CsrMatrix(ctx, rp, ci, v, (n, n))
    xd = ctx.malloc(n * 8); yd = ctx.malloc(n * 8)
    ctx.h2d(xd, np.ones(n))
    us = timed(torch, lambda: A.spmv(xd, yd))
    print(f"uniform n={n:8d} k=16: {us:8.1f} us  {us * 1e3 / (n * 16):.2f} ns/nnz", flush=True)
    A.close(); ctx.free(xd); ctx.free(yd)

n = 1_000_000
rp, ci, v = S.uniform(n, 16)
xd = ctx.malloc(n * 8); yd = ctx.malloc(n * 8)
ctx.h2d(xd, np.ones(n))
rows = np.repeat(np.arange(n), 16)
for nb in (2, 4, 8):
    mats = []
    for b in range(nb):
        lo, hi = b * n // nb, (b + 1) * n // nb
        m = (ci >= lo) & (ci < hi)
        cnt = np.bincount(rows[m], minlength=n)
        rpb = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int32)
        mats.append(E.CsrMatrix(ctx, rpb, ci[m], v[m], (n, n)))
    us = timed(torch, lambda: [M.spmv(xd, yd) for M in mats])
    print(f"uniform 1M split into {nb} column blocks: {us:8.1f} us", flush=True)
    for M in mats:
        M.close()
ctx.close()

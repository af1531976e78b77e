#!/usr/bin/env python3
"""Config 5 (1M complex upper-triangular, 16 nnz/row): time of the triangular factor's set-up
(ShiftedSession create: analysis + layout) on the device (default) and on the host
(EIGSOL_TRSV_HOST=1), and the end-to-end converged solve; checks that both builds give bitwise
the same solution."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pcsc_eigenvalue_solver_project_amd as E  # noqa: E402
from pcsc_eigenvalue_solver_project_amd import synthetic as S  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
ctx = E.Context(0)
rp, ci, v, _ = S.triu_complex(n, 16)
target = 1.5 * np.exp(0.7j)
sigma = target + 1e-3
x0 = S.start_vector(n, np.complex128)
A = E.CsrMatrix(ctx, rp, ci, v, (n, n))
out = {}
for mode in ("device", "host", "device"):   # the first pass loads the modules
    if mode == "host":
        os.environ["EIGSOL_TRSV_HOST"] = "1"
    else:
        os.environ.pop("EIGSOL_TRSV_HOST", None)
    t0 = time.perf_counter()
    s = E.ShiftedSession(A, sigma)
    t1 = time.perf_counter()
    s.begin(E.ShiftedSolverOptions(1000, 1e-12, sigma), x0)
    s.step(3)
    done, _ = s.query()
    while not done:
        s.step(2)
        done, _ = s.query()
    r = s.finish()
    t2 = time.perf_counter()
    info = s.kernel_info()
    s.close()
    out[mode] = {"create_s": round(t1 - t0, 4), "end_to_end_s": round(t2 - t0, 4), "iterations": r.iterations,
                 "eigenvalue": [r.eigenvalue.real, r.eigenvalue.imag], "variant": info["variant"],
                 "x": r.eigenvector}
assert np.array_equal(out["device"]["x"], out["host"]["x"]), "device and host builds differ"
for m in out.values():
    m.pop("x")
print(json.dumps({"n": n, **out}))

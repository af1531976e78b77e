"""long double power iteration on the 1M band matrix (bench.py's long_double_band1m), for a kernel trace:
python tools/r06_dd_power_prof.py [iterations]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pcsc_eigenvalue_solver_project_amd as E  # noqa: E402
from pcsc_eigenvalue_solver_project_amd import synthetic as S  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 30
n = 1_000_000
ctx = E.Context(0)
rp, ci, v = S.band(n, int(os.environ.get("DD_K", "10")))
A = E.CsrMatrix(ctx, rp, ci, v.astype(np.longdouble), (n, n))
sess = E.PowerSession(A)
sess.begin(E.SolverOptions(2**31 - 1, -1.0), S.start_vector(n).astype(np.longdouble))
sess.step(3)
ctx.synchronize()
t = time.perf_counter()
sess.step(iters)
ctx.synchronize()
print("ms per iteration %.4f" % ((time.perf_counter() - t) / iters * 1e3), flush=True)
sess.close()
A.close()
ctx.close()

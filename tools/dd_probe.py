"""Double-double (long double) power iteration speed on a band matrix: bench.py's
long_double_band1m extra on its own.  Usage: python tools/dd_probe.py [n]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
import pcsc_eigenvalue_solver_project_amd as E  # noqa: E402
from pcsc_eigenvalue_solver_project_amd import synthetic as S  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
ctx = E.Context(0)
print(json.dumps(bench.run_long_double_power(E, S, ctx, torch, n=n)))

#!/usr/bin/env python3
"""Profiling driver: N fused power iterations of a bench workload (no CPU baseline, no JSON)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import pcsc_eigenvalue_solver_project_amd as E  # noqa: E402
from pcsc_eigenvalue_solver_project_amd import synthetic as S  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--workload", default="band10m")
p.add_argument("--steps", type=int, default=20)
args = p.parse_args()
kind, rows, k = {"band10m": ("band", 10_000_000, 10), "uniform1m": ("uniform", 1_000_000, 16),
                 "band1m": ("band", 1_000_000, 16), "uniform10m": ("uniform", 10_000_000, 10)}[args.workload]
gen = S.band if kind == "band" else S.uniform
rp, ci, v = gen(rows, k)
ctx = E.Context(0)
A = E.CsrMatrix(ctx, rp, ci, v, (rows, rows))
s = E.PowerSession(A)
s.begin(E.SolverOptions(2**31 - 1, -1.0), S.start_vector(rows))
s.step(args.steps)
ctx.synchronize()
print("done", s.kernel_info())

"""Config-5 shifted inverse (1M complex triangular) and the general-sparse GMRES extra, timed as
bench.py times them, under the current environment (A/B of EIGSOL_TRSV_* knobs)."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
import bench
import pcsc_eigenvalue_solver_project_amd as E
from pcsc_eigenvalue_solver_project_amd import synthetic as S
st = torch.cuda.Stream(); torch.cuda.set_stream(st)
ctx = E.Context(0, stream=st.cuda_stream)
tag = {k: v for k, v in os.environ.items() if k.startswith("EIGSOL_TRSV")}
r5 = bench.run_config5(E, S, ctx, torch, st, True)
print(json.dumps({"env": tag, "config5_ms": r5.get("ms_per_iteration"), "converged": r5.get("converged")}), flush=True)
if len(sys.argv) > 1:
    rg = bench.run_config5_general(E, S, ctx)
    print(json.dumps({"env": tag, "gmres_ms": rg.get("ms_per_iteration"), "converged": rg.get("converged")}), flush=True)

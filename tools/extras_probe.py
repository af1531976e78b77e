"""Run selected bench.py extras legs alone: python tools/extras_probe.py config5 config5_general"""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
import bench as B
import pcsc_eigenvalue_solver_project_amd as E
from pcsc_eigenvalue_solver_project_amd import synthetic as S

st = torch.cuda.Stream()
torch.cuda.set_stream(st)
ctx = E.Context(0, stream=st.cuda_stream)
for name in sys.argv[1:]:
    if name == "config5":
        r = B.run_config5(E, S, ctx, torch, st, True)
    elif name == "config5_general":
        r = B.run_config5_general(E, S, ctx)
    else:
        raise SystemExit("unknown leg " + name)
    print(json.dumps({name: r}), flush=True)
ctx.close()

"""Print the library's HBM probe (eigsol_hbm_probe): read / copy / write GB/s and the best read grid."""
import ctypes as C, os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import pcsc_eigenvalue_solver_project_amd as E
from pcsc_eigenvalue_solver_project_amd import lib
ctx = E.Context(0)
rd, cp, wr, b = C.c_double(), C.c_double(), C.c_double(), C.c_int()
st = lib().eigsol_hbm_probe(ctx.handle, C.c_size_t(2 << 30), 10, C.byref(rd), C.byref(cp), C.byref(wr), C.byref(b))
print({"status": st, "read_GBps": rd.value, "copy_GBps": cp.value, "write_GBps": wr.value, "read_blocks_per_cu": b.value})

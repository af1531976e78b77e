#!/usr/bin/env python3
"""Benchmark of the MI355X power-iteration hot path (BASELINE.json metric).

metric : "power-iteration SpMV GB/s vs HBM roofline + eigvals/sec (QR), 1/2/4/8 GPU"
step   : one fused power iteration (y = A x / ||.||, ||y||^2, x^H y, device-side convergence
         test) over the workload's CSR matrix — powerMethodImpl's loop body
         (src/power_method/power_method.hpp:68-96) with the redundant second product fused away.
workload (default): BASELINE config "10M x 10M CSR ~10 nnz/row fp64, power_method row-sharded"
         — per GPU a 10,000,000-row block of the band generator, weak scaling:
         N GPUs hold an (N*10M) x (N*10M) matrix, one row block per rank.
value  : algorithmic bytes (12 nnz + 4 (n+1) + 16 n per iteration) x iterations
         x ranks / max-over-ranks wall time of the K timed iterations; inputs resident in HBM.

Run: python bench.py [--gpus N --steps K --warmup W]  (N>1 under torch.distributed.run).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "power-iteration SpMV GB/s vs HBM roofline + eigvals/sec (QR), 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)

WORKLOADS = {
    # name: (generator, rows per rank, nnz per row)
    "band10m": ("band", 10_000_000, 10),
    "uniform10m": ("uniform", 10_000_000, 10),
    "uniform1m": ("uniform", 1_000_000, 16),
    "band1m": ("band", 1_000_000, 16),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--workload", default="band10m", choices=sorted(WORKLOADS))
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--extras", action="store_true", help="also time config 3 (1M x 16 uniform)")
    return p.parse_args()


def gen(kind, n_global, k, row0, nrows):
    from pcsc_eigenvalue_solver_project_amd import synthetic as S
    if kind == "band":
        return S.band(n_global, k, row0=row0, nrows=nrows)
    return S.uniform(n_global, k, row0=row0, nrows=nrows)


def pmc_traffic(workload, kernel):
    """HBM bytes per launch of the same kernel on the same workload, from the committed rocprofv3
    PMC summary (profiles/, FETCH_SIZE x 2 + WRITE_SIZE per MI355X_MICROARCH.md); PMC counters
    cannot be read from inside a timed run, so the profile is a separate pass of this workload."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{workload}_*.json"))):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        kn = d.get("kernel") or ""
        if "hbm_traffic_bytes_per_launch" in d and kernel.split(" ")[0] in kn:
            best = {"hbm_traffic_bytes_per_launch": round(d["hbm_traffic_bytes_per_launch"]),
                    "source": os.path.relpath(f, ROOT)}
    return best


def cpu_baseline(kind, k, budget_s):
    """Reference algorithm (two CSC products per iteration, single thread) on a bounded sample."""
    from oracle import oracle as O
    from pcsc_eigenvalue_solver_project_amd import synthetic as S
    n = 1_000_000
    rp, ci, v = gen(kind, n, k, 0, n)
    cp, ri, vv = O.csr_to_csc(rp, ci, v, n)
    x0 = S.start_vector(n)
    t = time.perf_counter()
    O.power_csc(cp, ri, vv, x0, 2, -1.0)
    per_iter = (time.perf_counter() - t) / 2
    iters = max(3, int(budget_s / max(per_iter, 1e-6)))
    t = time.perf_counter()
    O.power_csc(cp, ri, vv, x0, iters, -1.0)
    dt = time.perf_counter() - t
    nbytes = S.csr_bytes_per_iteration(n, len(ci))
    return {
        "value": nbytes * iters / dt / 1e9,
        "unit": "GB/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{kind} {n}x{n}, {k} nnz/row (same generator), {iters} reference power "
                  f"iterations (2 CSC-scatter products each, oracle/eigsol_oracle.cpp, -O3, 1 thread), "
                  f"{dt:.1f}s",
        "ms_per_iteration": 1e3 * dt / iters,
    }


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("bench.py --gpus N>1 must run under torch.distributed.run")
    import torch
    import torch.distributed as dist

    if world > 1:
        dist.init_process_group("gloo")
    torch.cuda.set_device(local_rank)

    import pcsc_eigenvalue_solver_project_amd as E
    from pcsc_eigenvalue_solver_project_amd import synthetic as S

    kind, rows, k = WORKLOADS[args.workload]
    n_global = rows * world
    row0 = rows * rank
    # A dedicated (non-default) torch stream: the library's work and torch's timing events share it.
    torch_stream = torch.cuda.Stream()
    torch.cuda.set_stream(torch_stream)
    rp, ci, v = gen(kind, n_global, k, row0, rows)
    if world > 1:
        # one communicator per rank owned by the library (RCCL over xGMI); gloo only ships the id
        from pcsc_eigenvalue_solver_project_amd import dist as D
        ctx = D.torch_dist_context(local_rank, stream=torch_stream.cuda_stream)
        A, sess = D.sharded_power_session(ctx, rp, ci, v, n_global, row0)
    else:
        ctx = E.Context(local_rank, stream=torch_stream.cuda_stream)
        A = E.CsrMatrix(ctx, rp, ci, v, (rows, rows))
        sess = E.PowerSession(A)
    nnz = len(ci)
    del rp, ci, v
    x0 = S.start_vector(rows, np.float64, row0=row0)
    opts = E.SolverOptions(2**31 - 1, -1.0)   # tol < 0: the reference loop never stops early
    sess.begin(opts, x0)
    info = sess.kernel_info()
    sess.step(args.warmup)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(torch_stream)
    sess.step(args.steps)
    ev1.record(torch_stream)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    elapsed = t1 - t0
    ev_ms = ev0.elapsed_time(ev1)
    done, launches = sess.query()
    assert not done, "tol < 0 must never terminate"
    el = torch.tensor([elapsed, ev_ms / 1e3], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed_max, ev_max = float(el[0]), float(el[1])

    bytes_iter = info["bytes_per_iteration"]          # this rank's algorithmic bytes
    total_bytes = bytes_iter * args.steps * world
    value = total_bytes / elapsed_max / 1e9
    achieved = bytes_iter / (ev_ms / 1e3 / args.steps) / 1e9

    out = None
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed_max / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded generators of SURVEY §8d; x0 seed 7)",
            "config": {
                "workload": f"power_method CSR {args.workload}: {rows} rows x {k} nnz/row per GPU "
                            f"({kind} columns), global {n_global}x{n_global}",
                "rows_per_gpu": rows,
                "nnz_per_gpu": nnz,
                "n_global": n_global,
                "parallelism": f"row-block x{world}" if world > 1 else "single GPU",
                "bytes_per_iteration_per_gpu": bytes_iter,
                "grid_blocks": info["grid"],
                "row_tiles": info["tiles"],
            },
            "roofline": {
                "bound": "hbm",
                "kernel": info["kernel"] + ", fused power iteration",
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": None,
                "event_ms_per_launch": round(ev_ms / args.steps, 5),
                "algorithmic_bytes_per_launch": bytes_iter,
            },
            "cpu_baseline": None,
        }
    if rank == 0:
        pmc = pmc_traffic(args.workload, info["kernel"])
        if pmc:
            out["roofline"]["traffic"] = pmc["hbm_traffic_bytes_per_launch"]
            out["roofline"]["traffic_source"] = pmc["source"]
    if args.extras and world == 1:
        # config 3: 1M x 1M uniform, 16 nnz/row (working set < Infinity Cache: may exceed HBM bound)
        rp3, ci3, v3 = S.uniform(1_000_000, 16)
        A3 = E.CsrMatrix(ctx, rp3, ci3, v3, (1_000_000, 1_000_000))
        s3 = E.PowerSession(A3)
        s3.begin(opts, S.start_vector(1_000_000))
        s3.step(20)
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(torch_stream)
        s3.step(200)
        e1.record(torch_stream)
        torch.cuda.synchronize()
        b3 = s3.kernel_info()["bytes_per_iteration"]
        ms3 = e0.elapsed_time(e1) / 200
        out["extras"] = {"config3_uniform_1Mx16": {"GB/s": round(b3 / (ms3 / 1e3) / 1e9, 2),
                                                     "ms_per_iteration": round(ms3, 5),
                                                     "note": "212 MB working set fits the 256 MB Infinity Cache"}}
        s3.close()
        A3.close()
    sess.close()
    A.close()
    if rank == 0:
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(kind, k, args.cpu_seconds)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""MFMA utilisation of the QR path's GEMMs, from a rocprofv3 --kernel-trace --stats
summary of tools/prof_driver.py --workload qr4096:

  hessenberg : the blocked Hessenberg's trailing updates (hessenberg_blocked_f64): W0 = V^T A
               (split-K), M = V^T Y, W -= M V^T, W2^T = W^T T, and the single rank-2nb update
               A(:, c1:) -= [Y | V] [V | W2^T]^T (rankk_mfma<double>).  Useful flops only: the rank
               update's zero rows of V above the panel are not counted.
  rank_update: rankk_mfma<double> alone, flops it executes (2 n mt 2nb).
  francis    : the delayed window updates of the multishift sweeps (win_gemm_mfma); their sizes
               vary per window, so only their kernel time and share of the run are reported.

utilisation = flops / (kernel time x 78.6 TF/s, the MI355X dense fp64 matrix peak).

usage: tools/qr_mfma.py <run_kernel_stats.csv> <n> <out.json>
"""
import csv
import json
import sys

NB = 32                    # dev::kPanel (hessenberg.hip)
PEAK_F64_MFMA = 78.6e12    # MI355X dense fp64 matrix peak (MI355X_MICROARCH.md)


def hessenberg_flops(n):
    """Mirror of the GEMM calls in hessenberg_blocked_f64 (hessenberg.hip)."""
    useful = rank = 0
    last = n - 3
    for k in range(0, last + 1, NB):
        nbp = min(NB, last - k + 1)
        c1 = k + nbp
        mt = n - c1
        if mt <= 0:
            continue
        rows = n - (k + 1)
        useful += 2 * n * mt * nbp          # right: A(:, c1:) -= Y V^T
        useful += 2 * rows * mt * nbp       # left:  A(k+1:, c1:) -= V W2
        useful += 2 * nbp * mt * rows       # W0 = V^T A
        useful += 2 * nbp * nbp * rows      # M = V^T Y
        useful += 2 * nbp * mt * nbp        # W -= M V(c1:)^T
        useful += 2 * mt * nbp * nbp        # W2^T = W^T T
        rank += 2 * n * mt * 2 * nbp        # executed by rankk_mfma_f64
    return useful, rank


def main():
    stats, n, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    kernels = {}
    hess_ns = rank_ns = win_ns = total_ns = 0.0
    for r in csv.DictReader(open(stats)):
        t = float(r["TotalDurationNs"])
        kernels[r["Name"]] = {"calls": int(r["Calls"]), "total_ns": t}
        total_ns += t
        if "gemm_mfma_f64" in r["Name"] or "gemm_reduce" in r["Name"] or "rankk_mfma" in r["Name"]:
            hess_ns += t
        if "rankk_mfma" in r["Name"]:
            rank_ns += t
        if "win_gemm_mfma" in r["Name"]:
            win_ns += t
    useful, rank = hessenberg_flops(n)
    res = {"n": n, "panel": NB, "mfma_peak_TFLOPs": PEAK_F64_MFMA / 1e12,
           "hessenberg_gemm_flops": useful, "hessenberg_gemm_seconds": hess_ns * 1e-9,
           "hessenberg_gemm_TFLOPs": useful / (hess_ns * 1e-9) / 1e12 if hess_ns else None,
           "hessenberg_mfma_utilisation": useful / (hess_ns * 1e-9) / PEAK_F64_MFMA if hess_ns else None,
           "rank_update_flops": rank, "rank_update_seconds": rank_ns * 1e-9,
           "rank_update_TFLOPs": rank / (rank_ns * 1e-9) / 1e12 if rank_ns else None,
           "rank_update_mfma_utilisation": rank / (rank_ns * 1e-9) / PEAK_F64_MFMA if rank_ns else None,
           "francis_window_gemm_seconds": win_ns * 1e-9,
           "francis_window_gemm_share": win_ns / total_ns if total_ns else None,
           "kernels": kernels}
    # compatibility keys read by bench.py
    res["gemm_flops"] = useful
    res["gemm_TFLOPs"] = res["hessenberg_gemm_TFLOPs"]
    res["mfma_utilisation"] = res["hessenberg_mfma_utilisation"]
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "kernels"}))


if __name__ == "__main__":
    main()

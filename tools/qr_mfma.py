#!/usr/bin/env python3
"""MFMA utilisation of the blocked Hessenberg's trailing-update GEMMs:
sum(2 m n k over the GEMMs hessenberg_blocked_f64 issues) / (sum of gemm_mfma_f64 kernel time x 78.6 TF/s),
the kernel time taken from a rocprofv3 --kernel-trace --stats summary of tools/prof_driver.py --workload qr4096.

usage: tools/qr_mfma.py <run_kernel_stats.csv> <n> <out.json>
"""
import csv
import json
import sys

NB = 32                    # dev::kPanel (hessenberg.hip)
PEAK_F64_MFMA = 78.6e12    # MI355X dense fp64 matrix peak (MI355X_MICROARCH.md)


def gemm_flops(n):
    """Mirror of the GEMM calls in hessenberg_blocked_f64 (hessenberg.hip)."""
    f = 0
    last = n - 3
    for k in range(0, last + 1, NB):
        nbp = min(NB, last - k + 1)
        c1 = k + nbp
        mt = n - c1
        if mt <= 0:
            continue
        rows = n - (k + 1)
        f += 2 * n * mt * nbp          # A(:, c1:) -= Y V^T
        f += 2 * nbp * mt * rows       # W = V^T A
        f += 2 * nbp * mt * nbp        # W2 = T^T W
        f += 2 * rows * mt * nbp       # A -= V W2
    return f


def main():
    stats, n, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    gemm_ns = 0.0
    kernels = {}
    for r in csv.DictReader(open(stats)):
        kernels[r["Name"]] = {"calls": int(r["Calls"]), "total_ns": float(r["TotalDurationNs"])}
        if "gemm_mfma_f64" in r["Name"] or "gemm_reduce" in r["Name"]:
            gemm_ns += float(r["TotalDurationNs"])
    fl = gemm_flops(n)
    res = {"n": n, "panel": NB, "gemm_flops": fl, "gemm_seconds": gemm_ns * 1e-9,
           "gemm_TFLOPs": fl / (gemm_ns * 1e-9) / 1e12 if gemm_ns else None,
           "mfma_peak_TFLOPs": PEAK_F64_MFMA / 1e12,
           "mfma_utilisation": fl / (gemm_ns * 1e-9) / PEAK_F64_MFMA if gemm_ns else None,
           "kernels": kernels}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "kernels"}))


if __name__ == "__main__":
    main()

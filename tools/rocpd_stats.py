"""Per-kernel stats from a rocprofv3 rocpd database (the default output format).

rocprofv3 7.2 segfaults in its exit-time finaliser after a hipLaunchCooperativeKernel (standalone
repro: tools/coop_prof_repro.hip, no eigsol code involved), so its --stats CSV is never written
for the cooperative kernels; the rocpd database is complete before that point.  This prints the
same summary: name, calls, total / average / min / max ns, percentage.

usage: python tools/rocpd_stats.py <dir-or-db> [--csv out.csv] [--filter substring]
"""
import argparse, csv, glob, os, sqlite3, sys

ap = argparse.ArgumentParser()
ap.add_argument("path")
ap.add_argument("--csv")
ap.add_argument("--filter", default="")
args = ap.parse_args()
dbs = [args.path] if args.path.endswith(".db") else sorted(glob.glob(os.path.join(args.path, "**", "*.db"), recursive=True))
if not dbs:
    sys.exit(f"no .db under {args.path}")
agg = {}
for db in dbs:
    c = sqlite3.connect(db)
    for name, dur in c.execute("select name, duration from kernels"):
        a = agg.setdefault(name, [0, 0, None, None])
        a[0] += 1
        a[1] += dur
        a[2] = dur if a[2] is None else min(a[2], dur)
        a[3] = dur if a[3] is None else max(a[3], dur)
tot = sum(v[1] for v in agg.values()) or 1
rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
out = [["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage"]]
for name, (n, s, lo, hi) in rows:
    if args.filter in name:
        out.append([name, n, s, round(s / n, 1), lo, hi, round(100.0 * s / tot, 3)])
for r in out:
    print(",".join(str(x) for x in r) if r is out[0] else f"{r[1]:6d} {r[3]:12.1f} ns {r[6]:7.2f}%  {r[0][:120]}")
if args.csv:
    with open(args.csv, "w", newline="") as f:
        csv.writer(f).writerows(out)

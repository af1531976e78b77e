"""Kernel statistics from a rocprofv3 rocpd database (run_results.db): per kernel name the call
count, total and average duration; optional name filter and start-time window.
Usage: python tools/rocpd_stats.py DB [substring] [--top N]"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else ""
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 40
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name}, count(*), sum(end - start), avg(end - start) from kernels "
                     f"where {name} like ? group by {name} order by sum(end - start) desc", (f"%{filt}%",)).fetchall()
    tot = sum(r[2] for r in rows)
    print(f"{'calls':>7} {'total_ms':>10} {'avg_us':>10} {'pct':>6}  kernel")
    for r in rows[:top]:
        print(f"{r[1]:7d} {r[2] / 1e6:10.3f} {r[3] / 1e3:10.2f} {100 * r[2] / tot:6.1f}  {r[0][:150]}")
    print(f"total {tot / 1e6:.3f} ms over {sum(r[1] for r in rows)} dispatches")


if __name__ == "__main__":
    main()

"""GPU idle gaps of a rocprofv3 --kernel-trace CSV (rocprofv3 --kernel-trace --output-format csv):
the span from the first kernel's start to the last kernel's end, the busy time (union of kernel
intervals), and the idle time grouped by the kernel that ran before each gap.
usage: tools/gap_analysis.py <..._kernel_trace.csv> [name-filter]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
flt = sys.argv[2] if len(sys.argv) > 2 else ""
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows
            if flt in r["Kernel_Name"] or not flt)
if not ev:
    sys.exit("no kernels")
span = ev[-1][1] - ev[0][0]
busy, cur_s, cur_e = 0, ev[0][0], ev[0][1]
gaps = defaultdict(lambda: [0, 0])
prev = ev[0][2]
for s, e, name in ev[1:]:
    if s > cur_e:
        busy += cur_e - cur_s
        g = gaps[prev.split("(")[0][-60:]]
        g[0] += s - cur_e
        g[1] += 1
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
    prev = name
busy += cur_e - cur_s
print(f"kernels {len(ev)}  span {span / 1e6:.1f} ms  busy {busy / 1e6:.1f} ms  idle {(span - busy) / 1e6:.1f} ms")
for k, (t, c) in sorted(gaps.items(), key=lambda kv: -kv[1][0])[:12]:
    print(f"  idle after {k:62s} {t / 1e6:8.1f} ms in {c} gaps ({t / max(c, 1) / 1e3:.1f} us each)")

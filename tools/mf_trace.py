"""Per-dispatch timeline of the last multifrontal solve in a rocprofv3 --kernel-trace CSV
(rocprofv3 --kernel-trace --output-format csv -d DIR -o mft -- python3 tools/mf_probe.py 1000).
Usage: python tools/mf_trace.py DIR/mft_kernel_trace.csv"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "mf_gather_kernel" in r["Kernel_Name"]]
s, e = idx[-2], idx[-1]
t0 = int(rows[s]["Start_Timestamp"])
tot = 0.0
for r in rows[s:e]:
    nm = r["Kernel_Name"].split("(")[0].replace("void eigsol::dev::", "").replace("<eigsol::cplx>", "")
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += d
    wg = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])
    print(f"{(int(r['Start_Timestamp']) - t0) / 1e3:9.1f} {d:8.1f} {nm:28s} wg={wg}")
print("kernel sum", round(tot, 1), "us")

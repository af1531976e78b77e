"""Print a rocprofv3 kernel_stats.csv as a table: tools/prof_stats.py <dir>"""
import csv, glob, sys
f = sorted(glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True))[0]
for r in csv.DictReader(open(f)):
    print(r["Name"][:64].ljust(64), r["Calls"].rjust(7), "%10.1f ms" % (float(r["TotalDurationNs"]) / 1e6),
          "%9.1f us" % (float(r["AverageNs"]) / 1e3), "%6.2f%%" % float(r["Percentage"]))

"""Top kernels of rocprofv3 kernel_stats.csv files (tools/kstats.py DIR... [N])."""
import csv
import os
import sys

args = [a for a in sys.argv[1:] if not a.isdigit()]
n = int(next((a for a in sys.argv[1:] if a.isdigit()), 10))
for d in args:
    f = os.path.join(d, "run_kernel_stats.csv")
    print("==", d)
    for x in list(csv.DictReader(open(f)))[:n]:
        print("%-70s %6s %10.1f %8.1f" % (x["Name"][:70], x["Calls"], float(x["TotalDurationNs"]) / 1e3,
                                          float(x["AverageNs"]) / 1e3))

#!/usr/bin/env python3
"""Print the top kernels of a rocprofv3 --stats kernel_stats.csv."""
import csv
import sys

for path in sys.argv[1:]:
    rows = list(csv.DictReader(open(path)))
    print("==", path)
    for r in rows[:16]:
        print(r["Name"][:88].ljust(88), r["Calls"].rjust(5), "%9.1f us" % (float(r["AverageNs"]) / 1e3),
              "%6.2f%%" % float(r["Percentage"]))

"""Summarise a rocprofv3 kernel_stats.csv: name (shortened), calls, avg ms, total ms, share."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 15
for r in rows[:n]:
    name = re.sub(r"\(anonymous namespace\)::", "", r["Name"])
    name = re.sub(r"^void ", "", name)
    name = name.split("(")[0] if not name.startswith("__") else name
    print(f"{name[:90]:90s} {int(r['Calls']):6d} {float(r['AverageNs'])/1e6:9.3f} ms {float(r['TotalDurationNs'])/1e6:10.2f} ms {float(r['Percentage']):6.2f}%")

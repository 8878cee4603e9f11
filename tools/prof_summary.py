"""Per-step kernel summary of a rocprofv3 --stats csv: python tools/prof_summary.py <stats.csv> <steps> [top]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
tot = sum(float(r["TotalDurationNs"]) for r in rows) / 1e6 / steps
print("total kernel ms/step %.1f" % tot)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
    print("%7.2f %5.1f %s" % (float(r["TotalDurationNs"]) / 1e6 / steps, int(r["Calls"]) / steps, r["Name"][:100]))

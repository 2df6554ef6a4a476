"""Per-request device time by kernel from a rocprofv3 --stats kernel_stats.csv (diagnostic):
python tools/kstats_req.py <kernel_stats.csv> <calls per run>"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = float(sys.argv[2])
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    print(f"{r['Name'][:80]:80s} calls/req={int(r['Calls']) / n:6.2f} avg_us={float(r['AverageNs']) / 1e3:8.2f} "
          f"per_req_us={float(r['TotalDurationNs']) / n / 1e3:8.2f}")
print(f"total per request: {tot / n / 1e3:.1f} us")

"""Summarise a rocprofv3 run_kernel_stats.csv: top kernels by total time."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot / 1e6:.2f} ms in {sum(int(r['Calls']) for r in rows)} launches")
for r in rows[:top]:
    print(f"{float(r['TotalDurationNs']) / 1e6:9.2f} ms {int(r['Calls']):7d} x {float(r['AverageNs']) / 1e3:8.1f} us  "
          f"{float(r['Percentage']):5.1f}%  {r['Name'][:100]}")

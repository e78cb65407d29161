"""Per-step summary of a rocprofv3 --stats kernel table: python tools/prof_summary.py CSV STEPS [N]."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 14
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"kernel time per step: {tot / steps / 1e6:.3f} ms")
for r in rows[:top]:
    print(f"{float(r['TotalDurationNs']) / steps / 1e3:9.1f} us/step  calls/step {int(r['Calls']) / steps:5.1f}  "
          f"avg {float(r['AverageNs']) / 1e3:8.1f} us  {r['Name'][:96]}")

"""Effective GPU clock per launch (GRBM_GUI_ACTIVE / 8 XCDs / kernel wall time, MI355X_MICROARCH.md's
DVFS note) of the kernels matching a substring, for one or more rocprofv3 --pmc GRBM_GUI_ACTIVE runs
(e.g. the fused wide step and the drop-in path): is a kernel slower in one run because it does more
cycles or because the clock is lower?

    python tools/clk_table.py DIR [DIR ...] SUBSTRING
"""
import collections
import csv
import glob
import os
import sys

from pmc_table import short


def main():
    *dirs, sub = sys.argv[1:]
    for d in dirs:
        rows = collections.defaultdict(list)
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if sub in r["Kernel_Name"] and r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                    ns = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                    rows[short(r["Kernel_Name"])].append((float(r["Counter_Value"]), ns))
        print(os.path.basename(d.rstrip("/")))
        for k in sorted(rows):
            v = rows[k]
            cyc = sum(c for c, _ in v) / len(v) / 8
            ns = sum(n for _, n in v) / len(v)
            print(f"  {k:60s} n={len(v):3d}  {ns / 1e3:9.1f} us  {cyc / 1e6:8.3f} M cycles per XCD  "
                  f"{cyc / ns:6.3f} GHz")


if __name__ == "__main__":
    main()

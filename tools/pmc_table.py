"""Per-dispatch averages of rocprofv3 PMC counters for kernels matching a substring.

    python tools/pmc_table.py gpurun_out/pmc_TAG [substring]
"""
import collections
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else "gemm_"
    vals = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if sub in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k in sorted(vals):
        v = vals[k]
        print(f"{k:28s} {sum(v) / len(v):16.4g}   (n={len(v)})")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in vals and "GRBM_GUI_ACTIVE" in vals:
        mf = sum(vals["SQ_VALU_MFMA_BUSY_CYCLES"]) / len(vals["SQ_VALU_MFMA_BUSY_CYCLES"])
        gui = sum(vals["GRBM_GUI_ACTIVE"]) / len(vals["GRBM_GUI_ACTIVE"])
        print(f"MFMA busy per SIMD-cycle ~ {mf / (gui / 8 * 1024):.3f} (SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 x 1024 SIMDs))")


if __name__ == "__main__":
    main()

"""Per-dispatch averages of rocprofv3 PMC counters for kernels matching a substring, one block per
kernel (name up to its argument list).

    python tools/pmc_table.py gpurun_out/pmc_TAG [substring]
"""
import collections
import csv
import glob
import os
import sys


def short(name):
    name = name.replace("bnn::(anonymous namespace)::", "").replace("void ", "")
    depth, out = 0, []
    for ch in name:               # drop the parameter list, keep template arguments
        if ch == "(" and depth == 0:
            break
        depth += ch == "<"
        depth -= ch == ">"
        out.append(ch)
    return "".join(out)


def main():
    d = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else "gemm_"
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if sub in r["Kernel_Name"]:
                vals[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for kern in sorted(vals):
        print(kern)
        kv = vals[kern]
        for k in sorted(kv):
            v = kv[k]
            print(f"  {k:28s} {sum(v) / len(v):16.4g}   (n={len(v)})")
        avg = {k: sum(v) / len(v) for k, v in kv.items()}
        if "SQ_ACTIVE_INST_VALU" in avg and "SQ_WAVE_CYCLES" in avg:
            print(f"  VALU-active share of wave cycles {avg['SQ_ACTIVE_INST_VALU'] / avg['SQ_WAVE_CYCLES']:.3f}, "
                  f"waiting (s_waitcnt / barrier) {avg.get('SQ_WAIT_ANY', 0) / avg['SQ_WAVE_CYCLES']:.3f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in avg and "GRBM_GUI_ACTIVE" in avg:
            print(f"  MFMA busy per SIMD-cycle ~ {avg['SQ_VALU_MFMA_BUSY_CYCLES'] / (avg['GRBM_GUI_ACTIVE'] / 8 * 1024):.3f}")


if __name__ == "__main__":
    main()

"""Split a rocprofv3 --stats kernel table of `bench.py --dropin` (the reference's Net through the drop-in
modules: torch BatchNorm1d / Hardtanh / Dropout / Adam around libbnn's BinarizeLinear) into the libbnn
kernels and torch's, per training step.

    python tools/dropin_breakdown.py run_kernel_stats.csv STEPS
"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    steps = float(sys.argv[2])
    groups = {"libbnn": [], "torch / rocBLAS / runtime": []}
    for r in rows:
        us = float(r["TotalDurationNs"]) / steps / 1e3
        key = "libbnn" if "bnn::" in r["Name"] else "torch / rocBLAS / runtime"
        groups[key].append((us, float(r["Calls"]) / steps, r["Name"]))
    total = sum(us for g in groups.values() for us, _, _ in g)
    print(f"kernel time per step: {total / 1e3:.2f} ms")
    for k, g in groups.items():
        s = sum(us for us, _, _ in g)
        print(f"\n{k}: {s / 1e3:.2f} ms per step ({100 * s / total:.1f} %)")
        for us, calls, name in sorted(g, reverse=True)[:12]:
            short = name.replace("bnn::(anonymous namespace)::", "").replace("void ", "")
            print(f"  {us / 1e3:8.3f} ms  x{calls:4.1f}  {short[:110]}")


if __name__ == "__main__":
    main()

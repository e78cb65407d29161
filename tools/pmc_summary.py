"""Summarise rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) per kernel into a JSON that bench.py
reads for ``roofline.traffic``.

    python tools/pmc_summary.py --fetch gpurun_out/pmc_fetch_r01 --write gpurun_out/pmc_write_r01 \
        --out profiles/r01_pmc_traffic.json

Corrections (MI355X_MICROARCH.md, "HBM"): rocprofv3 reports both counters in KiB; on gfx950
FETCH_SIZE counts exactly half the bytes of a wide coalesced streaming read (128-B requests tallied
as 64 B), so fetched bytes = 2 * 1024 * FETCH_SIZE; WRITE_SIZE is exact for 16-B-per-lane stores,
bytes = 1024 * WRITE_SIZE.  Infinity-Cache hits are counted as fabric traffic (not excluded), so the
figure is an upper bound on HBM bytes.  Launches of one kernel instance are grouped by grid size
(the same template serves dX and dW of different shapes)."""
import argparse
import collections
import csv
import glob
import json
import os
import re


def short_name(k):
    k = re.sub(r"^void ", "", k)
    k = k.replace("bnn::(anonymous namespace)::", "")
    return k.split("(")[0]


def load(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    out = collections.defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            out[(short_name(r["Kernel_Name"]), int(r["Grid_Size"]))].append(float(r["Counter_Value"]))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--note", default="")
    a = ap.parse_args()
    fetch, write = load(a.fetch, "FETCH_SIZE"), load(a.write, "WRITE_SIZE")
    kernels = collections.defaultdict(dict)
    for key in sorted(set(fetch) | set(write)):
        name, grid = key
        if not ("bnn" in name or name.startswith(("gemm", "sign", "quant", "bn_", "adam", "col", "conv"))):
            continue
        f, w = fetch.get(key, []), write.get(key, [])
        fb = 2 * 1024 * sum(f) / len(f) if f else None
        wb = 1024 * sum(w) / len(w) if w else None
        kernels[name][str(grid)] = {"launches": max(len(f), len(w)),
                                    "fetch_bytes": round(fb) if fb is not None else None,
                                    "write_bytes": round(wb) if wb is not None else None}
    # per kernel: launch-weighted average over grids
    summary = {}
    for name, grids in kernels.items():
        n = sum(g["launches"] for g in grids.values())
        tot = sum(((g["fetch_bytes"] or 0) + (g["write_bytes"] or 0)) * g["launches"] for g in grids.values())
        summary[name] = {"traffic_bytes_per_launch": round(tot / n), "grids": grids}
    json.dump({"source": {"fetch": a.fetch, "write": a.write, "note": a.note,
                          "correction": "fetch = 2*1024*FETCH_SIZE, write = 1024*WRITE_SIZE (gfx950)"},
               "kernels": summary}, open(a.out, "w"), indent=1, sort_keys=True)
    for name, s in sorted(summary.items(), key=lambda kv: -kv[1]["traffic_bytes_per_launch"]):
        print(f"{s['traffic_bytes_per_launch'] / 1e9:9.3f} GB  {name}")


if __name__ == "__main__":
    main()

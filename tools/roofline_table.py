"""DESIGN.md §5's measured-roofline table from a rocprofv3 kernel-stats CSV of the wide step
(B = 65536, C = 8192) and a *_pmc_traffic.json of the same build: per kernel, average launch time,
the algorithmic work per launch (ops for the GEMMs, bytes for the streaming passes; E = 65536 x 8192
elements), the achieved rate and its fraction of the MI355X peak (FP4/FP6 MFMA 10.07 POPS dense,
int8 5.03 POPS, HBM 8 TB/s), and the PMC traffic per launch.

    python tools/roofline_table.py STATS.csv TRAFFIC.json
"""
import csv
import json
import sys

E = 65536 * 8192
GEMM_OPS = 2.0 * 65536 * 8192 * 8192
PIX_OPS = 2.0 * 65536 * 8192 * 832
FP4_PEAK, I8_PEAK, HBM = 10.07e15, 5.03e15, 8e12

# (name prefix as rocprofv3 lists it, label, kind, work per launch, passes)
ROWS = [
    ("gemm_fp6_k<2, 4, 2, 4, 2, 0, 2, 0, 0, 1>", "`gemm_fp6_k` dX + residual plane (fc2/fc3)", "mfma", GEMM_OPS, 5),
    ("gemm_fp6_k<2, 4, 2, 4, 2, 0, 2, 0, 0, 0>", "`gemm_fp6_k` dW (fc2/fc3)", "mfma", GEMM_OPS, 4),
    ("gemm_fp4_k<2, 4, 4, 2, 2, 128, 2, 1, 1>", "`gemm_fp4_k` fc2 + bn2 statistics", "mfma", GEMM_OPS, 1),
    ("gemm_fp4_k<2, 4, 4, 2, 2, 128, 2, 1, 0>", "`gemm_fp4_k` fc3 (int16 out)", "mfma", GEMM_OPS, 1),
    ("bn_bwd_apply_q6_k<0, true", "`bn_bwd_apply_q6_k<0>` bn2 bwd + FP6 digits + residual", "hbm", 12.7 * E, 0),
    ("bn_bwd_apply_q6_k<10, true", "`bn_bwd_apply_q6_k<10>` head bwd + digits + residual", "hbm", 8.7 * E, 0),
    ("bn_dz_quant_cols_t_k<2>", "`bn_dz_quant_cols_t_k<2>` dz1 -> int8 column digits", "hbm", 10.0 * E, 0),
    ("gemm_i8_v2_k<1, 1, 2, 4, 4, 2, 3, 64, 0, 0, 0, 1>", "`gemm_i8_v2_k` fc1 on pixels (+ bn1 statistics, s20 out)", "i8", PIX_OPS, 1),
    ("gemm_i8_v2_k<3, 1, 2, 4, 2, 2, 2, 128, 2, 0, 1, 0>", "`gemm_i8_v2_k<3,1>` dW1 on pixels", "i8", PIX_OPS, 3),
    ("adam_pack_fp4_k", "`adam_pack_fp4_k` (67 M weights)", "hbm", 1.95e9, 0),
    ("bn_reduce_k<2, 2>", "`bn_reduce_k<2>` bn1 bwd sums + maxima (s20)", "hbm", 7.0 * E, 0),
    ("bn_reduce_k<1, 1>", "`bn_reduce_k<1>` bn2 bwd sums (z16)", "hbm", 6.0 * E, 0),
    ("bn_head_reduce", "head statistics pass (+ dW4 partials)", "hbm", 2.0 * E, 0),
    ("bn_head_fwd_k<10, true", "`bn_head_fwd_k<10>` (f32 MFMA head)", "hbm", 2.0 * E, 0),
    ("bn_apply_pack_fp4_k<2>", "`bn_apply_pack_fp4_k` s20 in", "hbm", 4.0 * E, 0),
    ("bn_apply_pack_fp4_k<1>", "`bn_apply_pack_fp4_k` z16 in", "hbm", 3.0 * E, 0),
    ("bn_reduce_k<0, 1>", "`bn_reduce_k<0>` bn3 fwd statistics (+ keep bits)", "hbm", 2.0 * E, 0),
]


def short(name):
    name = name.replace("void ", "").replace("bnn::(anonymous namespace)::", "")
    return name.split("(")[0]


def main():
    stats = list(csv.DictReader(open(sys.argv[1])))
    traffic = json.load(open(sys.argv[2])) if len(sys.argv) > 2 else {}
    traffic = traffic.get("kernels", traffic)
    print("| kernel | µs per launch | work per launch | achieved | fraction of peak | PMC traffic per launch |")
    print("|---|---|---|---|---|---|")
    for prefix, label, kind, work, passes in ROWS:
        hits = [r for r in stats if short(r["Name"]).startswith(prefix)]
        if not hits:
            continue
        r = hits[0]
        us = float(r["AverageNs"]) / 1e3
        tr = next((v["traffic_bytes_per_launch"] for k, v in traffic.items() if k.startswith(prefix)), None)
        trs = f"{tr / 1e9:.2f} GB" if tr else "--"
        if kind == "hbm":
            rate = work / (us * 1e-6)
            print(f"| {label} | {us:.0f} | {work / 1e9:.2f} GB | {rate / 1e12:.2f} TB/s | {rate / HBM:.2f} of HBM | {trs} |")
        else:
            peak = FP4_PEAK if kind == "mfma" else I8_PEAK
            rate = work / (us * 1e-6)
            extra = f" ({rate * passes / peak:.2f} in {passes} MFMA passes)" if passes > 1 else ""
            print(f"| {label} | {us:.0f} | {work / 1e12:.2f} T ops | {rate / 1e15:.2f} POPS | "
                  f"{rate / peak:.3f}{extra} | {trs} |")


if __name__ == "__main__":
    main()

"""The three ternary-GEMM engines on the forward shapes (VERDICT n2): XNOR-popcount
on the VALU (gemm_xnor_k), int8 MFMA (gemm_i8 (1,1)) and FP4 MFMA (gemm_fp4), bit-exact against
each other, with their rates against their own roofline.

    python tools/xnor_probe.py [--reps 3]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-mnist-bnns_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from bnn_amd import functional as BF  # noqa: E402
from bench import MI355X_FP4_DENSE_TOPS, MI355X_INT8_DENSE_TOPS  # noqa: E402

# VALU popcount roofline: 5 VALU ops per 32 ternary MACs (and, xor, and, 2 x bcnt-accumulate),
# 64 lane-ops / clk / CU (4 SIMD x 16 lanes), 256 CUs, 2.4 GHz
XNOR_PEAK_TOPS = 64 * 256 * 2.4e9 * (2 * 32 / 5) / 1e12

SHAPES = {"fwd_fc2_wide": (65536, 8192, 8192), "fwd_fc2_mlp": (4096, 1536, 3072), "fwd_fc3_mlp": (4096, 768, 1536)}


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    g = torch.Generator(device="cuda").manual_seed(0)
    for name, (M, N, K) in SHAPES.items():
        x = torch.randint(-1, 2, (M, K), generator=g, device="cuda").float()
        w = torch.randint(-1, 2, (N, K), generator=g, device="cuda").float()
        xb, wb = BF.sign_pack_bits(x), BF.sign_pack_bits(w)
        xq, _ = BF.sign_pack(x, True, False)
        wq, _ = BF.sign_pack(w, True, False)
        x4, _ = BF.sign_pack_fp4(x)
        w4, _ = BF.sign_pack_fp4(w)
        ops = 2.0 * M * N * K
        res = {}
        outs = {}
        for eng, fn, peak in (("xnor", lambda: BF.gemm_xnor(xb, wb, M, N), XNOR_PEAK_TOPS),
                              ("int8", lambda: BF.gemm_i8(xq, 1, wq, 1, M, N, k_true=K), MI355X_INT8_DENSE_TOPS),
                              ("fp4", lambda: BF.gemm_fp4(x4, w4, M, N, k_true=K), MI355X_FP4_DENSE_TOPS)):
            outs[eng] = fn()
            ms = timeit(fn, args.reps)
            tops = ops / (ms * 1e-3) / 1e12
            res[eng] = {"ms": round(ms, 3), "tops": round(tops, 1), "peak_tops": round(peak, 1),
                        "frac": round(tops / peak, 3)}
        res["bit_exact"] = bool(torch.equal(outs["xnor"], outs["int8"]) and torch.equal(outs["fp4"], outs["int8"]))
        print(json.dumps({"shape": name, "M": M, "N": N, "K": K, **res}), flush=True)
        del x, w, xb, wb, xq, wq, x4, w4, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

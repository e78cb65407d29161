"""Time every bnn_gemm_i8 kernel variant on the wide-MLP shapes and check they agree bitwise.

    python tools/gemm_sweep.py [--reps 5]
Prints one JSON line per (shape, variant): avg ms, TOPS (int8 MFMA ops = 2*M*N*K*pairs) and the
fraction of the 5.03 POPS dense int8 peak."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-mnist-bnns_amd"))
import torch  # noqa: E402

from bnn_amd import _lib as L  # noqa: E402
from bnn_amd import functional as BF  # noqa: E402

PEAK = 256 * 4 * 2048 * 2.4e9 / 1e12

SHAPES = {  # name: (M, N, K, a_digits, b_digits)
    "fwd_fc2": (65536, 8192, 8192, 1, 1),
    "fwd_k128": (65536, 8192, 128, 1, 1),
    "fwd_fp4": (65536, 8192, 4096, 0, 0),
    "fc1_fwd": (65536, 8192, 832, 3, 1),
    "dx_fc2": (65536, 8192, 8192, 3, 1),
    "dw_fc2": (8192, 8192, 65536, 3, 1),
    "dw_fc1": (8192, 784, 65536, 3, 3),
    "mlp_fwd": (4096, 1536, 3072, 1, 1),
    "mlp_dx": (4096, 3072, 1536, 3, 1),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--variants", default="0,1,2,3,4,5,6,7,8,-1")
    ap.add_argument("--shapes", default=",".join(SHAPES))
    args = ap.parse_args()
    g = torch.Generator(device="cuda").manual_seed(0)
    for name in args.shapes.split(","):
        M, N, K, da, db = SHAPES[name]
        if da == 0:   # FP4 ternary form: random e2m1 codes in {0x0, 0x2, 0xA}, K in bytes
            codes = torch.tensor([0x0, 0x2, 0xA], dtype=torch.uint8, device="cuda")
            A = (codes[torch.randint(0, 3, (M, K), generator=g, device="cuda")] |
                 (codes[torch.randint(0, 3, (M, K), generator=g, device="cuda")] << 4))
            B = (codes[torch.randint(0, 3, (N, K), generator=g, device="cuda")] |
                 (codes[torch.randint(0, 3, (N, K), generator=g, device="cuda")] << 4))
            ref = None
            seen = set()
            for v in (int(x) for x in args.variants.split(",")):
                L.call("bnn_gemm_set_variant", v)
                kname = BF.gemm_kernel_name(0, 0, M, N, K)
                if kname in seen:
                    continue
                seen.add(kname)
                C = BF.gemm_fp4(A, B, M, N)
                torch.cuda.synchronize()
                same = True if ref is None else bool(torch.equal(C, ref))
                ref = C if ref is None else ref
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(args.reps):
                    BF.gemm_fp4(A, B, M, N)
                e.record()
                torch.cuda.synchronize()
                ms = s.elapsed_time(e) / args.reps
                tops = 2.0 * M * N * 2 * K / (ms * 1e-3) / 1e12
                print(json.dumps({"shape": name, "variant": v, "kernel": kname, "ms": round(ms, 3),
                                  "tops": round(tops, 1), "frac_fp4_peak": round(tops / (2 * PEAK), 3),
                                  "frac_int8_peak": round(tops / PEAK, 3), "matches_first": same}), flush=True)
            L.call("bnn_gemm_set_variant", -1)
            continue
        A = torch.randint(-128, 128, (da, M, K) if da > 1 else (M, K), generator=g, device="cuda",
                          dtype=torch.int8)
        if da > 1:
            A[2] = A[2] // 2        # top digit in [-64, 64)
        B = torch.randint(-1, 2, (db, N, K) if db > 1 else (N, K), generator=g, device="cuda", dtype=torch.int8)
        if db > 1:
            B = torch.randint(-128, 128, (db, N, K), generator=g, device="cuda", dtype=torch.int8)
            B[2] = B[2] // 2
        sa = torch.ones(M, device="cuda") if da > 1 else None
        ref = None
        pairs = BF.GEMM_PAIRS[(da, db)]
        seen = set()
        for v in (int(x) for x in args.variants.split(",")):
            L.call("bnn_gemm_set_variant", v)
            kname = BF.gemm_kernel_name(da, db, M, N, K)
            if kname in seen:
                continue
            seen.add(kname)
            C = BF.gemm_i8(A, da, B, db, M, N, a_scale=sa)
            torch.cuda.synchronize()
            same = True if ref is None else bool(torch.equal(C, ref))
            if kname.startswith("diag"):
                same = None
            if ref is None:
                ref = C
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(args.reps):
                BF.gemm_i8(A, da, B, db, M, N, a_scale=sa, out=C)
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e) / args.reps
            tops = 2.0 * M * N * K * pairs / (ms * 1e-3) / 1e12
            print(json.dumps({"shape": name, "variant": v, "kernel": kname,
                              "ms": round(ms, 3), "tops": round(tops, 1),
                              "frac": round(tops / PEAK, 3), "matches_first": same}), flush=True)
        L.call("bnn_gemm_set_variant", -1)
        del A, B, ref, C
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

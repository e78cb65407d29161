"""How many FP6 digit planes the backward GEMMs need.

Emulates the FP6 digit operand (bnn_fp6.h: per 32-element block, e with max|x| in [2^(e-1), 2^e),
I = rint(x * 2^(P*5 - 1 - e)), P balanced base-32 digits, each exact in e2m3) for P = 3 and 4 planes
on the gradients the wide step multiplies -- Gaussian rows and the heavy-tailed rows of
tests/test_gpu_fused.py (magnitudes spread over e^+-9) -- and measures dX = dY.W_b against float64
(the MFMA sums the digit products exactly per block; only the operand rounding is emulated).

    python tools/fp6_planes_bound.py [M] [K]
"""
import sys

import numpy as np


def quantise(x, planes):
    bits = 5 * planes - 1                       # |I| <= 2^bits (4 planes: 2^19)
    M, K = x.shape
    xb = x.reshape(M, K // 32, 32)
    amax = np.abs(xb).max(-1, keepdims=True)
    _, e = np.frexp(amax)                       # amax in [2^(e-1), 2^e)
    e = np.maximum(e, -111)
    I = np.rint(np.ldexp(xb, bits - e))
    return np.ldexp(I, e - bits).reshape(M, K)


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
    rng = np.random.default_rng(0)
    wb = np.sign(rng.uniform(-1, 1, (K, K)))
    cases = {
        "gaussian": rng.standard_normal((M, K)).astype(np.float32),
        "heavy-tailed e^+-9": (rng.standard_normal((M, K)) * np.exp(rng.uniform(-9, 9, (M, K)))).astype(np.float32),
    }
    print(f"dX = dY . W_b, M={M}, K=N={K}; bar 1e-5 norm-wise and per row")
    for name, x in cases.items():
        ref = x.astype(np.float64) @ wb
        for planes in (3, 4):
            got = quantise(x.astype(np.float64), planes) @ wb
            d = got - ref
            err = np.linalg.norm(d) / np.linalg.norm(ref)
            row = (np.linalg.norm(d, axis=1) / np.linalg.norm(ref, axis=1)).max()
            print(f"  {name:20s} {planes} planes: norm-wise {err:.2e}, worst row {row:.2e}"
                  f"  -> {'meets' if max(err, row) < 1e-5 else 'FAILS'} the bar")


if __name__ == "__main__":
    main()

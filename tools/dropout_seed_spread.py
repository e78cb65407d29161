"""does the dX residual plane (BNN_FP6_RES) or the dropout keep-bit plane move the
dropout-on MNIST accuracy, or is the libbnn / torch gap seed noise?  Runs the dropout loss-curve
workload of tests/test_gpu_loss_curve.py (t10k files, batch 100, 300 steps, p = 0.3) for several
seeds of each variant and prints per-seed training accuracies, means and standard errors.

    python tools/dropout_seed_spread.py [seeds per variant]
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "distributed-mnist-bnns_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import test_gpu_loss_curve as T  # noqa: E402


def stats(name, acc):
    a = np.array(acc)
    se = a.std(ddof=1) / np.sqrt(len(a))
    print(f"{name:28s} n={len(a)} mean {a.mean():.4f} sd {a.std(ddof=1):.4f} se {se:.4f}  "
          f"[{' '.join(f'{v:.4f}' for v in a)}]", flush=True)
    return a.mean(), se


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    from bnn_amd import functional as BF
    from bnn_amd import nets
    torch.manual_seed(5)
    state = {k: v.clone() for k, v in nets.MLP(*T.WIDTHS, p_drop=0.3).state_dict().items()}
    x, y, order = T._data()
    res = {}
    for name, res_on, kb in (("libbnn (residual, keep bits)", True, True), ("libbnn BNN_FP6_RES=0", False, True),
                             ("libbnn BNN_KEEP_BITS=0", True, False)):
        BF.FP6_RES, BF._KEEP_BITS[0] = res_on, kb
        res[name] = stats(name, [T._run_libbnn(state, x, y, order, p_drop=0.3, seed=100 + s)[1] for s in range(n)])
    BF.FP6_RES, BF._KEEP_BITS[0] = True, True
    res["torch"] = stats("torch fp32 (reference sem.)",
                         [T._run_torch(state, x, y, order, p_drop=0.3, seed=200 + s)[1] for s in range(n)])
    mt, st = res["torch"]
    for k, (m, s) in res.items():
        if k != "torch":
            print(f"{k:28s} - torch: {m - mt:+.4f} (se of the difference {np.hypot(s, st):.4f})")


if __name__ == "__main__":
    main()

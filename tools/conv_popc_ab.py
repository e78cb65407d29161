"""A/B timing of the binarised-input conv forward engines (bnn_conv_set_popc 0 / 1) on the BinCNN's
layers at the bench batch: bnn_conv2d_fwd_q (int16 sums, the compact hand-off the fused BinCNN
uses) and bnn_conv2d_fwd (fp32 + bias), HIP-event timed over many launches, plus one fused BinCNN
step per engine.  Prints one line per (layer, output, engine).

    python tools/conv_popc_ab.py [batch]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-mnist-bnns_amd"))

from bnn_amd import _lib as L  # noqa: E402


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    prev = L.lib().bnn_conv_set_popc(-1)
    g = torch.Generator(device="cuda").manual_seed(0)
    layers = {"conv1": (1, 28, 28, 16, 5, 2), "conv2": (16, 14, 14, 32, 5, 2)}
    for name, (C, H, W, Co, K, pad) in layers.items():
        x = torch.randn(N, C, H, W, generator=g, device="cuda")
        if C == 1:
            x = torch.where(x < 0.5, torch.zeros_like(x), x)           # pixel-like: 70 % zeros, rest > 0
        w = torch.randn(Co, C, K, K, generator=g, device="cuda")
        b = torch.randn(Co, generator=g, device="cuda")
        y = torch.empty(N, Co, H, W, device="cuda")
        yq = torch.empty(N, Co, H, W, dtype=torch.int16, device="cuda")
        res = {}
        for eng in (0, 1):
            L.call("bnn_conv_set_popc", eng)
            tq = timeit(lambda: L.call("bnn_conv2d_fwd_q", L.ptr(x), L.ptr(w), L.ptr(yq), 2, N, C, H, W, Co, K, K, 1,
                                       pad, 1, 1, L.stream()))
            rq = yq.clone()
            tf = timeit(lambda: L.call("bnn_conv2d_fwd", L.ptr(x), 1, L.ptr(w), L.ptr(b), L.ptr(y), N, C, H, W, Co,
                                       K, K, 1, pad, 1, 1, L.stream()))
            res[eng] = (rq, y.clone())
            out_bytes = yq.numel() * 2
            print(f"{name} N={N} engine={'popc' if eng else 'mfma/dot4'}  fwd_q(int16) {tq:8.1f} us "
                  f"({(x.numel() * 4 + out_bytes) / tq / 1e3:6.0f} GB/s)   fwd(fp32) {tf:8.1f} us", flush=True)
        assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1]), name
    from bnn_amd import nets
    from bnn_amd.data import synthetic_mnist
    torch.manual_seed(1)
    m = nets.BinCNN(org_protocol=False, mutate_input=False, fused_bn=True).cuda()
    x, y = synthetic_mnist(N, seed=2, device="cuda")

    def step():
        m.zero_grad(set_to_none=True)
        torch.nn.functional.cross_entropy(m(x), y).backward()

    for eng in (0, 1):
        L.call("bnn_conv_set_popc", eng)
        print(f"BinCNN fused fwd+bwd N={N} engine={'popc' if eng else 'mfma/dot4'}  {timeit(step, 20):8.1f} us",
              flush=True)
    L.call("bnn_conv_set_popc", prev)


if __name__ == "__main__":
    main()

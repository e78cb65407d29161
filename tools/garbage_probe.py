"""Uninitialised-memory probe: train the same fused model from the same init on the same batches
three times, each time after pre-filling the caching allocator's free blocks with a different
pattern (zeros, NaN, random), and compare every gradient bit for bit across the three runs.  A
kernel that reads memory it never wrote (a workspace, a padded plane) shows up as a difference
or a NaN; a deterministic path gives three identical runs.

    python tools/garbage_probe.py [cnn|config2|mlp|wide ...]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-mnist-bnns_amd"))

from bnn_amd import functional as BF  # noqa: E402
from bnn_amd import nets  # noqa: E402

KINDS = {
    # kind: (batch, steps)
    "cnn": (256, 3),
    "config2": (100, 3),
    "mlp": (512, 2),
    "wide": (1024, 2),
}


def make(kind):
    torch.manual_seed(100)
    if kind == "cnn":
        m = nets.BinCNN(org_protocol=False, mutate_input=False, fused_bn=True)
    elif kind == "config2":
        m = nets.Net(org_protocol=False, mutate_input=False, fused_bn=True)
    elif kind == "wide":
        m = nets.MLP(4096, 4096, 4096, p_drop=0.2, org_protocol=False, mutate_input=False, fused_bn=True)
    else:
        m = nets.MLP(512, 256, 256, p_drop=0.0, org_protocol=False, mutate_input=False, fused_bn=True)
    return m.cuda().train()


def fill(mode):
    """Allocate, fill and free blocks of many sizes, so the next allocations reuse them."""
    held = []
    sizes = [512 * 2 ** k for k in range(0, 12)] * 8 + [2 ** 24] * 16 + [2 ** 26] * 8
    for n in sizes:
        t = torch.empty(n // 4, dtype=torch.float32, device="cuda")
        if mode == "zero":
            t.zero_()
        elif mode == "nan":
            t.fill_(float("nan"))
        else:
            t.uniform_(-1e3, 1e3)
        held.append(t)
    torch.cuda.synchronize()
    del held


def run(kind, mode):
    batch, steps = KINDS[kind]
    m = make(kind)
    g = torch.Generator(device="cuda").manual_seed(1234)
    crit = torch.nn.CrossEntropyLoss()
    out = []
    for step in range(steps):
        u = torch.randint(0, 256, (batch, 1, 28, 28), generator=g, device="cuda").to(torch.uint8)
        u = torch.where(torch.rand(u.shape, generator=g, device="cuda") < 0.807, torch.zeros_like(u), u)
        x = u.float().div(255.0) if kind == "cnn" else u
        y = torch.randint(0, 10, (batch,), generator=g, device="cuda")
        for p in m.parameters():
            p.grad = None
        fill(mode)
        torch.manual_seed(1000 + 10 * step)
        crit(m(x), y).backward()
        out.append([(n, p.grad.detach().clone()) for n, p in m.named_parameters()])
        with torch.no_grad():
            for p in m.parameters():
                p.add_(p.grad, alpha=-0.01)
                BF.invalidate_packed(p)
    torch.cuda.synchronize()
    return out


def main():
    kinds = sys.argv[1:] or list(KINDS)
    bad = 0
    for kind in kinds:
        runs = {mode: run(kind, mode) for mode in ("zero", "nan", "rand")}
        for step in range(len(runs["zero"])):
            for i, (n, g0) in enumerate(runs["zero"][step]):
                line = []
                for mode in ("nan", "rand"):
                    g1 = runs[mode][step][i][1]
                    nan = bool(torch.isnan(g1).any())
                    d = float((g1 - g0).abs().max()) if not nan else float("nan")
                    ok = torch.equal(g0, g1)
                    bad += not ok
                    line.append(f"{mode}: {'==' if ok else 'DIFF'} nan={nan} max|d|={d:.3e}")
                print(f"{kind:8s} step {step} {n:22s} max|g|={float(g0.abs().max()):.2e}  " + "  ".join(line),
                      flush=True)
    print("GARBAGE_PROBE", "CLEAN" if bad == 0 else f"{bad} DIFFERENCES", flush=True)


if __name__ == "__main__":
    main()

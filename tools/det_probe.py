"""Determinism probe: two identical copies of a fused net, the same batch and dropout seed, one
forward + backward each (no exchange); prints every parameter whose gradient differs bit-wise.

    python tools/det_probe.py [config2|mlp|cnn] [batch]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-mnist-bnns_amd"))


def main():
    from bnn_amd import nets
    kind = sys.argv[1] if len(sys.argv) > 1 else "config2"
    batch = int(sys.argv[2]) if len(sys.argv) > 2 else 100

    def make():
        torch.manual_seed(100)
        if kind == "cnn":
            return nets.BinCNN(org_protocol=False, mutate_input=False, fused_bn=True).cuda().train()
        if kind == "config2":
            return nets.Net(org_protocol=False, mutate_input=False, fused_bn=True).cuda().train()
        return nets.MLP(512, 256, 256, p_drop=0.0, org_protocol=False, mutate_input=False, fused_bn=True).cuda().train()

    g = torch.Generator(device="cuda").manual_seed(1234)
    u = torch.randint(0, 256, (batch, 1, 28, 28), generator=g, device="cuda").to(torch.uint8)
    x = u.float().div(255.0) if kind == "cnn" else u
    y = torch.randint(0, 10, (batch,), generator=g, device="cuda")
    grads = []
    for rep in range(3):
        m = make() if rep < 2 else grads[0][2]
        for p in m.parameters():
            p.grad = None
        torch.manual_seed(7)
        torch.nn.functional.cross_entropy(m(x), y).backward()
        grads.append(({n: p.grad.detach().clone() for n, p in m.named_parameters()}, rep, m))
    for a, b, what in ((0, 1, "two copies"), (0, 2, "same copy twice")):
        bad = {n: float((grads[a][0][n] - grads[b][0][n]).abs().max()) for n in grads[a][0]
               if not torch.equal(grads[a][0][n], grads[b][0][n])}
        print(f"{kind} B={batch} {what}: {'identical' if not bad else bad}")


if __name__ == "__main__":
    main()

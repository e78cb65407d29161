"""Determinism probe: the fused MLP step's gradients over repeated runs and exchange modes."""
import os
import sys

import torch
import torch.distributed as dist

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "distributed-mnist-bnns_amd"), os.path.join(R, "tests")]
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29571")
dist.init_process_group("gloo", rank=0, world_size=1)
from test_gpu_exchange import _run  # noqa: E402

base, _ = _run((1024, 1024, 512), 1024, "none")
for it, mode in enumerate(["none", "accumulate", "direct", "none", "accumulate", "direct", "none"]):
    g, _ = _run((1024, 1024, 512), 1024, mode)
    bad = {k: (g[k] - base[k]).abs().max().item() for k in base if not torch.equal(g[k], base[k])}
    print(it, mode, "differs:", bad)

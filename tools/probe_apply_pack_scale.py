"""Probe: does the 64 x 64-tile BatchNorm apply-pack (sign_pack_tile_k<1, 1>) scale with the layer size?
Config 3's bn2 / bn3 passes both take ~20 us (profiles/r06_ac_mlpg_stats_head.txt).  Launches each
shape 50 times, with and without the transposed output; run under rocprofv3 --kernel-trace --stats
and read the per-kernel averages per shape from the trace (kernel names are the same, so the
shapes run in separate phases with a marker sync between them)."""
import sys, time
import torch
sys.path.insert(0, "distributed-mnist-bnns_amd")
from bnn_amd import _lib as L

def run(M, C, with_qt, reps=50):
    x = torch.randn(M, C, device="cuda")
    mean = torch.randn(C, device="cuda") * 0.1
    inv = torch.rand(C, device="cuda") + 0.5
    g = torch.randn(C, device="cuda"); b = torch.randn(C, device="cuda")
    q = torch.empty(M, ((C + 255) // 256) * 128, dtype=torch.uint8, device="cuda")
    qt = torch.empty(((C + 255) // 256) * 256, M // 2, dtype=torch.int8, device="cuda") if with_qt else None
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(reps):
        L.call("bnn_bn_apply_pack", L.ptr(x), M, C, L.ptr(mean), L.ptr(inv), None, L.ptr(g), L.ptr(b), 1, L.ptr(q),
               q.shape[1], L.ptr(qt) if qt is not None else None, qt.shape[1] if qt is not None else 0, 1, L.stream())
    ev1.record(); torch.cuda.synchronize()
    print(f"M={M} C={C} qt={int(with_qt)}: {ev0.elapsed_time(ev1) * 1000 / reps:.1f} us/launch (events, incl. host launch)", flush=True)
    time.sleep(0.05)

for M, C in [(4096, 768), (4096, 1536), (4096, 3072), (16384, 1536), (1024, 1536)]:
    run(M, C, True)
    run(M, C, False)

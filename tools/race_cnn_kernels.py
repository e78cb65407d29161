"""Localise a contention-only nondeterminism in the BinCNN's first block: P processes share the GPU,
each running the block's libbnn calls R times on fixed inputs and comparing every stage's output
with its first repetition, bit for bit -- conv1's int16 sums (bnn_conv2d_fwd_q), the BatchNorm2d
forward (mean, invstd, pooled y: bnn_bn2d_fwd_train_q), its backward statistics (dgamma, dbeta, sg,
sgx: bnn_bn2d_bwd_stats_q) and conv1's fused filter gradient (bnn_conv2d_bwd_filter_bn).

    python tools/race_cnn_kernels.py [processes] [repetitions] [batch] [seconds]

With seconds > 0 every process keeps repeating until that much wall time has passed (so the
processes overlap on the GPU), at least `repetitions` times.
"""
import os
import sys

import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "distributed-mnist-bnns_amd")


def _worker(rank, reps, N, q, secs=0.0):
    try:
        sys.path.insert(0, PKG)
        torch.cuda.set_device(0)
        from bnn_amd import _lib as L
        C, H, W, Co, K, pad = 1, 28, 28, 16, 5, 2
        g = torch.Generator(device="cuda").manual_seed(1234 + rank)
        u = torch.randint(0, 256, (N, 1, 28, 28), generator=g, device="cuda").to(torch.uint8)
        u = torch.where(torch.rand(u.shape, generator=g, device="cuda") < 0.807, torch.zeros_like(u), u)
        x = u.float().div(255.0)
        w = torch.randn(Co, C, K, K, generator=g, device="cuda") * 0.1
        cb = torch.randn(Co, generator=g, device="cuda") * 0.1
        gam = torch.rand(Co, generator=g, device="cuda") + 0.5
        bet = torch.randn(Co, generator=g, device="cuda") * 0.1
        dyp = torch.randn(N, Co, 14, 14, generator=g, device="cuda") * 1e-3
        first, bad = None, {}
        import time
        t_end = time.time() + secs
        r = -1
        while True:
            r += 1
            if r >= reps and time.time() >= t_end:
                break
            zq = torch.empty(N, Co, 28, 28, dtype=torch.int16, device="cuda")
            L.call("bnn_conv2d_fwd_q", L.ptr(x), L.ptr(w), L.ptr(zq), 2, N, C, H, W, Co, K, K, 1, pad, 1, 1, L.stream())
            rm, rv = torch.zeros(Co, device="cuda"), torch.ones(Co, device="cuda")
            mean, inv = torch.empty(Co, device="cuda"), torch.empty(Co, device="cuda")
            y = torch.empty(N, Co, 14, 14, device="cuda")
            ws = torch.empty((L.lib().bnn_bn2d_workspace(N, Co),), dtype=torch.uint8, device="cuda")
            L.call("bnn_bn2d_fwd_train_q", L.ptr(zq), L.ptr(cb), 2, N, Co, 28, 28, L.ptr(gam), L.ptr(bet), L.ptr(rm),
                   L.ptr(rv), 0.1, 1e-5, L.ptr(mean), L.ptr(inv), L.ptr(y), 1, 2, L.ptr(ws), L.stream())
            dg, db, sg, sgx = (torch.empty(Co, device="cuda") for _ in range(4))
            ws2 = torch.empty((L.lib().bnn_bn2d_workspace(N, Co),), dtype=torch.uint8, device="cuda")
            L.call("bnn_bn2d_bwd_stats_q", L.ptr(zq), L.ptr(cb), 2, L.ptr(dyp), N, Co, 28, 28, L.ptr(gam), L.ptr(bet),
                   L.ptr(mean), L.ptr(inv), 1, 2, L.ptr(dg), L.ptr(db), L.ptr(sg), L.ptr(sgx), L.ptr(ws2), L.stream())
            dw, dbc = torch.empty_like(w), torch.empty(Co, device="cuda")
            ws3 = torch.empty((L.lib().bnn_conv2d_bwd_filter_workspace(N, C, Co, K, K, 1),), dtype=torch.uint8,
                              device="cuda")
            L.call("bnn_conv2d_bwd_filter_bn", L.ptr(zq), L.ptr(cb), 2, L.ptr(dyp), L.ptr(mean), L.ptr(inv),
                   L.ptr(gam), L.ptr(bet), L.ptr(sg), L.ptr(sgx), 1.0 / (N * 28 * 28), 1, L.ptr(x), 1, L.ptr(dw),
                   L.ptr(dbc), L.ptr(ws3), N, C, H, W, Co, K, K, 1, pad, 1, 1, L.stream())
            torch.cuda.synchronize()
            cur = {"conv1 zq": zq, "bn mean": mean, "bn invstd": inv, "bn y": y, "running_mean": rm,
                   "running_var": rv, "dgamma": dg, "dbeta": db, "sg": sg, "sgx": sgx, "conv1 dw": dw, "conv1 db": dbc}
            if first is None:
                first = {k: v.clone() for k, v in cur.items()}
                continue
            for k, v in cur.items():
                if not torch.equal(v, first[k]):
                    d = (v.double() - first[k].double()).abs()
                    e = bad.setdefault(k, [0, 0.0, 0])
                    e[0] += 1
                    e[1] = max(e[1], float(d.max()))
                    e[2] = max(e[2], int((d > 0).sum()))
        reps = r
        lines = [f"rank {rank}: {reps} repetitions identical at every stage"] if not bad else []
        for k, (cnt, dmax, nel) in bad.items():
            lines.append(f"rank {rank}: {k:14s} differs in {cnt}/{reps - 1} reps, max|d| {dmax:.3e}, up to {nel} elements")
        q.put((rank, lines))
    except Exception:
        import traceback
        q.put((rank, ["ERR " + traceback.format_exc()]))


def main():
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    N = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    secs = float(sys.argv[4]) if len(sys.argv) > 4 else 0.0
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, R, N, q, secs)) for r in range(P)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=600) for _ in procs)
    for p in procs:
        p.join(timeout=30)
    for r in sorted(out):
        for line in out[r]:
            print(line, flush=True)


if __name__ == "__main__":
    main()

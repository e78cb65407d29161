"""Stage-by-stage trace of the BinCNN step under GPU contention: the forward / backward of every
libbnn autograd Function is wrapped to clone what it hands on (dense outputs, and the tensors a
compact placeholder carries), each of P processes repeats the same step R times, and the first
stage (in execution order) whose tensors differ from repetition 0 is reported per repetition.

    RACE_PROBE_FLAGS="C1BN=0" python tools/race_trace.py [processes] [repetitions] [batch]
"""
import os
import sys

import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "distributed-mnist-bnns_amd")


def _tensors(v):
    out = []
    if isinstance(v, torch.Tensor):
        if v.dim() > 0 and v.numel() > 1 and all(s == 0 for s in v.stride()):
            for attr in ("_bnn_zq", "_bnn_c1bn", "_bnn_q6", "_bnn_z16"):
                carried = getattr(v, attr, None)
                if carried is not None:
                    out += [c for c in carried if isinstance(c, torch.Tensor)]
        else:
            out.append(v)
    elif isinstance(v, (tuple, list)):
        for x in v:
            out += _tensors(x)
    return out


def _worker(rank, reps, N, q):
    try:
        sys.path.insert(0, PKG)
        torch.cuda.set_device(0)
        from bnn_amd import functional as BF
        from bnn_amd import nets
        for kv in filter(None, os.environ.get("RACE_PROBE_FLAGS", "").split(",")):
            k, v = kv.split("=")
            setattr(BF, k, bool(int(v)))
        trace = []

        def wrap(cls, name):
            fwd, bwd = cls.forward, cls.backward

            def f(ctx, *a, **k):
                y = fwd(ctx, *a, **k)
                trace.append((f"{name}.fwd", [t.detach().clone() for t in _tensors(y)]))
                return y

            def b(ctx, *g):
                r = bwd(ctx, *g)
                trace.append((f"{name}.bwd", [t.detach().clone() for t in _tensors(r)]))
                return r

            cls.forward, cls.backward = staticmethod(f), staticmethod(b)

        for cls in (BF.BinaryConv2dFunction, BF.BatchNorm2dHardtanhPoolFunction, BF.LinearNSmallFunction,
                    BF.CrossEntropyFunction):
            wrap(cls, cls.__name__.replace("Function", ""))
        # RACE_MITIGATE: sync_before / sync_after the BatchNorm2d forward, clone_zq (a fresh copy of the
        # compact input), zero_ws (workspaces and outputs zero-filled instead of torch.empty)
        mit = os.environ.get("RACE_MITIGATE", "")
        keep = []
        rereads = []
        evict_buf = torch.empty(2 ** 27, device="cuda") if "evict" in mit else None
        bnf = BF.BatchNorm2dHardtanhPoolFunction.forward

        def bn_fwd(ctx, x, *a):
            if "sync_before" in mit:
                torch.cuda.synchronize()
            if "evict" in mit:
                # stream 512 MiB through the caches (every XCD's L2 is 4 MiB) before the BatchNorm2d reads
                evict_buf.fill_(1.0)
                evict_buf.sum()
            if getattr(x, "_bnn_zq", None) is not None and ("clone_" in mit):
                zq = x._bnn_zq
                cq = "clone_zq" in mit or "clone_q" in mit
                cb = "clone_zq" in mit or "clone_b" in mit
                if "keep" in mit:
                    keep.append(zq)
                x._bnn_zq = (zq[0].clone() if cq else zq[0],
                             zq[1].clone() if (cb and zq[1] is not None) else zq[1], zq[2])
            y = bnf(ctx, x, *a)
            if "reread" in mit and getattr(x, "_bnn_zq", None) is not None:
                # the same compact input through bnn_bn2d_fwd_train_q again, 4 times: do repeated
                # reads of one buffer agree within this step?
                from bnn_amd import _lib as L
                zq = x._bnn_zq
                N, C, H, W = x.shape
                for _ in range(4):
                    y2 = torch.empty_like(y)
                    mean, inv = torch.empty(C, device=y.device), torch.empty(C, device=y.device)
                    ws = torch.empty((L.lib().bnn_bn2d_workspace(N, C),), dtype=torch.uint8, device=y.device)
                    L.call("bnn_bn2d_fwd_train_q", L.ptr(zq[0]), L.ptr(zq[1]), zq[2], N, C, H, W, L.ptr(a[0]),
                           L.ptr(a[1]), None, None, 0.1, float(a[6]), L.ptr(mean), L.ptr(inv), L.ptr(y2), 1, 2,
                           L.ptr(ws), L.stream())
                    if not torch.equal(y2, y):
                        rereads.append(int((y2 != y).sum()))
            if "sync_after" in mit:
                torch.cuda.synchronize()
            return y

        BF.BatchNorm2dHardtanhPoolFunction.forward = staticmethod(bn_fwd)
        if "zero_ws" in mit:
            _empty = torch.empty

            def zempty(*a, **k):
                return torch.zeros(*a, **k)

            BF.torch.empty = zempty
        torch.manual_seed(100)
        m = nets.BinCNN(org_protocol=False, mutate_input=False, fused_bn=True).cuda().train()
        g = torch.Generator(device="cuda").manual_seed(1234 + rank)
        u = torch.randint(0, 256, (N, 1, 28, 28), generator=g, device="cuda").to(torch.uint8)
        u = torch.where(torch.rand(u.shape, generator=g, device="cuda") < 0.807, torch.zeros_like(u), u)
        x = u.float().div(255.0)
        y = torch.randint(0, 10, (N,), generator=g, device="cuda")
        first, lines = None, []
        for r in range(reps):
            trace.clear()
            keep.clear()
            m.zero_grad(set_to_none=True)
            torch.nn.functional.cross_entropy(m(x), y).backward()
            torch.cuda.synchronize()
            cur = list(trace)
            if first is None:
                first = cur
                continue
            for i, ((n0, t0), (n1, t1)) in enumerate(zip(first, cur)):
                assert n0 == n1, (n0, n1)
                diff = [j for j, (a, b) in enumerate(zip(t0, t1)) if not torch.equal(a, b)]
                if diff:
                    j = diff[0]
                    d = (t1[j].double() - t0[j].double()).abs()
                    lines.append(f"rank {rank} rep {r}: first difference at stage {i} {n0} tensor {j} "
                                 f"{tuple(t0[j].shape)} {t0[j].dtype}: {int((d > 0).sum())} elements, max|d| "
                                 f"{float(d.max()):.3e}; differing tensors there {diff}")
                    break
        if "reread" in mit:
            lines.append(f"rank {rank}: re-reads of the same compact input that differed from the step's own "
                         f"BatchNorm2d output: {len(rereads)} (elements {rereads[:8]})")
        if not lines:
            lines.append(f"rank {rank}: {reps} repetitions identical at all {len(first)} stages "
                         f"({', '.join(n for n, _ in first)})")
        q.put((rank, lines))
    except Exception:
        import traceback
        q.put((rank, ["ERR " + traceback.format_exc()]))


def main():
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    N = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, R, N, q)) for r in range(P)]
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

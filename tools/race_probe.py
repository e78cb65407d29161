"""Run-to-run determinism of the fused training step under GPU contention: P processes share the
GPU, each recomputing the same forward + backward R times from the same state and comparing every
gradient (and the loss) with its first repetition, bit for bit.  A kernel with a race (a missing
barrier, an LDS hazard) that single-process scheduling hides shows up here as differing elements.

    python tools/race_probe.py [processes] [repetitions] [kinds...]

RACE_PROBE_FLAGS="C1BN=0,ZQ=0" sets functional's switches of those names before the runs.
"""
import os
import sys

import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "distributed-mnist-bnns_amd")

KINDS = {"cnn": 256, "config2": 100, "mlp": 512, "cnn4k": 4096}


def _make(kind):
    from bnn_amd import nets
    torch.manual_seed(100)
    if kind.startswith("cnn"):
        m = nets.BinCNN(org_protocol=False, mutate_input=False, fused_bn=True)
    elif kind == "config2":
        m = nets.Net(org_protocol=False, mutate_input=False, fused_bn=True)
    else:
        m = nets.MLP(512, 256, 256, p_drop=0.0, org_protocol=False, mutate_input=False, fused_bn=True)
    return m.cuda().train()


def _worker(rank, reps, kinds, q):
    try:
        sys.path.insert(0, PKG)
        torch.cuda.set_device(0)
        from bnn_amd import functional as BF
        for kv in filter(None, os.environ.get("RACE_PROBE_FLAGS", "").split(",")):
            k, v = kv.split("=")
            setattr(BF, k, bool(int(v)))
        lines = []
        for kind in kinds:
            batch = KINDS[kind]
            m = _make(kind)
            g = torch.Generator(device="cuda").manual_seed(1234 + rank)
            u = torch.randint(0, 256, (batch, 1, 28, 28), generator=g, device="cuda").to(torch.uint8)
            u = torch.where(torch.rand(u.shape, generator=g, device="cuda") < 0.807, torch.zeros_like(u), u)
            x = u.float().div(255.0) if kind.startswith("cnn") else u
            y = torch.randint(0, 10, (batch,), generator=g, device="cuda")
            first = None
            bad = {}
            for r in range(reps):
                for p in m.parameters():
                    p.grad = None
                torch.manual_seed(1000 + rank)
                loss = torch.nn.functional.cross_entropy(m(x), y)
                loss.backward()
                cur = [("loss", loss.detach().reshape(1).clone())] + [(n, p.grad.detach().clone())
                                                                    for n, p in m.named_parameters()]
                if first is None:
                    first = cur
                    continue
                for (n, a), (_, b) in zip(first, cur):
                    if not torch.equal(a, b):
                        d = (a - b).abs()
                        k = bad.setdefault(n, [0, 0.0, 0, float(a.abs().max())])
                        k[0] += 1
                        k[1] = max(k[1], float(d.max()))
                        k[2] = max(k[2], int((d > 0).sum()))
            torch.cuda.synchronize()
            if not bad:
                lines.append(f"rank {rank} {kind}: {reps} repetitions identical")
            for n, (cnt, dmax, nel, gmax) in bad.items():
                lines.append(f"rank {rank} {kind}: {n:20s} differs in {cnt}/{reps - 1} reps, max|d| {dmax:.3e} "
                             f"(max|g| {gmax:.2e}), up to {nel} elements")
        q.put((rank, lines))
    except Exception:
        import traceback
        q.put((rank, ["ERR " + traceback.format_exc()]))


def main():
    procs_n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    kinds = sys.argv[3:] or ["cnn", "config2", "mlp"]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, reps, kinds, q)) for r in range(procs_n)]
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

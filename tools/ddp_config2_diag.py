"""Two gloo ranks on one GPU, BASELINE config 2's Net (r = 3, batch 100 per rank): per step and per
copy (GradExchange / torch DDP / a plain copy) the hand-off counters that fired, and every
parameter's gradient against the exact average of the plain copies' gradients -- which copy
departs, at which step, on which parameter.  DIAG_EXCHANGE="direct_write=0,broadcast_buffers=0"
passes those GradExchange options.

    python tools/ddp_config2_diag.py [steps]
"""
import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "distributed-mnist-bnns_amd")
COUNTERS = ("Z16_HANDOFFS", "S20_HANDOFFS", "Q6_HANDOFFS", "I8C_HANDOFFS", "HEAD_CALLS")


def _worker(rank, world, port, steps, q):
    try:
        sys.path.insert(0, PKG)
        os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from bnn_amd import functional as BF
        from bnn_amd import nets
        from bnn_amd.parallel import GradExchange
        opts = {}
        for kv in filter(None, os.environ.get("DIAG_EXCHANGE", "").split(",")):
            k, v = kv.split("=")
            opts[k] = bool(int(v))

        def make():
            torch.manual_seed(100 + rank)
            return nets.Net(org_protocol=False, mutate_input=False, fused_bn=True).cuda().train()

        ours, ref, plain = make(), make(), make()
        ex = GradExchange(ours, bucket_mb=25.0, **opts)
        # record every bucket decrement and launch, in order
        names = {id(p): n for n, p in ours.named_parameters()}
        events = []
        _hook_orig, _gw_orig, _launch_orig = ex._make_hook, ex.grad_written, ex._launch_ready

        def _gw(p):
            events.append(("written", names[id(p)]))
            return _gw_orig(p)

        def _launch():
            before = ex._next
            _launch_orig()
            if ex._next != before:
                events.append(("launch", tuple(range(before, ex._next))))

        ex.grad_written, ex._launch_ready = _gw, _launch
        for h in ex._handles:
            h.remove()
        ex._handles = []
        for p in [p for p in ours.parameters() if p.requires_grad]:
            def mk(p):
                inner = _hook_orig(ex._param_buckets[p])

                def hook(pp):
                    events.append(("hook", names[id(pp)]))
                    return inner(pp)
                return hook
            ex._handles.append(p.register_post_accumulate_grad_hook(mk(p)))
        if ex.broadcast_buffers:
            ex._handles.append(ours.register_forward_pre_hook(lambda m, inp: ex.sync_buffers()))
        lines_b = [f"rank {rank} buckets: " + "; ".join(
            f"{i}: " + ",".join(n for n, p in ours.named_parameters() if i in ex._param_buckets[p])
            for i in range(len(ex.buckets)))]
        ddp = torch.nn.parallel.DistributedDataParallel(ref, device_ids=[0])
        for p in plain.parameters():
            dist.broadcast(p.data, src=0)
            BF.invalidate_packed(p)
        g = torch.Generator(device="cuda").manual_seed(1234 + rank)
        crit = torch.nn.CrossEntropyLoss()
        lines = list(lines_b)
        for step in range(steps):
            u = torch.randint(0, 256, (100, 1, 28, 28), generator=g, device="cuda").to(torch.uint8)
            u = torch.where(torch.rand(u.shape, generator=g, device="cuda") < 0.807, torch.zeros_like(u), u)
            y = torch.randint(0, 10, (100,), generator=g, device="cuda")
            ex.zero_grad()
            events.clear()
            ref.zero_grad(set_to_none=True)
            for p in plain.parameters():
                p.grad = None
            fired = {}
            for name, m_, fn in (("ours", ours, None), ("ddp", ddp, None), ("plain", plain, None)):
                c0 = {c: getattr(BF, c) for c in COUNTERS}
                torch.manual_seed(1000 + 10 * step + rank)
                crit(m_(u), y).backward()
                if name == "ours":
                    events.append(("finish", ""))
                    ex.finish()
                    lines.append(f"rank {rank} step {step} events: {events}")
                fired[name] = tuple(getattr(BF, c) - c0[c] for c in COUNTERS)
            lines.append(f"rank {rank} step {step} hand-offs {COUNTERS}: {fired}")
            for (n, p), q_, r_ in zip(ours.named_parameters(), ref.parameters(), plain.parameters()):
                gs = [torch.empty_like(r_.grad) for _ in range(world)]
                dist.all_gather(gs, r_.grad.contiguous())
                avg = sum(gs) / world
                for who, gg in (("exchange", p.grad), ("ddp", q_.grad)):
                    if not torch.equal(gg, avg):
                        d = (gg - avg).abs()
                        lines.append(f"rank {rank} step {step} {who:8s} {n:12s} differs: {int((d > 0).sum())} elements, "
                                     f"max|d| {float(d.max()):.3e}, max|g| {float(avg.abs().max()):.3e}")
                r_.grad = avg
            with torch.no_grad():
                for m_ in (ours, ref, plain):
                    for p in m_.parameters():
                        p.add_(p.grad, alpha=-0.01)
                        BF.invalidate_packed(p)
        ex.remove()
        q.put((rank, lines))
        dist.destroy_process_group()
    except Exception:
        import traceback
        q.put((rank, ["ERR " + traceback.format_exc()]))


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, steps, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=30)
    for r in sorted(out):
        for line in out[r]:
            print(line, flush=True)


if __name__ == "__main__":
    main()

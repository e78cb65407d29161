"""Two-rank gloo diagnostic on one GPU: three copies of a fused net per rank -- plain (no exchange),
ours (parallel.GradExchange) and ref (torch DDP) -- one step each on the same batch and dropout
seed; the plain gradients are all-gathered and averaged by hand; prints, per parameter, whether
ours / ref equal that average (and plain equals ours' local gradient before the exchange).

    python tools/ddp_diag.py [config2|mlp|cnn]
"""
import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "distributed-mnist-bnns_amd")


def worker(rank, port, kind, q):
    sys.path.insert(0, PKG)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    from bnn_amd import nets
    from bnn_amd.parallel import GradExchange
    batch = {"config2": 100, "mlp": 512, "cnn": 256}[kind]

    def make():
        torch.manual_seed(100 + (rank if "perrank" in sys.argv else 0))
        if kind == "cnn":
            m = nets.BinCNN(org_protocol=False, mutate_input=False, fused_bn=True)
        elif kind == "config2":
            m = nets.Net(org_protocol=False, mutate_input=False, fused_bn=True)
        else:
            m = nets.MLP(512, 256, 256, p_drop=0.0, org_protocol=False, mutate_input=False, fused_bn=True)
        return m.cuda().train()

    g = torch.Generator(device="cuda").manual_seed(1234 + rank)
    u = torch.randint(0, 256, (batch, 1, 28, 28), generator=g, device="cuda").to(torch.uint8)
    x = u.float().div(255.0) if kind == "cnn" else u
    y = torch.randint(0, 10, (batch,), generator=g, device="cuda")
    crit = torch.nn.CrossEntropyLoss()
    plain, ours, ref = make(), make(), make()
    from bnn_amd import functional as BF
    for p in plain.parameters():                 # rank 0's weights, as the exchange / DDP broadcast them
        dist.broadcast(p.data, src=0)
        BF.invalidate_packed(p)
    for b in plain.buffers():
        dist.broadcast(b, src=0)
    ex = GradExchange(ours, bucket_mb=1.0)
    ddp = torch.nn.parallel.DistributedDataParallel(ref, device_ids=[0])
    torch.manual_seed(7 + rank)
    crit(plain(x), y).backward()
    ex.zero_grad()
    torch.manual_seed(7 + rank)
    crit(ours(x), y).backward()
    local = {n: p.grad.detach().clone() for n, p in ours.named_parameters()}
    ex.finish()
    torch.manual_seed(7 + rank)
    crit(ddp(x), y).backward()
    lines = []
    for (n, p), po, pr in zip(plain.named_parameters(), ours.parameters(), ref.parameters()):
        gs = [torch.zeros_like(p.grad) for _ in range(2)]
        dist.all_gather(gs, p.grad.detach().contiguous())
        avg = (gs[0] + gs[1]) / 2
        avg2 = gs[0] / 2 + gs[1] / 2
        d = lambda a, b: float((a - b).abs().max())   # noqa: E731
        lines.append(f"r{rank} {n:18s} plain=ours_local {torch.equal(p.grad, local[n])} "
                     f"ours=avg {torch.equal(po.grad, avg)} ({d(po.grad, avg):.1e}) ref=avg {torch.equal(pr.grad, avg)} "
                     f"({d(pr.grad, avg):.1e}) avg=avg2 {torch.equal(avg, avg2)}")
    q.put("\n".join(lines))
    ex.remove()
    dist.destroy_process_group()


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "cnn"
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, port, kind, q)) for r in range(2)]
    for p in ps:
        p.start()
    for _ in ps:
        print(q.get(timeout=120))
    for p in ps:
        p.join(timeout=30)


if __name__ == "__main__":
    main()

"""One-rank gloo: the fused BinCNN under torch DDP vs the same model alone -- hand-off counters and
the conv weight gradients (does DDP keep the conv1 / BatchNorm2d hand-off?)."""
import os
import socket
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-mnist-bnns_amd"))


def main():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(s.getsockname()[1])
    s.close()
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=0, world_size=1)
    from bnn_amd import functional as BF
    from bnn_amd import nets

    def make():
        torch.manual_seed(100)
        return nets.BinCNN(org_protocol=False, mutate_input=False, fused_bn=True).cuda().train()

    g = torch.Generator(device="cuda").manual_seed(5)
    x = torch.randint(0, 256, (256, 1, 28, 28), generator=g, device="cuda").float().div(255.0)
    y = torch.randint(0, 10, (256,), generator=g, device="cuda")
    plain, ref = make(), make()
    ddp = torch.nn.parallel.DistributedDataParallel(ref, device_ids=[0])
    for name, m in (("plain", plain), ("ddp", ddp)):
        c0 = (BF.C1BN_HANDOFFS, BF.ZQ_HANDOFFS)
        out = m(x)
        print(name, "output type", type(out), out.requires_grad, "grad_fn", type(out.grad_fn).__name__)
        torch.nn.functional.cross_entropy(out, y).backward()
        print(name, "C1BN / ZQ hand-offs", BF.C1BN_HANDOFFS - c0[0], BF.ZQ_HANDOFFS - c0[1])
    for (n, p), q in zip(plain.named_parameters(), ref.parameters()):
        print(f"{n:18s} equal {torch.equal(p.grad, q.grad)} max|d| {float((p.grad - q.grad).abs().max()):.2e} "
              f"max|g| {float(p.grad.abs().max()):.2e}")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

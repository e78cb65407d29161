"""Which form of the one-rank RCCL step is not repeatable?  (tests/test_gpu_rccl.py::
test_rccl_exchange_captured_in_graph[mlp] failed once in round 6: the 3rd loss of the eager run and
of the graph replays differed by 1.1e-5.)  One process, no other GPU work: the fused MLP of that
test (1024-512-512, dropout 0.3, batch 1024) trained 5 steps from the same state REPS times in each of
three forms -- eager without exchange, eager with the one-rank RCCL exchange, GraphedStep with the
exchange -- and every run's losses and final parameters compared with the form's first run and
across forms.

    python tools/det_rccl_probe.py [reps]
"""
import os
import socket
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-mnist-bnns_amd"))


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(s.getsockname()[1])
    s.close()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    from bnn_amd.parallel import init_rccl
    init_rccl(dev, 0, 1)
    import torch.distributed as dist
    from bnn_amd import functional as BF
    from bnn_amd import nets
    from bnn_amd.data import synthetic_mnist
    from bnn_amd.graph import GraphedStep
    from bnn_amd.optim import LatentAdam
    from bnn_amd.parallel import GradExchange
    x, y = synthetic_mnist(1024, seed=321, device=dev)
    crit = torch.nn.CrossEntropyLoss()

    def run(form):
        torch.manual_seed(7)
        m = nets.MLP(1024, 512, 512, p_drop=0.3, org_protocol=False, mutate_input=False, fused_bn=True).to(dev).train()
        torch.manual_seed(99)
        ds = BF.DeviceStep(dev).activate()
        try:
            ex = GradExchange(m, bucket_mb=0.5, force_collectives=True) if form != "eager" else None
            opt = LatentAdam(m.parameters(), lr=0.01, clamp_params=nets.binary_params(m), device_step=ds)

            def step():
                if ex is not None:
                    ex.zero_grad()
                else:
                    for p in m.parameters():
                        p.grad = None
                loss = crit(m(x), y)
                loss.backward()
                if ex is not None:
                    ex.finish()
                opt.step()
                return loss
            losses = []
            if form == "graph":
                g = GraphedStep(step, opt, ds, warmup=2)
                for _ in range(3):
                    losses.append(float(g().item()))
            else:
                for i in range(5):
                    loss = step()
                    if i >= 2:
                        losses.append(float(loss.item()))
            torch.cuda.synchronize()
            state = [v.detach().cpu().numpy().copy() for v in m.state_dict().values()]
            if ex is not None:
                ex.remove()
            return losses, state
        finally:
            ds.deactivate()

    results = {}
    for form in ("eager", "exchange", "graph"):
        results[form] = [run(form) for _ in range(reps)]
    ref_l, ref_s = results["eager"][0]
    for form, rs in results.items():
        l0, s0 = rs[0]
        diffs = []
        for i, (l, st) in enumerate(rs):
            same = l == l0 and all(np.array_equal(a, b) for a, b in zip(st, s0))
            diffs.append("=" if same else "X")
        cross = l0 == ref_l and all(np.array_equal(a, b) for a, b in zip(s0, ref_s))
        print(f"{form:9s}: runs vs its first run {''.join(diffs)}; first run == eager's first run: {cross}; "
              f"losses {['%.8f' % v for v in l0]}", flush=True)
        for i, (l, st) in enumerate(rs):
            if l != l0:
                print(f"   run {i}: losses {['%.8f' % v for v in l]}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

"""The training loop's criterion on libbnn (bnn_cross_entropy_*, bnn_amd.nn.CrossEntropyLoss):
torch.nn.CrossEntropyLoss() (reduction 'mean') applied to the nets' LogSoftmax output, as the
reference's training loop does (mnist-dist2.py:118-137).

* the loss within 1e-6 (relative) of torch's and of a float64 restatement, the input gradient within
  1e-6 of torch's (elementwise, relative to the largest entry), over row counts from 1 to the wide
  batch and every supported class count;
* deterministic (fixed-order sums: two runs bit-identical); a target outside [0, C) gives NaN;
* non-default arguments fall back to torch; a HIP-graph-captured step with it replays equal to
  the eager device-step steps bit for bit.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def F():
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    from bnn_amd import functional
    return functional


def _case(M, C, seed, logprob=True):
    g = torch.Generator(device="cuda").manual_seed(seed)
    z = torch.randn(M, C, generator=g, device="cuda") * 3.0
    p = torch.log_softmax(z, dim=1) if logprob else z
    y = torch.randint(0, C, (M,), generator=g, device="cuda")
    return p, y


@pytest.mark.parametrize("M,C", [(1, 10), (7, 10), (300, 10), (4096, 10), (65536, 10), (1000, 2), (513, 16),
                                 (256, 32), (1000, 64)])
def test_cross_entropy_matches_torch(F, M, C):
    for logprob in (True, False):
        p, y = _case(M, C, M * 7 + C, logprob)
        a = p.clone().requires_grad_(True)
        b = p.clone().requires_grad_(True)
        la = F.cross_entropy(a, y)
        lb = torch.nn.functional.cross_entropy(b, y)
        la.backward()
        lb.backward()
        ref = float(torch.nn.functional.cross_entropy(p.double(), y))
        assert abs(float(la) - float(lb)) <= 1e-6 * max(1.0, abs(float(lb)))
        assert abs(float(la) - ref) <= 1e-6 * max(1.0, abs(ref))
        ga, gb = a.grad, b.grad
        assert (ga - gb).abs().max().item() <= 1e-6 * gb.abs().max().item()


def test_cross_entropy_deterministic_and_nan_target(F):
    p, y = _case(65536, 10, 3)
    l1 = F.cross_entropy(p, y)
    l2 = F.cross_entropy(p, y)
    assert torch.equal(l1, l2)
    y2 = y.clone()
    y2[123] = 10                       # outside [0, C)
    assert torch.isnan(F.cross_entropy(p, y2)).item()


@pytest.mark.parametrize("M", [300, 65536])
@pytest.mark.parametrize("ignore", [-100, 3])
def test_cross_entropy_ignore_index_matches_torch(F, M, ignore):
    """nn.CrossEntropyLoss(ignore_index=...) semantics: ignored rows add no loss term and get a zero
    gradient row, the mean is over the others (they used to be counted / NaN)."""
    from bnn_amd.nn import CrossEntropyLoss
    p, y = _case(M, 10, 11)
    y = y.clone()
    y[::7] = ignore
    a = p.clone().requires_grad_(True)
    b = p.clone().requires_grad_(True)
    la = CrossEntropyLoss(ignore_index=ignore)(a, y)
    lb = torch.nn.functional.cross_entropy(b, y, ignore_index=ignore)
    la.backward()
    lb.backward()
    assert abs(float(la) - float(lb)) <= 1e-6 * max(1.0, abs(float(lb)))
    assert (a.grad - b.grad).abs().max().item() <= 1e-6 * b.grad.abs().max().item()
    assert bool((a.grad[::7] == 0).all())
    yall = torch.full_like(y, ignore)                        # every row ignored: torch's 0 / 0
    c = p.clone().requires_grad_(True)
    lc = CrossEntropyLoss(ignore_index=ignore)(c, yall)
    lc.backward()
    assert torch.isnan(lc).item() and bool((c.grad == 0).all())


def test_module_routes_and_falls_back(F):
    from bnn_amd.nn import CrossEntropyLoss
    p, y = _case(300, 10, 9)
    assert torch.equal(CrossEntropyLoss()(p, y), F.cross_entropy(p, y))
    s = CrossEntropyLoss(reduction="sum")(p, y)              # torch's path
    assert abs(float(s) - float(torch.nn.functional.cross_entropy(p, y, reduction="sum"))) <= 1e-4
    q, yq = _case(300, 7, 9)                                 # C = 7: torch's path
    assert abs(float(CrossEntropyLoss()(q, yq)) - float(torch.nn.functional.cross_entropy(q, yq))) <= 1e-6


def test_mlp_step_with_libbnn_cross_entropy(F):
    """A fused-MLP training step with the libbnn criterion against the same step with torch's: loss
    within 1e-6, every parameter gradient within 1e-5 of torch's (the criterion's gradient enters
    the backward at ~1e-7); the biases ahead of a BatchNorm, analytically zero, within 1e-7."""
    from bnn_amd import nets
    from bnn_amd.nn import CrossEntropyLoss
    g = torch.Generator(device="cuda").manual_seed(4)
    u = torch.randint(0, 256, (2048, 1, 28, 28), generator=g, device="cuda").to(torch.uint8)
    y = torch.randint(0, 10, (2048,), generator=g, device="cuda")
    res = []
    for crit in (CrossEntropyLoss(), torch.nn.CrossEntropyLoss()):
        torch.manual_seed(0)
        m = nets.MLP(512, 256, 128, p_drop=0.0, org_protocol=False, mutate_input=False, fused_bn=True).cuda().train()
        loss = crit(m(u), y)
        loss.backward()
        res.append((float(loss), {k: p.grad.detach().clone() for k, p in m.named_parameters()}))
    (la, ga), (lb, gb) = res
    assert abs(la - lb) <= 1e-6 * max(1.0, abs(lb))
    for k in gb:
        if k in ("fc1.bias", "fc2.bias", "fc3.bias"):   # ahead of a BatchNorm: analytically zero
            assert (ga[k] - gb[k]).abs().max().item() <= 1e-7, k
            continue
        err = (ga[k] - gb[k]).norm().item() / max(gb[k].norm().item(), 1e-30)
        assert err <= 1e-5, (k, err)


def test_graph_replays_with_libbnn_cross_entropy(F):
    from bnn_amd import nets
    from bnn_amd.graph import GraphedStep
    from bnn_amd.nets import binary_params
    from bnn_amd.nn import CrossEntropyLoss
    from bnn_amd.optim import LatentAdam
    g = torch.Generator(device="cuda").manual_seed(3)
    u = torch.randint(0, 256, (256, 1, 28, 28), generator=g, device="cuda").to(torch.uint8)
    y = torch.randint(0, 10, (256,), generator=g, device="cuda")
    crit = CrossEntropyLoss()
    runs = []
    for graphed in (False, True):
        torch.manual_seed(5)
        m = nets.MLP(256, 128, 64, p_drop=0.3, org_protocol=False, mutate_input=False, fused_bn=True).cuda().train()
        torch.manual_seed(99)
        ds = F.DeviceStep().activate()
        try:
            opt = LatentAdam(m.parameters(), lr=0.01, clamp_params=binary_params(m), device_step=ds)

            def step():
                for p in m.parameters():
                    p.grad = None
                loss = crit(m(u), y)
                loss.backward()
                opt.step()
                return loss
            losses = []
            if graphed:
                gs = GraphedStep(step, opt, ds, warmup=2)
                for _ in range(3):
                    losses.append(float(gs().item()))
            else:
                for i in range(5):
                    loss = step()
                    if i >= 2:
                        losses.append(float(loss.item()))
            torch.cuda.synchronize()
            runs.append(({k: v.detach().cpu().numpy().copy() for k, v in m.state_dict().items()}, losses))
        finally:
            ds.deactivate()
    (a, la), (b, lb) = runs
    assert la == lb
    for k in a:
        assert np.array_equal(a[k], b[k]), k

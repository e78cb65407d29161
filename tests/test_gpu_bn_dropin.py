"""bnn_amd.nn.BatchNorm1d: torch.nn.BatchNorm1d's module on libbnn's BatchNorm passes, the drop-in a
user of the reference swaps for the Nets' bn1..bn3 (mnist-dist2.py:52-57).  Checked against torch's
own module on the same inputs, parameters and buffers: outputs, the three gradients, running
statistics and num_batches_tracked, in every mode torch's _BatchNorm.forward has (momentum /
cumulative average, track_running_stats off, affine off, eval), and the reference Net with the
swapped modules through the unchanged mnist-dist2 loop."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def NN():
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    from bnn_amd import nn as bnn_nn
    return bnn_nn


def _pair(NN, C, **kw):
    ref = torch.nn.BatchNorm1d(C, **kw).cuda()
    ours = NN.BatchNorm1d(C, **kw).cuda()
    with torch.no_grad():
        if ref.affine:
            ref.weight.uniform_(0.5, 1.5)
            ref.bias.uniform_(-0.5, 0.5)
    ours.load_state_dict(ref.state_dict())
    return ref, ours


@pytest.mark.parametrize("M,C,kw", [
    (4096, 3072, {}),
    (100, 768, {}),
    (257, 192, {"momentum": None}),
    (64, 192, {"track_running_stats": False}),
    (512, 256, {"affine": False}),
    (1000, 1536, {"momentum": 0.3, "eps": 1e-3}),
])
def test_bn_dropin_matches_torch(NN, M, C, kw):
    g = torch.Generator(device="cuda").manual_seed(M + C)
    ref, ours = _pair(NN, C, **kw)
    for step in range(3):
        x = (torch.randn(M, C, generator=g, device="cuda") * 3 + 1.5)
        gy = torch.randn(M, C, generator=g, device="cuda")
        xr, xo = x.clone().requires_grad_(), x.clone().requires_grad_()
        yr, yo = ref(xr), ours(xo)
        assert torch.allclose(yo, yr, atol=1e-5, rtol=1e-5), (step, float((yo - yr).abs().max()))
        yr.backward(gy)
        yo.backward(gy)
        assert torch.allclose(xo.grad, xr.grad, atol=1e-5, rtol=1e-4), float((xo.grad - xr.grad).abs().max())
        if ref.affine:
            # batch sums over M rows: relative to the gradient's scale
            for a, b in ((ours.weight.grad, ref.weight.grad), (ours.bias.grad, ref.bias.grad)):
                assert torch.allclose(a, b, atol=1e-5 * M ** 0.5, rtol=1e-5), float((a - b).abs().max())
                a.zero_()
                b.zero_()
        for k, v in ref.state_dict().items():
            o = ours.state_dict()[k]
            if v.dtype == torch.long:
                assert torch.equal(o, v), k
            else:
                assert torch.allclose(o, v, atol=1e-6, rtol=1e-5), (k, float((o - v).abs().max()))
    ref.eval()
    ours.eval()
    x = torch.randn(M, C, generator=g, device="cuda")
    yr, yo = ref(x), ours(x)
    assert torch.allclose(yo, yr, atol=1e-5, rtol=1e-5), float((yo - yr).abs().max())


def test_bn_dropin_net_step_matches_torch_bn(NN):
    """The reference Net (r = 3) through the drop-in modules and the unchanged mnist-dist2 loop
    (.org protocol, torch.optim.Adam, CrossEntropyLoss), once with torch's BatchNorm1d and once with
    the libbnn drop-in.  Step 0 (identical weights): loss, every gradient and the BatchNorm buffers
    within fp32 BatchNorm rounding.  Two more steps: the losses stay within 1e-4 (the latents near 0
    may take different signs after an update, so later buffers are not compared element-wise)."""
    from bnn_amd import nets
    from bnn_amd.data import synthetic_mnist
    from bnn_amd.optim import org_protocol_step
    x, y = synthetic_mnist(256, seed=5, device="cuda")
    torch.manual_seed(3)
    a = nets.Net(p_drop=0.0).cuda().train()
    b = nets.Net(p_drop=0.0, dropin_bn=True).cuda().train()
    b.load_state_dict(a.state_dict())
    assert isinstance(b.bn1, NN.BatchNorm1d) and not isinstance(a.bn1, NN.BatchNorm1d)
    opts = [torch.optim.Adam(m.parameters(), lr=0.01) for m in (a, b)]
    crit = torch.nn.CrossEntropyLoss()
    from bnn_amd import functional as BF
    h0 = BF.Q6_HANDOFFS
    for step in range(3):
        losses = []
        for m, opt in zip((a, b), opts):
            opt.zero_grad()
            loss = crit(m(x), y)
            loss.backward()
            if step == 0:
                m._grads = {k: p.grad.detach().clone() for k, p in m.named_parameters()}
            org_protocol_step(m, opt)
            losses.append(float(loss.detach()))
        assert abs(losses[0] - losses[1]) <= 1e-4 * max(1.0, abs(losses[0])), (step, losses)
        if step == 0:
            for k, ga in a._grads.items():
                gb = b._grads[k]
                # a bias in front of a BatchNorm has an exactly-zero gradient in exact arithmetic
                # (fc*.bias: ~1e-11 of rounding either way), hence the absolute floor
                scale = float(ga.abs().max())
                assert float((gb - ga).abs().max()) <= max(1e-4 * scale, 1e-7), (k, float((gb - ga).abs().max()), scale)
            # the buffers (the parameters are compared through their gradients above: Adam's first
            # step moves each by ~lr * sign(grad), which rounding flips where the gradient is ~0)
            sa, sb = a.state_dict(), b.state_dict()
            for k in sa:
                if k.startswith("bn") and ("running" in k or "num_batches" in k):
                    assert torch.allclose(sb[k].float(), sa[k].float(), atol=1e-5, rtol=1e-4), k
    # bn2's gradient reached fc2 with its FP6 digits (no second quantising pass over it)
    assert BF.Q6_HANDOFFS > h0


def test_bn_dropin_handoff_with_a_second_consumer(NN):
    """fc's output feeding the drop-in BatchNorm AND another op: autograd sums the two gradients, so
    fc's backward receives a tensor without the BatchNorm's digits and quantises the sum itself --
    the gradients equal those with torch's BatchNorm1d in the same graph."""
    from models.binarized_modules import BinarizeLinear
    g = torch.Generator(device="cuda").manual_seed(11)
    x = torch.randn(512, 256, generator=g, device="cuda")
    grads = []
    for bn_cls in (torch.nn.BatchNorm1d, NN.BatchNorm1d):
        torch.manual_seed(2)
        fc = BinarizeLinear(256, 128).cuda()
        fc.org_protocol = False
        bn = bn_cls(128).cuda()
        y = fc(x.clone())
        loss = (bn(y) * torch.linspace(-1, 1, 128, device="cuda")).sum() + 0.5 * (y * y).mean()
        loss.backward()
        grads.append((fc.weight.grad.clone(), fc.bias.grad.clone()))
    (wa, ba), (wb, bb) = grads
    assert float((wb - wa).abs().max()) <= 1e-4 * float(wa.abs().max()), float((wb - wa).abs().max())
    assert float((bb - ba).abs().max()) <= 1e-4 * float(ba.abs().max()) + 1e-6


"""GPU parity of the fused head (functional.DropoutBNHardtanhLinearFunction: drop -> bn3 -> htanh3
-> fc4, mnist-dist2.py:69-76) against the unfused libbnn path (dropout_batch_norm_hardtanh + torch
nn.Linear) on the same inputs and dropout seed, and against a float64 restatement.

Bars: output and every gradient norm-wise within 1e-5 (f32 products on the MFMA, f32 sums in
another order than rocBLAS); running statistics bit-identical (the same statistics pass).
"""
import numpy as np
import pytest
import torch

from conftest import rel_err

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def F():
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    from bnn_amd import functional
    return functional


def host(t):
    torch.cuda.synchronize()
    return t.detach().cpu().numpy()


def _modules(C, seed):
    torch.manual_seed(seed)
    bn = torch.nn.BatchNorm1d(C).cuda().train()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.2, 0.2)
    fc = torch.nn.Linear(C, 10).cuda()
    return bn, fc


@pytest.mark.parametrize("M,C,p", [(512, 256, 0.3), (1000, 512, 0.0), (64, 1024, 0.3), (4096, 768, 0.3), (33, 256, 0.3)])
def test_head_matches_unfused(F, M, C, p):
    g = torch.Generator(device="cuda").manual_seed(M + C)
    z0 = (torch.randint(-30, 31, (M, C), generator=g, device="cuda").float() + 0.25)
    dy = torch.randn(M, 10, generator=g, device="cuda")
    outs = []
    for fused in (True, False):
        bn, fc = _modules(C, 3)
        z = z0.clone().requires_grad_(True)
        torch.manual_seed(77)                        # the dropout seed draw
        if fused:
            y = F.dropout_bn_hardtanh_linear(z, p, bn, fc)
        else:
            y = fc(F.dropout_batch_norm_hardtanh(z, p, bn) if p > 0 else F.batch_norm_hardtanh(z, bn))
        y.backward(dy)
        outs.append({"y": host(y), "dz": host(z.grad), "dgw": host(bn.weight.grad), "dgb": host(bn.bias.grad),
                     "dw4": host(fc.weight.grad), "db4": host(fc.bias.grad), "rm": host(bn.running_mean),
                     "rv": host(bn.running_var)})
    a, b = outs
    for k in ("y", "dz", "dgw", "dgb", "dw4", "db4"):
        assert rel_err(a[k], b[k]) <= 1e-5, (k, rel_err(a[k], b[k]))
    assert np.array_equal(a["rm"], b["rm"]) and np.array_equal(a["rv"], b["rv"])


def test_head_against_float64(F):
    """No dropout: y = htanh(BN(z)) W4^T + b4 and its gradients against float64 autograd."""
    M, C = 300, 256
    g = torch.Generator(device="cuda").manual_seed(9)
    z0 = torch.randn(M, C, generator=g, device="cuda") * 3
    dy = torch.randn(M, 10, generator=g, device="cuda")
    bn, fc = _modules(C, 4)
    z = z0.clone().requires_grad_(True)
    y = F.dropout_bn_hardtanh_linear(z, 0.0, bn, fc)
    y.backward(dy)
    zd = z0.double().cpu().requires_grad_(True)
    wd = fc.weight.detach().double().cpu().requires_grad_(True)
    bd = fc.bias.detach().double().cpu().requires_grad_(True)
    gd = bn.weight.detach().double().cpu().requires_grad_(True)
    ed = bn.bias.detach().double().cpu().requires_grad_(True)
    mu = zd.mean(0)
    var = zd.var(0, unbiased=False)
    h = torch.clamp((zd - mu) / torch.sqrt(var + bn.eps) * gd + ed, -1, 1)
    yd = h @ wd.T + bd
    yd.backward(dy.double().cpu())
    assert rel_err(host(y), yd.detach().numpy()) <= 1e-5
    assert rel_err(host(z.grad), zd.grad.numpy()) <= 1e-5
    assert rel_err(host(fc.weight.grad), wd.grad.numpy()) <= 1e-5
    assert rel_err(host(fc.bias.grad), bd.grad.numpy()) <= 1e-6
    assert rel_err(host(bn.weight.grad), gd.grad.numpy()) <= 1e-5


def test_wide_step_with_fused_head_equals_unfused(F):
    """A whole training step of the MLP with and without the fused head: parameter gradients
    within 1e-5 (the head's sums are ordered differently; everything upstream sees dz within it)."""
    from bnn_amd import nets
    grads = []
    for fused in (True, False):
        torch.manual_seed(0)
        m = nets.MLP(512, 256, 128, org_protocol=False, mutate_input=False, fused_bn=True).cuda().train()
        m.fused_head = fused
        g = torch.Generator(device="cuda").manual_seed(5)
        u = torch.randint(0, 256, (1024, 1, 28, 28), generator=g, device="cuda").to(torch.uint8)
        y = torch.randint(0, 10, (1024,), generator=g, device="cuda")
        torch.manual_seed(1)
        torch.nn.CrossEntropyLoss()(m(u), y).backward()
        grads.append({k: host(p.grad) for k, p in m.named_parameters()})
    for k in grads[0]:
        a, b = grads[0][k], grads[1][k]
        if k in ("fc1.bias", "fc2.bias", "fc3.bias"):
            # a bias feeding a BatchNorm has a mathematically zero gradient: both are rounding noise,
            # bounded against the layer's weight gradient instead
            ref = np.linalg.norm(grads[1][k.replace("bias", "weight")])
            assert np.linalg.norm(a - b) <= 1e-5 * ref, k
        else:
            assert rel_err(a, b) <= 2e-5, (k, rel_err(a, b))


@pytest.mark.parametrize("M,N,ld", [(4096, 10, 10), (1, 10, 10), (65, 3, 16), (32768, 16, 16)])
def test_col_sums_narrow_matches_torch(M, N, ld):
    """bnn_col_sums_narrow (the fused head's bias gradient db4 = dY4.sum(0)): the column sums of a
    narrow matrix against float64, within fp32 rounding of the result; repeat calls bit-identical."""
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    from bnn_amd import _lib as L
    g = torch.Generator(device="cuda").manual_seed(M + N)
    y = torch.randn(M, ld, generator=g, device="cuda")
    out = torch.empty(N, device="cuda")
    L.call("bnn_col_sums_narrow", L.ptr(y), M, N, ld, L.ptr(out), L.stream())
    ref = y[:, :N].double().sum(0)
    assert float((out.double() - ref).abs().max()) <= 1e-6 * max(1.0, float(ref.abs().max()))
    out2 = torch.empty_like(out)
    L.call("bnn_col_sums_narrow", L.ptr(y), M, N, ld, L.ptr(out2), L.stream())
    assert torch.equal(out, out2)

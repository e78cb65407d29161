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


def test_dropout_bits_equal_hash_mask(F):
    """bnn_dropout_bits: bit i of the materialised mask = keep(i) of the hash the passes evaluate
    (bnn_dropout_mask), for a ragged n and a seed with all 64 bits used."""
    from bnn_amd import _lib as L
    for n, p, seed in ((1000003, 0.3, 0x9E3779B97F4A7C15), (64 * 64 * 8, 0.5, 7), (77, 0.3, 1)):
        bits = torch.empty(((n + 63) // 64 * 2,), dtype=torch.int32, device="cuda")
        L.call("bnn_dropout_bits", n, p, seed, L.ptr(bits), L.stream())
        L.call("bnn_dropout_bits_clear")
        keep = (F.dropout_mask(n, p, seed) > 0).cpu().numpy()
        w = bits.cpu().numpy().view(np.uint32)
        got = ((w[np.arange(n) >> 5] >> (np.arange(n) & 31).astype(np.uint32)) & 1).astype(bool)
        assert np.array_equal(got, keep), (n, p)


@pytest.mark.parametrize("M,C,z16", [(4096, 768, False), (2048, 1024, True)])
def test_head_with_dropout_bits_bit_identical(F, M, C, z16, monkeypatch):
    """The fused head (and the unfused dropout BatchNorm) with the mask materialised as bits
    (functional.DROP_BITS) equals the per-pass hash bit for bit: output, every gradient, the FP6
    digit hand-off and the running statistics."""
    g = torch.Generator(device="cuda").manual_seed(M)
    z0 = (torch.randint(-30, 31, (M, C), generator=g, device="cuda").float() + 0.25)
    dy = torch.randn(M, 10, generator=g, device="cuda")
    runs = []
    for bits in (False, True):
        monkeypatch.setattr(F, "DROP_BITS", bits)
        for fused in (True, False):
            bn, fc = _modules(C, 5)
            z = z0.clone().requires_grad_(True)
            zin = z
            if z16:     # an int16-carried pre-activation, as fc3's FP4 GEMM hands it to the head
                zin = F._z16_carrier(z0.round().to(torch.int16), torch.full((C,), 0.25, device="cuda"))
            torch.manual_seed(78)
            n0 = F.DROP_BITS_USES
            if fused:
                y = F.dropout_bn_hardtanh_linear(zin if z16 else z, 0.3, bn, fc)
            else:
                y = fc(F.dropout_batch_norm_hardtanh(z, 0.3, bn))
            assert F.DROP_BITS_USES - n0 == int(bits)
            y.backward(dy)
            out = {"y": host(y), "dgw": host(bn.weight.grad), "dgb": host(bn.bias.grad), "dw4": host(fc.weight.grad),
                   "rm": host(bn.running_mean), "rv": host(bn.running_var)}
            if not (fused and z16):
                out["dz"] = host(z.grad)
            runs.append(out)
    for a, b in zip(runs[:2], runs[2:]):
        for k in a:
            assert np.array_equal(a[k], b[k]), k

"""GPU parity of the fused BatchNorm backward + FP6 quantise pass (bnn_bn_bwd_q6) and of the
autograd hand-off that feeds its digits to the next BinarizeLinear backward
(functional._bn_bwd_q6 / _q6_take).

Bars: dz, dgamma, dbeta and every digit byte bit-identical to bnn_bn_bwd (/ bnn_bn_dropout_bwd)
followed by bnn_quant6_rows and bnn_quant6_cols_t on the same dz; the bias gradient (a double
column sum, summed in another order) within 1e-6; a whole training step's parameter gradients
bit-identical with and without the hand-off, bias gradients of the consuming layers within 1e-6.
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


@pytest.mark.parametrize("M,C", [(1000, 192), (100, 64), (333, 128), (4096, 1024), (64, 3072)])
@pytest.mark.parametrize("p", [0.0, 0.3])
def test_bn_bwd_q6_matches_separate_passes(F, M, C, p):
    from bnn_amd import _lib as L
    g = torch.Generator(device="cuda").manual_seed(M + C)
    z = torch.randint(-40, 41, (M, C), generator=g, device="cuda").float() + 0.5 * torch.randn(M, C, generator=g, device="cuda")
    dh = torch.randn(M, C, generator=g, device="cuda") * torch.exp(torch.randn(1, C, generator=g, device="cuda") * 3)
    gw = torch.rand(C, generator=g, device="cuda") + 0.5
    gb = torch.randn(C, generator=g, device="cuda") * 0.1
    rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    mean, invstd, mlo = F._bn_stat_buffers(C, "cuda")
    ws = F._bn_ws(M, C, "cuda")
    seed = 1234
    L.call("bnn_bn_dropout_fwd_train", L.ptr(z), M, C, L.ptr(gw), L.ptr(gb), L.ptr(rm), L.ptr(rv), 0.1, 1e-5,
           L.ptr(mean), L.ptr(invstd), L.ptr(mlo), None, 1, float(p), seed, L.ptr(ws), L.stream())
    # reference: the separate passes
    dz = torch.empty_like(z)
    dgw, dgb = torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
    L.call("bnn_bn_dropout_bwd", L.ptr(z), L.ptr(dh), M, C, L.ptr(gw), L.ptr(gb), L.ptr(mean), L.ptr(invstd),
           L.ptr(mlo), 1, float(p), seed, L.ptr(dz), L.ptr(dgw), L.ptr(dgb), L.ptr(ws), L.stream())
    rows = F.quant6_rows(dz)
    cols, cs = F.quant6_cols_t(dz, want_colsum=True)
    # fused
    dgw2, dgb2 = torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
    dz2 = F._bn_bwd_q6(z, dh, M, C, gw, gb, mean, invstd, mlo, True, p, seed, dgw2, dgb2, F._bn_ws(M, C, "cuda"),
                       "bn_bwd_q6")
    rows2, cols2, cs2 = F._q6_take(dz2)
    assert torch.equal(dz2, dz) and torch.equal(dgw2, dgw) and torch.equal(dgb2, dgb)
    for a, b in ((rows, rows2), (cols, cols2)):
        assert a.Kp == b.Kp and a.rows == b.rows
        assert torch.equal(a.lo, b.lo) and torch.equal(a.hi, b.hi)
        n = a.rows
        assert torch.equal(a.sc[:, :n], b.sc[:, :n])
    assert rel_err(host(cs2), host(dz).astype(np.float64).sum(0)) <= 1e-6
    assert rel_err(host(cs2), host(cs)) <= 1e-6
    assert F._q6_take(dz2) is None                   # taken once


def _wide_step(F, handoff, M=512, width=1024, seed=0):
    from bnn_amd import nets
    F.Q6_HANDOFF = handoff
    try:
        torch.manual_seed(seed)
        m = nets.MLP(width, width, width, org_protocol=False, mutate_input=False, fused_bn=True).cuda().train()
        g = torch.Generator(device="cuda").manual_seed(7)
        u = torch.randint(0, 256, (M, 1, 28, 28), generator=g, device="cuda").to(torch.uint8)
        y = torch.randint(0, 10, (M,), generator=g, device="cuda")
        timer = F.KernelTimer()
        with F.timing(timer):
            torch.nn.CrossEntropyLoss()(m(u), y).backward()
        names = set(timer.summary())
        return {k: host(p.grad) for k, p in m.named_parameters()}, names
    finally:
        F.Q6_HANDOFF = True


def test_training_step_with_handoff_equals_without(F):
    g1, names1 = _wide_step(F, True)
    g0, names0 = _wide_step(F, False)
    assert "bn_bwd_q6" in names1 and names1 & {"bn_dropout_bwd_q6", "bn_head_bwd_q6"}   # the hand-off ran
    assert "quant6_rows_k" not in names1 and "quant6_cols_t_k" not in names1
    assert "bn_bwd_q6" not in names0 and "quant6_rows_k" in names0
    for k in g0:
        if k in ("fc2.bias", "fc3.bias"):             # column sums folded in another order
            assert rel_err(g1[k], g0[k]) <= 1e-6, k
        else:
            assert np.array_equal(g1[k], g0[k]), k

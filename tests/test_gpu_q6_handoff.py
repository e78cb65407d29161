"""GPU parity of the fused BatchNorm backward + FP6 quantise pass (bnn_bn_bwd_q6) and of the
autograd hand-off that feeds its digits to the next BinarizeLinear backward
(functional._bn_bwd_q6 / _q6_take).

Bars: dz, dgamma, dbeta and every digit byte (the rows' residual plane included: the fused pass forms
it with magic fmas, bnn_quant6_rows with rint) bit-identical to bnn_bn_bwd (/ bnn_bn_dropout_bwd)
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
    # the residual plane at every size here (the networks add it from FP6_RES_MIN_ROWS rows on)
    prev = functional.FP6_RES_MIN_ROWS
    functional.FP6_RES_MIN_ROWS = 0
    yield functional
    functional.FP6_RES_MIN_ROWS = prev


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
           L.ptr(mean), L.ptr(invstd), L.ptr(mlo), None, 1, float(p), seed, None, L.ptr(ws), L.stream())
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
        assert (a.res is None) == (b.res is None) and (a.res is None or torch.equal(a.res, b.res))
        n = a.rows
        assert torch.equal(a.sc[:, :n], b.sc[:, :n])
    assert rel_err(host(cs2), host(dz).astype(np.float64).sum(0)) <= 1e-6
    assert rel_err(host(cs2), host(cs)) <= 1e-6
    assert F._q6_take(dz2) is None                   # taken once


def _wide_step(F, handoff, M=512, width=1024, seed=0, bn_epi=False):
    from bnn_amd import nets
    epi0 = F.BN_EPI
    F.Q6_HANDOFF = handoff
    F.BN_EPI = bn_epi           # the statistics' summation order must match for bit-equality
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
        F.BN_EPI = epi0


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


@pytest.mark.parametrize("x_i16,mode", [(False, 1), (True, 1), (False, 2)])
def test_gemm_fp6_bnstats_epilogue(F, x_i16, mode):
    """bnn_gemm_fp6_bnstats: C bit-identical to the plain panel GEMM; its per-tile-row partials of
    sum g, sum g*xhat (g = dy masked by -1 < BN(x) < 1) within 1e-6 of float64 sums of the same
    fp32 quantities; mode 2's max|g| / max|xhat| exact; the folded statistics (bnn_bn_bwd_stats_pre)
    within 1e-6 of bn_bwd's own reduction."""
    from bnn_amd import _lib as L
    M, N, K = 4100, 8192, 2048                    # ragged last tile row; >= 1 round of tiles (unsplit)
    g = torch.Generator(device="cuda").manual_seed(11 + mode)
    dyq = torch.randn(M, K, generator=g, device="cuda")
    w = torch.randint(-1, 2, (N, K), generator=g, device="cuda").float()
    A = F.quant6_rows(dyq)
    P = F.fp4_panels(F.sign_pack_fp4(w)[0], N, K)
    xi = torch.randint(-300, 301, (M, N), generator=g, device="cuda").to(torch.int16)
    xb = torch.randn(N, generator=g, device="cuda")
    x = xi.float() + xb if x_i16 else torch.randn(M, N, generator=g, device="cuda") * 3
    mean, invstd, mlo = F._bn_stat_buffers(N, "cuda")
    rm, rv = torch.zeros(N, device="cuda"), torch.ones(N, device="cuda")
    gam = torch.rand(N, generator=g, device="cuda") + 0.5
    bet = torch.randn(N, generator=g, device="cuda") * 0.2
    L.call("bnn_bn_fwd_train", L.ptr(x), M, N, L.ptr(gam), L.ptr(bet), L.ptr(rm), L.ptr(rv), 0.1, 1e-5,
           L.ptr(mean), L.ptr(invstd), L.ptr(mlo), None, 1, L.ptr(F._bn_ws(M, N, "cuda")), L.stream())
    C0 = F.gemm_fp6(A, None, N, panels=P, panel_ks=K // 64)
    C1, part, R = F.gemm_fp6_bnstats(A, P, K // 64, N, xi if x_i16 else x, xb if x_i16 else None, x_i16, mean,
                                     mlo, invstd, gam, bet, mode)
    assert torch.equal(C0, C1)
    xh = ((x - mean) - mlo) * invstd
    yv = (xh.double() * gam.double() + bet.double()).float()   # fmaf(xh, gamma, beta): one rounding
    gg = torch.where((yv > -1) & (yv < 1), C0, torch.zeros_like(C0))
    pr = part.view(-1, R, N)
    assert rel_err(host(pr[0]).astype(np.float64).sum(0), host(gg).astype(np.float64).sum(0)) < 1e-6
    assert rel_err(host(pr[1]).astype(np.float64).sum(0), (host(gg).astype(np.float64) * host(xh)).sum(0)) < 1e-6
    if mode == 2:
        assert torch.equal(pr[2].max(0).values, gg.abs().max(0).values)
        assert torch.equal(pr[3].max(0).values, xh.abs().max(0).values)
    # the fold against bn_bwd's own statistics (dgamma = sum g*xhat, dbeta = sum g)
    ws = F._bn_ws(M, N, "cuda")
    dg0, db0, dg1, db1 = (torch.empty(N, device="cuda") for _ in range(4))
    L.call("bnn_bn_bwd", L.ptr(x), L.ptr(C0), M, N, L.ptr(gam), L.ptr(bet), L.ptr(mean), L.ptr(invstd), L.ptr(mlo),
           1, None, L.ptr(dg0), L.ptr(db0), L.ptr(ws), L.stream())
    sc, ds = torch.empty(N, device="cuda"), torch.empty(N, dtype=torch.int64, device="cuda")
    L.call("bnn_bn_bwd_stats_pre", L.ptr(part), R, M, N, mode, L.ptr(gam), L.ptr(invstd), L.ptr(dg1), L.ptr(db1),
           L.ptr(sc) if mode == 2 else None, L.ptr(ds) if mode == 2 else None, L.ptr(F._bn_ws(M, N, "cuda")),
           L.stream())
    assert rel_err(host(dg1), host(dg0)) < 1e-6 and rel_err(host(db1), host(db0)) < 1e-6


def test_training_step_bn_epilogue_statistics(F):
    """A fused wide step with the BatchNorm-backward statistics taken from the dX GEMMs' epilogues
    (functional.BN_EPI) against the same step with the separate statistics pass: the forward and
    loss identical, every gradient within 1e-6 norm-wise (the sums differ only in order)."""
    n0 = F.BN_EPI_USES
    # 64 x 4 tiles of 128 x 512 on the dX GEMMs: one round of the chip, so their plan is unsplit
    g1, names1 = _wide_step(F, True, M=8192, width=2048, bn_epi=True)
    assert F.BN_EPI_USES - n0 >= 1
    g0, _ = _wide_step(F, True, M=8192, width=2048, bn_epi=False)
    for k in g0:
        assert rel_err(g1[k], g0[k]) <= 1e-6 or np.abs(g1[k] - g0[k]).max() <= 1e-7, k

"""GPU parity of fc1 on u8 pixels (bnn_pixels.hip + bnn_gemm_i8_affine): the reference's first
BinarizeLinear (models/binarized_modules.py:68-85, input kept since size(1) == 784) fed by
ToTensor (mnist-dist2.py:96-99) or ToTensor + Normalize (mnist-distributed-BNNS2.py:82).

Bars:
* pixels_pack, row sums, digit column sums, the offset GEMM: exact (integers);
* forward against float64 of the reference's fp32 pixels: norm-wise <= 1e-6 (its only roundings
  are the scale by a and the fp32 bias add, both after the exact integer sum);
* dW, db against float64: <= 1e-5 (the dY digits); a pixel column that is zero across the batch
  gets an exactly zero weight gradient, as the reference's fp32 GEMM gives (ToTensor).
Real pixels: the MNIST test images the reference ships (tests/golden, a fixture).
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, rel_err
from oracle import bnn_np as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def F():
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    from bnn_amd import functional
    return functional


@pytest.fixture(scope="module")
def t10k():
    from bnn_amd.data import read_idx
    return read_idx(os.path.join(GOLDEN, "t10k-images-idx3-ubyte.gz")).reshape(10000, 784)


def host(t):
    torch.cuda.synchronize()
    return t.detach().cpu().numpy()


def _pixels(rng, M, K):
    u = rng.integers(1, 256, (M, K)).astype(np.uint8)
    u[rng.random((M, K)) < 0.807] = 0
    return u


@pytest.mark.parametrize("M,K", [(5, 784), (300, 784), (64, 784), (1000, 100), (7, 33), (0, 784)])
@pytest.mark.parametrize("which", ["both", "q", "qt"])
def test_pixels_pack_exact(F, M, K, which):
    rng = np.random.default_rng(M * 7 + K)
    u = _pixels(rng, M, K)
    q, qt = F.pixels_pack(torch.as_tensor(u).cuda(), want_q=which != "qt", want_qt=which != "q")
    v = u.astype(np.int16) - 128
    if which != "qt":
        qh = host(q)
        assert qh.shape == (M, F.round_up(K)) and np.array_equal(qh[:, :K], v) and not qh[:, K:].any()
    if which != "q":
        th = host(qt)
        assert th.shape == (K, F.round_up(M)) and np.array_equal(th[:, :M], v.T) and not th[:, M:].any()


def test_row_sums_exact(F):
    rng = np.random.default_rng(3)
    q = rng.integers(-1, 2, (1000, 832)).astype(np.int8)
    q[:, 784:] = 0
    out = host(F.row_sums(torch.as_tensor(q).cuda(), 784))
    assert out.dtype == np.int64 and np.array_equal(out, q[:, :784].sum(1, dtype=np.int64))


@pytest.mark.parametrize("M,N", [(300, 200), (1000, 37), (64, 8192), (4096, 64)])
def test_quant_cols_t_digit_sums_exact(F, M, N):
    rng = np.random.default_rng(M + N)
    x = (rng.standard_normal((M, N)) * np.exp(rng.uniform(-8, 8, (1, N)))).astype(np.float32)
    x[:, 3] = 0.0
    dg, sc, cs, ds = F.quant_cols_t(torch.as_tensor(x).cuda(), want_colsum=True, want_dsum=True)
    d = host(dg).astype(np.int64)
    comb = d[2] * 65536 + d[1] * 256 + d[0]
    assert np.array_equal(host(ds), comb.sum(1))
    assert host(ds)[3] == 0


def test_gemm_i8_affine_offsets_exact(F):
    """(1,1) with col_off and (3,1) with row_off against the int64 formula, scales of 1."""
    rng = np.random.default_rng(11)
    M, N, K = 300, 200, 832
    A = rng.integers(-128, 128, (M, K)).astype(np.int8)
    B = rng.integers(-1, 2, (N, K)).astype(np.int8)
    co = rng.integers(-784, 785, N).astype(np.int64)
    ro = rng.integers(-2 ** 30, 2 ** 30, M).astype(np.int64)
    dv = lambda a: torch.as_tensor(a).cuda()   # noqa: E731
    C = host(F.gemm_i8_affine(dv(A), 1, dv(B), 1, M, N, col_off=dv(co), off_mul=128.0))
    exact = A.astype(np.int64) @ B.astype(np.int64).T + 128 * co[None, :]
    assert np.array_equal(C, exact.astype(np.float32))
    A3 = rng.integers(-128, 128, (3, M, K)).astype(np.int8)
    C3 = host(F.gemm_i8_affine(dv(A3), 3, dv(B), 1, M, N, row_off=dv(ro), off_mul=128.0))
    comb = (A3[2].astype(np.int64) * 65536 + A3[1].astype(np.int64) * 256 + A3[0]) @ B.astype(np.int64).T
    exact3 = comb + 128 * ro[:, None]
    assert np.array_equal(C3, exact3.astype(np.float64).astype(np.float32))


def _layer(F, u, w, b, normalize, want_grad=True):
    ut = torch.as_tensor(u).cuda()
    wt = torch.as_tensor(w).cuda().requires_grad_(want_grad)
    bt = torch.as_tensor(b).cuda().requires_grad_(want_grad)
    y = F.binary_linear_pixels(ut, wt, bt, normalize)
    return y, wt, bt


@pytest.mark.parametrize("normalize", [None, (0.1307, 0.3081)])
@pytest.mark.parametrize("M,N", [(512, 3072), (64, 192), (2048, 1000), (1, 10)])
def test_fc1_pixels_forward_backward(F, t10k, normalize, M, N):
    rng = np.random.default_rng(M + N)
    u = t10k[rng.choice(10000, M, replace=False)]
    w = rng.uniform(-1, 1, (N, 784)).astype(np.float32)
    w[:, ::97] = 0.0                                               # ternary zeros
    b = rng.standard_normal(N).astype(np.float32)
    y, wt, bt = _layer(F, u, w, b, normalize)
    x = O.to_tensor(u, normalize).astype(np.float64)                # the reference's fp32 pixels
    wb = np.sign(w).astype(np.float64)
    ref = x @ wb.T + b
    assert rel_err(host(y), ref) <= 1e-6
    dy = rng.standard_normal((M, N)).astype(np.float32) * np.exp(rng.uniform(-4, 4, (1, N))).astype(np.float32)
    y.backward(torch.as_tensor(dy).cuda())
    dw_ref = dy.astype(np.float64).T @ x
    assert rel_err(host(wt.grad), dw_ref) <= 1e-5
    assert rel_err(host(bt.grad), dy.astype(np.float64).sum(0)) <= 1e-6
    if normalize is None:
        dead = ~u.any(0)                                           # pixel columns dark in the whole batch
        assert dead.any()
        assert not host(wt.grad)[:, dead].any()                     # exactly zero, as fp32 GEMM gives


def test_fc1_pixels_matches_fp32_path(F, t10k):
    """The u8 path and the fp32-pixel path (int8 digit planes of u/255) agree to the bar."""
    rng = np.random.default_rng(5)
    u = t10k[:256]
    w = rng.uniform(-1, 1, (512, 784)).astype(np.float32)
    b = rng.standard_normal(512).astype(np.float32)
    y8 = host(F.binary_linear_pixels(torch.as_tensor(u).cuda(), torch.as_tensor(w).cuda(), torch.as_tensor(b).cuda()))
    yf = host(F.binary_linear(torch.as_tensor(O.to_tensor(u)).cuda(), torch.as_tensor(w).cuda(),
                              torch.as_tensor(b).cuda(), binarize_input=False))
    assert rel_err(y8, yf) <= 2e-6


def test_dropin_fc1_recognises_totensor_images(F, t10k):
    """The drop-in BinarizeLinear(784, N) handed fp32 ToTensor images (x = fl(u / 255), as
    mnist-dist2.py's loader makes them on the host, or fl(u * fl(1 / 255)), torch's division by a
    scalar on the GPU) runs the u8-pixel GEMMs: output
    and weight / bias gradients bit-identical to binary_linear_pixels on the bytes, within 2e-6 of
    the fp32-digit path; dead pixel columns get exactly zero weight gradient.  Inputs that are not
    such images (one element off by an ulp, a Normalize'd image, an input that needs its own
    gradient) keep the fp32 path."""
    from models.binarized_modules import BinarizeLinear
    rng = np.random.default_rng(11)
    u = t10k[:300]
    torch.manual_seed(3)
    lin = BinarizeLinear(784, 256).cuda()
    w0 = lin.weight.detach().clone()
    for where in ("host", "gpu"):
        xt = torch.as_tensor(O.to_tensor(u)).cuda() if where == "host" else \
            torch.as_tensor(u).cuda().float().div(255.0)
        n0 = F.UNIT_PIXELS
        lin.weight.grad = lin.bias.grad = None
        y = lin(xt)
        assert F.UNIT_PIXELS == n0 + 1, where
        g = torch.as_tensor(rng.standard_normal((300, 256)).astype(np.float32)).cuda()
        y.backward(g)
        w8 = w0.clone().requires_grad_(True)
        b8 = lin.bias.detach().clone().requires_grad_(True)
        y8 = F.binary_linear_pixels(torch.as_tensor(u).cuda(), w8, b8)
        y8.backward(g)
        assert torch.equal(y, y8) and torch.equal(lin.weight.grad, w8.grad) and torch.equal(lin.bias.grad, b8.grad)
        yf = F.binary_linear(xt, w0, lin.bias.detach(), binarize_input=False)
        assert rel_err(host(y), host(yf)) <= 2e-6
        dead = ~u.any(0)
        assert not host(lin.weight.grad)[:, dead].any()
        lin.weight.data = w0.clone()
        del lin.weight.org
    for name, xt in (("ulp", torch.as_tensor(O.to_tensor(u)).cuda()),
                     ("normalize", (torch.as_tensor(O.to_tensor(u)).cuda() - 0.1307) / 0.3081)):
        if name == "ulp":     # 2 ulps: the host and GPU roundings of u / 255 differ by at most one
            two = torch.tensor(2.0, device="cuda")
            xt.view(-1)[12345] = torch.nextafter(torch.nextafter(xt.view(-1)[12345], two), two)
        n0 = F.UNIT_PIXELS
        lin(xt)
        assert F.UNIT_PIXELS == n0, name
    xg = torch.as_tensor(O.to_tensor(u)).cuda().requires_grad_(True)
    n0 = F.UNIT_PIXELS
    lin(xg).sum().backward()
    assert F.UNIT_PIXELS == n0 and xg.grad is not None


def test_fc1_pixels_empty_batch(F):
    w = torch.randn(16, 784, device="cuda", requires_grad=True)
    b = torch.randn(16, device="cuda", requires_grad=True)
    y = F.binary_linear_pixels(torch.zeros((0, 784), dtype=torch.uint8, device="cuda"), w, b)
    assert y.shape == (0, 16)
    y.sum().backward()
    assert not w.grad.any() and not b.grad.any()


def test_net_on_pixels_drop_in(F, t10k):
    """nets.MLP given the bytes equals the same MLP given ToTensor(bytes) at fc1, and a training
    step of the fused trainer path runs on them (loss finite, dead-pixel weights unchanged)."""
    from bnn_amd import nets
    from bnn_amd.optim import LatentAdam
    torch.manual_seed(0)
    m = nets.MLP(256, 128, 64, org_protocol=False, mutate_input=False, fused_bn=True).cuda().train()
    u = torch.as_tensor(t10k[:512].reshape(512, 1, 28, 28)).cuda()
    y = torch.randint(0, 10, (512,), device="cuda")
    h8 = m.fc1(u.view(-1, 784))
    hf = m.fc1(torch.as_tensor(O.to_tensor(t10k[:512])).cuda())
    assert rel_err(host(h8), host(hf)) <= 2e-6
    w0 = host(m.fc1.weight).copy()
    opt = LatentAdam(m.parameters(), lr=0.01, clamp_params=nets.binary_params(m))
    loss = torch.nn.CrossEntropyLoss()(m(u), y)
    loss.backward()
    opt.step()
    assert np.isfinite(float(loss))
    dead = ~t10k[:512].any(0)
    w1 = host(m.fc1.weight)
    assert np.array_equal(w1[:, dead], w0[:, dead]) and not np.array_equal(w1, w0)


@pytest.mark.parametrize("M,C", [(1000, 512), (4096, 768), (77, 64)])
def test_bn_bwd_i8cols_vs_written_dz(F, M, C):
    """bnn_bn_bwd_i8cols (dz formed from x, dy after the statistics pass, never stored; column
    scale from the a-priori bound of bn_reduce_k MODE 2) against bnn_bn_bwd's written dz:
    dgamma / dbeta bit for bit; every digit decodes to dz within half its scale; the scale lies
    between the true-max scale and a few bits above it; the digit sums (T) are exact; the column
    sums (dB) match float64."""
    from bnn_amd import _lib as L
    g = torch.Generator(device="cuda").manual_seed(M + C)
    x = (torch.randint(-40, 41, (M, C), generator=g, device="cuda").float() + 0.37)
    x[M // 3, 5] = 900.0                              # an outlier row: max|xhat| far above typical
    dy = torch.randn(M, C, generator=g, device="cuda")
    dy[:, 3] = 0.0                                    # an all-zero gradient column: scale 0
    dy[:, 7] *= torch.exp(4 * torch.randn(M, generator=g, device="cuda"))   # heavy-tailed column
    gam = torch.rand(C, generator=g, device="cuda") + 0.5
    bet = torch.rand(C, generator=g, device="cuda") - 0.5
    mean, invstd, lo = (torch.empty(C, device="cuda") for _ in range(3))
    ws = torch.empty((L.lib().bnn_bn_workspace(M, C),), dtype=torch.uint8, device="cuda")
    L.call("bnn_bn_fwd_train", L.ptr(x), M, C, L.ptr(gam), L.ptr(bet), None, None, -1.0, 1e-5, L.ptr(mean),
           L.ptr(invstd), L.ptr(lo), None, 1, L.ptr(ws), L.stream())
    dz = torch.empty(M, C, device="cuda")
    dg_a, db_a = torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
    L.call("bnn_bn_bwd", L.ptr(x), L.ptr(dy), M, C, L.ptr(gam), L.ptr(bet), L.ptr(mean), L.ptr(invstd), L.ptr(lo), 1,
           L.ptr(dz), L.ptr(dg_a), L.ptr(db_a), L.ptr(ws), L.stream())
    _, sc_ref, _ = F.quant_cols_t(dz, want_colsum=False)
    dg_b, db_b = torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
    out = F._bn_bwd_i8c(x, dy, M, C, gam, bet, mean, invstd, lo, dg_b, db_b)
    dt, sc, cs, ds = (host(t) for t in F._i8c_take(out))
    assert torch.equal(dg_a, dg_b) and torch.equal(db_a, db_b)
    z64, sc_ref = host(dz).astype(np.float64), host(sc_ref)
    assert sc[3] == 0 and sc_ref[3] == 0 and not dt[:, 3].any()
    live = sc_ref > 0
    assert np.all(sc[live] >= sc_ref[live]) and np.all(sc[live] <= 64 * sc_ref[live])
    d = dt[:, :, :M].astype(np.int64)
    v = d[2] * 65536 + d[1] * 256 + d[0]                        # [C][M]
    assert np.all(np.abs(v * sc[:, None].astype(np.float64) - z64.T) <= sc[:, None] / 2 * (1 + 1e-6))
    assert not dt[:, :, M:].any()
    assert np.array_equal(ds, v.sum(1))
    assert rel_err(cs, z64.sum(0)) < 1e-6


def test_mlp_step_with_i8cols_handoff_equals_unfused(F):
    """A fused MLP training step on u8 pixels with the fc1 weight gradient fed by the int8
    column-digit hand-off equals the step with the hand-off off (dz written, re-read, quantised):
    every other gradient bit for bit; fc1's weight and bias gradients (digits scaled by the
    a-priori bound, column sums in another order) within 1e-6 norm-wise; dead pixels exact zeros."""
    from bnn_amd import nets
    g = torch.Generator(device="cuda").manual_seed(7)
    u = torch.randint(0, 256, (2048, 1, 28, 28), generator=g, device="cuda").to(torch.uint8)
    u[:, :, :3] = 0                                   # dead pixels: exact-zero weight gradients
    y = torch.randint(0, 10, (2048,), generator=g, device="cuda")
    grads = []
    epi0 = F.BN_EPI
    for on in (True, False):
        F.I8C_HANDOFF = on
        F.BN_EPI = False          # both steps reduce the BatchNorm statistics in the same order
        try:
            torch.manual_seed(0)
            m = nets.MLP(1024, 512, 256, org_protocol=False, mutate_input=False, fused_bn=True).cuda().train()
            torch.manual_seed(1)
            n0 = F.I8C_HANDOFFS
            torch.nn.CrossEntropyLoss()(m(u), y).backward()
            assert F.I8C_HANDOFFS - n0 == (1 if on else 0)
            grads.append({k: p.grad.detach().clone() for k, p in m.named_parameters()})
        finally:
            F.I8C_HANDOFF = True
            F.BN_EPI = epi0
    for k in grads[0]:
        if k in ("fc1.weight", "fc1.bias"):
            assert rel_err(host(grads[0][k]), host(grads[1][k]).astype(np.float64)) < 1e-6, k
        else:
            assert torch.equal(grads[0][k], grads[1][k]), k
    dead = grads[0]["fc1.weight"].view(1024, 28, 28)[:, :3]
    assert not dead.any()


@pytest.mark.parametrize("M,N,normalize", [(8192, 4096, None), (1000, 3072, None), (4100, 1024, (0.1307, 0.3081)),
                                           (77, 200, None)])
def test_pixels_gemm_bn_forward_statistics(F, t10k, M, N, normalize):
    """bnn_gemm_i8_affine_bnstats: C bit-identical to bnn_gemm_i8_affine; the chunk partials equal
    float64 chunk sums / M2 of z = a*(S + s0*R) + b computed from the exact integer sums; the
    final (bnn_bn_fwd_final_parts) within 1e-6 of bnn_bn_fwd_train's statistics of the stored z
    (which differ only by z's fp32 rounding), running statistics likewise."""
    from bnn_amd import _lib as L
    rng = np.random.default_rng(M + N)
    u = t10k[rng.integers(0, 10000, M)]
    w = rng.uniform(-1, 1, (N, 784)).astype(np.float32)
    w[:, ::97] = 0.0
    b = rng.standard_normal(N).astype(np.float32)
    ut, wt, bt = (torch.as_tensor(v).cuda() for v in (u, w, b))
    a, s0 = F.pixel_affine(normalize)
    q, _ = F.pixels_pack(ut, want_q=True, want_qt=False)
    wq, _ = F.packed_weight(wt, "i8", True, False, False)
    R = F.row_sums(wq, 784)
    bs = F._const_vec(a, N, "cuda")
    y0 = F.gemm_i8_affine(q, 1, wq, 1, M, N, b_scale=bs, bias=bt, col_off=R, off_mul=s0, k_true=784)
    y1 = F._pixels_fwd_with_stats(q, wq, M, N, 784, bs, bt, R, s0)
    assert torch.equal(y0, y1)
    part, rows, chunk = getattr(y1, F._FSTATS_ATTR)[:3]
    # exact integer sums (|S| <= 128*784: exact in the float64 product)
    S = (u.astype(np.float64) - 128) @ np.sign(w).astype(np.float64).T
    z = float(np.float32(a)) * (S + float(s0) * host(R).astype(np.float64)[None, :]) + b.astype(np.float64)
    ph = host(part)
    for r in range(rows):
        zc = z[r * chunk:(r + 1) * chunk]
        assert rel_err(ph[0, r], zc.sum(0)) <= 1e-12
        assert rel_err(ph[1, r], ((zc - zc.mean(0)) ** 2).sum(0)) <= 1e-9
    mean0, istd0, lo0 = F._bn_stat_buffers(N, "cuda")
    mean1, istd1, lo1 = (t.clone() for t in F._bn_stat_buffers(N, "cuda"))
    rm0, rv0 = torch.zeros(N, device="cuda"), torch.ones(N, device="cuda")
    rm1, rv1 = rm0.clone(), rv0.clone()
    L.call("bnn_bn_fwd_train", L.ptr(y0), M, N, None, None, L.ptr(rm0), L.ptr(rv0), 0.1, 1e-5, L.ptr(mean0),
           L.ptr(istd0), L.ptr(lo0), None, 1, L.ptr(F._bn_ws(M, N, "cuda")), L.stream())
    L.call("bnn_bn_fwd_final_parts", L.ptr(part), rows, chunk, M, N, L.ptr(rm1), L.ptr(rv1), 0.1, 1e-5,
           L.ptr(mean1), L.ptr(istd1), L.ptr(lo1), L.stream())
    m0 = host(mean0).astype(np.float64) + host(lo0)
    m1 = host(mean1).astype(np.float64) + host(lo1)
    assert np.abs(m1 - z.mean(0)).max() <= 1e-12 * np.abs(z).max() + 1e-12
    sd = z.std(0)
    assert np.all(np.abs(m1 - m0) <= 1e-6 * sd + 1e-30)
    assert rel_err(host(istd1), host(istd0)) <= 1e-6
    assert rel_err(host(rm1), host(rm0)) <= 1e-6 and rel_err(host(rv1), host(rv0)) <= 1e-6


def test_mlp_step_pixel_statistics_epilogue(F):
    """A fused MLP training step on pixels with bn1's forward statistics from the fc1 epilogue
    (functional.PIX_STATS) against the same step with the statistics pass: loss within 1e-6, bn1's
    batch statistics within 1e-6, every gradient within 1e-4 norm-wise (a BatchNorm near-tie may
    resolve differently: the two means differ by z's fp32 rounding)."""
    from bnn_amd import nets
    g = torch.Generator(device="cuda").manual_seed(3)
    u = torch.randint(0, 256, (4096, 1, 28, 28), generator=g, device="cuda").to(torch.uint8)
    y = torch.randint(0, 10, (4096,), generator=g, device="cuda")
    out = []
    on0 = F.PIX_STATS
    for on in (True, False):
        F.PIX_STATS = on
        try:
            torch.manual_seed(0)
            m = nets.MLP(2048, 1024, 512, org_protocol=False, mutate_input=False, fused_bn=True).cuda().train()
            n0 = F.PIX_STATS_USES
            loss = torch.nn.CrossEntropyLoss()(m(u), y)
            loss.backward()
            assert F.PIX_STATS_USES - n0 == (1 if on else 0)
            out.append((float(loss), {k: host(p.grad) for k, p in m.named_parameters()},
                        host(m.bn1.running_mean), host(m.bn1.running_var)))
        finally:
            F.PIX_STATS = on0
    (l1, g1, rm1, rv1), (l0, g0, rm0, rv0) = out
    assert abs(l1 - l0) <= 1e-6 * abs(l0)
    assert rel_err(rm1, rm0) <= 1e-6 and rel_err(rv1, rv0) <= 1e-6
    for k in g0:   # fc1.bias: analytically zero ahead of a batch-statistics BatchNorm (~1e-11 noise)
        assert rel_err(g1[k], g0[k]) <= 1e-4 or np.abs(g1[k] - g0[k]).max() <= 1e-9, k

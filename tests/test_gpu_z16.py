"""GPU parity of the compact pre-activation path (z16, functional.Z16): a hidden BinarizeLinear's
output z = F.linear(sign(h), W_b) + bias (binarized_modules.py:80-83) carried as int16 dot products
plus the bias into the BatchNorm passes that consume it (mnist-dist2.py:66-70).

Every *_i16 entry reads x = fl(I + bias), the value the fp32 GEMM epilogue stores, so each result
must be BIT-IDENTICAL to the fp32 entry on the fp32 z: statistics, FP4 rows/transpose, the fused
quantising backward (dz, its FP6 digits, column sums, dgamma/dbeta), the fused head forward and
backward, and a whole training step of the MLP with and without the hand-off.
"""
import numpy as np
import pytest
import torch

from conftest import rel_err

pytestmark = pytest.mark.gpu


def host(t):
    torch.cuda.synchronize()
    return t.detach().cpu().numpy()


@pytest.fixture(scope="module")
def F():
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    from bnn_amd import functional
    # the quantised row operands carry the residual plane at every size here (the networks add it
    # from functional.FP6_RES_MIN_ROWS rows on), so the fused passes' residual output is compared too
    prev = functional.FP6_RES_MIN_ROWS
    functional.FP6_RES_MIN_ROWS = 0
    yield functional
    functional.FP6_RES_MIN_ROWS = prev


def eq(a, b):
    torch.cuda.synchronize()
    return (a is None and b is None) or (a is not None and b is not None and torch.equal(a, b))


def _z(M, K, N, seed, with_bias=True):
    """int16 dot products of a ternary GEMM (and the fp32 z the fp32 path sees)."""
    from bnn_amd import functional as F
    g = torch.Generator(device="cuda").manual_seed(seed)
    h = torch.randint(-1, 2, (M, K), generator=g, device="cuda").float()
    w = torch.randint(-1, 2, (N, K), generator=g, device="cuda").float()
    q4, _ = F.sign_pack_fp4(h)
    w4, _ = F.sign_pack_fp4(w)
    bias = (torch.rand(N, generator=g, device="cuda") - 0.5) * 2 if with_bias else None
    z16 = F.gemm_fp4_i16(q4, w4, M, N, k_true=K)
    z = F.gemm_fp4(q4, w4, M, N, bias=bias, k_true=K)
    return z16, bias, z


@pytest.mark.parametrize("M,K,N", [(300, 512, 256), (1024, 8192, 512), (64, 256, 768)])
@pytest.mark.parametrize("with_bias", [True, False])
def test_gemm_fp4_i16_is_the_fp32_output_minus_bias(F, M, K, N, with_bias):
    z16, bias, z = _z(M, K, N, M + K + N, with_bias)
    assert z16.dtype == torch.int16 and int(z16.abs().max()) <= K
    zf = z16.float() + (bias if bias is not None else 0.0)
    assert eq(zf, z)


def _stats(F, z, z16, bias, M, C, p=0.0, seed=0):
    from bnn_amd import _lib as L
    outs = []
    for form in ("f32", "i16"):
        rm = torch.zeros(C, device="cuda")
        rv = torch.ones(C, device="cuda")
        mean, invstd, lo = (torch.empty(C, device="cuda") for _ in range(3))
        ws = torch.empty((L.lib().bnn_bn_workspace(M, C),), dtype=torch.uint8, device="cuda")
        gam = torch.linspace(0.5, 1.5, C, device="cuda")
        bet = torch.linspace(-0.2, 0.2, C, device="cuda")
        if form == "f32":
            L.call("bnn_bn_dropout_fwd_train", L.ptr(z), M, C, L.ptr(gam), L.ptr(bet), L.ptr(rm), L.ptr(rv), 0.1,
                   1e-5, L.ptr(mean), L.ptr(invstd), L.ptr(lo), None, 1, float(p), int(seed), None, L.ptr(ws),
                   L.stream())
        else:
            L.call("bnn_bn_fwd_train_i16", L.ptr(z16), L.ptr(bias), M, C, L.ptr(gam), L.ptr(bet), L.ptr(rm),
                   L.ptr(rv), 0.1, 1e-5, L.ptr(mean), L.ptr(invstd), L.ptr(lo), float(p), int(seed), None,
                   L.ptr(ws), L.stream())
        outs.append((mean, invstd, lo, rm, rv, gam, bet))
    return outs


@pytest.mark.parametrize("M,C,p", [(1000, 512, 0.0), (4096, 768, 0.3), (77, 256, 0.0)])
def test_statistics_i16_bit_identical(F, M, C, p):
    z16, bias, z = _z(M, 384, C, 7 * M + C)
    a, b = _stats(F, z, z16, bias, M, C, p, seed=99)
    for x, y in zip(a, b):
        assert eq(x, y)


@pytest.mark.parametrize("M,C", [(300, 256), (8200, 8192)])
def test_apply_pack_i16_bit_identical(F, M, C):
    from bnn_amd import _lib as L
    z16, bias, z = _z(M, 512, C, M + 3 * C)
    (mean, invstd, lo, _, _, gam, bet), _ = _stats(F, z, z16, bias, M, C)
    res = []
    for form in ("f32", "i16"):
        q = torch.full((M, C // 2), 0x55, dtype=torch.uint8, device="cuda")
        qt = torch.full((C, F.round_up(M, 256) // 2), 0x55, dtype=torch.uint8, device="cuda")
        if form == "f32":
            L.call("bnn_bn_apply_pack", L.ptr(z), M, C, L.ptr(mean), L.ptr(invstd), L.ptr(lo), L.ptr(gam), L.ptr(bet),
                   1, L.ptr(q), q.shape[1], L.ptr(qt), qt.shape[1], 1, L.stream())
        else:
            L.call("bnn_bn_apply_pack_i16", L.ptr(z16), L.ptr(bias), M, C, L.ptr(mean), L.ptr(invstd), L.ptr(lo),
                   L.ptr(gam), L.ptr(bet), L.ptr(q), q.shape[1], L.ptr(qt), qt.shape[1], 0, L.stream())
        res.append((q, qt))
    assert eq(res[0][0], res[1][0]) and eq(res[0][1], res[1][1])


def _fp6_bufs(F, M, C):
    rows = F.Fp6Operand(*F._fp6_buffers(M, C, "cuda"), M, C, F._res_buffer(M, C, "cuda"))
    Mp = F.round_up(M)
    cols = F.Fp6Operand(*F._fp6_buffers(C, Mp, "cuda"), C, Mp)
    for t in (rows.lo, rows.hi, rows.sc, rows.res, cols.lo, cols.hi, cols.sc):
        if t is not None:
            t.fill_(0x5A)
    return rows, cols


@pytest.mark.parametrize("M,C,p", [(512, 256, 0.0), (1000, 512, 0.3)])
def test_bwd_q6_i16_bit_identical(F, M, C, p):
    from bnn_amd import _lib as L
    z16, bias, z = _z(M, 256, C, 5 * M + C)
    (mean, invstd, lo, _, _, gam, bet), _ = _stats(F, z, z16, bias, M, C, p, seed=11)
    dy = torch.randn(M, C, device="cuda", generator=torch.Generator(device="cuda").manual_seed(M))
    res = []
    for form in ("f32", "i16"):
        dx = torch.empty(M, C, device="cuda")
        dg, db, cs = (torch.empty(C, device="cuda") for _ in range(3))
        rows, cols = _fp6_bufs(F, M, C)
        ws = torch.empty((L.lib().bnn_bn_workspace(M, C),), dtype=torch.uint8, device="cuda")
        common = [M, C, L.ptr(gam), L.ptr(bet), L.ptr(mean), L.ptr(invstd), L.ptr(lo), 1, float(p), 11, L.ptr(dx),
                  L.ptr(dg), L.ptr(db), L.ptr(rows.lo), L.ptr(rows.hi), L.ptr(rows.sc), L.ptr(rows.res),
                  L.ptr(cols.lo), L.ptr(cols.hi), L.ptr(cols.sc), L.ptr(cs), L.ptr(ws), L.stream()]
        if form == "f32":
            L.call("bnn_bn_bwd_q6", L.ptr(z), L.ptr(dy), *common)
        else:
            L.call("bnn_bn_bwd_q6_i16", L.ptr(z16), L.ptr(bias), L.ptr(dy), *common)
        res.append([dx, dg, db, cs, rows.lo, rows.hi, rows.sc, rows.res, cols.lo, cols.hi, cols.sc])
    for x, y in zip(*res):
        assert eq(x, y)


@pytest.mark.parametrize("M,C", [(512, 256), (1000, 1024)])
def test_head_i16_bit_identical(F, M, C):
    from bnn_amd import _lib as L
    p, seed = 0.3, 1234
    z16, bias, z = _z(M, 256, C, 9 * M + C)
    (mean, invstd, lo, _, _, gam, bet), _ = _stats(F, z, z16, bias, M, C, p, seed)
    g = torch.Generator(device="cuda").manual_seed(C)
    w4 = torch.randn(10, C, device="cuda", generator=g) * 0.05
    b4 = torch.randn(10, device="cuda", generator=g)
    dy4 = torch.randn(M, 10, device="cuda", generator=g)
    res = []
    for form in ("f32", "i16"):
        y4 = torch.empty(M, 10, device="cuda")
        if form == "f32":
            L.call("bnn_bn_head_fwd", L.ptr(z), M, C, L.ptr(mean), L.ptr(invstd), L.ptr(lo), L.ptr(gam), L.ptr(bet),
                   p, seed, None, L.ptr(w4), 10, L.ptr(b4), L.ptr(y4), L.stream())
        else:
            L.call("bnn_bn_head_fwd_i16", L.ptr(z16), L.ptr(bias), M, C, L.ptr(mean), L.ptr(invstd), L.ptr(lo),
                   L.ptr(gam), L.ptr(bet), p, seed, None, L.ptr(w4), 10, L.ptr(b4), L.ptr(y4), L.stream())
        dx = torch.empty(M, C, device="cuda")
        dg, db, cs = (torch.empty(C, device="cuda") for _ in range(3))
        dw4 = torch.empty(10, C, device="cuda")
        rows, cols = _fp6_bufs(F, M, C)
        ws = torch.empty((L.lib().bnn_bn_head_workspace(M, C, 10),), dtype=torch.uint8, device="cuda")
        common = [L.ptr(dy4), L.ptr(w4), 10, M, C, L.ptr(gam), L.ptr(bet), L.ptr(mean), L.ptr(invstd), L.ptr(lo), p,
                  seed, None, L.ptr(dx), L.ptr(dg), L.ptr(db), L.ptr(dw4), L.ptr(rows.lo), L.ptr(rows.hi), L.ptr(rows.sc),
                  L.ptr(rows.res), L.ptr(cols.lo), L.ptr(cols.hi), L.ptr(cols.sc), L.ptr(cs), L.ptr(ws), L.stream()]
        if form == "f32":
            L.call("bnn_bn_head_bwd_q6", L.ptr(z), *common)
        else:
            L.call("bnn_bn_head_bwd_q6_i16", L.ptr(z16), L.ptr(bias), *common)
        res.append([y4, dx, dg, db, dw4, cs, rows.lo, rows.hi, rows.sc, rows.res, cols.lo, cols.hi, cols.sc])
    for x, y in zip(*res):
        assert eq(x, y)


def test_mlp_step_with_z16_equals_fp32(F):
    """A whole training step (forward, loss, backward, fused Adam + re-pack) of a 4096-wide MLP at
    batch 32768 -- large enough that z16_ok hands fc2's and fc3's outputs on as int16 -- equals the
    same step with the hand-off disabled, bit for bit: loss, every parameter, Adam moment and
    BatchNorm buffer."""
    from bnn_amd import nets
    from bnn_amd.nets import binary_params
    from bnn_amd.optim import LatentAdam
    M, W = 32768, 4096
    assert F.z16_ok(M, W, W)
    g = torch.Generator(device="cuda").manual_seed(3)
    u = torch.randint(0, 256, (M, 1, 28, 28), generator=g, device="cuda").to(torch.uint8)
    y = torch.randint(0, 10, (M,), generator=g, device="cuda")
    states = []
    for z16 in (True, False):
        F.Z16 = z16
        try:
            torch.manual_seed(0)
            m = nets.MLP(W, W, W, org_protocol=False, mutate_input=False, fused_bn=True).cuda().train()
            opt = LatentAdam(m.parameters(), lr=0.01, clamp_params=binary_params(m))
            losses = []
            n0 = F.Z16_HANDOFFS
            for _ in range(2):
                for p in m.parameters():
                    p.grad = None
                torch.manual_seed(1)
                loss = torch.nn.CrossEntropyLoss()(m(u), y)
                loss.backward()
                opt.step()
                losses.append(float(loss.item()))
            assert F.Z16_HANDOFFS - n0 == (4 if z16 else 0)     # fc2 and fc3, two steps
            st = {k: v.detach().clone() for k, v in m.state_dict().items()}
            for i, p in enumerate(m.parameters()):
                for k in ("exp_avg", "exp_avg_sq"):
                    st[f"opt{i}.{k}"] = opt.state[p][k].clone()
            states.append((losses, st))
            del m, opt
        finally:
            F.Z16 = True
    (la, a), (lb, b) = states
    assert la == lb
    for k in a:
        assert torch.equal(a[k], b[k]), k


@pytest.mark.parametrize("M,K,N,i16", [(65536 // 4, 2048, 4096, True), (65536 // 4, 2048, 4096, False),
                                       (1000, 768, 1536, True), (333, 512, 256, False)])
def test_gemm_fp4_bnstats_epilogue(F, M, K, N, i16):
    """bnn_gemm_fp4_bnstats: C (fp32 + bias) / C16 bit-identical to bnn_gemm_fp4 / bnn_gemm_fp4_i16;
    chunk sums of the stored z = fl(I + b) equal float64 sums of the same fp32 values (the double
    sum is exact), M2 within 1e-9; the final (bnn_bn_fwd_final_parts) mean hi/lo bit-identical to
    bnn_bn_fwd_train's on the same z, invstd and running statistics within 1e-6."""
    from bnn_amd import _lib as L
    g = torch.Generator(device="cuda").manual_seed(M + K + N)
    h = torch.randint(-1, 2, (M, K), generator=g, device="cuda").float()
    w = torch.randint(-1, 2, (N, K), generator=g, device="cuda").float()
    b = torch.randn(N, generator=g, device="cuda")
    q, _ = F.sign_pack_fp4(h)
    wq, _ = F.sign_pack_fp4(w)
    chunk = int(L.lib().bnn_gemm_fp4_bnstats_chunk(M, N, q.shape[1]))
    assert chunk in (64, 128)
    if i16:
        c0 = F.gemm_fp4_i16(q, wq, M, N, k_true=K)
        c1, fst = F._fp4_fwd_with_stats(q, wq, M, N, K, None, b, chunk, True)
        z = c0.float() + b
    else:
        c0 = F.gemm_fp4(q, wq, M, N, bias=b, k_true=K)
        c1, fst = F._fp4_fwd_with_stats(q, wq, M, N, K, b, b, chunk, False)
        z = c0
    assert torch.equal(c0, c1)
    part, rows = fst[0], fst[1]
    zh = host(z).astype(np.float64)
    ph = host(part)
    for r in range(rows):
        zc = zh[r * chunk:(r + 1) * chunk]
        assert np.array_equal(ph[0, r], zc.sum(0)) or rel_err(ph[0, r], zc.sum(0)) <= 1e-15
        assert rel_err(ph[1, r], ((zc - zc.mean(0)) ** 2).sum(0)) <= 1e-9
    mean0, istd0, lo0 = F._bn_stat_buffers(N, "cuda")
    mean1, istd1, lo1 = (t.clone() for t in F._bn_stat_buffers(N, "cuda"))
    rm0, rv0 = torch.zeros(N, device="cuda"), torch.ones(N, device="cuda")
    rm1, rv1 = rm0.clone(), rv0.clone()
    L.call("bnn_bn_fwd_train", L.ptr(z.contiguous()), M, N, None, None, L.ptr(rm0), L.ptr(rv0), 0.1, 1e-5,
           L.ptr(mean0), L.ptr(istd0), L.ptr(lo0), None, 1, L.ptr(F._bn_ws(M, N, "cuda")), L.stream())
    L.call("bnn_bn_fwd_final_parts", L.ptr(part), rows, chunk, M, N, L.ptr(rm1), L.ptr(rv1), 0.1, 1e-5,
           L.ptr(mean1), L.ptr(istd1), L.ptr(lo1), L.stream())
    assert torch.equal(mean0, mean1) and torch.equal(lo0, lo1)
    assert rel_err(host(istd1), host(istd0)) <= 1e-6
    assert rel_err(host(rm1), host(rm0)) <= 1e-6 and rel_err(host(rv1), host(rv0)) <= 1e-6


def test_mlp_step_fp4_statistics_epilogue(F):
    """A fused MLP training step with bn2's forward statistics from fc2's FP4 epilogue
    (functional.FP4_STATS) against the statistics pass: loss within 1e-6, bn2's running buffers
    within 1e-6, gradients within 1e-4 norm-wise (invstd may differ in its last bit)."""
    from bnn_amd import nets
    g = torch.Generator(device="cuda").manual_seed(4)
    u = torch.randint(0, 256, (8192, 1, 28, 28), generator=g, device="cuda").to(torch.uint8)
    y = torch.randint(0, 10, (8192,), generator=g, device="cuda")
    out = []
    on0 = F.FP4_STATS
    for on in (True, False):
        F.FP4_STATS = on
        try:
            torch.manual_seed(0)
            m = nets.MLP(2048, 2048, 1024, org_protocol=False, mutate_input=False, fused_bn=True).cuda().train()
            n0 = F.FP4_STATS_USES
            loss = torch.nn.CrossEntropyLoss()(m(u), y)
            loss.backward()
            uses = F.FP4_STATS_USES - n0
            out.append((float(loss), {k: host(p.grad) for k, p in m.named_parameters()},
                        host(m.bn2.running_mean), host(m.bn2.running_var), uses))
        finally:
            F.FP4_STATS = on0
    (l1, g1, rm1, rv1, u1), (l0, g0, rm0, rv0, u0) = out
    assert u1 == 1 and u0 == 0              # bn2 took fc2's epilogue statistics
    assert abs(l1 - l0) <= 1e-6 * abs(l0)
    assert rel_err(rm1, rm0) <= 1e-6 and rel_err(rv1, rv0) <= 1e-6
    for k in g0:
        assert rel_err(g1[k], g0[k]) <= 1e-4 or np.abs(g1[k] - g0[k]).max() <= 1e-9, k


@pytest.mark.parametrize("i16", [True, False])
def test_gemm_fp4_bnstats_dropout(F, i16):
    """The dropout form of bnn_gemm_fp4_bnstats: its final (bnn_bn_fwd_final_parts) against
    bnn_bn_dropout_fwd_train on the fp32 z with the same p and seed -- mean hi / lo bit-identical
    (both sum the same dropped fp32 values exactly in double), invstd and running statistics within
    1e-6; a different seed gives other statistics."""
    from bnn_amd import _lib as L
    M, K, N, p, seed = 8192, 2048, 1024, 0.3, 123456789
    g = torch.Generator(device="cuda").manual_seed(99)
    h = torch.randint(-1, 2, (M, K), generator=g, device="cuda").float()
    w = torch.randint(-1, 2, (N, K), generator=g, device="cuda").float()
    b = torch.randn(N, generator=g, device="cuda")
    q, _ = F.sign_pack_fp4(h)
    wq, _ = F.sign_pack_fp4(w)
    chunk = int(L.lib().bnn_gemm_fp4_bnstats_chunk(M, N, q.shape[1]))
    z = F.gemm_fp4(q, wq, M, N, bias=b, k_true=K)
    res = []
    for sd in (seed, seed + 1):
        c1, fst = F._fp4_fwd_with_stats(q, wq, M, N, K, None if i16 else b, b, chunk, i16, (p, sd))
        mean1, istd1, lo1 = (t.clone() for t in F._bn_stat_buffers(N, "cuda"))
        rm1, rv1 = torch.zeros(N, device="cuda"), torch.ones(N, device="cuda")
        L.call("bnn_bn_fwd_final_parts", L.ptr(fst[0]), fst[1], chunk, M, N, L.ptr(rm1), L.ptr(rv1), 0.1, 1e-5,
               L.ptr(mean1), L.ptr(istd1), L.ptr(lo1), L.stream())
        res.append((mean1, istd1, lo1, rm1, rv1))
    mean0, istd0, lo0 = F._bn_stat_buffers(N, "cuda")
    rm0, rv0 = torch.zeros(N, device="cuda"), torch.ones(N, device="cuda")
    L.call("bnn_bn_dropout_fwd_train", L.ptr(z), M, N, None, None, L.ptr(rm0), L.ptr(rv0), 0.1, 1e-5, L.ptr(mean0),
           L.ptr(istd0), L.ptr(lo0), None, 1, p, seed, None, L.ptr(F._bn_ws(M, N, "cuda")), L.stream())
    mean1, istd1, lo1, rm1, rv1 = res[0]
    assert torch.equal(mean0, mean1) and torch.equal(lo0, lo1)
    assert rel_err(host(istd1), host(istd0)) <= 1e-6
    assert rel_err(host(rm1), host(rm0)) <= 1e-6 and rel_err(host(rv1), host(rv0)) <= 1e-6
    assert not torch.equal(res[1][0], mean0)

"""GPU parity of the dropout keep-bit plane (bnn_dropout_keep_bits_bytes, Drop::bits): the fused
dropout in front of bn3 (mnist-dist2.py:69-70, fc3 -> drop -> bn3 -> htanh3 -> fc4) is evaluated
once, by the forward statistics pass, which stores the keep mask as bits; the head's forward,
statistics and quantising backward passes read the bits instead of hashing every element again.

Bars: the stored bits are exactly the mask bnn_dropout_mask regenerates (fused 8-row batches and the
standalone kernel, ragged row counts), and every head output -- y4, dx, dgamma, dbeta, dW4, the FP6
digit records, residual planes and column sums -- is BIT-IDENTICAL with and without the plane.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

# (M, C): 8-row statistics chunks (fused writer), a ragged tail, 1-row chunks (standalone writer),
# 64-row chunks
SHAPES = [(4096, 1024), (4100, 1024), (1000, 512), (16384, 2048)]


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


def _inputs(F, M, C, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    h = torch.randint(-1, 2, (M, 512), generator=g, device="cuda").float()
    w = torch.randint(-1, 2, (C, 512), generator=g, device="cuda").float()
    q4, _ = F.sign_pack_fp4(h)
    w4, _ = F.sign_pack_fp4(w)
    bias = (torch.rand(C, generator=g, device="cuda") - 0.5) * 2
    z16 = F.gemm_fp4_i16(q4, w4, M, C, k_true=512)
    z = F.gemm_fp4(q4, w4, M, C, bias=bias, k_true=512)
    return z16, bias, z


def _expected_words(M, C, p, seed):
    """The keep mask of bnn_dropout_mask packed as keep_word does: word (r / 8, c / 4), bit 4 i + j."""
    from bnn_amd import _lib as L
    m = torch.empty(M * C, device="cuda")
    L.call("bnn_dropout_mask", M * C, float(p), int(seed), L.ptr(m), L.stream())
    keep = (m > 0).view(M, C).to(torch.int64)
    M8 = (M + 7) // 8 * 8
    k = torch.zeros(M8, C, dtype=torch.int64, device="cuda")
    k[:M] = keep
    k = k.view(M8 // 8, 8, C // 4, 4)
    sh = (4 * torch.arange(8, device="cuda").view(1, 8, 1, 1) + torch.arange(4, device="cuda").view(1, 1, 1, 4))
    words = (k << sh).sum(dim=(1, 3))
    return words.to(torch.int64) & 0xFFFFFFFF


def _stats(F, form, z, z16, bias, M, C, p, seed, kb):
    from bnn_amd import _lib as L
    rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    mean, invstd, lo = (torch.empty(C, device="cuda") for _ in range(3))
    ws = torch.empty((L.lib().bnn_bn_workspace(M, C),), dtype=torch.uint8, device="cuda")
    gam = torch.linspace(0.5, 1.5, C, device="cuda")
    bet = torch.linspace(-0.2, 0.2, C, device="cuda")
    if form == "f32":
        L.call("bnn_bn_dropout_fwd_train", L.ptr(z), M, C, L.ptr(gam), L.ptr(bet), L.ptr(rm), L.ptr(rv), 0.1, 1e-5,
               L.ptr(mean), L.ptr(invstd), L.ptr(lo), None, 1, float(p), int(seed), L.ptr(kb), L.ptr(ws), L.stream())
    else:
        L.call("bnn_bn_fwd_train_i16", L.ptr(z16), L.ptr(bias), M, C, L.ptr(gam), L.ptr(bet), L.ptr(rm), L.ptr(rv),
               0.1, 1e-5, L.ptr(mean), L.ptr(invstd), L.ptr(lo), float(p), int(seed), L.ptr(kb), L.ptr(ws),
               L.stream())
    return mean, invstd, lo, rm, rv, gam, bet


def _keep_buffer(M, C):
    from bnn_amd import _lib as L
    n = int(L.lib().bnn_dropout_keep_bits_bytes(M, C))
    assert n == (M + 7) // 8 * (C // 4) * 4
    return torch.full((n // 4,), -1, dtype=torch.int32, device="cuda")   # poisoned: every word is written


@pytest.mark.parametrize("M,C", SHAPES)
@pytest.mark.parametrize("form", ["f32", "i16"])
def test_statistics_pass_writes_the_keep_mask(F, M, C, form):
    p, seed = 0.3, 4321 + M
    z16, bias, z = _inputs(F, M, C, M + C)
    kb = _keep_buffer(M, C)
    got = _stats(F, form, z, z16, bias, M, C, p, seed, kb)
    ref = _stats(F, form, z, z16, bias, M, C, p, seed, None)
    for a, b in zip(got, ref):        # writing the plane leaves the statistics unchanged
        assert eq(a, b)
    words = kb.to(torch.int64).view((M + 7) // 8, C // 4) & 0xFFFFFFFF
    assert eq(words, _expected_words(M, C, p, seed))


def test_keep_bits_bytes_rejects_bad_shapes(F):
    from bnn_amd import _lib as L
    assert L.lib().bnn_dropout_keep_bits_bytes(0, 256) < 0
    assert L.lib().bnn_dropout_keep_bits_bytes(16, 258) < 0
    assert L.lib().bnn_dropout_keep_bits_bytes(9, 8) == 2 * 2 * 4


@pytest.mark.parametrize("M,C", SHAPES)
@pytest.mark.parametrize("form", ["f32", "i16"])
def test_head_passes_with_keep_bits_bit_identical(F, M, C, form):
    """With and without the plane, under either form of the statistics pass (4 or 2 columns per
    thread, bnn_bn_set_head_reduce_cols): all four runs bit-identical."""
    from bnn_amd import _lib as L
    p, seed = 0.3, 99 + C
    z16, bias, z = _inputs(F, M, C, 3 * M + C)
    g = torch.Generator(device="cuda").manual_seed(C + 7)
    w4 = torch.randn(10, C, device="cuda", generator=g) * 0.05
    b4 = torch.randn(10, device="cuda", generator=g)
    dy4 = torch.randn(M, 10, device="cuda", generator=g)
    res = []
    saved = L.lib().bnn_bn_set_head_reduce_cols(-1)
    try:
        for cols in (4, 2):
            assert L.lib().bnn_bn_set_head_reduce_cols(cols) == 0
            for use_bits in (False, True):
                kb = _keep_buffer(M, C) if use_bits else None
                mean, invstd, lo, _, _, gam, bet = _stats(F, form, z, z16, bias, M, C, p, seed, kb)
                y4 = torch.empty(M, 10, device="cuda")
                if form == "f32":
                    L.call("bnn_bn_head_fwd", L.ptr(z), M, C, L.ptr(mean), L.ptr(invstd), L.ptr(lo), L.ptr(gam),
                           L.ptr(bet), p, seed, L.ptr(kb), L.ptr(w4), 10, L.ptr(b4), L.ptr(y4), L.stream())
                else:
                    L.call("bnn_bn_head_fwd_i16", L.ptr(z16), L.ptr(bias), M, C, L.ptr(mean), L.ptr(invstd),
                           L.ptr(lo), L.ptr(gam), L.ptr(bet), p, seed, L.ptr(kb), L.ptr(w4), 10, L.ptr(b4),
                           L.ptr(y4), L.stream())
                dx = torch.empty(M, C, device="cuda") if form == "f32" else None
                dg, db, cs = (torch.empty(C, device="cuda") for _ in range(3))
                dw4 = torch.empty(10, C, device="cuda")
                rows = F.Fp6Operand(*F._fp6_buffers(M, C, "cuda"), M, C, F._res_buffer(M, C, "cuda"))
                Mp = F.round_up(M)
                cols_op = F.Fp6Operand(*F._fp6_buffers(C, Mp, "cuda"), C, Mp)
                for t in (rows.lo, rows.hi, rows.sc, rows.res, cols_op.lo, cols_op.hi, cols_op.sc):
                    if t is not None:
                        t.fill_(0x5A)
                ws = torch.empty((L.lib().bnn_bn_head_workspace(M, C, 10),), dtype=torch.uint8, device="cuda")
                common = [L.ptr(dy4), L.ptr(w4), 10, M, C, L.ptr(gam), L.ptr(bet), L.ptr(mean), L.ptr(invstd),
                          L.ptr(lo), p, seed, L.ptr(kb), L.ptr(dx), L.ptr(dg), L.ptr(db), L.ptr(dw4), L.ptr(rows.lo),
                          L.ptr(rows.hi), L.ptr(rows.sc), L.ptr(rows.res), L.ptr(cols_op.lo), L.ptr(cols_op.hi),
                          L.ptr(cols_op.sc), L.ptr(cs), L.ptr(ws), L.stream()]
                if form == "f32":
                    L.call("bnn_bn_head_bwd_q6", L.ptr(z), *common)
                else:
                    L.call("bnn_bn_head_bwd_q6_i16", L.ptr(z16), L.ptr(bias), *common)
                out = [y4, dg, db, dw4, cs, rows.lo, rows.hi, rows.sc, rows.res, cols_op.lo, cols_op.hi, cols_op.sc]
                res.append(out + ([dx] if dx is not None else []))
    finally:
        L.lib().bnn_bn_set_head_reduce_cols(saved)
    for other in res[1:]:
        for a, b in zip(res[0], other):
            assert eq(a, b)


def test_head_reduce_cols_switch_rejects_bad_values(F):
    from bnn_amd import _lib as L
    assert L.lib().bnn_bn_set_head_reduce_cols(3) != 0
    assert L.lib().bnn_bn_set_head_reduce_cols(-1) in (2, 4)


@pytest.mark.parametrize("M,C", [(4096, 1024), (1000, 512)])
def test_fused_head_function_keep_bits_on_off(F, M, C):
    """dropout_bn_hardtanh_linear forward + backward with the plane (the default) and with
    BNN_KEEP_BITS=0's hashing passes: identical outputs and gradients."""
    torch.manual_seed(M)
    x0 = torch.randn(M, C, device="cuda") * 3
    res = []
    for on in (False, True):
        saved = F._KEEP_BITS[0]
        F._KEEP_BITS[0] = on
        try:
            torch.manual_seed(5)
            bn = torch.nn.BatchNorm1d(C).cuda().train()
            fc = torch.nn.Linear(C, 10).cuda()
            x = x0.clone().requires_grad_(True)
            y = F.dropout_bn_hardtanh_linear(x, 0.3, bn, fc, seed=777)
            y.backward(torch.linspace(-1, 1, M * 10, device="cuda").view(M, 10))
            res.append([y.detach(), x.grad, bn.weight.grad, bn.bias.grad, fc.weight.grad, fc.bias.grad,
                        bn.running_mean, bn.running_var])
        finally:
            F._KEEP_BITS[0] = saved
    for a, b in zip(*res):
        assert eq(a, b)

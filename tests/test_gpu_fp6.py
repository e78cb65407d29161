"""GPU parity of the FP6 digit GEMMs (csrc/bnn_gemm6.hip): fp32 operand x ternary operand on
v_mfma_scale_f32_32x32x64_f8f6f4 -- the backward GEMMs of BinarizeLinear (dX = dY.W_b,
dW = dY^T.X_b) and the first layer's forward (models/binarized_modules.py:80).

Bars:
* quantisers: decoded on the host, every element within max|x_block| * 2^-19 of x (the a-priori
  bound), digits in range, padding zero, column sums to fp32 rounding of the double sum; the row
  operands' residual FP4 plane (bnn_fp6.h): digits in [-4, 4] and the five planes' value EXACTLY
  rint(x 2^(22-e)) 2^(e-22) (within max|x_block| * 2^-23 of x);
* GEMM: against float64 products of the DECODED digits norm-wise <= 2e-6 (fp32 accumulation of
  exact block partial sums), against the float64 product of x itself <= 1e-5 (the gradient bar).
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
    # the row operands here carry the residual plane at every size (the networks add it from
    # functional.FP6_RES_MIN_ROWS rows on); restored after the module
    prev = functional.FP6_RES_MIN_ROWS
    functional.FP6_RES_MIN_ROWS = 0
    yield functional
    functional.FP6_RES_MIN_ROWS = prev


def host(t):
    torch.cuda.synchronize()
    return t.detach().cpu().numpy()


def _codes(lo, hi, rows, nblk):
    """[rows, nblk, 4 planes, 32] e2m3 codes from the lo / hi byte arrays (element i of a plane
    at bits 6i..6i+5 of its 6 dwords: 4 in lo, 2 in hi)."""
    lo = lo.reshape(rows, nblk, 4, 16)
    hi = hi.reshape(rows, nblk, 4, 8)
    words = np.ascontiguousarray(np.concatenate([lo, hi], axis=-1)).view(np.uint32).astype(np.uint64)
    codes = np.zeros(words.shape[:-1] + (32,), np.int64)
    for i in range(32):
        w, o = (6 * i) // 32, (6 * i) % 32
        c = words[..., w] >> np.uint64(o)
        if o > 26:
            c |= words[..., w + 1] << np.uint64(32 - o)
        codes[..., i] = (c & np.uint64(63)).astype(np.int64)
    return codes


def _e2m3_digit(c):
    s = np.where(c & 0x20, -1, 1)
    e = (c >> 3) & 3
    m = c & 7
    v8 = np.where(e == 0, m, (8 + m) << np.maximum(e - 1, 0))      # value * 8
    return s * v8


def residual_digits(op, rows):
    """[rows, nblk, 32] digits in [-4, 4] of the residual FP4 plane (element i at bits 4i: byte i/2,
    low nibble for even i; e2m1 code of d/2 = |d|, sign bit 3)."""
    nblk = op.Kp // 32
    r = host(op.res).reshape(-1, nblk, 16)[:rows].astype(np.int64)
    nib = np.stack([r & 15, r >> 4], axis=-1).reshape(rows, nblk, 32)
    assert np.all((nib & 7) <= 4)
    return np.where(nib & 8, -(nib & 7), nib & 7)


def decode(op, rows, residual=True):
    """Host decode of an Fp6Operand: [rows, Kp] float64 values and the digits (with the residual
    plane, scaled by plane 0's scale / 32, when the operand has one)."""
    nblk = op.Kp // 32
    d = _e2m3_digit(_codes(host(op.lo), host(op.hi), rows, nblk))     # [rows, nblk, 4, 32]
    sc = host(op.sc)                                                  # [Kp/64, rows_pad, 2]
    E = np.stack([sc[b // 2, :rows, b % 2] for b in range(nblk)], axis=1).astype(np.int64)   # [rows, nblk]
    val = np.zeros((rows, nblk, 32))
    for j in range(4):
        val += d[:, :, j, :] * np.ldexp(1.0, (E + 5 * j - 130))[..., None]
    if residual and op.res is not None:
        val += residual_digits(op, rows) * np.ldexp(1.0, E - 133)[..., None]
    return val.reshape(rows, nblk * 32), d, E


def _check_quant(x, val, d, E, bits=19):
    rows, K = x.shape
    nblk = val.shape[1] // 32
    assert np.all(np.abs(d[..., :3, :]) <= 16) and np.all(np.abs(d[..., 3, :]) <= 16)
    assert np.all(d[..., :3, :] < 16)                    # balanced: d0..d2 in [-16, 15]
    xp = np.zeros((rows, nblk * 32))
    xp[:, :K] = x
    amax = np.abs(xp.reshape(rows, nblk, 32)).max(-1)
    bound = np.repeat(amax * 2.0 ** -bits, 32, axis=1)
    assert np.all(np.abs(val - xp) <= bound + 1e-300)
    assert not val[:, K:].any()
    nz = amax > 0
    e = E - 111
    assert np.all((np.ldexp(1.0, e - 1) <= amax)[nz]) and np.all((amax < np.ldexp(1.0, e))[nz])


@pytest.mark.parametrize("M,K", [(5, 64), (300, 1000), (64, 784), (1, 8192), (257, 33)])
def test_quant6_rows_decodes_within_bound(F, M, K):
    rng = np.random.default_rng(M + K)
    x = (rng.standard_normal((M, K)) * np.exp(rng.uniform(-12, 12, (M, K)))).astype(np.float32)
    x[:, ::7] = 0.0
    if M > 3:
        x[3] = 0.0
    op = F.quant6_rows(torch.as_tensor(x).cuda())
    val4, d, E = decode(op, M, residual=False)
    _check_quant(x.astype(np.float64), val4, d, E)
    assert op.res is not None                            # the row operands carry the residual plane
    val, d, E = decode(op, M)
    _check_quant(x.astype(np.float64), val, d, E, bits=22)
    # the five planes are rint(x 2^(22-e)) 2^(e-22) exactly (e = E - 111 from the block max)
    xp = np.zeros((M, op.Kp))
    xp[:, :K] = x
    step = np.repeat(np.ldexp(1.0, E - 111 - 22), 32, axis=1)
    want = np.rint(xp / step) * step
    assert np.array_equal(val, want)


@pytest.mark.parametrize("M,N", [(300, 200), (64, 8192), (1000, 37), (33, 64)])
def test_quant6_cols_t_decodes_within_bound(F, M, N):
    rng = np.random.default_rng(M * N)
    x = (rng.standard_normal((M, N)) * np.exp(rng.uniform(-10, 10, (M, 1)))).astype(np.float32)
    op, cs = F.quant6_cols_t(torch.as_tensor(x).cuda(), want_colsum=True)
    val, d, E = decode(op, N)
    _check_quant(x.T.astype(np.float64), val, d, E)
    assert rel_err(host(cs), x.astype(np.float64).sum(0)) < 1e-6


@pytest.mark.parametrize("M,N,K", [(300, 200, 256), (257, 520, 1000), (64, 64, 64), (1000, 129, 1024),
                                   (2048, 1024, 8192), (3, 7, 784)])
def test_gemm_fp6_every_variant(F, M, N, K):
    from bnn_amd import _lib as L
    rng = np.random.default_rng(M + 3 * N + K)
    x = (rng.standard_normal((M, K)) * np.exp(rng.uniform(-6, 6, (M, 1)))).astype(np.float32)
    w = rng.integers(-1, 2, (N, K)).astype(np.float32)
    bias = rng.standard_normal(N).astype(np.float32)
    xt = torch.as_tensor(x).cuda()
    op = F.quant6_rows(xt)
    op4 = F.Fp6Operand(op.lo, op.hi, op.sc, op.rows, op.Kp)    # the four digit planes alone
    w4, _ = F.sign_pack_fp4(torch.as_tensor(w).cuda())
    val, _, _ = decode(op4, M)
    exact_q = val[:, :K] @ w.astype(np.float64).T + bias        # what the MFMA sums (no rounding)
    exact_x = x.astype(np.float64) @ w.astype(np.float64).T + bias
    bt = torch.as_tensor(bias).cuda()
    names = set()
    try:
        for v in range(0, 16):
            L.call("bnn_gemm_fp6_set_variant", v)
            name = L.lib().bnn_gemm_fp6_kernel(M, N).decode()
            if name in names:
                continue
            names.add(name)
            C = host(F.gemm_fp6(op4, w4, N, bias=bt))
            assert rel_err(C, exact_q) < 2e-6, (name, rel_err(C, exact_q))
            assert rel_err(C, exact_x) < 1e-5, (name, rel_err(C, exact_x))
    finally:
        L.call("bnn_gemm_fp6_set_variant", -1)
    assert len(names) >= 3
    # the default kernel with the residual plane (a fifth MFMA pass): the five-plane product
    val5, _, _ = decode(op, M)
    exact_q5 = val5[:, :K] @ w.astype(np.float64).T + bias
    C5 = host(F.gemm_fp6(op, w4, N, bias=bt))
    assert rel_err(C5, exact_q5) < 2e-6 and rel_err(C5, exact_x) < 2e-6, (rel_err(C5, exact_q5), rel_err(C5, exact_x))


@pytest.mark.parametrize("M,N,K", [(768, 1536, 4096), (1536, 3072, 4096), (4096, 1536, 768), (200, 132, 8192),
                                   (64, 64, 1024), (300, 520, 512), (1000, 36, 1024)])
def test_gemm_fp6_split_k(F, M, N, K):
    """Split-K (tile grids below one round of the chip: the MLP's backward GEMMs at batch 4096,
    config 3): per-split fp32 partials folded in split order with the bias.  Equal to the digit
    product within fp32 rounding, deterministic (two runs bit-identical), shape-only (an unaligned,
    strided C -- a gradient-bucket view -- gets the same bits), and a workspace too small falls
    back to the unsplit grid.  Shapes: 2-32 splits, ragged M / N."""
    from bnn_amd import _lib as L
    rng = np.random.default_rng(M + N + K)
    x = (rng.standard_normal((M, K)) * np.exp(rng.uniform(-6, 6, (M, 1)))).astype(np.float32)
    w = rng.integers(-1, 2, (N, K)).astype(np.float32)
    bias = rng.standard_normal(N).astype(np.float32)
    wsb = L.lib().bnn_gemm_fp6_workspace(M, N, K)
    assert wsb > 0 and "split-K" in L.lib().bnn_gemm_fp6_kernel_k(M, N, K).decode()
    op = F.quant6_rows(torch.as_tensor(x).cuda())
    w4, _ = F.sign_pack_fp4(torch.as_tensor(w).cuda())
    val, _, _ = decode(op, M)
    exact_q = val[:, :K] @ w.astype(np.float64).T + bias
    exact_x = x.astype(np.float64) @ w.astype(np.float64).T + bias
    bt = torch.as_tensor(bias).cuda()
    C1, C2 = host(F.gemm_fp6(op, w4, N, bias=bt)), host(F.gemm_fp6(op, w4, N, bias=bt))
    assert np.array_equal(C1, C2)
    assert rel_err(C1, exact_q) < 2e-6 and rel_err(C1, exact_x) < 1e-5
    big = torch.full((M * (N + 3) + 1,), float("nan"), device="cuda")
    Cv = big[1:].view(M, N + 3)[:, :N]                 # 4-B aligned only, row pitch N + 3
    F.gemm_fp6(op, w4, N, bias=bt, out=Cv)
    assert np.array_equal(host(Cv), C1)
    C0 = torch.empty(M, N, device="cuda")               # no workspace: the unsplit grid
    L.call("bnn_gemm_fp6_ws", L.ptr(op.lo), L.ptr(op.hi), L.ptr(op.sc), op.sc.shape[1], L.ptr(op.res), L.ptr(w4),
           w4.shape[1],
           L.ptr(bt), L.ptr(C0), N, M, N, op.Kp, None, 0, L.stream())
    assert rel_err(host(C0), exact_q) < 2e-6


def test_gemm_fp6_propagates_nan(F):
    """A NaN in the fp32 operand makes its block's E8M0 scale NaN: every output that sums over it
    is NaN (as the reference's fp32 GEMM gives), the others are unaffected."""
    x = torch.randn(40, 128, device="cuda")
    x[7, 100] = float("nan")
    w = torch.randint(-1, 2, (24, 128), device="cuda").float()
    C = F.gemm_fp6(F.quant6_rows(x), F.sign_pack_fp4(w)[0], 24)
    isn = torch.isnan(C)
    assert bool(isn[7].all()) and int(isn.sum()) == 24


@pytest.mark.parametrize("M,N,K", [(300, 600, 320), (2048, 1024, 8192), (768, 1536, 4096), (64, 37, 64)])
def test_fp4_panels_and_panel_gemm(F, M, N, K):
    """The FP4 panel layout [ceil(N/512)][K/64][512][32 B] (zero rows beyond N) equals a host
    re-tiling of the row-major operand, and the GEMM staged from panels is bit-identical to the one
    staged from rows (only the staging source changes), split-K shapes included."""
    from bnn_amd import _lib as L
    rng = np.random.default_rng(M * 7 + N + K)
    x = (rng.standard_normal((M, K)) * np.exp(rng.uniform(-4, 4, (M, 1)))).astype(np.float32)
    w = rng.integers(-1, 2, (N, K)).astype(np.float32)
    w4, _ = F.sign_pack_fp4(torch.as_tensor(w).cuda())
    P = F.fp4_panels(w4, N, K)
    rows = host(w4)[:, :K // 2]
    npan = (N + 511) // 512
    ref = np.zeros((npan * 512, K // 2), np.uint8)
    ref[:N] = rows
    ref = ref.reshape(npan, 512, K // 64, 32).transpose(0, 2, 1, 3).reshape(-1)
    assert np.array_equal(host(P), ref)
    op = F.quant6_rows(torch.as_tensor(x).cuda())
    bt = torch.as_tensor(rng.standard_normal(N).astype(np.float32)).cuda()
    C_rows = host(F.gemm_fp6(op, w4, N, bias=bt, panels=None)) if M * N * K < F.PANEL_MIN_MACS else None
    if C_rows is None:                                  # force the row-major staging for the comparison
        C0 = torch.empty(M, N, device="cuda")
        wsb = L.lib().bnn_gemm_fp6_workspace(M, N, op.Kp)
        ws = torch.empty((max(wsb, 1),), dtype=torch.uint8, device="cuda")
        L.call("bnn_gemm_fp6_ws", L.ptr(op.lo), L.ptr(op.hi), L.ptr(op.sc), op.sc.shape[1], L.ptr(op.res), L.ptr(w4),
           w4.shape[1],
               L.ptr(bt), L.ptr(C0), N, M, N, op.Kp, L.ptr(ws), wsb, L.stream())
        C_rows = host(C0)
    C_pan = host(F.gemm_fp6(op, w4, N, bias=bt, panels=P))
    assert np.array_equal(C_pan, C_rows)
    val, _, _ = decode(op, M)
    assert rel_err(C_pan, val[:, :K] @ w.astype(np.float64).T + host(bt)) < 2e-6


@pytest.mark.parametrize("M,N,K", [(16384, 4096, 1024), (16512, 4096, 1088), (8192, 8192, 4096)])
@pytest.mark.parametrize("res", [True, False])
def test_fp6_persistent_gemm_bit_identical(F, M, N, K, res):
    """The persistent form of the default tile (gemm_fp6_pers_k: one workgroup per CU, loading and
    storing waves split so a tile's stores drain under the next tile's k loop; an A/B switch, off by
    default) against one workgroup per tile: C bit-identical, with and without the residual plane; grids of
    4-5 tiles per workgroup, an uneven tile count (129 tile rows) and an odd number of k-steps (17:
    the two-slot ring's parity carries across tiles), and within 2e-6 of the float64 product of the
    decoded operand."""
    from bnn_amd import _lib as L
    rng = np.random.default_rng(M + N + K + res)
    x = (rng.standard_normal((M, K)) * np.exp(rng.uniform(-3, 3, (M, 1)))).astype(np.float32)
    w = rng.integers(-1, 2, (N, K)).astype(np.float32)
    w4, _ = F.sign_pack_fp4(torch.as_tensor(w).cuda())
    P = F.fp4_panels(w4, N, K)
    op = F.quant6_rows(torch.as_tensor(x).cuda())
    if not res:
        op.res = None
    prev = L.lib().bnn_gemm_fp6_set_persistent(-1)
    ks = P.numel() // (((N + 511) // 512) * 512 * 32)
    try:
        L.call("bnn_gemm_fp6_set_persistent", 1)
        assert "pers" in L.lib().bnn_gemm_fp6_kernel_k(M, N, op.Kp).decode()
        C1 = F.gemm_fp6(op, None, N, panels=P, panel_ks=ks)
        L.call("bnn_gemm_fp6_set_persistent", 0)
        assert "pers" not in L.lib().bnn_gemm_fp6_kernel_k(M, N, op.Kp).decode()
        C0 = F.gemm_fp6(op, None, N, panels=P, panel_ks=ks)
        torch.cuda.synchronize()
    finally:
        L.call("bnn_gemm_fp6_set_persistent", prev)
    assert torch.equal(C0, C1)
    op_head = F.quant6_rows(torch.as_tensor(x[:2048]).cuda())      # rows quantise independently
    if not res:
        op_head.res = None
    val, _, _ = decode(op_head, 2048, residual=res)
    assert rel_err(host(C1)[:2048], val[:, :K] @ w.astype(np.float64).T) < 2e-6


@pytest.mark.parametrize("M,N,K", [(8192, 4096, 1024), (16384, 4096, 1088), (8256, 4096, 512)])
@pytest.mark.parametrize("res", [True, False])
def test_fp6_half_tile_gemm_bit_identical(F, M, N, K, res):
    """The half-tile form (64 x 512 tiles, two 4-wave workgroups per CU, the default for the
    residual-plane dX launches; bnn_gemm_fp6_set_half) against the 128 x 512 tile, with and without
    a first-round stagger: C bit-identical with and without the residual plane, on grids of >= 2
    rounds, an odd number of 64-row tile rows (8256 = 129 x 64) and an odd number of k-steps (17);
    within 2e-6 of the float64 product of the decoded operand."""
    from bnn_amd import _lib as L
    rng = np.random.default_rng(M + N + K + res + 7)
    x = (rng.standard_normal((M, K)) * np.exp(rng.uniform(-3, 3, (M, 1)))).astype(np.float32)
    w = rng.integers(-1, 2, (N, K)).astype(np.float32)
    w4, _ = F.sign_pack_fp4(torch.as_tensor(w).cuda())
    P = F.fp4_panels(w4, N, K)
    op = F.quant6_rows(torch.as_tensor(x).cuda())
    if not res:
        op.res = None
    prev = L.lib().bnn_gemm_fp6_set_half(-1, 0.0)
    ks = P.numel() // (((N + 511) // 512) * 512 * 32)
    outs = {}
    try:
        for mode, st in ((0, 0.0), (2, 0.0), (2, 60.0)):
            L.call("bnn_gemm_fp6_set_half", mode, st)
            name = L.lib().bnn_gemm_fp6_kernel_kr(M, N, op.Kp, int(res)).decode()
            assert ("<1, 4, 2, 4, 2>" in name) == (mode > 0), (mode, name)
            outs[(mode, st)] = F.gemm_fp6(op, None, N, panels=P, panel_ks=ks)
        torch.cuda.synchronize()
    finally:
        L.call("bnn_gemm_fp6_set_half", prev, 0.0)
    C0 = outs[(0, 0.0)]
    for k, C in outs.items():
        assert torch.equal(C, C0), k
    op_head = F.quant6_rows(torch.as_tensor(x[:2048]).cuda())
    if not res:
        op_head.res = None
    val, _, _ = decode(op_head, 2048, residual=res)
    assert rel_err(host(C0)[:2048], val[:, :K] @ w.astype(np.float64).T) < 2e-6

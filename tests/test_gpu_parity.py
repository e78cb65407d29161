"""GPU parity: libbnn (through its C ABI) against the oracle and the reference's golden outputs.

Bars (written here, per BASELINE.json north_star):
* binarised forward (ternary x ternary + bias): bit-exact (np.array_equal);
* fp32-input forward (fc1 / RGB conv): norm-wise relative error <= 1e-6 vs float64;
* gradients: norm-wise relative error <= 1e-5 vs the float64 oracle.
"""
import numpy as np
import pytest
import torch

from conftest import close, load_golden, rel_err
from oracle import bnn_np as O

pytestmark = pytest.mark.gpu

GRAD_TOL = 1e-5
FP_FWD_TOL = 1e-6


@pytest.fixture(scope="module")
def F():
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    from bnn_amd import functional
    return functional


def dev(a):
    return torch.as_tensor(np.ascontiguousarray(a)).cuda()


def host(t):
    torch.cuda.synchronize()
    return t.detach().cpu().numpy()


def run_linear(F, x, w, b, dy, binarize, backend="mfma"):
    xt = dev(x).requires_grad_(True)
    wt = dev(w).requires_grad_(True)
    bt = dev(b).requires_grad_(True) if b is not None else None
    y = F.binary_linear(xt, wt, bt, binarize_input=binarize, backend=backend)
    y.backward(dev(dy))
    return (host(y), host(xt.grad), host(wt.grad), host(bt.grad) if bt is not None else None)


@pytest.mark.parametrize("name", ["linear_first", "linear_hidden", "linear_nobias_zw"])
@pytest.mark.parametrize("backend", ["fp4", "mfma", "xnor"])
def test_linear_matches_reference_golden(F, name, backend):
    """The reference's own BinarizeLinear fixtures through every engine; "fp4" is the default one
    (FP4 MFMA forward, FP6 digit-plane backward GEMMs)."""
    g = load_golden(name)
    binarize = not O.first_layer(g["x"])
    b = g["bias"] if g["has_bias"] else None
    y, dx, dw, db = run_linear(F, g["x"], g["w_latent"], b, g["dy"], binarize, backend)
    if binarize:
        assert np.array_equal(y, g["y"])
    else:
        y64 = g["x"].astype(np.float64) @ np.sign(g["w_latent"]).astype(np.float64).T + (b if b is not None else 0)
        assert rel_err(y, y64) < FP_FWD_TOL
        assert rel_err(y, g["y"]) < FP_FWD_TOL
    _, w64, _ = O.linear_backward(g["x_after"], g["w_latent"], g["dy"], need_dx=False)
    dx64 = g["dy"].astype(np.float64) @ np.sign(g["w_latent"]).astype(np.float64)
    dw64 = g["dy"].astype(np.float64).T @ g["x_after"].astype(np.float64)
    assert rel_err(dx, dx64) < GRAD_TOL and rel_err(dx, g["dx"]) < GRAD_TOL
    assert rel_err(dw, dw64) < GRAD_TOL and rel_err(dw, g["dw"]) < GRAD_TOL
    if b is not None:
        assert rel_err(db, g["db"]) < GRAD_TOL


SHAPES = [(1, 64, 1), (3, 100, 37), (64, 256, 128), (100, 3072, 1536), (129, 1000, 257), (257, 784, 300),
          (512, 1536, 768)]


@pytest.mark.parametrize("M,K,N", SHAPES)
@pytest.mark.parametrize("backend", ["mfma", "xnor", "fp4"])
def test_linear_random_shapes(F, M, K, N, backend):
    rng = np.random.default_rng(M * 131 + K * 7 + N)
    x = rng.standard_normal((M, K)).astype(np.float32)
    x[rng.random((M, K)) < 0.05] = 0.0                     # sign(0) = 0 -> ternary
    w = rng.uniform(-1, 1, (N, K)).astype(np.float32)
    w[rng.random((N, K)) < 0.01] = 0.0
    b = rng.standard_normal(N).astype(np.float32)
    dy = rng.standard_normal((M, N)).astype(np.float32)
    binarize = K != 784
    y, dx, dw, db = run_linear(F, x, w, b, dy, binarize, backend)
    y_ref, xu = O.linear_forward(x, w, b)
    if binarize:
        assert np.array_equal(y, y_ref)
    else:
        y64 = x.astype(np.float64) @ np.sign(w).astype(np.float64).T + b
        assert rel_err(y, y64) < FP_FWD_TOL
    dx64 = dy.astype(np.float64) @ np.sign(w).astype(np.float64)
    dw64 = dy.astype(np.float64).T @ xu.astype(np.float64)
    assert rel_err(dx, dx64) < GRAD_TOL
    assert rel_err(dw, dw64) < GRAD_TOL
    assert rel_err(db, dy.astype(np.float64).sum(0)) < GRAD_TOL


def test_mfma_and_xnor_agree_bitwise(F):
    rng = np.random.default_rng(5)
    x = dev(np.where(rng.random((300, 2048)) < 0.1, 0, rng.standard_normal((300, 2048))).astype(np.float32))
    w = dev(rng.uniform(-1, 1, (200, 2048)).astype(np.float32))
    b = dev(rng.standard_normal(200).astype(np.float32))
    y1 = F.binary_linear(x, w, b, True, "mfma")
    y2 = F.binary_linear(x, w, b, True, "xnor")
    y3 = F.binary_linear(x, w, b, True, "fp4")
    assert torch.equal(y1, y2)
    assert torch.equal(y1, y3)


@pytest.mark.parametrize("M,N,K", [(300, 200, 256), (257, 520, 1000), (64, 64, 64), (2048, 1024, 8192)])
def test_every_fp4_variant_is_exact(F, M, N, K):
    """FP4 (e2m1) ternary GEMM variants against exact integer products."""
    from bnn_amd import _lib
    rng = np.random.default_rng(M + N + K)
    x = rng.integers(-1, 2, (M, K)).astype(np.float32)
    w = rng.integers(-1, 2, (N, K)).astype(np.float32)
    bias = rng.standard_normal(N).astype(np.float32)
    ref = (x.astype(np.int64) @ w.astype(np.int64).T).astype(np.float32) + bias
    x4, _ = F.sign_pack_fp4(dev(x))
    w4, _ = F.sign_pack_fp4(dev(w))
    names = set()
    try:
        for v in range(0, 7):
            _lib.call("bnn_gemm_set_variant", v)
            name = F.gemm_kernel_name(0, 0, M, N, x4.shape[1])
            if name in names:
                continue
            names.add(name)
            assert np.array_equal(host(F.gemm_fp4(x4, w4, M, N, bias=dev(bias))), ref), name
    finally:
        _lib.call("bnn_gemm_set_variant", -1)


def test_sign_pack_layouts(F):
    rng = np.random.default_rng(1)
    x = rng.standard_normal((70, 130)).astype(np.float32)
    x[::3, ::5] = 0.0
    q, qt = F.sign_pack(dev(x), True, True)
    q, qt = host(q), host(qt)
    s = np.sign(x).astype(np.int8)
    assert q.shape == (70, 192) and qt.shape == (130, 128)
    assert np.array_equal(q[:, :130], s) and not q[:, 130:].any()
    assert np.array_equal(qt[:, :70], s.T) and not qt[:, 70:].any()
    sb, nz = F.sign_pack_bits(dev(x))
    sb, nz = host(sb).view(np.uint32), host(nz).view(np.uint32)
    for k in (0, 31, 32, 129):
        assert np.array_equal((sb[:, k // 32] >> (k % 32)) & 1, (x[:, k] < 0).astype(np.uint32))
        assert np.array_equal((nz[:, k // 32] >> (k % 32)) & 1, (x[:, k] != 0).astype(np.uint32))
    assert not sb[:, 5:].any() and not nz[:, 5:].any()


def test_sign_of_nan_is_zero(F):
    """Documented deviation: the ternary kernels map sign(NaN) to 0 where the
    reference's Tensor.sign() (binarized_modules.py:13) would propagate NaN.  Pinned for every
    packed form and through a binarised forward: a NaN latent weight acts as a zero weight."""
    rng = np.random.default_rng(11)
    x = rng.standard_normal((67, 300)).astype(np.float32)
    x[::4, ::7] = np.nan
    z = np.where(np.isnan(x), np.float32(0), x)
    for want_qt in (False, True):
        a, b = F.sign_pack(dev(x), True, want_qt), F.sign_pack(dev(z), True, want_qt)
        assert all(torch.equal(p, q) for p, q in zip(a, b) if p is not None)
    a, b = F.sign_pack_fp4(dev(x), want_qt=True), F.sign_pack_fp4(dev(z), want_qt=True)
    assert all(torch.equal(p, q) for p, q in zip(a, b) if p is not None)
    a, b = F.sign_pack_bits(dev(x)), F.sign_pack_bits(dev(z))
    assert all(torch.equal(p, q) for p, q in zip(a, b))
    h = np.sign(rng.standard_normal((33, 300))).astype(np.float32)
    bias = rng.standard_normal(67).astype(np.float32)
    y_nan, *_ = run_linear(F, h, x, bias, np.zeros((33, 67), np.float32), True, backend="fp4")
    y_zero, *_ = run_linear(F, h, z, bias, np.zeros((33, 67), np.float32), True, backend="fp4")
    assert np.array_equal(y_nan, y_zero) and np.isfinite(y_nan).all()


def _recon(d, s):
    d = d.astype(np.float64)
    return (d[2] * 65536 + d[1] * 256 + d[0]) * s


def test_digit_quantisation(F):
    rng = np.random.default_rng(2)
    x = (rng.standard_normal((50, 300)) * np.exp(rng.uniform(-20, 20, (50, 1)))).astype(np.float32)
    x[3] = 0.0
    d, s = F.quant_rows(dev(x))
    d, s = host(d), host(s)
    assert d[:, :, 300:].sum() == 0 and s[3] == 0 and np.all(np.abs(d[2]) <= 65)
    r = _recon(d[:, :, :300], s[:, None])
    amax = np.abs(x).max(1, keepdims=True)
    assert np.all(np.abs(r - x) <= amax * 2.0 ** -22 + 1e-45)
    dt, sc, cs = F.quant_cols_t(dev(x), want_colsum=True)
    dt, sc, cs = host(dt), host(sc), host(cs)
    r = _recon(dt[:, :, :50], sc[:, None]).T
    amax = np.abs(x).max(0, keepdims=True)
    assert np.all(np.abs(r - x) <= amax * 2.0 ** -22 + 1e-45)
    assert rel_err(cs, x.astype(np.float64).sum(0)) < 1e-6


@pytest.mark.parametrize("name", ["conv_c1", "conv_c16", "conv_c3", "conv_sdg"])
def test_conv_matches_reference_golden(F, name):
    g = load_golden(name)
    s, p, d, gr = (int(v) for v in g["conv"])
    binarize = O.conv_binarizes_input(g["x"])
    xt = dev(g["x"]).requires_grad_(True)
    wt = dev(g["w_latent"]).requires_grad_(True)
    bt = dev(g["bias"]).requires_grad_(True) if g["has_bias"] else None
    y = F.binary_conv2d(xt, wt, bt, binarize, s, p, d, gr)
    y.backward(dev(g["dy"]))
    if binarize:
        assert np.array_equal(host(y), g["y"])
    else:
        assert rel_err(host(y), g["y"]) < FP_FWD_TOL
    dx64, dw64, db64 = O.conv2d_backward(g["x_after"], g["w_latent"], g["dy"], s, p, d, gr)
    assert rel_err(host(xt.grad), g["dx"]) < GRAD_TOL
    assert rel_err(host(wt.grad), g["dw"]) < GRAD_TOL
    if bt is not None:
        assert rel_err(host(bt.grad), g["db"]) < GRAD_TOL


def test_conv_cnn_shapes_vs_oracle(F):
    rng = np.random.default_rng(3)
    x = np.where(rng.random((6, 16, 14, 14)) < 0.3, 0, rng.standard_normal((6, 16, 14, 14))).astype(np.float32)
    w = rng.uniform(-1, 1, (32, 16, 5, 5)).astype(np.float32)
    b = rng.standard_normal(32).astype(np.float32)
    dy = rng.standard_normal((6, 32, 14, 14)).astype(np.float32)
    xt, wt, bt = dev(x).requires_grad_(True), dev(w).requires_grad_(True), dev(b).requires_grad_(True)
    y = F.binary_conv2d(xt, wt, bt, True, 1, 2, 1, 1)
    y.backward(dev(dy))
    y_ref, xu = O.conv2d_forward(x, w, b, 1, 2, 1, 1)
    assert np.array_equal(host(y), y_ref)
    dx64, dw64, db64 = O.conv2d_backward(xu, w, dy, 1, 2, 1, 1)
    assert rel_err(host(xt.grad), dx64) < GRAD_TOL
    assert rel_err(host(wt.grad), dw64) < GRAD_TOL
    assert rel_err(host(bt.grad), db64) < GRAD_TOL


@pytest.mark.parametrize("shape", [
    # (N, C, H, W, Co, K, pad, bias, binarize) -- LDS-tiled fast path (stride 1, pad <= K-1) ...
    (1, 1, 28, 28, 16, 5, 2, True, True),
    (9, 16, 14, 14, 32, 5, 2, True, True),
    (17, 3, 13, 11, 8, 3, 1, True, False),      # the C == 3 rule: fp32 input
    (5, 7, 10, 9, 5, 3, 0, False, True),
    (3, 33, 8, 8, 40, 3, 2, True, True),
    (2, 64, 6, 7, 64, 1, 0, True, True),
    (11, 3, 9, 12, 3, 7, 3, False, False),
    (4, 20, 5, 5, 64, 5, 4, True, True),
    # ... and shapes that take the generic kernels (stride 2 / pad > K-1 / C > 64)
    (3, 4, 9, 9, 6, 3, 3, True, True),
    (2, 80, 5, 5, 8, 3, 1, True, True),
])
def test_conv_tiled_and_generic_shapes_vs_oracle(F, shape):
    N, C, H, W, Co, K, pad, has_bias, binarize = shape
    rng = np.random.default_rng(N * 1000 + C)
    x = np.where(rng.random((N, C, H, W)) < 0.2, 0, rng.standard_normal((N, C, H, W))).astype(np.float32)
    w = np.where(rng.random((Co, C, K, K)) < 0.1, 0, rng.uniform(-1, 1, (Co, C, K, K))).astype(np.float32)
    b = rng.standard_normal(Co).astype(np.float32) if has_bias else None
    xt, wt = dev(x).requires_grad_(True), dev(w).requires_grad_(True)
    bt = dev(b).requires_grad_(True) if has_bias else None
    assert binarize == O.conv_binarizes_input(x)
    y = F.binary_conv2d(xt, wt, bt, binarize, 1, pad, 1, 1)
    y_ref, xu = O.conv2d_forward(x, w, b, 1, pad, 1, 1)   # float64 sums
    if binarize:
        assert np.array_equal(host(y), y_ref)
    else:
        assert rel_err(host(y), y_ref) < FP_FWD_TOL
    dy = rng.standard_normal(tuple(y.shape)).astype(np.float32)
    y.backward(dev(dy))
    dx64, dw64, db64 = O.conv2d_backward(xu, w, dy, 1, pad, 1, 1)
    assert rel_err(host(xt.grad), dx64) < GRAD_TOL
    assert rel_err(host(wt.grad), dw64) < GRAD_TOL
    if has_bias:
        assert rel_err(host(bt.grad), db64) < GRAD_TOL


@pytest.mark.parametrize("shape", [
    (9, 16, 14, 14, 32, 5, 2, True),     # BinCNN conv2
    (10, 1, 28, 28, 16, 5, 2, True),     # BinCNN conv1 (binarised C=1 input)
    (5, 3, 12, 10, 8, 3, 1, False),      # C == 3: fp32 input
    (3, 20, 9, 7, 40, 3, 0, True),
    (2, 32, 6, 6, 64, 1, 0, True),
])
def test_conv_backward_mfma_matches_valu(F, shape):
    """The MFMA implicit-GEMM conv kernels (int8 forward; backward data on bf16x3 (mode 1) or f32
    (mode 2), backward filter on f32) against the float64 oracle and against the VALU kernels
    (bnn_conv_set_mfma(0)) on the same inputs."""
    from bnn_amd import _lib as L
    N, C, H, W, Co, K, pad, binarize = shape
    rng = np.random.default_rng(N + C + Co)
    x = np.where(rng.random((N, C, H, W)) < 0.3, 0, rng.standard_normal((N, C, H, W))).astype(np.float32)
    w = np.where(rng.random((Co, C, K, K)) < 0.1, 0, rng.uniform(-1, 1, (Co, C, K, K))).astype(np.float32)
    b = rng.standard_normal(Co).astype(np.float32)
    grads = []
    try:
        for on in (1, 2, 0):
            L.call("bnn_conv_set_mfma", on)
            xt, wt, bt = dev(x).requires_grad_(True), dev(w).requires_grad_(True), dev(b).requires_grad_(True)
            y = F.binary_conv2d(xt, wt, bt, binarize, 1, pad, 1, 1)
            dy = np.random.default_rng(1).standard_normal(tuple(y.shape)).astype(np.float32)
            y.backward(dev(dy))
            grads.append((host(xt.grad), host(wt.grad), host(bt.grad), host(y)))
    finally:
        L.call("bnn_conv_set_mfma", 1)
    _, xu = O.conv2d_forward(x, w, b, 1, pad, 1, 1)
    dx64, dw64, db64 = O.conv2d_backward(xu, w, dy, 1, pad, 1, 1)
    assert np.array_equal(grads[0][3], grads[2][3])      # forward: int8-MFMA conv == VALU conv, bitwise
    for g in grads:
        assert rel_err(g[0], dx64) < GRAD_TOL
        assert rel_err(g[1], dw64) < GRAD_TOL
        assert rel_err(g[2], db64) < GRAD_TOL


@pytest.mark.parametrize("shape", [
    (4096, 16, 14, 14, 32, 5, 2),    # BinCNN conv2 at the bench batch: 16 samples per workgroup
    (4096, 1, 28, 28, 16, 5, 2),     # BinCNN conv1
])
def test_conv_backward_full_batch_vs_float64(F, shape):
    """The bf16x3 conv backward at the bench's batch (the 16-samples-per-workgroup schedule, one
    round over the CUs) against float64 torch convolutions of the binarised operands on the GPU."""
    N, C, H, W, Co, K, pad = shape
    g = torch.Generator(device="cuda").manual_seed(N + C)
    x = torch.randn(N, C, H, W, device="cuda", generator=g)
    x = torch.where(torch.rand(N, C, H, W, device="cuda", generator=g) < 0.3, torch.zeros_like(x), x)
    w = torch.rand(Co, C, K, K, device="cuda", generator=g) * 2 - 1
    b = torch.randn(Co, device="cuda", generator=g)
    dy = torch.randn(N, Co, H, W, device="cuda", generator=g)
    xt, wt, bt = x.clone().requires_grad_(True), w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    F.binary_conv2d(xt, wt, bt, True, 1, pad, 1, 1).backward(dy)
    xs, ws, d64 = torch.sign(x).double(), torch.sign(w).double(), dy.double()
    dw64 = torch.nn.grad.conv2d_weight(xs, tuple(w.shape), d64, padding=pad)
    dx64 = torch.nn.grad.conv2d_input(tuple(x.shape), ws, d64, padding=pad)
    db64 = d64.sum((0, 2, 3))
    for got, want in ((wt.grad, dw64), (xt.grad, dx64), (bt.grad, db64)):
        err = float((got.double() - want).norm() / want.norm())
        assert err < GRAD_TOL, err


@pytest.mark.parametrize("shape", [
    (5, 1, 28, 28, 16, 5, 2),      # BinCNN conv1, a ragged last workgroup
    (7, 1, 12, 16, 8, 3, 1),
    (3, 1, 20, 8, 32, 5, 0),
    (9, 1, 28, 28, 64, 3, 1),
    (6, 1, 10, 12, 4, 5, 4),       # pad = K - 1
])
def test_conv1_filter_valu_vs_float64(F, shape):
    """The one-input-channel filter gradient (conv_bwd_filter_c1_k, bnn_conv_set_c1_filter) against
    float64 torch on the binarised operands and against the MFMA kernel on the same inputs."""
    from bnn_amd import _lib as L
    N, C, H, W, Co, K, pad = shape
    g = torch.Generator(device="cuda").manual_seed(N * 7 + Co)
    x = torch.randn(N, C, H, W, device="cuda", generator=g)
    x = torch.where(torch.rand(N, C, H, W, device="cuda", generator=g) < 0.3, torch.zeros_like(x), x)
    w = torch.rand(Co, C, K, K, device="cuda", generator=g) * 2 - 1
    b = torch.randn(Co, device="cuda", generator=g)
    OH, OW = H + 2 * pad - K + 1, W + 2 * pad - K + 1
    dy = torch.randn(N, Co, OH, OW, device="cuda", generator=g)
    xs, d64 = torch.sign(x).double(), dy.double()
    dw64 = torch.nn.grad.conv2d_weight(xs, tuple(w.shape), d64, padding=pad)
    db64 = d64.sum((0, 2, 3))
    got = []
    try:
        for on in (1, 0):
            L.call("bnn_conv_set_c1_filter", on)
            wt, bt = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
            F.binary_conv2d(x, wt, bt, True, 1, pad, 1, 1).backward(dy)
            got.append((wt.grad.double(), bt.grad.double()))
    finally:
        L.call("bnn_conv_set_c1_filter", 1)
    for gw, gb in got:
        assert float((gw - dw64).norm() / dw64.norm()) < GRAD_TOL
        assert float((gb - db64).norm() / db64.norm()) < GRAD_TOL


def test_hardtanh_backward(F):
    x = torch.tensor([-2.0, -1.0, -0.5, 0.0, 0.5, 1.0, 3.0] * 11, device="cuda")
    g = torch.randn_like(x)
    out = F.hardtanh_backward(x, g)
    xr = x.clone().requires_grad_(True)
    torch.nn.functional.hardtanh(xr).backward(g)
    assert torch.equal(out, xr.grad)


def test_adam_clamp_matches_torch(F):
    torch.manual_seed(0)
    p0 = torch.empty(10007, device="cuda").uniform_(-1.2, 1.2)
    p_ref = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([p_ref], lr=0.01)
    p = p0.clone()
    m = torch.zeros_like(p)
    v = torch.zeros_like(p)
    for step in range(1, 6):
        g = torch.randn_like(p)
        p_ref.grad = g.clone()
        opt.step()
        with torch.no_grad():
            p_ref.clamp_(-1, 1)
        F.adam_clamp_(p, g, m, v, step, lr=0.01)
    assert close(host(p), host(p_ref), 1e-6, 0.0)


def test_adam_clamp_multi_equals_single(F):
    """bnn_adam_clamp_multi (LatentAdam's one launch for the small parameters): p, m, v bit-identical
    to one bnn_adam_clamp per tensor, for 19 tensors (two launches), mixed sizes (incl. empty),
    clamp flags and step counts."""
    torch.manual_seed(3)
    sizes = [10, 8192, 1, 0, 3072, 257, 65536, 10, 5, 40000, 1536, 768, 100, 2, 7, 31, 512, 9, 4096]
    single, multi = [], []
    for i, n in enumerate(sizes):
        p = torch.empty(n, device="cuda").uniform_(-1.3, 1.3)
        m, v = torch.randn(n, device="cuda") * 1e-3, torch.rand(n, device="cuda") * 1e-6
        g = torch.randn(n, device="cuda")
        single.append([p.clone(), g, m.clone(), v.clone(), 3 + i % 4, i % 3 != 0])
        multi.append([p.clone(), g, m.clone(), v.clone(), 3 + i % 4, i % 3 != 0])
    for p, g, m, v, st, cl in single:
        F.adam_clamp_(p, g, m, v, st, lr=0.01, clamp=cl)
    F.adam_clamp_multi_([tuple(t) for t in multi], 0.01)
    for a, b in zip(single, multi):
        for x, y in zip(a[:4], b[:4]):
            assert torch.equal(x, y)


def test_large_forward_exact_vs_rocblas(F):
    """Size-independent property at wide-MLP scale: ternary products are integers < 2^24, so an
    fp32 GEMM in any order is exact; libbnn must equal it bit-for-bit (plus the same bias add)."""
    torch.manual_seed(1)
    x = torch.randn(2048, 8192, device="cuda")
    x[x.abs() < 0.01] = 0
    w = torch.empty(8192, 8192, device="cuda").uniform_(-1, 1)
    b = torch.randn(8192, device="cuda")
    y = F.binary_linear(x, w, b, True)
    ref = (torch.sign(x) @ torch.sign(w).t()) + b
    assert torch.equal(y, ref)


@pytest.mark.parametrize("M,C", [(7, 12), (300, 64), (1000, 1536)])
@pytest.mark.parametrize("hardtanh", [True, False])
def test_batchnorm_hardtanh_vs_oracle(F, M, C, hardtanh):
    """Fused BatchNorm1d(+Hardtanh) (mnist-dist2.py:52-74) against the float64 oracle and torch."""
    rng = np.random.default_rng(M + C)
    x = (rng.integers(-40, 40, (M, C)) + rng.standard_normal(C) * 3).astype(np.float32)
    gamma = rng.uniform(0.5, 1.5, C).astype(np.float32)
    beta = rng.uniform(-0.2, 0.2, C).astype(np.float32)
    g = rng.standard_normal((M, C)).astype(np.float32)
    bn = torch.nn.BatchNorm1d(C).cuda()
    with torch.no_grad():
        bn.weight.copy_(dev(gamma))
        bn.bias.copy_(dev(beta))
    xt = dev(x).requires_grad_(True)
    y = F.batch_norm_hardtanh(xt, bn, hardtanh)
    y.backward(dev(g))
    yr, cache, rm, rv = O.batchnorm_train(x, gamma, beta, np.zeros(C), np.ones(C))
    yo = O.hardtanh(yr) if hardtanh else yr
    assert rel_err(host(y), yo) < 1e-6
    np.testing.assert_allclose(host(bn.running_mean), rm, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(host(bn.running_var), rv, rtol=1e-5, atol=1e-6)
    assert int(bn.num_batches_tracked) == 1
    gm = O.hardtanh_backward(yr, g) if hardtanh else g
    dx, dgam, dbet = O.batchnorm_backward(cache, gm)
    assert rel_err(host(xt.grad), dx) < GRAD_TOL
    assert rel_err(host(bn.weight.grad), dgam) < GRAD_TOL
    assert rel_err(host(bn.bias.grad), dbet) < GRAD_TOL
    # eval mode uses the running statistics
    bn.eval()
    ye = F.batch_norm_hardtanh(dev(x), bn, hardtanh)
    ref = torch.nn.functional.batch_norm(dev(x), bn.running_mean, bn.running_var, bn.weight, bn.bias, False,
                                         0.0, bn.eps)
    if hardtanh:
        ref = ref.clamp(-1, 1)
    assert rel_err(host(ye), host(ref)) < 1e-6


@pytest.mark.parametrize("N,C,H,W", [(5, 16, 28, 28), (64, 32, 14, 14), (3, 8, 6, 10)])
@pytest.mark.parametrize("pool", [2, 0])
def test_batchnorm2d_hardtanh_pool_vs_oracle(F, N, C, H, W, pool):
    """Fused BatchNorm2d -> Hardtanh -> MaxPool2d(2) (the BinCNN block) against the float64 oracle
    (tie-free input so the argmax is unambiguous) and torch's modules in eval mode."""
    rng = np.random.default_rng(N * C + H + pool)
    x = (rng.standard_normal((N, C, H, W)) * 2 + rng.standard_normal((1, C, 1, 1))).astype(np.float32)
    gamma = rng.uniform(0.5, 1.5, C).astype(np.float32)
    beta = rng.uniform(-0.2, 0.2, C).astype(np.float32)
    bn = torch.nn.BatchNorm2d(C).cuda()
    with torch.no_grad():
        bn.weight.copy_(dev(gamma))
        bn.bias.copy_(dev(beta))
    xt = dev(x).requires_grad_(True)
    y = F.batch_norm2d_hardtanh_pool(xt, bn, True, pool)
    yr, cache, rm, rv = O.batchnorm2d_train(x, gamma, beta, np.zeros(C), np.ones(C))
    h = O.hardtanh(yr)
    if pool:
        yo, arg = O.maxpool2_forward(h)
    else:
        yo = h
    assert y.shape == yo.shape
    assert rel_err(host(y), yo) < 1e-6
    np.testing.assert_allclose(host(bn.running_mean), rm, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(host(bn.running_var), rv, rtol=1e-5, atol=1e-6)
    g = rng.standard_normal(yo.shape).astype(np.float32)
    y.backward(dev(g))
    gf = O.maxpool2_backward(g, arg, x.shape) if pool else g
    dx, dgam, dbet = O.batchnorm2d_backward(cache, O.hardtanh_backward(yr, gf))
    assert rel_err(host(xt.grad), dx) < GRAD_TOL
    assert rel_err(host(bn.weight.grad), dgam) < GRAD_TOL
    assert rel_err(host(bn.bias.grad), dbet) < GRAD_TOL
    bn.eval()
    ye = F.batch_norm2d_hardtanh_pool(dev(x), bn, True, pool)
    ref = torch.nn.functional.hardtanh(bn(dev(x)))
    if pool:
        ref = torch.nn.functional.max_pool2d(ref, 2, 2)
    assert rel_err(host(ye), host(ref)) < 1e-6


@pytest.mark.parametrize("batch", [512, 37])
def test_bn2d_row_kernels_match_window_kernels(F, batch):
    """The row forms of the pooled BatchNorm2d passes (bnn_bn2d_set_rows) in a fused BinCNN step on
    compact conv outputs, against the window-per-thread kernels: forward output and loss
    bit-identical (same statistics, same per-window arithmetic), every gradient within 1e-6 (the
    backward statistics are summed per row instead of per window group).  Batch 37: 37 x 16 x 14
    row pairs leave a ragged last workgroup in the LDS-staged row kernels (Rows16)."""
    from bnn_amd import _lib as L
    from bnn_amd import nets
    from bnn_amd.data import synthetic_mnist
    x, y = synthetic_mnist(batch, seed=3)
    x, y = x.cuda(), y.cuda()
    res = []
    try:
        for on in (1, 0):
            L.call("bnn_bn2d_set_rows", on)
            torch.manual_seed(11)
            m = nets.BinCNN(org_protocol=False, mutate_input=False, fused_bn=True).cuda()
            out = m(x)
            loss = torch.nn.functional.nll_loss(out, y)
            loss.backward()
            res.append((host(out), float(loss), {k: host(p.grad) for k, p in m.named_parameters()}))
    finally:
        L.call("bnn_bn2d_set_rows", 1)
    (o1, l1, g1), (o0, l0, g0) = res
    assert np.array_equal(o1, o0) and l1 == l0
    for k in g0:
        # a conv bias ahead of a BatchNorm has an analytically zero gradient (~1e-8 of summation
        # noise here): compared absolutely
        assert rel_err(g1[k], g0[k]) <= 1e-6 or np.abs(g1[k] - g0[k]).max() <= 1e-7, k


def test_conv1_bn2d_handoff_matches_unfused(F):
    """The BinCNN's conv1 weight gradient formed straight from its BatchNorm2d + Hardtanh + MaxPool2d
    backward (functional.C1BN: bnn_bn2d_bwd_stats_q + bnn_conv2d_bwd_filter_bn, the layer's fp32 dY
    never written) against the unfused path (bnn_bn2d_bwd_q's dx into bnn_conv2d_bwd_filter): the
    hand-off fires once per step; loss, layer 2 and the classifier bit-identical; layer 1's BatchNorm
    gradients identical (same statistics pass); conv1's weight gradient within 1e-6 (another
    summation order), its bias gradient (analytically zero ahead of a BatchNorm) within 1e-7."""
    from bnn_amd import nets
    from bnn_amd.data import synthetic_mnist
    x, y = synthetic_mnist(1024, seed=5)
    res = []
    for on in (True, False):
        F.C1BN = on
        try:
            torch.manual_seed(17)
            m = nets.BinCNN(org_protocol=False, mutate_input=False, fused_bn=True).cuda()
            n0 = F.C1BN_HANDOFFS
            loss = torch.nn.functional.nll_loss(m(x.cuda()), y.cuda())
            loss.backward()
            res.append((float(loss), {k: host(p.grad) for k, p in m.named_parameters()}, F.C1BN_HANDOFFS - n0))
        finally:
            F.C1BN = True
    (l1, g1, h1), (l0, g0, h0) = res
    assert h1 == 1 and h0 == 0
    assert l1 == l0
    for k in g0:
        if k == "layer1.0.weight":
            assert rel_err(g1[k], g0[k]) <= 1e-6, k
        elif k == "layer1.0.bias":
            assert np.abs(g1[k] - g0[k]).max() <= 1e-7, k
        else:
            assert np.array_equal(g1[k], g0[k]), k


def test_conv1_filter_switch_between_forward_and_backward(F):
    """The conv1 / BatchNorm2d hand-off is decided in the forward.  Switching the one-channel filter
    kernel off after it (bnn_conv_set_c1_filter(0) between forward and backward) falls back to the
    BatchNorm2d dx + the regular filter kernel instead of failing, and the BNN_CONV_C1F=0 knob is
    applied before the first conv forward (so that forward does not opt into the hand-off): both
    steps equal the default one (conv1's weight gradient -- then from the bf16x3 MFMA filter kernel
    instead of the VALU one -- within the 1e-5 gradient bar, its bias within 1e-7, the rest
    bit-identical)."""
    from bnn_amd import _lib as L
    from bnn_amd import nets
    from bnn_amd.data import synthetic_mnist
    x, y = synthetic_mnist(512, seed=6)
    x, y = x.cuda(), y.cuda()

    def step(mode):
        torch.manual_seed(21)
        m = nets.BinCNN(org_protocol=False, mutate_input=False, fused_bn=True).cuda()
        n0 = F.C1BN_HANDOFFS
        if mode == "env":
            F._CONV_C1F[0] = "0"
        loss = torch.nn.functional.nll_loss(m(x), y)
        if mode == "switch":
            L.call("bnn_conv_set_c1_filter", 0)
        loss.backward()
        return float(loss), {k: host(p.grad) for k, p in m.named_parameters()}, F.C1BN_HANDOFFS - n0

    try:
        ref = step("default")
        sw = step("switch")
        L.call("bnn_conv_set_c1_filter", 1)
        env = step("env")
    finally:
        F._CONV_C1F[0] = None
        L.call("bnn_conv_set_c1_filter", 1)
    assert ref[2] == 1 and sw[2] == 0 and env[2] == 0, (ref[2], sw[2], env[2])
    for l, g, _ in (sw, env):
        assert l == ref[0]
        for k in g:
            if k == "layer1.0.weight":
                assert rel_err(g[k], ref[1][k]) <= 1e-5, k
            elif k == "layer1.0.bias":
                assert np.abs(g[k] - ref[1][k]).max() <= 1e-7, k
            else:
                assert np.array_equal(g[k], ref[1][k]), k


def test_fused_cnn_step_matches_torch_modules(F):
    """BinCNN with the fused BatchNorm2d+Hardtanh+MaxPool2d op against the same net through torch's
    BatchNorm2d / Hardtanh / MaxPool2d modules (integer-valued conv outputs: pooling ties resolved
    by the same first-max rule), one forward + backward."""
    from bnn_amd import nets
    from bnn_amd.data import synthetic_mnist
    torch.manual_seed(5)
    a = nets.BinCNN(org_protocol=False, mutate_input=False).cuda()
    b = nets.BinCNN(org_protocol=False, mutate_input=False, fused_bn=True).cuda()
    b.load_state_dict(a.state_dict())
    x, y = synthetic_mnist(96, seed=7, device="cuda")
    la = torch.nn.functional.cross_entropy(a(x), y)
    la.backward()
    lb = torch.nn.functional.cross_entropy(b(x), y)
    lb.backward()
    assert abs(la.item() - lb.item()) < 1e-5
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        # a conv bias feeding BatchNorm has an exactly-zero true gradient (both sides are ~1e-8
        # rounding noise), so it is compared absolutely
        assert rel_err(host(pb.grad), host(pa.grad)) < 1e-4 or close(host(pb.grad), host(pa.grad), 0.0, 1e-6), n
    for (n, ba), bb in zip(a.named_buffers(), b.buffers()):
        assert close(host(ba), host(bb), 1e-5, 1e-6), n


@pytest.mark.parametrize("shape", [(37, 1, 28, 28, 16, 5, 2), (19, 16, 14, 14, 32, 5, 2), (5, 32, 8, 8, 24, 3, 1)])
def test_conv_fwd_compact_sums(F, shape):
    """bnn_conv2d_fwd_q writes the exact binary-conv sums as int8 (C*KH*KW <= 127) / int16: adding
    the bias in fp32 reproduces bnn_conv2d_fwd's fp32 output bit for bit (the BinCNN's conv1 / conv2
    and a 3x3 shape)."""
    from bnn_amd import _lib as L
    N, C, H, W, Co, K, pad = shape
    g = torch.Generator(device="cuda").manual_seed(N * C)
    x = torch.randn(N, C, H, W, generator=g, device="cuda")
    x[0, 0, 3, :5] = 0.0                                  # exact zeros: sign 0
    w = torch.randn(Co, C, K, K, generator=g, device="cuda")
    b = torch.randn(Co, generator=g, device="cuda")
    y = torch.empty(N, Co, H + 2 * pad - K + 1, W + 2 * pad - K + 1, device="cuda")
    L.call("bnn_conv2d_fwd", L.ptr(x), 1, L.ptr(w), L.ptr(b), L.ptr(y), N, C, H, W, Co, K, K, 1, pad, 1, 1, L.stream())
    fmt = 1 if C * K * K <= 127 else 2
    yq = torch.empty(y.shape, dtype=torch.int8 if fmt == 1 else torch.int16, device="cuda")
    L.call("bnn_conv2d_fwd_q", L.ptr(x), L.ptr(w), L.ptr(yq), fmt, N, C, H, W, Co, K, K, 1, pad, 1, 1, L.stream())
    assert torch.equal(yq.float() + b.view(1, -1, 1, 1), y)


def test_fused_cnn_compact_outputs_bit_identical(F):
    """The fused BinCNN with its conv outputs travelling as int16 sums + bias
    (functional.ZQ) against the same net with fp32 conv outputs: loss, every gradient and the
    BatchNorm running buffers bit-identical, two hand-offs per forward."""
    from bnn_amd import nets
    from bnn_amd.data import synthetic_mnist
    torch.manual_seed(6)
    a = nets.BinCNN(org_protocol=False, mutate_input=False, fused_bn=True).cuda()
    b = nets.BinCNN(org_protocol=False, mutate_input=False, fused_bn=True).cuda()
    b.load_state_dict(a.state_dict())
    x, y = synthetic_mnist(200, seed=9, device="cuda")
    try:
        F.C1BN = False            # conv1's BatchNorm hand-off sums in another order (its own test)
        F.ZQ = False
        la = torch.nn.functional.cross_entropy(a(x), y)
        la.backward()
        F.ZQ = True
        n0 = F.ZQ_HANDOFFS
        lb = torch.nn.functional.cross_entropy(b(x), y)
        lb.backward()
        assert F.ZQ_HANDOFFS - n0 == 2
    finally:
        F.ZQ = True
        F.C1BN = True
    assert la.item() == lb.item()
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        assert torch.equal(pa.grad, pb.grad), n
    for (n, ba), bb in zip(a.named_buffers(), b.buffers()):
        assert torch.equal(ba, bb), n


def test_compact_conv_falls_back_when_refused(F):
    """emit_compact only when bnn_conv2d_fwd_q takes the shape (bnn_conv2d_fwd_q_ok, the kernel
    choice itself): with the MFMA conv kernels switched off (bnn_conv_set_mfma(0)) and for a
    C = 16 layer whose 20x20 output exceeds the MFMA forward's 256-pixel tile, the fused BinCNN
    block takes the fp32 conv output instead of raising, with the same loss."""
    from bnn_amd import _lib as L
    from bnn_amd import nets
    from bnn_amd.data import synthetic_mnist
    assert L.lib().bnn_conv2d_fwd_q_ok(2, 8, 16, 14, 14, 32, 5, 5, 1, 2, 1, 1) == 1
    assert L.lib().bnn_conv2d_fwd_q_ok(2, 8, 16, 20, 20, 32, 5, 5, 1, 2, 1, 1) == 0
    torch.manual_seed(6)
    a = nets.BinCNN(org_protocol=False, mutate_input=False, fused_bn=True).cuda()
    x, y = synthetic_mnist(64, seed=9, device="cuda")
    la = torch.nn.functional.cross_entropy(a(x), y).item()
    try:
        L.call("bnn_conv_set_mfma", 0)
        assert L.lib().bnn_conv2d_fwd_q_ok(2, 8, 16, 14, 14, 32, 5, 5, 1, 2, 1, 1) == 0
        n0 = F.ZQ_HANDOFFS
        lb = torch.nn.functional.cross_entropy(a(x), y).item()
        assert F.ZQ_HANDOFFS == n0
    finally:
        L.call("bnn_conv_set_mfma", 1)
    assert abs(la - lb) <= 1e-6 * max(1.0, abs(la))
    # a C = 16 input whose 20x20 output the compact kernels refuse: the fp32 path, no error
    conv = nets.BinarizeConv2d(16, 32, 5, padding=2).cuda()
    conv.org_protocol = False
    xb = torch.randn(4, 16, 20, 20, device="cuda")
    n0 = F.ZQ_HANDOFFS
    out = conv(xb, emit_compact=True)
    assert F.ZQ_HANDOFFS == n0 and out.stride() != (0, 0, 0, 0)
    ref = F.binary_conv2d(xb, conv.weight, conv.bias, True, 1, 2, 1, 1)
    assert torch.equal(out, ref)


def test_fused_mlp_step_matches_unfused(F):
    """The build's trainer path (fused BN+Hardtanh, latent Adam) against the drop-in path
    (torch BatchNorm1d/Hardtanh, torch Adam + .org protocol) on one step, dropout off."""
    from bnn_amd import nets
    from bnn_amd.data import synthetic_mnist
    from bnn_amd.optim import LatentAdam, org_protocol_step
    torch.manual_seed(3)
    a = nets.MLP(256, 128, 64, p_drop=0.0).cuda()
    b = nets.MLP(256, 128, 64, p_drop=0.0, org_protocol=False, mutate_input=False, fused_bn=True).cuda()
    b.load_state_dict(a.state_dict())
    x, y = synthetic_mnist(128, seed=11, device="cuda")
    oa = torch.optim.Adam(a.parameters(), lr=0.01)
    ob = LatentAdam(b.parameters(), lr=0.01, clamp_params=nets.binary_params(b))
    la = torch.nn.functional.cross_entropy(a(x), y)
    la.backward()
    lb = torch.nn.functional.cross_entropy(b(x), y)
    lb.backward()
    assert abs(la.item() - lb.item()) < 1e-5
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        assert close(host(pa.grad), host(pb.grad), 1e-4, 1e-6), n
    org_protocol_step(a, oa)
    ob.step()
    for k in ("fc1", "fc2", "fc3"):
        wa = getattr(a, k).weight.org
        wb = getattr(b, k).weight
        assert close(host(wa), host(wb), 1e-4, 0.0), k


@pytest.mark.parametrize("cfg", [(1, 1), (3, 1), (3, 3)])
@pytest.mark.parametrize("M,N,K", [(300, 200, 256), (257, 520, 384), (64, 64, 64), (1000, 129, 1024)])
def test_every_gemm_variant_is_exact(F, cfg, M, N, K):
    """Every kernel in the bnn_gemm_i8 variant table (tools/gemm_sweep.py) against an exact int64
    reference, including K not a multiple of 128 and ragged M, N."""
    from bnn_amd import _lib
    da, db = cfg
    rng = np.random.default_rng(M + N + K + da + db)
    A = rng.integers(-128, 128, (da, M, K)).astype(np.int8)
    B = (rng.integers(-1, 2, (db, N, K)) if db == 1 else rng.integers(-128, 128, (db, N, K))).astype(np.int8)
    if da == 3:
        A[2] //= 2
    if db == 3:
        B[2] //= 2
    bias = rng.standard_normal(N).astype(np.float32)
    sa = np.exp2(rng.integers(-30, -10, M)).astype(np.float32) if da == 3 else None
    sb = np.exp2(rng.integers(-30, -10, N)).astype(np.float32) if db == 3 else None
    w = [1 << (8 * d) for d in range(3)]
    acc = np.zeros((M, N), np.float64)
    for i in range(da):
        for j in range(db):
            if da == 3 and db == 3 and i + j < 2:
                continue                      # pairs the kernel drops (weight <= 2^-24 of the top)
            acc += (w[i] if da == 3 else 1) * (w[j] if db == 3 else 1) * (
                A[i].astype(np.int64) @ B[j].astype(np.int64).T).astype(np.float64)
    if sa is not None:
        acc *= sa[:, None]
    if sb is not None:
        acc *= sb[None, :]
    ref = acc.astype(np.float32) + bias
    At = dev(A if da == 3 else A[0])
    Bt = dev(B if db == 3 else B[0])
    names = set()
    try:
        for v in range(0, 10):
            _lib.call("bnn_gemm_set_variant", v)
            name = F.gemm_kernel_name(da, db, M, N, K)
            if name in names:
                continue
            names.add(name)
            C = host(F.gemm_i8(At, da, Bt, db, M, N, a_scale=dev(sa) if sa is not None else None,
                               b_scale=dev(sb) if sb is not None else None, bias=dev(bias)))
            if cfg == (1, 1):
                assert np.array_equal(C, ref), name
            else:
                assert rel_err(C, ref) < 1e-6, name
    finally:
        _lib.call("bnn_gemm_set_variant", -1)


@pytest.mark.parametrize("backend", ["fp4", "mfma", "xnor"])
def test_empty_and_single_sample_batches(F, backend):
    """Edge batches through the drop-in path: an empty batch returns an empty output (as torch's
    F.linear / F.conv2d do) with empty gradients, and a batch of one is exact."""
    from models.binarized_modules import BinarizeConv2d, BinarizeLinear
    torch.manual_seed(9)
    lin = BinarizeLinear(256, 96).cuda()
    lin.backend = backend
    for m in (0, 1):
        x = torch.randn(m, 256, device="cuda", requires_grad=True)
        xr = x.detach().clone()
        y = lin(x)
        assert y.shape == (m, 96)
        y.sum().backward()
        assert x.grad.shape == (m, 256)
        if m:
            ref = torch.sign(xr) @ torch.sign(lin.weight.org).t() + lin.bias.detach()
            assert torch.equal(y.detach(), ref)
    conv = BinarizeConv2d(16, 32, kernel_size=5, padding=2).cuda()
    for n in (0, 1):
        x = torch.randn(n, 16, 14, 14, device="cuda", requires_grad=True)
        xr = x.detach().clone()
        y = conv(x)
        assert y.shape == (n, 32, 14, 14)
        y.sum().backward()
        assert x.grad.shape == (n, 16, 14, 14)
        if n:
            ref = torch.nn.functional.conv2d(torch.sign(xr).double().cpu(), torch.sign(conv.weight.org).double().cpu(),
                                             None, padding=2) + conv.bias.detach().double().cpu().view(1, -1, 1, 1)
            assert torch.equal(y.detach().cpu(), ref.float())   # integer sum, then one fp32 bias add


@pytest.mark.parametrize("M,C,p", [(1000, 768, 0.3), (64, 12, 0.5)])
def test_dropout_batchnorm_hardtanh_vs_explicit_mask(F, M, C, p):
    """Fused Dropout -> BatchNorm1d -> Hardtanh (mnist-dist2.py:69-74) against torch's BatchNorm1d +
    Hardtanh applied to x * mask, with the mask the fused passes regenerate (bnn_dropout_mask):
    outputs, running stats and all gradients, and the keep fraction ~ 1 - p."""
    torch.manual_seed(M + C)
    x = (torch.randn(M, C, device="cuda") * 3 + torch.randn(C, device="cuda")).requires_grad_(True)
    bn_a = torch.nn.BatchNorm1d(C).cuda()
    with torch.no_grad():
        bn_a.weight.uniform_(0.5, 1.5)
        bn_a.bias.uniform_(-0.2, 0.2)
    bn_b = torch.nn.BatchNorm1d(C).cuda()
    bn_b.load_state_dict(bn_a.state_dict())
    seed = 123456789 + M
    y = F.dropout_batch_norm_hardtanh(x, p, bn_a, seed=seed)
    g = torch.randn_like(y)
    y.backward(g)
    mask = F.dropout_mask(M * C, p, seed).view(M, C)
    keep = (mask > 0).float().mean().item()
    assert abs(keep - (1 - p)) < 0.02 + 3 / (M * C) ** 0.5
    assert torch.all((mask == 0) | (mask == torch.tensor(1.0 / (1.0 - p), device="cuda")))
    xr = x.detach().clone().requires_grad_(True)
    yr = torch.nn.functional.hardtanh(bn_b(xr * mask))
    yr.backward(g)
    assert rel_err(host(y), host(yr)) < 1e-5
    assert rel_err(host(x.grad), host(xr.grad)) < GRAD_TOL
    assert rel_err(host(bn_a.weight.grad), host(bn_b.weight.grad)) < GRAD_TOL
    assert rel_err(host(bn_a.bias.grad), host(bn_b.bias.grad)) < GRAD_TOL
    assert close(host(bn_a.running_mean), host(bn_b.running_mean), 1e-5, 1e-6)
    assert close(host(bn_a.running_var), host(bn_b.running_var), 1e-5, 1e-6)


def test_dropout_mask_statistics(F):
    """The fused passes' keep mask (bnn_dropout_mask regenerates it): keep fraction within 5 sigma
    of 1 - p on 2^24 elements, and no correlation (|r| < 5/sqrt(n)) between neighbouring elements,
    elements one wide-MLP row apart, or the masks of consecutive seeds / device-step seeds."""
    n, p = 1 << 24, 0.3
    seed = 987654321
    a = (F.dropout_mask(n, p, seed) > 0).double()
    keep = a.mean().item()
    assert abs(keep - (1 - p)) < 5 * (p * (1 - p) / n) ** 0.5

    def corr(u, v):
        u = u - u.mean()
        v = v - v.mean()
        return (u * v).mean().item() / (u.std().item() * v.std().item())

    lim = 5 / n ** 0.5
    assert abs(corr(a[:-1], a[1:])) < lim
    assert abs(corr(a[:-8192], a[8192:])) < lim
    for s2 in (seed + 1, seed + 0xD1B54A32D192ED03 % (1 << 64), seed ^ (1 << 40)):
        b = (F.dropout_mask(n, p, s2 % (1 << 64)) > 0).double()
        assert abs(corr(a, b)) < lim, s2

"""The binarised-input conv forward's popcount engine (csrc/bnn_conv_popc.hip, bnn_conv_set_popc)
against the int8-MFMA / dot4 engine and against F.conv2d(sign(x), sign(w)) + bias on the CPU
(binarized_modules.py:93-105): exact integer sums, so every comparison is bit for bit -- the fp32
output of bnn_conv2d_fwd, the int8 / int16 sums of bnn_conv2d_fwd_q, and a fused BinCNN step
(loss, every gradient, the BatchNorm buffers) with either engine."""
import pytest
import torch

pytestmark = pytest.mark.gpu

# (N, C, H, W, Co, K, pad): the BinCNN's conv1 / conv2, ragged batches, 3x3 / 7x7 / 1x1, a 20 x 30
# single-channel image (padded width 32), pad < (K - 1) / 2 and pad = K - 1
SHAPES = [
    (256, 1, 28, 28, 16, 5, 2), (37, 1, 28, 28, 16, 5, 2), (9, 1, 20, 30, 8, 3, 1), (5, 1, 12, 12, 24, 5, 4),
    (256, 16, 14, 14, 32, 5, 2), (33, 16, 14, 14, 32, 5, 2), (17, 16, 9, 11, 24, 3, 0), (8, 16, 7, 7, 16, 7, 3),
    (5, 16, 6, 6, 10, 1, 0), (3, 16, 14, 14, 64, 5, 1),
]


def _inputs(shape, seed):
    N, C, H, W, Co, K, pad = shape
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.randn(N, C, H, W, generator=g, device="cuda")
    x = torch.where(torch.rand(x.shape, generator=g, device="cuda") < 0.3, torch.zeros_like(x), x)   # sign 0
    x[0, 0, 0, :3] = -0.0                                                                         # sign(-0) = 0
    w = torch.randn(Co, C, K, K, generator=g, device="cuda")
    w[0, 0, 0, 0] = 0.0
    b = torch.randn(Co, generator=g, device="cuda")
    return x, w, b


def _fwd(x, w, b, shape, popc):
    from bnn_amd import _lib as L
    N, C, H, W, Co, K, pad = shape
    y = torch.empty(N, Co, H + 2 * pad - K + 1, W + 2 * pad - K + 1, device="cuda")
    prev = L.lib().bnn_conv_set_popc(-1)
    L.call("bnn_conv_set_popc", int(popc))
    try:
        L.call("bnn_conv2d_fwd", L.ptr(x), 1, L.ptr(w), L.ptr(b), L.ptr(y), N, C, H, W, Co, K, K, 1, pad, 1, 1,
               L.stream())
        out = {0: y}
        for fmt in (1, 2):
            if fmt == 1 and C * K * K > 127:
                continue
            if not L.lib().bnn_conv2d_fwd_q_ok(fmt, N, C, H, W, Co, K, K, 1, pad, 1, 1):
                continue
            yq = torch.empty(y.shape, dtype=torch.int8 if fmt == 1 else torch.int16, device="cuda")
            L.call("bnn_conv2d_fwd_q", L.ptr(x), L.ptr(w), L.ptr(yq), fmt, N, C, H, W, Co, K, K, 1, pad, 1, 1,
                   L.stream())
            out[fmt] = yq
        torch.cuda.synchronize()
    finally:
        L.call("bnn_conv_set_popc", prev)
    return out


@pytest.mark.parametrize("shape", SHAPES)
def test_popc_conv_forward_bit_identical(shape):
    from bnn_amd import _lib as L
    N, C, H, W, Co, K, pad = shape
    x, w, b = _inputs(shape, N * 131 + C * 7 + K)
    a = _fwd(x, w, b, shape, popc=False)
    p = _fwd(x, w, b, shape, popc=True)
    # exact sums on the CPU (float64: every partial sum an integer far below 2^53)
    ref_i = torch.nn.functional.conv2d(torch.sign(x).double().cpu(), torch.sign(w).double().cpu(), padding=pad)
    ref = (ref_i.float() + b.cpu().view(1, -1, 1, 1))
    assert torch.equal(p[0].cpu(), ref)
    assert torch.equal(a[0].cpu(), ref)
    for fmt, yq in p.items():
        if fmt:
            assert torch.equal(yq.cpu().long(), ref_i.long()), fmt
            if fmt in a:
                assert torch.equal(yq, a[fmt]), fmt
    if C == 16 or (C == 1 and K <= 5):
        assert 2 in p                 # the popcount engine takes every compact shape listed


def test_popc_conv_refuses_other_geometry():
    """Shapes outside the popcount kernels (C = 3, stride 2, even K, a wide single-channel image) stay
    on the other engine with the switch on, with the same results."""
    from bnn_amd import _lib as L
    for shape in [(4, 3, 16, 16, 8, 3, 1), (4, 1, 40, 40, 8, 5, 2), (4, 32, 8, 8, 16, 3, 1)]:
        x, w, b = _inputs(shape, 7)
        a = _fwd(x, w, b, shape, popc=False)
        p = _fwd(x, w, b, shape, popc=True)
        assert torch.equal(a[0], p[0]), shape
    assert L.lib().bnn_conv_set_popc(-1) in (0, 1)


def test_popc_fused_bincnn_step_bit_identical():
    """A fused BinCNN training step (compact conv outputs, conv1 / BatchNorm2d hand-off) with the
    popcount engine against the MFMA / dot4 engine: loss, gradients and buffers bit-identical."""
    from bnn_amd import _lib as L
    from bnn_amd import nets
    from bnn_amd.data import synthetic_mnist
    torch.manual_seed(3)
    a = nets.BinCNN(org_protocol=False, mutate_input=False, fused_bn=True).cuda()
    b = nets.BinCNN(org_protocol=False, mutate_input=False, fused_bn=True).cuda()
    b.load_state_dict(a.state_dict())
    x, y = synthetic_mnist(512, seed=4, device="cuda")
    prev = L.lib().bnn_conv_set_popc(-1)
    L.call("bnn_conv_set_popc", 0)
    try:
        la = torch.nn.functional.cross_entropy(a(x), y)
        la.backward()
    finally:
        L.call("bnn_conv_set_popc", prev)
    L.call("bnn_conv_set_popc", 1)
    try:
        lb = torch.nn.functional.cross_entropy(b(x), y)
        lb.backward()
        torch.cuda.synchronize()
    finally:
        L.call("bnn_conv_set_popc", prev)
    assert la.item() == lb.item()
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        assert torch.equal(pa.grad, pb.grad), n
    for (n, ba), bb in zip(a.named_buffers(), b.buffers()):
        assert torch.equal(ba, bb), n

"""GPU parity of fc1's compact output (s20, functional.S20): the u8-pixel BinarizeLinear's
z1 = F.linear(x, W_b) + bias (binarized_modules.py:80-83, input kept at size(1) == 784, x = u/255)
carried as the exact integer sums S = sum_k u_k sign(w_k) in 20 bits (an int16 plane + a nibble
plane) into the fused bn1 -> fc2 op that consumes it (mnist-dist2.py:64-66).

Every *_s20 entry reads z = fl(fl(S * a) + b), the value the fp32 GEMM epilogue stores, so each
result must be BIT-IDENTICAL to the fp32 entry on the fp32 z1: the decoded z1 and the epilogue
statistics, the FP4 rows / transpose of the apply-pack, the int8-column-digit BatchNorm backward
(digits, scale, digit sums, bias / BatchNorm gradients), and a whole training step with and
without the hand-off.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def F():
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    from bnn_amd import functional
    return functional


def eq(a, b):
    torch.cuda.synchronize()
    return torch.equal(a, b)


def _fc1(F, M, N, seed, with_bias=True, extreme=None):
    """(fp32 z1 with its statistics, the s20 placeholder with its statistics) of one pixel layer."""
    g = torch.Generator(device="cuda").manual_seed(seed)
    K = 784
    if extreme is None:
        u = torch.randint(0, 256, (M, K), generator=g, device="cuda").to(torch.uint8)
        w = torch.randn(N, K, generator=g, device="cuda")
    else:   # |S| at its bound: every pixel 255, every weight +1 (or -1)
        u = torch.full((M, K), 255, dtype=torch.uint8, device="cuda")
        w = torch.full((N, K), float(extreme), device="cuda")
    b = (torch.rand(N, generator=g, device="cuda") - 0.5) if with_bias else None
    a, s0 = F.pixel_affine(None)
    q, _ = F.pixels_pack(u, want_q=True, want_qt=False)
    wq, _ = F.packed_weight(w, "i8", True, False, cache=False)
    R = F.row_sums(wq, K)
    assert F.L.lib().bnn_gemm_i8_s20_ok(M, N, q.shape[1], K, float(s0)) == 1
    z = F._pixels_fwd_with_stats(q, wq, M, N, K, F._const_vec(a, N, "cuda"), b, R, s0)
    zs = F._pixels_fwd_s20(q, wq, M, N, K, a, b, R, s0)
    return z, zs


def test_s20_ok_bounds(F):
    L = F.L.lib()
    assert L.bnn_gemm_i8_s20_ok(65536, 8192, 832, 784, 128.0) == 1
    assert L.bnn_gemm_i8_s20_ok(65536, 8192, 832, 784, 94.6715) == 0      # Normalize: s0 not integral
    assert L.bnn_gemm_i8_s20_ok(65536, 8190, 832, 784, 128.0) == 0        # N % 4
    assert L.bnn_gemm_i8_s20_ok(64, 256, 2048, 2047, 128.0) == 1          # 2047 * 256 < 2^19
    assert L.bnn_gemm_i8_s20_ok(64, 256, 2112, 2049, 128.0) == 0


@pytest.mark.parametrize("M,N,with_bias", [(300, 256, True), (8200, 8192, True), (1000, 512, False)])
def test_pixels_s20_decodes_to_the_fp32_z1(F, M, N, with_bias):
    z, zs = _fc1(F, M, N, M + N, with_bias)
    lo, hi, bias, scale = F._s20_of(zs)
    assert lo.dtype == torch.int16 and hi.dtype == torch.uint8 and hi.shape == (M, N // 2)
    assert eq(F.dense_preact(zs), z)
    fz, fs = getattr(z, F._FSTATS_ATTR), getattr(zs, F._FSTATS_ATTR)
    assert eq(fz[0], fs[0]) and fz[1:] == fs[1:]                 # identical epilogue statistics


@pytest.mark.parametrize("sign", [1.0, -1.0])
def test_pixels_s20_at_the_sum_bound(F, sign):
    z, zs = _fc1(F, 256, 256, 7, True, extreme=sign)
    assert eq(F.dense_preact(zs), z)
    lo, hi, _, _ = F._s20_of(zs)
    S = (lo.to(torch.int32) & 0xFFFF) | ((hi[:, :1].to(torch.int32) & 15) << 16)
    assert int(S[0, 0]) == (255 * 784 if sign > 0 else (1 << 20) - 255 * 784)


def _bn_stats(F, z, M, C):
    from bnn_amd import _lib as L
    mean, invstd, lo = F._bn_stat_buffers(C, "cuda")
    rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    gam = torch.linspace(0.5, 1.5, C, device="cuda")
    bet = torch.linspace(-0.2, 0.2, C, device="cuda")
    L.call("bnn_bn_fwd_train", L.ptr(z), M, C, L.ptr(gam), L.ptr(bet), L.ptr(rm), L.ptr(rv), 0.1, 1e-5,
           L.ptr(mean), L.ptr(invstd), L.ptr(lo), None, 1, L.ptr(F._bn_ws(M, C, "cuda")), L.stream())
    return mean, invstd, lo, gam, bet


@pytest.mark.parametrize("M,C,panel", [(300, 256, 0), (8200, 8192, 1), (1000, 512, 1)])
def test_apply_pack_s20_bit_identical(F, M, C, panel):
    from bnn_amd import _lib as L
    z, zs = _fc1(F, M, C, 3 * M + C)
    lo, hi, bias, scale = F._s20_of(zs)
    mean, invstd, mlo, gam, bet = _bn_stats(F, z, M, C)
    res = []
    for form in ("f32", "s20"):
        q = torch.full((M, C // 2), 0x55, dtype=torch.uint8, device="cuda")
        qt = (F._qt_buffer(C, M, "fp4p", "cuda") if panel else
              torch.full((C, F.round_up(M, 256) // 2), 0x55, dtype=torch.uint8, device="cuda"))
        if form == "f32":
            L.call("bnn_bn_apply_pack", L.ptr(z), M, C, L.ptr(mean), L.ptr(invstd), L.ptr(mlo), L.ptr(gam),
                   L.ptr(bet), 1, L.ptr(q), q.shape[1], L.ptr(qt), qt.shape[1], 2 if panel else 1, L.stream())
        else:
            L.call("bnn_bn_apply_pack_s20", L.ptr(lo), L.ptr(hi), L.ptr(bias), scale, M, C, L.ptr(mean),
                   L.ptr(invstd), L.ptr(mlo), L.ptr(gam), L.ptr(bet), L.ptr(q), q.shape[1], L.ptr(qt), qt.shape[1],
                   panel, L.stream())
        res.append((q, qt))
    assert eq(res[0][0], res[1][0]) and eq(res[0][1], res[1][1])


@pytest.mark.parametrize("M,C", [(300, 256), (8200, 8192)])
def test_bwd_i8cols_s20_bit_identical(F, M, C):
    z, zs = _fc1(F, M, C, 5 * M + C)
    lo, hi, bias, scale = F._s20_of(zs)
    mean, invstd, mlo, gam, bet = _bn_stats(F, z, M, C)
    dy = torch.randn(M, C, device="cuda", generator=torch.Generator(device="cuda").manual_seed(M)) * 1e-3
    res = []
    for form in ("f32", "s20"):
        dgw, dgb = torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
        dz = F._bn_bwd_i8c(z, dy, M, C, gam, bet, mean, invstd, mlo, dgw, dgb,
                           s20=(lo, hi, bias, scale) if form == "s20" else None)
        ent = getattr(dz, F._I8C_ATTR)
        res.append([dgw, dgb, *ent[1:]])
    for x, y in zip(*res):
        assert eq(x, y)


def test_mlp_step_with_s20_equals_fp32(F):
    """Two training steps (forward, loss, backward, fused Adam + re-pack) of a fused MLP on u8
    pixels with fc1's output as s20 equal the same steps with the hand-off off, bit for bit: loss,
    every parameter, Adam moment and BatchNorm buffer."""
    from bnn_amd import nets
    from bnn_amd.nets import binary_params
    from bnn_amd.optim import LatentAdam
    M, W = 16384, 2048            # >= Z16_MIN_TILES 256x256 tiles: the hand-off fires
    g = torch.Generator(device="cuda").manual_seed(5)
    u = torch.randint(0, 256, (M, 1, 28, 28), generator=g, device="cuda").to(torch.uint8)
    y = torch.randint(0, 10, (M,), generator=g, device="cuda")
    states = []
    for s20 in (True, False):
        F.S20 = s20
        try:
            torch.manual_seed(0)
            m = nets.MLP(W, W, W // 2, org_protocol=False, mutate_input=False, fused_bn=True).cuda().train()
            opt = LatentAdam(m.parameters(), lr=0.01, clamp_params=binary_params(m))
            losses = []
            n0 = F.S20_HANDOFFS
            for _ in range(2):
                for p in m.parameters():
                    p.grad = None
                torch.manual_seed(1)
                loss = torch.nn.CrossEntropyLoss()(m(u), y)
                loss.backward()
                opt.step()
                losses.append(float(loss.item()))
            assert F.S20_HANDOFFS - n0 == (2 if s20 else 0)
            st = {k: v.detach().clone() for k, v in m.state_dict().items()}
            for i, p in enumerate(m.parameters()):
                for k in ("exp_avg", "exp_avg_sq"):
                    st[f"opt{i}.{k}"] = opt.state[p][k].clone()
            states.append((losses, st))
            del m, opt
        finally:
            F.S20 = True
    (la, a), (lb, b) = states
    assert la == lb
    for k in a:
        assert torch.equal(a[k], b[k]), k


def test_compact_bias_is_guarded_not_copied(F):
    """The compact carriers hold the producing layer's bias itself (no per-step snapshot copy): an
    in-place update of it between forward and backward is refused by torch's saved-tensor check."""
    from bnn_amd import nets
    M, W = 16384, 2048
    g = torch.Generator(device="cuda").manual_seed(8)
    u = torch.randint(0, 256, (M, 1, 28, 28), generator=g, device="cuda").to(torch.uint8)
    y = torch.randint(0, 10, (M,), generator=g, device="cuda")
    m = nets.MLP(W, W, W, org_protocol=False, mutate_input=False, fused_bn=True).cuda().train()
    n0 = F.S20_HANDOFFS
    loss = torch.nn.CrossEntropyLoss()(m(u), y)
    assert F.S20_HANDOFFS - n0 == 1
    with torch.no_grad():
        m.fc1.bias.add_(1.0)
    with pytest.raises(RuntimeError, match="modified by an inplace operation"):
        loss.backward()


def test_compact_bias_guard_fires_after_latent_adam(F):
    """LatentAdam writes the parameters through raw pointers (bnn_adam_clamp_multi / _pack) and bumps
    their versions as a torch in-place op would: a backward of a forward taken before the update is
    refused instead of rebuilding z from the updated bias."""
    from bnn_amd import nets
    from bnn_amd.optim import LatentAdam
    M, W = 16384, 2048                     # the s20 carrier's grid (>= 512 tiles), as above
    g = torch.Generator(device="cuda").manual_seed(9)
    u = torch.randint(0, 256, (M, 1, 28, 28), generator=g, device="cuda").to(torch.uint8)
    y = torch.randint(0, 10, (M,), generator=g, device="cuda")
    m = nets.MLP(W, W, W, org_protocol=False, mutate_input=False, fused_bn=True).cuda().train()
    n0 = F.S20_HANDOFFS
    loss = torch.nn.CrossEntropyLoss()(m(u), y)
    assert F.S20_HANDOFFS - n0 == 1
    for p in m.parameters():
        p.grad = torch.zeros_like(p)
    v0 = m.fc1.bias._version
    LatentAdam(m.parameters(), lr=0.01, clamp_params=nets.binary_params(m)).step()
    assert m.fc1.bias._version > v0
    with pytest.raises(RuntimeError, match="modified by an inplace operation"):
        loss.backward()

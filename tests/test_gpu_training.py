"""GPU training parity: the reference's own 3-step training traces replayed through libbnn.

``tests/golden/trace_org.npz`` / ``trace_frozen.npz`` were produced by importing the reference
operator module and running the mnist-dist2.py:118-137 loop (org restore -> Adam -> clamp) and
the mnist-dist3.py:113-119 loop (no org protocol: binary weights frozen) on CPU, widths
48/32/24, batch 16, dropout p = 0, Adam lr 0.01 (tests/golden/make_golden.py:121-164).

Two GPU paths replay them:

(i)  the drop-in: ``models.binarized_modules`` layers in ``nets.MLP`` (its nn.BatchNorm1d /
     nn.Hardtanh modules executed by libbnn's BatchNorm+Hardtanh kernels), ``torch.optim.Adam``
     and ``optim.org_protocol_step`` -- the reference scripts' exact call pattern;
(ii) the build's fused trainer path (what bench.py times): ``org_protocol = False``,
     ``fused_bn = True`` (libbnn BatchNorm+Hardtanh, BN -> sign-pack -> FP4 GEMM), ``LatentAdam``
     (fused Adam + clamp + re-pack of the next forward's weight operands).

BatchNorm near-ties.  The hidden pre-activations are integers plus a per-column bias, so values
within an ulp of the batch mean are common (7-17 per step in these traces); the next layer's
sign() turns the last-ulp rounding of the mean into +-1 flips.  The reference (torch CPU,
double-accumulated BatchNorm statistics) resolves every one of them as exact arithmetic does --
checked against the fixtures' recorded binarized activations (``s*/act/fc2_in``,
``s*/act/fc3_in``) -- and so do libbnn's BatchNorm kernels (batch sum in double, mean kept as
an fp32 hi + lo pair, x - mean = (x - hi) - lo).  The replays therefore assert the binarized
activations EQUAL the reference's at every step.  torch's own GPU BatchNorm1d (float mean) does
not resolve them that way: ``test_trace_replay_dropin_torch_batchnorm`` states a looser band.

Tolerances:
* loss per step: |loss - loss_ref| <= 1e-5 (absolute; losses are ~2.3);
* log-probs: norm-wise <= 1e-5 at step 0, 1e-4 after an optimizer step;
* gradients at step 0 (same initial weights, nothing chaotic yet): norm-wise <= 1e-5 against
  the reference's fp32 CPU gradients;
* after an update: norm-wise <= 1e-4.  Adam divides by sqrt(v) + eps, so parameters whose true
  gradient is tiny move by about +-lr whatever the sign of rounding noise: the BinarizeLinear
  biases feed BatchNorm, their exact gradient is 0 and both sides hold ~1e-8 rounding noise.
  Those biases (and the BatchNorm running means, which carry them) are checked for range /
  loosely, as tests/test_oracle_golden.py does for the CPU oracle.
"""
import os
import numpy as np
import pytest
import torch

from conftest import close, load_golden, rel_err

pytestmark = pytest.mark.gpu

LOSS_TOL = 1e-5
STEP0_TOL = 1e-5
LATER_TOL = 1e-4
FC_BIAS = ("fc1.bias", "fc2.bias", "fc3.bias")   # exact gradient 0 (BatchNorm follows)
BINARY_W = ("fc1.weight", "fc2.weight", "fc3.weight")


@pytest.fixture(scope="module")
def nets():
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    from bnn_amd import nets as N
    return N


def host(t):
    torch.cuda.synchronize()
    return t.detach().cpu().numpy()


def _init_state(g):
    sd = {}
    for k, v in g.items():
        if k.startswith("init/"):
            t = torch.as_tensor(np.asarray(v))
            sd[k[len("init/"):]] = t
    return sd


def _make_model(nets, g, fused, libbnn_bn=True):
    w = [int(v) for v in g["meta/widths"]]
    if fused:
        m = nets.MLP(*w, p_drop=0.0, org_protocol=False, mutate_input=False, fused_bn=True, backend="fp4")
    else:
        m = nets.MLP(*w, p_drop=0.0, fused_bn=libbnn_bn)
    m.load_state_dict(_init_state(g))
    return m.cuda().train()


def _record_acts(model):
    """The binarized inputs of fc2 / fc3 (the drop-in leaves sign(input) in the caller's tensor,
    binarized_modules.py:75-76) and the BatchNorm inputs z2 (for the near-tie analysis)."""
    acts = {}

    def keep(name):
        def hook(mod, inp, out):
            acts[name] = host(inp[0]).astype(np.int8)
        return hook

    model.fc2.register_forward_hook(keep("fc2_in"))
    model.fc3.register_forward_hook(keep("fc3_in"))
    model.bn1.register_forward_pre_hook(lambda m, inp: acts.__setitem__("z1", host(inp[0]).astype(np.float64)))
    model.bn2.register_forward_pre_hook(lambda m, inp: acts.__setitem__("z2", host(inp[0]).astype(np.float64)))
    return acts


def _check_step(s, g, loss, out, named, org_of, tol):
    assert abs(float(loss) - float(g[f"s{s}/loss"])) < LOSS_TOL, (s, float(loss), float(g[f"s{s}/loss"]))
    assert rel_err(host(out), g[f"s{s}/out"]) < tol, (s, rel_err(host(out), g[f"s{s}/out"]))
    for k, p in named.items():
        gref = g[f"s{s}/grad/{k}"]
        if k in FC_BIAS:
            assert close(host(p.grad), gref, 0.0, 1e-5), (s, k)       # both ~0 (rounding noise)
            continue
        assert rel_err(host(p.grad), gref) < tol, (s, k, rel_err(host(p.grad), gref))


def _check_update(s, g, org_of, named, tol, org_protocol):
    for k in BINARY_W:
        ref = g[f"s{s}/org/{k}"]
        got = host(org_of(k))
        if org_protocol:
            assert close(got, ref, tol, 0.0), (s, k, rel_err(got, ref))
            assert np.abs(got).max() <= 1.0
        else:                                    # frozen: latent = initial weights, unchanged
            assert np.array_equal(np.sign(got), np.sign(g[f"init/{k}"])), (s, k)
    for k in FC_BIAS:
        got = host(named[k])
        if org_protocol:
            assert np.abs(got).max() <= 1.0      # clamped with the weights (mnist-dist2.py:135-137)
    for k in ("bn1.weight", "bn2.weight", "bn3.weight", "fc4.weight", "fc4.bias"):
        assert close(host(named[k]), g[f"s{s}/data/{k}"], tol, 1e-6), (s, k)


def _check_buffers(s, g, model):
    bufs = dict(model.named_buffers())
    for k in ("bn1.running_var", "bn2.running_var", "bn3.running_var"):
        assert close(host(bufs[k]), g[f"s{s}/buf/{k}"], 1e-5, 1e-7), (s, k)
    for k in ("bn1.running_mean", "bn2.running_mean", "bn3.running_mean"):
        # running_mean carries the fc bias, whose Adam update is driven by rounding noise
        assert close(host(bufs[k]), g[f"s{s}/buf/{k}"], 1e-3, 0.0), (s, k)


@pytest.mark.parametrize("name", ["trace_org", "trace_frozen"])
def test_trace_replay_dropin(nets, name):
    """Path (i): reference call pattern, torch Adam (+ the .org protocol for trace_org)."""
    from bnn_amd.optim import org_protocol_step
    g = load_golden(name)
    org = bool(g["meta/org_protocol"])
    model = _make_model(nets, g, fused=False)
    acts = _record_acts(model)
    opt = torch.optim.Adam(model.parameters(), lr=float(g["meta/lr"]))
    crit = torch.nn.CrossEntropyLoss()
    named = dict(model.named_parameters())
    for s in range(3):
        x = torch.as_tensor(g[f"s{s}/x"]).cuda()
        t = torch.as_tensor(g[f"s{s}/target"]).cuda()
        opt.zero_grad()
        out = model(x)
        loss = crit(out, t)
        loss.backward()
        for k in ("fc2_in", "fc3_in"):          # near-ties resolved as the reference resolves them
            assert np.array_equal(acts[k], g[f"s{s}/act/{k}"]), (s, k, int((acts[k] != g[f"s{s}/act/{k}"]).sum()))
        tol = STEP0_TOL if s == 0 else LATER_TOL
        _check_step(s, g, loss.item(), out, named, None, tol)
        if org:
            org_protocol_step(model, opt)          # mnist-dist2.py:131-137
        else:
            opt.step()                             # mnist-dist3.py:116-119
        _check_update(s, g, lambda k: named[k].org, named, LATER_TOL, org)
        _check_buffers(s, g, model)


@pytest.mark.parametrize("name", ["trace_org", "trace_frozen"])
def test_trace_replay_fused_trainer(nets, name):
    """Path (ii): the fused trainer path bench.py times.  The frozen trace (mnist-dist3.py: Adam
    updates the binarised copy that the next forward overwrites) is the same as leaving the
    binary weights out of the optimizer and clamping nothing."""
    from bnn_amd.optim import LatentAdam
    g = load_golden(name)
    org = bool(g["meta/org_protocol"])
    model = _make_model(nets, g, fused=True)
    named = dict(model.named_parameters())
    if org:
        opt = LatentAdam(model.parameters(), lr=float(g["meta/lr"]), clamp_params=nets.binary_params(model))
    else:
        opt = LatentAdam([p for k, p in named.items() if k not in BINARY_W], lr=float(g["meta/lr"]))
    crit = torch.nn.CrossEntropyLoss()
    for s in range(3):
        x = torch.as_tensor(g[f"s{s}/x"]).cuda()
        t = torch.as_tensor(g[f"s{s}/target"]).cuda()
        for p in model.parameters():
            p.grad = None
        out = model(x)
        loss = crit(out, t)
        loss.backward()
        tol = STEP0_TOL if s == 0 else LATER_TOL
        _check_step(s, g, loss.item(), out, named, None, tol)
        opt.step()
        _check_update(s, g, lambda k: named[k], named, LATER_TOL, org)
        _check_buffers(s, g, model)


@pytest.mark.parametrize("name", ["trace_org", "trace_frozen"])
def test_trace_replay_dropin_torch_batchnorm(nets, name):
    """The drop-in with torch's own GPU BatchNorm1d kernels between the libbnn layers.  torch's
    GPU BN computes the batch mean in fp32, so it resolves BatchNorm near-ties (see module doc)
    by rounding, not as the reference does.  Stated band: at step 0 (identical weights) every
    binarized activation that differs from the reference's sits at a near-tie
    (|z - mean| <= 1e-5 * max|z|), and every step's loss is within 0.05 of the reference's
    (one flipped +-1 activation moves a 16-sample loss by ~1e-3)."""
    from bnn_amd.optim import org_protocol_step
    g = load_golden(name)
    org = bool(g["meta/org_protocol"])
    model = _make_model(nets, g, fused=False, libbnn_bn=False)
    acts = _record_acts(model)
    opt = torch.optim.Adam(model.parameters(), lr=float(g["meta/lr"]))
    crit = torch.nn.CrossEntropyLoss()
    for s in range(3):
        x = torch.as_tensor(g[f"s{s}/x"]).cuda()
        t = torch.as_tensor(g[f"s{s}/target"]).cuda()
        opt.zero_grad()
        loss = crit(model(x), t)
        loss.backward()
        if s == 0:
            for k, zk in (("fc2_in", "z1"), ("fc3_in", "z2")):
                z = acts[zk]
                near = np.abs(z - z.mean(0)) <= 1e-5 * np.abs(z).max()
                bad = acts[k] != g[f"s{s}/act/{k}"]
                assert not (bad & ~near).any(), (k, int((bad & ~near).sum()))
        assert abs(loss.item() - float(g[f"s{s}/loss"])) < 0.05, (s, loss.item())
        if org:
            org_protocol_step(model, opt)
        else:
            opt.step()


def test_fused_trainer_uses_repacked_weights(nets):
    """The fused latent update rewrites the next forward's packed weight operands in place
    (bnn_adam_clamp_pack): a run that drops the cache before every forward (so every forward
    re-packs sign(w) from scratch) must produce bit-identical losses, gradients and weights."""
    from bnn_amd import functional as BF
    from bnn_amd.data import synthetic_mnist
    from bnn_amd.optim import LatentAdam
    torch.manual_seed(21)
    runs = []
    for drop_cache in (False, True):
        torch.manual_seed(21)
        model = nets.MLP(320, 192, 128, p_drop=0.0, org_protocol=False, mutate_input=False, fused_bn=True).cuda()
        opt = LatentAdam(model.parameters(), lr=0.01, clamp_params=nets.binary_params(model))
        rec = []
        for s in range(4):
            x, y = synthetic_mnist(256, seed=100 + s, device="cuda")
            if drop_cache:
                for p in model.parameters():
                    BF.invalidate_packed(p)
            for p in model.parameters():
                p.grad = None
            loss = torch.nn.functional.cross_entropy(model(x), y)
            loss.backward()
            rec.append(loss.item())
            opt.step()
        rec += [host(p) for p in model.parameters()]
        if not drop_cache:
            assert getattr(model.fc2.weight, "_bnn_pack", None) is not None
        runs.append(rec)
    for a, b in zip(*runs):
        assert np.array_equal(np.asarray(a), np.asarray(b))


@pytest.mark.parametrize("N,K", [(300, 1000), (64, 784), (8192, 784), (100, 37), (512, 768), (2048, 4096)])
@pytest.mark.parametrize("fmt", [0, 1])
@pytest.mark.parametrize("qt_fmt", [0, 1])
def test_adam_clamp_pack_matches_unfused(nets, N, K, fmt, qt_fmt):
    """bnn_adam_clamp_pack: p, m, v bit-identical to bnn_adam_clamp; q / qt bit-identical to
    sign-packing the updated weight (padding zero)."""
    from bnn_amd import _lib as L
    from bnn_amd import functional as F
    torch.manual_seed(N + K + fmt)
    p0 = torch.empty(N, K, device="cuda").uniform_(-1.1, 1.1)
    p0[torch.rand_like(p0) < 0.01] = 0.0
    g = torch.randn_like(p0)
    m0 = torch.randn_like(p0) * 0.1
    v0 = torch.rand_like(p0) * 0.01
    a = [p0.clone(), m0.clone(), v0.clone()]
    F.adam_clamp_(a[0], g, a[1], a[2], 3, lr=0.01)
    b = [p0.clone(), m0.clone(), v0.clone()]
    if fmt == 1:
        q = torch.full((N, F.round_up(K, 256) // 2), 0x77, dtype=torch.uint8, device="cuda")
    else:
        q = torch.full((N, F.round_up(K)), 7, dtype=torch.int8, device="cuda")
    if qt_fmt == 1:
        qt = torch.full((K, F.round_up(N, 256) // 2), 0x77, dtype=torch.uint8, device="cuda")
    else:
        qt = torch.full((K, F.round_up(N)), 7, dtype=torch.int8, device="cuda")
    L.call("bnn_adam_clamp_pack", L.ptr(b[0]), L.ptr(g), L.ptr(b[1]), L.ptr(b[2]), N, K, 0.01, 0.9, 0.999, 1e-8,
           3, 1.0, 1, fmt, L.ptr(q), q.shape[1], L.ptr(qt), qt.shape[1], qt_fmt, L.stream())
    for x, y in zip(a, b):
        assert torch.equal(x, y)
    if fmt == 1:
        q_ref, _ = F.sign_pack_fp4(a[0])
    else:
        q_ref, _ = F.sign_pack(a[0], True, False)
    _, qt_ref = F.sign_pack_fp4(a[0], want_qt=True, qt_fmt="fp4" if qt_fmt == 1 else "i8", want_q=False)
    assert torch.equal(q, q_ref)
    assert torch.equal(qt, qt_ref)


@pytest.mark.parametrize("N,K,qt_fmt", [(512, 768, 1), (1024, 2048, 2), (8192, 8192, 2), (768, 1536, 1)])
def test_adam_pack_tile256_equals_tile64(nets, N, K, qt_fmt):
    """The 256 x 256-tile form of bnn_adam_clamp_pack (whole tiles, FP4 rows + FP4 / panel
    transpose) against the 64 x 64-tile kernel (bnn_adam_pack_set_tile256(0)): p, m, v, q, qt
    bit-identical."""
    from bnn_amd import _lib as L
    torch.manual_seed(N + K)
    p0 = torch.empty(N, K, device="cuda").uniform_(-1.1, 1.1)
    p0[torch.rand_like(p0) < 0.01] = 0.0
    g = torch.randn_like(p0)
    m0 = torch.randn_like(p0) * 0.1
    v0 = torch.rand_like(p0) * 0.01
    outs = []
    try:
        for tile256 in (2, 0):                # 2: the big tile at any whole-tile shape
            L.call("bnn_adam_pack_set_tile256", tile256)
            b = [p0.clone(), m0.clone(), v0.clone()]
            q = torch.full((N, K // 2), 0x77, dtype=torch.uint8, device="cuda")
            qt = torch.full((K, N // 2), 0x77, dtype=torch.uint8, device="cuda")
            L.call("bnn_adam_clamp_pack", L.ptr(b[0]), L.ptr(g), L.ptr(b[1]), L.ptr(b[2]), N, K, 0.01, 0.9, 0.999,
                   1e-8, 3, 1.0, 1, 1, L.ptr(q), q.shape[1], L.ptr(qt), qt.shape[1], qt_fmt, L.stream())
            outs.append(b + [q, qt])
    finally:
        L.call("bnn_adam_pack_set_tile256", int(os.environ.get("BNN_ADAM_TILE256", "1") != "0"))
    for x, y in zip(*outs):
        assert torch.equal(x, y)

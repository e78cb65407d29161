"""GPU training parity at widths where every fusion of the benched path fires.

``tests/golden/trace_wide.npz`` is the reference's own 10-step training run
(tests/golden/make_golden.py ``trace_wide_case``: ``models/binarized_modules.py`` imported as is,
the mnist-dist2.py:46-76 Net at widths 256/256/256, the :118-137 loop with the .org protocol,
Adam lr 0.01, dropout p = 0, batch 256, input = ToTensor of u8 pixels).

Two GPU paths replay it:

(i)  the drop-in: ``models.binarized_modules`` layers with the .org protocol, fp32 input u/255,
     libbnn BatchNorm+Hardtanh, ``torch.optim.Adam`` + ``optim.org_protocol_step`` -- the
     reference script's call pattern;
(ii) the trainer / bench.py path: u8 pixels in HBM (fc1 on the bytes), BN -> sign-pack -> FP4
     GEMM, int16 pre-activations (z16, forced on at this size by ``Z16_MIN_TILES = 0``), the FP6
     digit hand-offs from the BatchNorm backward (q6), the fused drop->bn3->htanh3->fc4 head, the
     int8 column-digit hand-off to fc1's weight gradient (i8cols) and the fused
     ``LatentAdam`` (Adam + clamp + re-pack).  The test asserts every one of those hand-offs
     fired on every step.

Tolerances:
* loss, every step: |loss - loss_ref| <= 1e-5 (losses ~2.3);
* log-probs: norm-wise <= 1e-5 at step 0, <= 1e-4 afterwards;
* step-0 gradients of every parameter: norm-wise <= 1e-5 against the reference's fp32 CPU
  gradients (the fc biases feed BatchNorm: exact gradient 0, both sides ~1e-8 noise: absolute);
* per-step gradients of the BatchNorm affine parameters and fc4: norm-wise <= 1e-4;
* latent weights after each step: the sign pattern (the next forward's binarized weights) may
  differ in at most ``SIGN_BUDGET`` elements per tensor, and the float64 digest (sum |w|,
  sum w^2) within 1e-5 relative; final latent weights norm-wise <= 1e-4.  Adam turns a gradient
  whose true value is within rounding noise of 0 into a +-lr step whichever sign the noise has,
  so a latent weight that also sits within 2*lr of 0 may land on the other side of it.  The
  float64 oracle replays this trace with 0 sign differences (tests/test_oracle_golden.py).
* binarized activations of fc2 / fc3 (drop-in path): equal to the reference's at every step.
"""
import numpy as np
import pytest
import torch

from conftest import close, load_golden, rel_err

pytestmark = pytest.mark.gpu

LOSS_TOL = 1e-5
STEP0_TOL = 1e-5
LATER_TOL = 1e-4
SIGN_BUDGET = 4
FC_BIAS = ("fc1.bias", "fc2.bias", "fc3.bias")
BINARY_W = ("fc1.weight", "fc2.weight", "fc3.weight")
SMALL = ("bn1.weight", "bn1.bias", "bn2.weight", "bn2.bias", "bn3.weight", "bn3.bias", "fc4.weight", "fc4.bias")


@pytest.fixture(scope="module")
def wide():
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    return load_golden("trace_wide")


def host(t):
    torch.cuda.synchronize()
    return t.detach().cpu().numpy()


def _model(g, fused):
    from bnn_amd import nets
    w = [int(v) for v in g["meta/widths"]]
    if fused:
        m = nets.MLP(*w, p_drop=0.0, org_protocol=False, mutate_input=False, fused_bn=True, backend="fp4")
    else:
        m = nets.MLP(*w, p_drop=0.0, fused_bn=True)
    m.load_state_dict({k[5:]: torch.as_tensor(np.asarray(v)) for k, v in g.items() if k.startswith("init/")})
    return m.cuda().train()


def _sign_diff(w, packed):
    return int(np.unpackbits(np.packbits((np.asarray(w) > 0).reshape(-1)) ^ packed).sum())


def _check_step(s, g, loss, out, named, latent, report):
    dl = abs(float(loss) - float(g[f"s{s}/loss"]))
    eo = rel_err(host(out), g[f"s{s}/out"])
    row = {"step": s, "dloss": dl, "out": eo}
    assert dl <= LOSS_TOL, (s, float(loss), float(g[f"s{s}/loss"]))
    assert eo <= (STEP0_TOL if s == 0 else LATER_TOL), (s, eo)
    for k in (named if s == 0 else SMALL):
        got, ref = host(named[k].grad), g[f"s{s}/grad/{k}"]
        if k in FC_BIAS:
            assert close(got, ref, 0.0, 1e-5), (s, k)
            continue
        e = rel_err(got, ref)
        row["g:" + k] = e
        assert e <= (STEP0_TOL if s == 0 else LATER_TOL), (s, k, e)
    return row


def _check_latent(s, g, latent, row):
    for k in BINARY_W:
        o = host(latent(k)).astype(np.float64)
        nd = _sign_diff(o, g[f"s{s}/orgsign/{k}"])
        row["sign:" + k] = nd
        assert nd <= SIGN_BUDGET, (s, k, nd)
        assert int((o == 0).sum()) == int(g[f"s{s}/orgzero/{k}"])
        dg = g[f"s{s}/orgdigest/{k}"]
        for i in (1, 2):
            got = (np.abs(o).sum(), (o * o).sum())[i - 1]
            assert abs(got - dg[i]) <= 1e-5 * abs(dg[i]), (s, k, i, got, dg[i])
        assert np.abs(o).max() <= 1.0


def _check_final(g, named, latent, model):
    for k in BINARY_W:
        assert close(host(latent(k)), g[f"final/data/{k}"], LATER_TOL, 0.0), (k, rel_err(host(latent(k)), g[f"final/data/{k}"]))
    for k in SMALL:
        assert close(host(named[k]), g[f"final/data/{k}"], LATER_TOL, 1e-6), k
    for k in FC_BIAS:
        assert np.abs(host(named[k])).max() <= 1.0
    bufs = dict(model.named_buffers())
    for k in ("bn1.running_var", "bn2.running_var", "bn3.running_var"):
        assert close(host(bufs[k]), g[f"final/buf/{k}"], 1e-4, 1e-7), k


def test_wide_trace_dropin(wide):
    """Path (i): the reference's call pattern on fp32 input; binarized activations equal."""
    from bnn_amd.optim import org_protocol_step
    g = wide
    model = _model(g, fused=False)
    acts = {}

    def keep(nm):
        def hook(mod, inp, out):
            acts[nm] = host(inp[0])
        return hook

    model.fc2.register_forward_hook(keep("fc2_in"))
    model.fc3.register_forward_hook(keep("fc3_in"))
    opt = torch.optim.Adam(model.parameters(), lr=float(g["meta/lr"]))
    crit = torch.nn.CrossEntropyLoss()
    named = dict(model.named_parameters())
    rows = []
    for s in range(int(g["meta/steps"])):
        x = torch.as_tensor(g[f"s{s}/u8"]).cuda().float().div_(255.0)        # transforms.ToTensor()
        t = torch.as_tensor(g[f"s{s}/target"]).cuda()
        opt.zero_grad()
        out = model(x)
        loss = crit(out, t)
        loss.backward()
        row = _check_step(s, g, loss.item(), out, named, None, rows)
        for k in ("fc2_in", "fc3_in"):
            nd = _sign_diff(acts[k], g[f"s{s}/act/{k}"])
            row["act:" + k] = nd
            assert nd == 0 and int((acts[k] == 0).sum()) == int(g[f"s{s}/act0/{k}"]), (s, k, nd)
        org_protocol_step(model, opt)                       # mnist-dist2.py:131-137
        _check_latent(s, g, lambda k: named[k].org, row)
        rows.append(row)
    print("\nwide trace, drop-in:", *rows, sep="\n  ")
    _check_final(g, named, lambda k: named[k].org, model)


def test_wide_trace_fused_trainer(wide, monkeypatch):
    """Path (ii): what bench.py / the trainer run, with every hand-off asserted per step."""
    from bnn_amd import functional as BF
    from bnn_amd import nets
    from bnn_amd.optim import LatentAdam
    monkeypatch.setattr(BF, "Z16_MIN_TILES", 0)            # z16 at this grid size too
    g = wide
    model = _model(g, fused=True)
    named = dict(model.named_parameters())
    opt = LatentAdam(model.parameters(), lr=float(g["meta/lr"]), clamp_params=nets.binary_params(model))
    crit = torch.nn.CrossEntropyLoss()
    rows = []
    for s in range(int(g["meta/steps"])):
        u = torch.as_tensor(g[f"s{s}/u8"]).cuda()                           # resident u8 pixels
        t = torch.as_tensor(g[f"s{s}/target"]).cuda()
        c0 = (BF.Z16_HANDOFFS, BF.Q6_HANDOFFS, BF.I8C_HANDOFFS, BF.HEAD_CALLS)
        for p in model.parameters():
            p.grad = None
        out = model(u)
        loss = crit(out, t)
        loss.backward()
        fired = [a - b for a, b in zip((BF.Z16_HANDOFFS, BF.Q6_HANDOFFS, BF.I8C_HANDOFFS, BF.HEAD_CALLS), c0)]
        # z16: fc2 and fc3 outputs; q6: dz of fc3 (head bwd) and fc2 (bn2 bwd) taken by the FP6 GEMMs;
        # i8cols: bn1 bwd -> fc1's dW; one fused head
        assert fired == [2, 2, 1, 1], (s, fired)
        row = _check_step(s, g, loss.item(), out, named, None, rows)
        opt.step()
        _check_latent(s, g, lambda k: named[k], row)
        assert getattr(model.fc2.weight, "_bnn_pack", None) is not None    # re-packed by the fused update
        rows.append(row)
    print("\nwide trace, fused trainer path:", *rows, sep="\n  ")
    _check_final(g, named, lambda k: named[k], model)

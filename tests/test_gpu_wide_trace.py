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

Binarized-weight teacher forcing.  Adam turns a gradient whose true value is within rounding
noise of 0 into a +-lr step whichever sign the noise has, so a latent weight that also sits within
2*lr of 0 can land on the other side of 0 than the reference's (the float64 oracle never does on
this trace; any other fp32 GEMM can -- test_wide_trace_free_running calibrates it with torch fp32
on this GPU).  One such flip changes the next forward's binarized weights and the trajectories
split (observed: the loss moves by ~3e-4, BatchNorm-parameter gradients by several %).  The
replays therefore compare every step FROM THE REFERENCE'S BINARIZED WEIGHTS: before each forward,
a latent weight whose sign differs from the reference's recorded sign pattern is negated (at most
``SIGN_BUDGET`` per tensor and step, counted in the printed rows), so each step is held to the
same-trajectory bars:
* loss |loss - loss_ref| <= 1e-5 (losses ~2.3);
* log-probs norm-wise <= 1e-5 at step 0, <= 1e-4 afterwards;
* step-0 gradients of every parameter norm-wise <= 1e-5 against the reference's fp32 CPU
  gradients (the fc biases feed BatchNorm: exact gradient 0, both sides ~1e-8 noise: absolute);
* per-step gradients of the BatchNorm affine parameters and fc4 norm-wise <= 1e-4;
* latent weights after each step: float64 digest (sum |w|, sum w^2) within 1e-4 relative (the
  forced elements keep their own magnitude), final latent weights norm-wise <= 1e-3;
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
FREE_SPLIT_LOSS_TOL = 0.1   # free-running, after the first split: a sanity bound
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


def _step_row(s, g, loss, out, named):
    """Per-step comparison numbers (asserted by _assert_row)."""
    row = {"step": s, "dloss": abs(float(loss) - float(g[f"s{s}/loss"])), "out": rel_err(host(out), g[f"s{s}/out"])}
    for k in (named if s == 0 else SMALL):
        got, ref = host(named[k].grad), g[f"s{s}/grad/{k}"]
        if k in FC_BIAS:
            row["g:" + k] = float(np.linalg.norm(got - ref))          # absolute: exact gradient 0
        else:
            row["g:" + k] = rel_err(got, ref)
    return row


def _latent_row(s, g, latent, row):
    for k in BINARY_W:
        o = host(latent(k)).astype(np.float64)
        row["sign:" + k] = _sign_diff(o, g[f"s{s}/orgsign/{k}"])
        row["zero:" + k] = int((o == 0).sum()) - int(g[f"s{s}/orgzero/{k}"])
        dg = g[f"s{s}/orgdigest/{k}"]
        row["dig:" + k] = max(abs(np.abs(o).sum() - dg[1]) / dg[1], abs((o * o).sum() - dg[2]) / dg[2])
        row["max:" + k] = float(np.abs(o).max())


def _assert_row(row):
    s = row["step"]
    tol = STEP0_TOL if s == 0 else LATER_TOL
    assert row["dloss"] <= LOSS_TOL, row
    assert row["out"] <= tol, row
    for k, v in row.items():
        if k.startswith("g:"):
            assert v <= (1e-5 if k[2:] in FC_BIAS else tol), (k, row)
        if k.startswith("forced:"):
            assert v <= SIGN_BUDGET, row
    for k in BINARY_W:
        assert row["zero:" + k] == 0 and row["max:" + k] <= 1.0, row
        assert row["dig:" + k] <= 1e-4, row


def _force_signs(s, g, latent, row):
    """Negate the latent weights whose sign differs from the reference's after step s - 1."""
    for k in BINARY_W:
        t = latent(k)
        o = host(t)
        ref = np.unpackbits(g[f"s{s - 1}/orgsign/{k}"])[:o.size].astype(bool)
        idx = np.nonzero(((o.reshape(-1) > 0) != ref) & (o.reshape(-1) != 0))[0]
        row["forced:" + k] = int(idx.size)
        if idx.size:
            with torch.no_grad():
                t.view(-1)[torch.as_tensor(idx, device=t.device)] *= -1.0


def _check_final(g, named, latent, model):
    for k in BINARY_W:
        assert close(host(latent(k)), g[f"final/data/{k}"], 1e-3, 0.0), (k, rel_err(host(latent(k)), g[f"final/data/{k}"]))
    for k in SMALL:
        assert close(host(named[k]), g[f"final/data/{k}"], LATER_TOL, 1e-6), k
    for k in FC_BIAS:
        assert np.abs(host(named[k])).max() <= 1.0
    bufs = dict(model.named_buffers())
    for k in ("bn1.running_var", "bn2.running_var", "bn3.running_var"):
        assert close(host(bufs[k]), g[f"final/buf/{k}"], LATER_TOL, 1e-7), k


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
    for s in range(int(g["meta/steps"])):
        x = torch.as_tensor(g[f"s{s}/u8"]).cuda().float().div_(255.0)        # transforms.ToTensor()
        t = torch.as_tensor(g[f"s{s}/target"]).cuda()
        forced = {}
        if s > 0:
            _force_signs(s, g, lambda k: named[k].org, forced)
        opt.zero_grad()
        out = model(x)
        loss = crit(out, t)
        loss.backward()
        row = {**_step_row(s, g, loss.item(), out, named), **forced}
        for k in ("fc2_in", "fc3_in"):
            row["act:" + k] = _sign_diff(acts[k], g[f"s{s}/act/{k}"]) + abs(
                int((acts[k] == 0).sum()) - int(g[f"s{s}/act0/{k}"]))
        org_protocol_step(model, opt)                       # mnist-dist2.py:131-137
        _latent_row(s, g, lambda k: named[k].org, row)
        print(f"  drop-in {row}", flush=True)
        assert row["act:fc2_in"] == 0 and row["act:fc3_in"] == 0, row
        _assert_row(row)
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
    for s in range(int(g["meta/steps"])):
        u = torch.as_tensor(g[f"s{s}/u8"]).cuda()                           # resident u8 pixels
        t = torch.as_tensor(g[f"s{s}/target"]).cuda()
        forced = {}
        if s > 0:
            _force_signs(s, g, lambda k: named[k], forced)   # (an in-place op: the packed cache re-packs)
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
        row = {**_step_row(s, g, loss.item(), out, named), **forced}
        opt.step()
        _latent_row(s, g, lambda k: named[k], row)
        print(f"  fused {row}", flush=True)
        _assert_row(row)
        assert getattr(model.fc2.weight, "_bnn_pack", None) is not None    # re-packed by the fused update
    _check_final(g, named, lambda k: named[k], model)


def _free_run(g, model, opt, step_fn, latent):
    """Free-running replay: (per-step |dloss|, step of the first binarized-weight split or None)."""
    dl, split = [], None
    for s in range(int(g["meta/steps"])):
        loss = step_fn(s)
        dl.append(abs(loss - float(g[f"s{s}/loss"])))
        if split is None and any(_sign_diff(host(latent(k)), g[f"s{s}/orgsign/{k}"]) for k in BINARY_W):
            split = s + 1                     # the next forward uses different binarized weights
    return dl, split


def test_wide_trace_free_running(wide):
    """No forcing: the fused path and, as calibration, the reference's own semantics on torch fp32
    GEMMs on this GPU (oracle/bnn_torch.py: sign() + F.linear, BatchNorm1d, Adam + the .org
    protocol) replay the trace freely.  Bar: |dloss| <= 1e-5 on every step before the first
    binarized-weight split.  After it the trajectories are decorrelated (measured: 3e-4, then
    1e-2 .. 5e-2 by steps 7-9; the FP6 digit gradients (~3e-6 norm-wise) flip a near-zero
    gradient's sign sooner than an fp32 GEMM (~1e-7): torch fp32 on the GPU has not split by
    step 9), so only a sanity bound is asserted; the loss-curve criterion is the windowed one of
    test_gpu_loss_curve.py."""
    from bnn_amd import nets
    from bnn_amd.optim import LatentAdam
    from oracle.bnn_torch import RefMLP, train_step
    g = wide
    crit = torch.nn.CrossEntropyLoss()
    model = _model(g, fused=True)
    named = dict(model.named_parameters())
    opt = LatentAdam(model.parameters(), lr=float(g["meta/lr"]), clamp_params=nets.binary_params(model))

    def fused_step(s):
        for p in model.parameters():
            p.grad = None
        loss = crit(model(torch.as_tensor(g[f"s{s}/u8"]).cuda()), torch.as_tensor(g[f"s{s}/target"]).cuda())
        loss.backward()
        opt.step()
        return loss.item()

    dl, split = _free_run(g, model, opt, fused_step, lambda k: named[k])
    ref = RefMLP(*[int(v) for v in g["meta/widths"]], p_drop=0.0)
    ref.load_state_dict({k[5:]: torch.as_tensor(np.asarray(v)) for k, v in g.items() if k.startswith("init/")})
    ref = ref.cuda().train()
    ropt = torch.optim.Adam(ref.parameters(), lr=float(g["meta/lr"]))
    rnamed = dict(ref.named_parameters())

    def torch_step(s):
        x = torch.as_tensor(g[f"s{s}/u8"]).cuda().float().div_(255.0)
        return train_step(ref, ropt, x, torch.as_tensor(g[f"s{s}/target"]).cuda(), True)

    tdl, tsplit = _free_run(g, ref, ropt, torch_step, lambda k: rnamed[k].org)
    print(f"\nfree-running |dloss| per step, libbnn fused (first split before step {split}):",
          " ".join(f"{v:.1e}" for v in dl))
    print(f"free-running |dloss| per step, torch fp32 on the GPU (first split before step {tsplit}):",
          " ".join(f"{v:.1e}" for v in tdl))
    for s, v in enumerate(dl):
        assert v <= (LOSS_TOL if split is None or s < split else FREE_SPLIT_LOSS_TOL), (s, v, split)

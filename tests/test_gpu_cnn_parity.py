"""Whole-network parity of the BinCNN (BASELINE config 4) against the reference.

``tests/golden/trace_cnn.npz`` is the reference's own 8-step training run (make_golden.py
``trace_cnn_case``: ``models/binarized_modules.py``'s BinarizeConv2d imported as is, in the
config-4 topology -- conv5x5(1->16, p2) -> BatchNorm2d -> Hardtanh -> MaxPool2d(2), conv5x5(16->32,
p2) -> ..., Linear(1568, 10), LogSoftmax -- trained by the mnist-dist2.py:118-137 loop with the
.org protocol, Adam lr 0.01, batch 256, input ToTensor of u8 pixels).  It is replayed on the GPU by

(i)  the drop-in path: the reference's call pattern (.org protocol, ``torch.optim.Adam`` +
     ``optim.org_protocol_step``), conv2's binarized input compared with the reference's;
(ii) the bench's fused path: ``nets.BinCNN(fused_bn=True)`` with the latent weights in the
     Parameters, the conv outputs travelling as int16 sums + bias into the fused
     BatchNorm2d+Hardtanh+MaxPool2d (zq hand-offs asserted on every step), the narrow-classifier
     kernels and LatentAdam.

Both replay from the reference's binarized weights (teacher forcing, as test_gpu_wide_trace.py
does: a latent conv weight whose sign differs from the reference's after the previous step is
negated before the forward, at most SIGN_BUDGET per tensor and step).  Bars per step: loss
|d| <= 1e-5 * max(1, loss); log-probs <= 1e-5 at step 0, <= 1e-4 after; step-0 gradients <= 1e-5
against the fixture (the conv weights: within the reference's own fp32 accumulation error,
tests/test_oracle_t64.py CONV_W_REF_TOL; conv biases absolute: exact gradient 0); per-step
gradients of BatchNorm2d and the classifier <= 1e-4.

test_cnn_one_step_bench_batch_vs_float64: one training step of the bench's CNN workload (batch
4096, bench.build("cnn"), bench's synthetic data) against the float64 oracle (oracle/bnn_t64.py
CNNOracle) on the GPU -- no continuous-input layer exists in this net (conv1 binarises the
pixels), so the whole step is compared from the raw input: loss / log-probs <= 1e-5, every
gradient <= 1e-5, except where the same oracle step with its convolution backward contractions
in fp32 (the reference's arithmetic for them: torch fp32 GEMMs of the fp32 gradient and the ternary
operand) is itself further than 1e-5 from float64 -- the conv weight gradients contract B*28*28
(conv1: 3.2 M at B = 4096) / B*14*14 products of a BatchNorm2d gradient that sums to 0 per channel
-- and then that fp32 calibration is the bar (named in the assertion); the update = Adam (float64)
+ clamp on the GPU's own gradient elementwise <= 1e-7.
"""
import numpy as np
import pytest
import torch

from conftest import close, load_golden, rel_err
from test_oracle_t64 import CONV_W_REF_TOL

pytestmark = pytest.mark.gpu

CONV_W = ("layer1.0.weight", "layer2.0.weight")
CONV_B = ("layer1.0.bias", "layer2.0.bias")
SMALL = ("layer1.1.weight", "layer1.1.bias", "layer2.1.weight", "layer2.1.bias", "fc.weight", "fc.bias")
SIGN_BUDGET = 4
LR = 0.01


@pytest.fixture(scope="module")
def trace():
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    return load_golden("trace_cnn")


def host(t):
    torch.cuda.synchronize()
    return t.detach().cpu().numpy()


def _model(g, fused):
    from bnn_amd import nets
    if fused:
        m = nets.BinCNN(org_protocol=False, mutate_input=False, fused_bn=True)
    else:
        m = nets.BinCNN(fused_bn=True)
    m.load_state_dict({k[5:]: torch.as_tensor(np.asarray(v)) for k, v in g.items() if k.startswith("init/")})
    return m.cuda().train()


def _x(g, s):
    return torch.as_tensor(g[f"s{s}/u8"]).cuda().view(-1, 1, 28, 28).float().div_(255.0)   # ToTensor()


def _force(s, g, latent, row):
    for k in CONV_W:
        t = latent(k)
        o = host(t).reshape(-1)
        ref = np.unpackbits(g[f"s{s - 1}/orgsign/{k}"])[:o.size].astype(bool)
        idx = np.nonzero(((o > 0) != ref) & (o != 0))[0]
        row["forced:" + k] = int(idx.size)
        if idx.size:
            with torch.no_grad():
                t.view(-1)[torch.as_tensor(idx, device=t.device)] *= -1.0


def _force_bias(s, g, named, row):
    """The conv biases' true gradient is 0 (BatchNorm2d removes the mean): Adam turns their
    rounding-noise gradients into +-lr steps whose signs every implementation draws differently
    (the reference's own fp32 included), and the running means carry them.  They are held to the
    reference's values after each step (the largest move recorded), as the latent signs are."""
    for k in CONV_B:
        ref = torch.as_tensor(g[f"s{s - 1}/data/{k}"]).to(named[k].device)
        with torch.no_grad():
            row["bias:" + k] = float((named[k] - ref).abs().max())
            named[k].copy_(ref)


def _row(s, g, loss, out, named):
    row = {"step": s, "dloss": abs(float(loss) - float(g[f"s{s}/loss"])), "out": rel_err(host(out), g[f"s{s}/out"])}
    for k in named:
        if s > 0 and k not in SMALL:
            continue
        got, ref = host(named[k].grad), g[f"s{s}/grad/{k}"]
        row["g:" + k] = float(np.linalg.norm(got - ref)) if k in CONV_B else rel_err(got, ref)
    return row


def _check(row, latent, g):
    s = row["step"]
    tol = 1e-5 if s == 0 else 1e-4
    assert row["dloss"] <= 1e-5 * max(1.0, float(g[f"s{s}/loss"])), row
    assert row["out"] <= tol, row
    for k, v in row.items():
        if k.startswith("g:"):
            name = k[2:]
            assert v <= (1e-5 if name in CONV_B else CONV_W_REF_TOL.get(name, tol)), (k, row)
        if k.startswith("forced:"):
            assert v <= SIGN_BUDGET, row
    for k in CONV_W:
        o = host(latent(k))
        assert np.abs(o).max() <= 1.0
        assert close(o, g[f"s{s}/data/{k}"], 1e-3, 0.0), (k, rel_err(o, g[f"s{s}/data/{k}"]))


def test_cnn_trace_dropin(trace):
    from bnn_amd.optim import org_protocol_step
    g = trace
    model = _model(g, fused=False)
    named = dict(model.named_parameters())
    acts = {}
    model.layer2[0].register_forward_hook(lambda mod, inp, out: acts.__setitem__("conv2_in", host(inp[0])))
    opt = torch.optim.Adam(model.parameters(), lr=LR)
    crit = torch.nn.CrossEntropyLoss()
    for s in range(int(g["meta/steps"])):
        forced = {}
        if s > 0:
            _force(s, g, lambda k: named[k].org, forced)
        opt.zero_grad()
        out = model(_x(g, s))
        loss = crit(out, torch.as_tensor(g[f"s{s}/target"]).cuda())
        loss.backward()
        row = {**_row(s, g, loss.item(), out, named), **forced}
        a = acts["conv2_in"]
        row["act:conv2_in"] = int(np.unpackbits(np.packbits((a > 0).reshape(-1)) ^ g[f"s{s}/act/conv2_in"]).sum()) + abs(
            int((a == 0).sum()) - int(g[f"s{s}/act0/conv2_in"]))
        org_protocol_step(model, opt)                       # mnist-dist2.py:131-137
        print(f"  drop-in {row}", flush=True)
        assert row["act:conv2_in"] == 0, row
        _check(row, lambda k: named[k].org, g)


def test_cnn_trace_fused(trace):
    from bnn_amd import functional as BF
    from bnn_amd import nets
    from bnn_amd.optim import LatentAdam
    g = trace
    model = _model(g, fused=True)
    named = dict(model.named_parameters())
    opt = LatentAdam(model.parameters(), lr=LR, clamp_params=nets.binary_params(model))
    crit = torch.nn.CrossEntropyLoss()
    for s in range(int(g["meta/steps"])):
        forced = {}
        if s > 0:
            _force(s, g, lambda k: named[k], forced)
            _force_bias(s, g, named, forced)
        for p in model.parameters():
            p.grad = None
        z0 = BF.ZQ_HANDOFFS
        out = model(_x(g, s))
        loss = crit(out, torch.as_tensor(g[f"s{s}/target"]).cuda())
        loss.backward()
        assert BF.ZQ_HANDOFFS - z0 == 2, s             # both conv outputs as int16 sums + bias
        row = {**_row(s, g, loss.item(), out, named), **forced}
        opt.step()
        print(f"  fused {row}", flush=True)
        _check(row, lambda k: named[k], g)
    bufs = dict(model.named_buffers())
    last = int(g["meta/steps"]) - 1
    for k in ("layer1.1.running_var", "layer2.1.running_var"):
        assert close(host(bufs[k]), g[f"s{last}/buf/{k}"], 1e-4, 1e-7), k
    # with the conv biases held to the reference's (_force_bias) the running means follow it too
    for k in ("layer1.1.running_mean", "layer2.1.running_mean"):
        assert close(host(bufs[k]), g[f"s{last}/buf/{k}"], 1e-4, 1e-7), (k, rel_err(host(bufs[k]), g[f"s{last}/buf/{k}"]))


def test_cnn_one_step_bench_batch_vs_float64():
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    import bench
    from bnn_amd import functional as BF
    from bnn_amd.data import synthetic_mnist
    from bnn_amd.nets import binary_params
    from bnn_amd.optim import LatentAdam
    from oracle import bnn_t64 as T
    batch = bench.CONFIGS["cnn"][1]
    torch.manual_seed(0)
    model = bench.build("cnn", "fp4").cuda().train()
    x, y = synthetic_mnist(batch, seed=1234, device=torch.device("cuda"), as_u8=False)
    state = {k: v.detach().clone() for k, v in model.state_dict().items()}
    named = dict(model.named_parameters())
    opt = LatentAdam(model.parameters(), lr=LR, clamp_params=binary_params(model))
    for p in model.parameters():
        p.grad = None
    z0 = BF.ZQ_HANDOFFS
    out = model(x)
    loss = torch.nn.functional.cross_entropy(out, y)
    loss.backward()
    assert BF.ZQ_HANDOFFS - z0 == 2
    grads = {k: p.grad.detach().clone() for k, p in named.items()}
    opt.step()
    orc = T.CNNOracle(state, lr=LR, device="cuda")
    loss_ref, out_ref, g_ref = orc.step(x, y, update=False)
    dloss, eout = abs(float(loss) - loss_ref), T.rel_err(out.detach(), out_ref)

    def errors(gr):
        return {k: float(torch.linalg.vector_norm(gr[k].double() - g_ref[k])) if k in CONV_B
                else T.rel_err(gr[k], g_ref[k]) for k in named}

    errs = errors(grads)
    # calibration: the same float64 step with the convolution backward contractions in fp32 (torch
    # fp32 matmul / einsum of the fp32 gradient and the ternary operand, as the reference's F.conv2d
    # backward computes them)
    torch.backends.cuda.matmul.allow_tf32 = False

    def fp32(kind, j, gf, o):
        if kind == "dw":
            return torch.einsum("nol,nkl->ok", gf.float(), o.float()).double()
        return (o.float().T @ gf.float()).double()

    _, _, g32 = T.CNNOracle(state, lr=LR, device="cuda").step(x, y, update=False, bwd=fp32)
    cerrs = {k: float(torch.linalg.vector_norm(g32[k] - g_ref[k])) if k in CONV_B else T.rel_err(g32[k], g_ref[k])
             for k in named}
    print(f"\nBinCNN step B={batch}: loss {float(loss):.6f} vs {loss_ref:.6f} (d {dloss:.1e}), log-probs {eout:.1e}")
    print("  libbnn vs float64:         ", {k: f"{v:.1e}" for k, v in errs.items()})
    print("  fp32-GEMM backward vs f64: ", {k: f"{v:.1e}" for k, v in cerrs.items()})
    assert dloss <= 1e-5, (float(loss), loss_ref)
    assert eout <= 1e-5, eout
    for k, v in errs.items():
        bar = max(1e-5, cerrs[k])
        assert v <= bar, (k, v, f"bar {bar:.2e}: 1e-5, or the fp32-GEMM calibration {cerrs[k]:.2e} where that "
                          "exceeds it")
    upd = {}
    for k in named:
        gk = grads[k].double()
        m, v = 0.1 * gk, 0.001 * gk * gk
        want = state[k].double() - (LR / 0.1) * m / (torch.sqrt(v) / np.sqrt(0.001) + 1e-8)
        if k in CONV_W or k in CONV_B:
            want.clamp_(-1, 1)
        upd[k] = float((named[k].detach().double() - want).abs().max())
        assert upd[k] <= 1e-7, (k, upd[k])
    print(f"  update max {max(upd.values()):.1e}")

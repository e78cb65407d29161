"""Whole-network parity at the BASELINE MLP configurations.

``nets.Net()`` = the reference's ``Net`` at infl_ratio 3 (mnist-dist2.py:46-76: 784-3072-1536-768-10)
runs ONE training step (:118-137, dropout 0) through libbnn and is compared with the float64
oracle (``oracle.bnn_np.MLPOracle``, itself pinned to the reference's traces) at

* batch 100 -- BASELINE config 1's workload (the reference's CPU run);
* batch 4096 -- BASELINE config 3 (``bench.py --config mlp``).

Both GPU paths run: the drop-in (reference call pattern: .org protocol, fp32 input u/255,
torch.optim.Adam + org_protocol_step) and the fused trainer path (u8 pixels, BN -> sign-pack ->
FP4 GEMM, FP6 / int8 hand-offs, fused head, LatentAdam).

Checks:
* fc1's output z1 (continuous: fp32 pixels, or u8 pixels through the exact integer path) against
  float64: norm-wise <= 1e-6;
* everything downstream of z1 against the oracle run FROM THE SAME z1 (MLPOracle.step(z1=...)).
  fc1's input is continuous, so z1 carries fp32 rounding (the reference's own CPU sgemm differs
  from float64 too), and an element within an ulp-scale window of bn1's batch mean takes whichever
  sign that rounding gives it -- a handful of such BatchNorm near-ties per step at batch 4096, each
  moving one sample's output by ~1e-3.  From the same z1 the near-ties resolve identically (libbnn
  keeps the batch mean as an exact hi + lo pair), and the bars are: loss |d| <= 1e-5, log-probs
  norm-wise <= 1e-5, every gradient norm-wise <= 1e-5 (the fc biases feed BatchNorm: exact
  gradient 0, checked absolute);
* the update: every parameter after the step equals torch's Adam (float64) + the clamp applied
  to the GPU's own gradient, elementwise to 1e-7.  The first Adam step moves a weight by
  lr * g / (|g| + eps): for |g| near eps it amplifies the gradient's elementwise rounding, so the
  update is checked on the gradient the step actually had (the gradient is checked above); the
  count of latents that land off the oracle's own update by > 1e-6 is printed.
"""
import numpy as np
import pytest
import torch

from conftest import close, rel_err
from oracle import bnn_np as O

pytestmark = pytest.mark.gpu

TOL = 1e-5
FC_BIAS = ("fc1.bias", "fc2.bias", "fc3.bias")
BINARY_W = ("fc1.weight", "fc2.weight", "fc3.weight")
LR = 0.01
_CACHE = {}


def host(t):
    torch.cuda.synchronize()
    return t.detach().cpu().numpy()


def _case(batch):
    """(initial state, u8 pixels, targets), made once per batch on the host."""
    if batch in _CACHE:
        return _CACHE[batch]
    from bnn_amd import nets
    torch.manual_seed(1000 + batch)
    m = nets.Net(p_drop=0.0)
    state = {k: v.detach().numpy().copy() for k, v in m.state_dict().items()}
    rng = np.random.default_rng(batch)
    u8 = np.where(rng.random((batch, 784)) < 0.807, 0, rng.integers(1, 256, (batch, 784))).astype(np.uint8)
    tgt = rng.integers(0, 10, batch).astype(np.int64)
    _CACHE[batch] = (state, u8, tgt)
    return _CACHE[batch]


def _adam1(p0, g, clamp):
    """torch.optim.Adam's first step (lr LR, betas (0.9, 0.999), eps 1e-8) in float64, + clamp."""
    g = np.asarray(g, np.float64)
    m, v = 0.1 * g, 0.001 * g * g
    new = np.asarray(p0, np.float64) - (LR / 0.1) * m / (np.sqrt(v) / np.sqrt(0.001) + 1e-8)
    return np.clip(new, -1, 1) if clamp else new


@pytest.mark.parametrize("path", ["dropin", "fused"])
@pytest.mark.parametrize("batch", [100, 4096])
def test_net_r3_one_step_vs_oracle(batch, path):
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    from bnn_amd import functional as BF
    from bnn_amd import nets
    from bnn_amd.optim import LatentAdam, org_protocol_step
    state, u8, tgt = _case(batch)
    fused = path == "fused"
    if fused:
        model = nets.Net(p_drop=0.0, org_protocol=False, mutate_input=False, fused_bn=True)
    else:
        model = nets.Net(p_drop=0.0, fused_bn=True)
    model.load_state_dict({k: torch.as_tensor(v) for k, v in state.items()})
    model = model.cuda().train()
    named = dict(model.named_parameters())
    z1 = {}
    model.fc1.register_forward_hook(
        lambda mod, inp, out: z1.__setitem__("z", host(BF.dense_preact(out)).astype(np.float32)))
    if fused:
        opt = LatentAdam(model.parameters(), lr=LR, clamp_params=nets.binary_params(model))
        x = torch.as_tensor(u8).cuda()
        for p in model.parameters():
            p.grad = None
    else:
        opt = torch.optim.Adam(model.parameters(), lr=LR)
        x = torch.as_tensor(u8).cuda().float().div_(255.0)
        opt.zero_grad()
    c0 = (BF.Q6_HANDOFFS, BF.I8C_HANDOFFS, BF.HEAD_CALLS)
    out = model(x)
    loss = torch.nn.functional.cross_entropy(out, torch.as_tensor(tgt).cuda())
    loss.backward()
    if fused:     # the benched fusions ran: two FP6 digit hand-offs, the int8 one to fc1, the head
        assert [a - b for a, b in zip((BF.Q6_HANDOFFS, BF.I8C_HANDOFFS, BF.HEAD_CALLS), c0)] == [2, 1, 1]
    grads = {k: host(p.grad) for k, p in named.items()}
    # fc1 forward against float64 (x = ToTensor(u8) in fp32, as the reference's loader makes it)
    x64 = O.to_tensor(u8).astype(np.float64)
    z1_64 = x64 @ np.sign(state["fc1.weight"]).astype(np.float64).T + state["fc1.bias"]
    ez1 = rel_err(z1["z"], z1_64)
    assert ez1 <= 1e-6, ez1
    # the oracle from the same z1
    orc = O.MLPOracle({k: v for k, v in state.items() if "num_batches" not in k}, lr=LR)
    loss_ref, out_ref, g_ref = orc.step(O.to_tensor(u8), tgt, z1=z1["z"])
    assert abs(loss.item() - loss_ref) <= TOL, (loss.item(), loss_ref)
    assert rel_err(host(out), out_ref) <= TOL
    errs = {}
    for k in named:
        if k in FC_BIAS:
            assert close(grads[k], g_ref[k], 0.0, 1e-5), k
            continue
        errs[k] = rel_err(grads[k], g_ref[k])
        assert errs[k] <= TOL, (k, errs[k])
    if fused:
        opt.step()
    else:
        org_protocol_step(model, opt)
    clamp = set(BINARY_W) | set(FC_BIAS)
    moved = {}
    for k in named:
        got = host(named[k] if fused or k not in BINARY_W else named[k].org).astype(np.float64)
        want = _adam1(state[k], grads[k], k in clamp)
        d = float(np.abs(got - want).max())
        assert d <= 1e-7, (k, d)
        if k in BINARY_W:     # informational: latents off the oracle's own update
            moved[k] = int((np.abs(got - orc.org[k]) > 1e-6).sum())
    print(f"\nNet r=3 batch {batch} {path}: z1 {ez1:.1e}, dloss {abs(loss.item() - loss_ref):.1e}, "
          f"grads {max(errs.values()):.1e}, latents off the oracle's update by >1e-6 (|g| near eps): {moved}")

"""Whole-network parity at the BASELINE MLP configurations.

``nets.Net()`` = the reference's ``Net`` at infl_ratio 3 (mnist-dist2.py:46-76: 784-3072-1536-768-10)
runs ONE training step (:118-137, dropout 0) through libbnn and is compared with the float64
oracle (``oracle.bnn_np.MLPOracle``, itself pinned to the reference's traces) at

* batch 100 -- BASELINE config 1's workload (the reference's CPU run);
* batch 4096 -- BASELINE config 3 (``bench.py --config mlp``).

Both GPU paths run: the drop-in (reference call pattern: .org protocol, fp32 input u/255,
torch.optim.Adam + org_protocol_step) and the fused trainer path (u8 pixels, BN -> sign-pack ->
FP4 GEMM, FP6 / int8 hand-offs, fused head, LatentAdam).

Bars: loss |d| <= 1e-5; log-probs norm-wise <= 1e-5; every step-0 gradient norm-wise <= 1e-5
(the fc biases feed BatchNorm, exact gradient 0: absolute); after the update every latent
weight equals the oracle's to 1e-6 except where the oracle's gradient is within 1e-5 * max|g| of
0 (Adam's first step moves a weight by lr * g / (|g| + eps) ~ +-lr, so a gradient whose sign is
decided by rounding moves it by +-lr either way: tie-aware, as test_gpu_training.py).
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
    """(initial state, u8 pixels, targets, oracle loss / log-probs / grads / latent weights after the
    step), computed once per batch on the host."""
    if batch in _CACHE:
        return _CACHE[batch]
    from bnn_amd import nets
    torch.manual_seed(1000 + batch)
    m = nets.Net(p_drop=0.0)
    state = {k: v.detach().numpy().copy() for k, v in m.state_dict().items()}
    rng = np.random.default_rng(batch)
    u8 = np.where(rng.random((batch, 784)) < 0.807, 0, rng.integers(1, 256, (batch, 784))).astype(np.uint8)
    tgt = rng.integers(0, 10, batch).astype(np.int64)
    orc = O.MLPOracle({k: v for k, v in state.items() if "num_batches" not in k}, lr=LR)
    loss, out, grads = orc.step(O.to_tensor(u8), tgt)
    res = (state, u8, tgt, loss, out, grads, {k: orc.org[k].copy() for k in BINARY_W},
           {k: orc.p[k].copy() for k in orc.p})
    _CACHE[batch] = res
    return res


@pytest.mark.parametrize("path", ["dropin", "fused"])
@pytest.mark.parametrize("batch", [100, 4096])
def test_net_r3_one_step_vs_oracle(batch, path):
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    from bnn_amd import functional as BF
    from bnn_amd import nets
    from bnn_amd.optim import LatentAdam, org_protocol_step
    state, u8, tgt, loss_ref, out_ref, g_ref, org_ref, p_ref = _case(batch)
    fused = path == "fused"
    if fused:
        model = nets.Net(p_drop=0.0, org_protocol=False, mutate_input=False, fused_bn=True)
    else:
        model = nets.Net(p_drop=0.0, fused_bn=True)
    model.load_state_dict({k: torch.as_tensor(v) for k, v in state.items()})
    model = model.cuda().train()
    named = dict(model.named_parameters())
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
    assert abs(loss.item() - loss_ref) <= TOL, (loss.item(), loss_ref)
    assert rel_err(host(out), out_ref) <= TOL
    errs = {}
    for k, p in named.items():
        got = host(p.grad)
        if k in FC_BIAS:
            assert close(got, g_ref[k], 0.0, 1e-5), k
            continue
        errs[k] = rel_err(got, g_ref[k])
        assert errs[k] <= TOL, (k, errs[k])
    if fused:
        opt.step()
    else:
        org_protocol_step(model, opt)
    flips = {}
    for k in BINARY_W:
        got = host(named[k] if fused else named[k].org).astype(np.float64)
        g = g_ref[k]
        tie = np.abs(g) <= 1e-5 * np.abs(g).max()
        bad = np.abs(got - org_ref[k]) > 1e-6
        assert not (bad & ~tie).any(), (k, int((bad & ~tie).sum()))
        flips[k] = int(bad.sum())
    for k in ("bn1.weight", "bn2.weight", "bn3.weight", "fc4.weight", "fc4.bias"):
        assert close(host(named[k]), p_ref[k], 1e-6, 1e-7), k
    print(f"\nNet r=3 batch {batch} {path}: dloss {abs(loss.item() - loss_ref):.1e}, "
          f"grads {max(errs.values()):.1e}, tie-moved latents {flips}")

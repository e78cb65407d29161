"""Whole-step parity at BASELINE config 5's real size -- the bench's own workload.

``bench.py`` times ``nets.MODELS["wide"]`` (784-8192x3-10, dropout 0.3) at 65,536 samples per GPU
on u8 pixels, through the fused path: fc1 on the bytes with bn1's forward statistics from its
epilogue (PIX_STATS), fc2's FP4 GEMM with bn2's statistics from its epilogue (FP4_STATS), int16
pre-activations (z16), the drop->bn3->htanh3->fc4 head, the FP6 digit hand-offs of the BatchNorm
backwards (q6), the int8 column digits to fc1's weight gradient (i8cols), and the fused
Adam + clamp + FP4 re-pack.  At that size several of those kernels run far beyond what the
kernel-level tests cover (5.4e8 elements per activation, > 2^31 bytes of fp32).

test_wide_step_config5_vs_float64 runs ONE such step (model and batch built exactly as bench.py
builds them: bench.build, bench.CONFIGS, data.synthetic_mnist seed 1234) and checks it against the
float64 oracle (oracle/bnn_t64.py, pinned to the reference's traces on the CPU) on the GPU:

* every fusion above fired (hand-off counters);
* fc1's output z1 against float64 (<= 1e-6 norm-wise); everything downstream against the oracle
  run FROM THE GPU's z1 (fc1's input is continuous, so z1's fp32 rounding decides bn1's
  near-ties; see test_gpu_net_configs.py) with the GPU's own dropout keep mask injected (the
  build's masks come from a hash, not torch's Philox stream: DESIGN.md §8) -- loss |d| <= 1e-5,
  log-probs <= 1e-5, every gradient <= 1e-5 norm-wise (the fc biases feed BatchNorm: exact
  gradient 0, checked absolute) except the hidden BatchNorm biases, <= 5e-5 (cancellation:
  BN_BIAS_TOL);
* Hardtanh-boundary columns: at this batch a few columns of a BatchNorm hold elements whose output
  lies within 2^-20 of +-1 (oracle.bnn_t64.TAU), where the strict backward mask 1[-1 < y < 1] is
  decided by the last bits of y: fp32 (libbnn, the reference) and float64 can disagree there, and
  the column's gradient then differs by one whole masked term (observed: 2 of 8192 columns of bn1,
  their fc1 weight-gradient rows 1e-2 off; every other row <= 1e-5).  Those columns' entries of
  bn_i's gradients and rows of fc_i's weight gradient are compared separately (reported, at most
  1 % of the columns), every other entry at 1e-5 -- as BatchNorm near-ties are resolved by
  anchoring on the GPU's z1;
* the reference's own arithmetic, torch fp32 (oracle/bnn_torch.py RefMLP, same state, input and
  mask, against float64 from ITS z1), is reported beside it for scale;
* the update: every parameter after LatentAdam equals torch's Adam (float64) + the clamp on the
  GPU's own gradient, elementwise <= 1e-7.

test_wide_bench_loss_vs_reference_semantics records the loss of the bench's first 25 steps (its
batch, seed, lr and dropout) beside the reference semantics on torch fp32 on the same GPU
(oracle/bnn_torch.py RefMLP + the .org protocol, torch's dropout) run twice with different
dropout seeds: the spread of those two is the band the fused path is held to (mean of the last 10
steps), and the curves are printed (why the loss of this workload sits above ln 10).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

TOL = 1e-5
# A hidden BatchNorm's bias gradient is the batch sum of its (masked) upstream gradient dy, and dy
# is the next BatchNorm's gradient multiplied through a linear layer: it sums to ~0 over the batch
# (BatchNorm's backward output does exactly), so |dbeta| is orders below sum|dy| and the FP6
# operand's 2^-19-of-block-maximum rounding of dy (~2e-6 per element) is amplified in it.  At
# B = 65,536 measured 1.5e-5 / 1.6e-5 (bn2 / bn1; every other gradient <= 3.1e-6); the reference's
# own fp32 arithmetic lands 1.2e-2..1.8e-2 from float64 on these same entries.
BN_BIAS_TOL = {"bn1.bias": 5e-5, "bn2.bias": 5e-5, "bn3.bias": 5e-5}
FC_BIAS = ("fc1.bias", "fc2.bias", "fc3.bias")
BINARY_W = ("fc1.weight", "fc2.weight", "fc3.weight")
LR = 0.01


def _bench_setup():
    import bench
    from bnn_amd.data import synthetic_mnist
    batch = bench.CONFIGS["wide"][1]
    torch.manual_seed(0)                                   # bench.main: seed, then build
    model = bench.build("wide", "fp4").cuda().train()
    x, y = synthetic_mnist(batch, seed=1234, device=torch.device("cuda"), as_u8=True)
    return model, x, y


def _counters(BF):
    return {k: getattr(BF, k) for k in ("PIX_STATS_USES", "FP4_STATS_USES", "Z16_HANDOFFS", "Q6_HANDOFFS",
                                         "I8C_HANDOFFS", "HEAD_CALLS", "S20_HANDOFFS")}


class _MaskDrop(torch.nn.Module):
    """nn.Dropout with a given scaled keep mask: fl(x * mask) in fp32, as torch's dropout forms it."""

    def __init__(self, mask):
        super().__init__()
        self.mask = mask

    def forward(self, x):
        return x * self.mask


def _errors(grads, g_ref, names):
    """Norm-wise relative error per parameter (the fc biases feed BatchNorm: exact gradient 0,
    absolute norm)."""
    from oracle import bnn_t64 as T
    out = {}
    for k in names:
        if k in FC_BIAS:
            out[k] = float(torch.linalg.vector_norm(grads[k].double() - g_ref[k]))
        else:
            out[k] = T.rel_err(grads[k], g_ref[k])
    return out


def _row_errors(a, b):
    """Per-row relative errors of a [N, K] gradient against float64 b: (median, max, rows > 1e-4)."""
    d = torch.linalg.vector_norm(a.double() - b, dim=1) / torch.linalg.vector_norm(b, dim=1).clamp_min(1e-300)
    return float(d.median()), float(d.max()), int((d > 1e-4).sum())


def test_wide_step_config5_vs_float64(monkeypatch):
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    from bnn_amd import functional as BF
    from bnn_amd.nets import binary_params
    from bnn_amd.optim import LatentAdam
    from oracle import bnn_t64 as T
    from oracle.bnn_torch import RefMLP
    model, x, y = _bench_setup()
    B, C = x.shape[0], model.fc2.in_features
    p_drop = model.drop.p
    assert (B, C, p_drop) == (65536, 8192, 0.3)
    state = {k: v.detach().clone() for k, v in model.state_dict().items()}
    named = dict(model.named_parameters())
    opt = LatentAdam(model.parameters(), lr=LR, clamp_params=binary_params(model))
    seeds = []
    draw = BF.dropout_seed
    monkeypatch.setattr(BF, "dropout_seed", lambda: seeds.append(draw()) or seeds[-1])
    z1 = {}
    hook = model.fc1.register_forward_hook(lambda mod, inp, out: z1.__setitem__("z", BF.dense_preact(out).detach()))
    c0 = _counters(BF)
    for p in model.parameters():
        p.grad = None
    out = model(x)
    loss = torch.nn.functional.cross_entropy(out, y)
    loss.backward()
    hook.remove()
    c1 = _counters(BF)
    fired = {k: c1[k] - c0[k] for k in c0}
    assert fired == {"PIX_STATS_USES": int(BF.PIX_STATS), "FP4_STATS_USES": int(BF.FP4_STATS), "Z16_HANDOFFS": 2,
                     "Q6_HANDOFFS": 2, "I8C_HANDOFFS": 1, "HEAD_CALLS": 1,
                     "S20_HANDOFFS": int(BF.S20 and BF.PIX_STATS)}, fired
    assert len(seeds) == 1, seeds
    grads = {k: p.grad.detach().clone() for k, p in named.items()}
    out = out.detach()
    loss_gpu = float(loss)
    opt.step()
    torch.cuda.synchronize()
    after = {k: p.detach().clone() for k, p in named.items()}
    del opt, loss, model
    torch.cuda.empty_cache()

    # fc1's output against float64 (x = ToTensor(u8) in fp32, as the reference's loader makes it)
    xf = x.view(B, 784).float().div(255.0)
    z1_64 = xf.double() @ torch.sign(state["fc1.weight"].double()).T + state["fc1.bias"].double()
    ez1 = T.rel_err(z1["z"], z1_64)
    del z1_64
    # the oracle from the GPU's z1, with the GPU's dropout mask
    mask = BF.dropout_mask(B * C, p_drop, seeds[0]).view(B, C)
    orc = T.MLPOracle(state, lr=LR, device="cuda")
    loss_ref, out_ref, g_ref = orc.step(xf, y, z1=z1["z"], drop=mask, update=False)
    del z1
    dloss = abs(loss_gpu - loss_ref)
    eout = T.rel_err(out, out_ref)
    errs = _errors(grads, g_ref, named)
    rows1 = _row_errors(grads["fc1.weight"], g_ref["fc1.weight"])
    # the Hardtanh-boundary columns of each hidden BatchNorm, and the errors without them
    bcols = [b > 0 for b in orc.boundary]
    inner = {}
    for i, l in enumerate(("fc1", "fc2", "fc3")):
        keep = ~bcols[i]
        for k in (f"{l}.weight", f"bn{i + 1}.weight", f"bn{i + 1}.bias"):
            inner[k] = T.rel_err(grads[k][keep], g_ref[k][keep])
        for k in (f"{l}.weight", f"bn{i + 1}.weight", f"bn{i + 1}.bias"):
            if bool(bcols[i].any()):
                errs[k + "@boundary"] = T.rel_err(grads[k][bcols[i]], g_ref[k][bcols[i]])
    nbound = [int(b.sum()) for b in bcols]
    del g_ref, out_ref
    del orc
    torch.cuda.empty_cache()

    # for scale: the reference's own arithmetic (torch fp32 F.linear / BatchNorm1d / autograd,
    # oracle/bnn_torch.py RefMLP) on the same state, input and dropout mask, against the float64
    # oracle run from ITS z1 -- how far an fp32 implementation of the reference is from float64 here
    ref = RefMLP(C, C, C, p_drop=0.0)
    ref.load_state_dict({k: v.cpu() for k, v in state.items()})
    ref.drop = _MaskDrop(mask)
    ref = ref.cuda().train()
    zr = {}
    ref.fc1.register_forward_hook(lambda mod, inp, o: zr.__setitem__("z", o.detach().clone()))
    lt = torch.nn.functional.cross_entropy(ref(xf.clone()), y)
    lt.backward()
    tgrads = {k: p.grad.detach() for k, p in ref.named_parameters()}
    orc = T.MLPOracle(state, lr=LR, device="cuda")
    tloss_ref, _, tg_ref = orc.step(xf, y, z1=zr["z"], drop=mask, update=False)
    terrs = _errors(tgrads, tg_ref, named)
    trows1 = _row_errors(tgrads["fc1.weight"], tg_ref["fc1.weight"])
    del orc, tg_ref, tgrads, ref, zr
    torch.cuda.empty_cache()
    print(f"\nconfig 5 step (B={B}, p={p_drop}): z1 {ez1:.1e}, loss {loss_gpu:.6f} vs {loss_ref:.6f} (d {dloss:.1e}), "
          f"log-probs {eout:.1e}")
    print("  libbnn vs float64:     ", {k: f"{v:.1e}" for k, v in errs.items()})
    print(f"  Hardtanh-boundary columns per hidden BatchNorm: {nbound}; without them:",
          {k: f"{v:.1e}" for k, v in inner.items()})
    print("  torch fp32 vs float64: ", {k: f"{v:.1e}" for k, v in terrs.items()},
          f"(loss d {abs(float(lt) - tloss_ref):.1e})")
    print(f"  fc1.weight per-row error (median, max, rows > 1e-4): libbnn {rows1}, torch fp32 {trows1}")
    assert ez1 <= 1e-6, ez1
    assert dloss <= TOL, (loss_gpu, loss_ref)
    assert eout <= TOL, eout
    for n, h in zip(nbound, (C, C, C)):
        assert n <= h // 100, nbound
    for k, v in errs.items():
        if "@" in k:
            continue
        assert inner.get(k, v) <= BN_BIAS_TOL.get(k, TOL), (k, v, inner.get(k))
    # the update: torch.optim.Adam's first step in float64 on the GPU's own gradient, + clamp
    clamp = set(BINARY_W) | set(FC_BIAS)
    upd = {}
    for k in named:
        g = grads[k].double()
        m, v = 0.1 * g, 0.001 * g * g
        want = state[k].double() - (LR / 0.1) * m / (torch.sqrt(v) / np.sqrt(0.001) + 1e-8)
        if k in clamp:
            want.clamp_(-1, 1)
        upd[k] = float((after[k].double() - want).abs().max())
        assert upd[k] <= 1e-7, (k, upd[k])
    print(f"  update max {max(upd.values()):.1e}")


STEPS = 25


def test_wide_bench_loss_vs_reference_semantics():
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    from bnn_amd.nets import binary_params
    from bnn_amd.optim import LatentAdam
    from oracle.bnn_torch import RefMLP, train_step
    model, x, y = _bench_setup()
    state = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    opt = LatentAdam(model.parameters(), lr=LR, clamp_params=binary_params(model))
    crit = torch.nn.CrossEntropyLoss()
    L = []
    for _ in range(STEPS):                                # bench.main's step()
        for p in model.parameters():
            p.grad = None
        loss = crit(model(x), y)
        loss.backward()
        opt.step()
        L.append(loss.detach())
    L = np.array([float(v) for v in L])
    del model, opt
    torch.cuda.empty_cache()
    xf = x.float().div(255.0)
    curves = []
    for seed in (100, 200):
        torch.manual_seed(seed)                           # torch's dropout masks (Philox)
        ref = RefMLP(8192, 8192, 8192, p_drop=0.3)
        ref.load_state_dict(state)
        ref = ref.cuda().train()
        ropt = torch.optim.Adam(ref.parameters(), lr=LR)
        curves.append(np.array([train_step(ref, ropt, xf.clone(), y, True) for _ in range(STEPS)]))
        del ref, ropt
        torch.cuda.empty_cache()
    T1, T2 = curves
    tail = lambda a: float(a[-10:].mean())   # noqa: E731
    band = max(2 * abs(tail(T1) - tail(T2)), 0.05 * tail(T1))
    print("\nwide bench workload, loss per step (libbnn fused, hash dropout):", " ".join(f"{v:.3f}" for v in L))
    print("reference semantics torch fp32, dropout seed 100             :", " ".join(f"{v:.3f}" for v in T1))
    print("reference semantics torch fp32, dropout seed 200             :", " ".join(f"{v:.3f}" for v in T2))
    print(f"mean of the last 10 steps: libbnn {tail(L):.4f}, torch {tail(T1):.4f} / {tail(T2):.4f} (band {band:.4f}); "
          f"step 0: {L[0]:.5f} / {T1[0]:.5f} / {T2[0]:.5f}")
    assert abs(L[0] - T1[0]) <= 0.01 and abs(T1[0] - T2[0]) <= 0.01    # same init, masks differ
    assert abs(tail(L) - tail(T1)) <= band

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
  build's masks come from a hash, not torch's Philox stream: DESIGN.md §8);
* anchored on the GPU's Hardtanh decisions at the boundary: an element whose BatchNorm output lies
  within 2^-20 of +-1 (oracle.bnn_t64.TAU) gets the strict backward mask 1[-1 < y < 1] from the
  last bits of y, which fp32 (libbnn, the reference) and float64 can decide differently (observed:
  64 of bn1's 8192 columns hold such elements, 2 of them decided differently, each moving a whole
  fc1 weight-gradient row by 1e-2).  The oracle takes those elements' masks from y formed with
  libbnn's fp32 arithmetic (bn_dz1: ((z - mean) - mean_lo) * invstd, fma with gamma, beta) on the
  GPU's own batch statistics (functional.STATS_TAP), and asserts every element OUTSIDE the window
  gets the same decision from that y as from float64's (so the anchor changes nothing but the
  window);
* then: loss |d| <= 1e-5, log-probs <= 1e-5, EVERY gradient <= 1e-5 norm-wise, all columns
  included (the fc biases feed BatchNorm: exact gradient 0, checked absolute);
* calibration of the backward GEMMs' arithmetic (printed, and the bar where it exceeds 1e-5): the
  same anchored oracle step with the dX / dW products in fp32 (torch fp32 matmul of the fp32 dz
  and the ternary operand -- the reference's arithmetic for these GEMMs), and in emulations of
  libbnn's operand: dz rounded per 32-element block to 2^(e-19) (FP6 4 digit planes), with a
  float64 or an fp32 product, and with 5 planes.  A gradient whose fp32-GEMM calibration itself
  exceeds 1e-5 is held to that number (named in the assertion);
* the update: every parameter after LatentAdam equals torch's Adam (float64) + the clamp on the
  GPU's own gradient, elementwise <= 1e-7.

test_wide_bench_loss_same_masks records the loss of the bench's first 25 steps (its batch, seed,
lr and dropout) beside the reference semantics on torch fp32 on the same GPU (oracle/bnn_torch.py
RefMLP + the .org protocol) driven by libbnn's own dropout masks, so the two differ only in
arithmetic; the band is the spread of the reference run under row permutations of the batch, and
the curves are printed (why the loss of this workload sits above ln 10).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

TOL = 1e-5
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


def libbnn_y(stats, gamma, beta):
    """The BatchNorm output as libbnn's backward passes form it for the Hardtanh mask (csrc
    bnn_common.h bn_dz1: xh = ((x - mean) - mean_lo) * invstd, y = fma(xh, gamma, beta)), from the
    GPU's fp32 statistics: each torch fp32 op rounds once; the fma's product is exact in float64
    and its sum rounds once there, then to fp32."""
    mean, invstd, mlo = stats[0], stats[1], stats[2]
    g64, b64 = gamma.double(), beta.double()

    def f(z):
        xh = ((z.float() - mean) - mlo) * invstd
        return (xh.double() * g64 + b64).float()
    return f


def fp6_round(g, dim, planes=4):
    """libbnn's FP6 digit operand of an fp32 gradient, emulated in float64: each 32-element block
    along ``dim`` (the GEMM's contraction) rounded to the step 2^(e - 19 - 5 (planes - 4)), e the
    exponent with max|block| in [2^(e-1), 2^e) (bnn_fp6.h block_scale, rint)."""
    x = g.float().double().movedim(dim, -1)
    shp = x.shape
    blk = x.reshape(*shp[:-1], shp[-1] // 32, 32)
    amax = blk.abs().amax(-1, keepdim=True)
    e = torch.frexp(amax).exponent
    step = torch.ldexp(torch.ones_like(amax), e - 19 - 5 * (planes - 4))
    q = torch.where(amax > 0, torch.round(blk / step) * step, torch.zeros_like(blk))
    return q.reshape(shp).movedim(-1, dim)


def calib_bwd(mode):
    """Backward GEMM arithmetic of a calibration run (oracle ``bwd``): "fp32" = torch fp32 matmul
    of the fp32 dz and the ternary operand; "fp6" / "fp6_f32acc" / "fp6_rows5" = libbnn's FP6 digit
    operand (column digits for dW, row digits for dX) with a float64 / fp32 product / 5 planes on
    the dX operand.  fc1's weight gradient (libbnn: int8 column digits) stays exact in the FP6
    emulations."""
    def f(kind, i, g, o):
        if mode == "fp32":
            a = g.float()
            return (a.T @ o.float() if kind == "dw" else a @ o.float()).double()
        if kind == "dw":
            if i == 0:
                return g.T @ o
            q = fp6_round(g, 0)
            return (q.float().T @ o.float()).double() if mode == "fp6_f32acc" else q.T @ o
        q = fp6_round(g, 1, 5 if mode == "fp6_rows5" else 4)
        return (q.float() @ o.float()).double() if mode == "fp6_f32acc" else q @ o
    return f


CALIB = ("fp32", "fp6", "fp6_f32acc", "fp6_rows5")


def test_wide_step_config5_vs_float64(monkeypatch):
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    from bnn_amd import functional as BF
    from bnn_amd.nets import binary_params
    from bnn_amd.optim import LatentAdam
    from oracle import bnn_t64 as T
    torch.backends.cuda.matmul.allow_tf32 = False
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
    stats = []
    monkeypatch.setattr(BF, "STATS_TAP", stats)
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
    assert len(stats) == 3 and all(s.shape == (3, C) for s in stats), [s.shape for s in stats]
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
    # the oracle from the GPU's z1, with the GPU's dropout mask, anchored on its Hardtanh decisions
    mask = BF.dropout_mask(B * C, p_drop, seeds[0]).view(B, C)
    ys = [libbnn_y(stats[i], state[f"bn{i + 1}.weight"], state[f"bn{i + 1}.bias"]) for i in range(3)]
    anchor = lambda i, z: ys[i](z)      # noqa: E731

    def run(bwd=None):
        orc = T.MLPOracle(state, lr=LR, device="cuda")
        r = orc.step(xf, y, z1=z1["z"], drop=mask, update=False, anchor=anchor, bwd=bwd)
        return r, orc.boundary, orc.anchored

    (loss_ref, out_ref, g_ref), boundary, anchored = run()
    dloss = abs(loss_gpu - loss_ref)
    eout = T.rel_err(out, out_ref)
    errs = _errors(grads, g_ref, named)
    rows1 = _row_errors(grads["fc1.weight"], g_ref["fc1.weight"])
    nbound = [int(b.gt(0).sum()) for b in boundary]
    del out_ref
    torch.cuda.empty_cache()
    calib = {}
    for mode in CALIB:
        (_, _, gc), _, _ = run(calib_bwd(mode))
        calib[mode] = _errors(gc, g_ref, named)
        del gc
        torch.cuda.empty_cache()
    del g_ref
    print(f"\nconfig 5 step (B={B}, p={p_drop}): z1 {ez1:.1e}, loss {loss_gpu:.6f} vs {loss_ref:.6f} "
          f"(d {dloss:.1e}), log-probs {eout:.1e}")
    print(f"  Hardtanh-boundary columns per hidden BatchNorm: {nbound}; anchored (changed in window, "
          f"differing outside): {anchored}")
    print(f"  fc1.weight per-row error (median, max, rows > 1e-4): {rows1}")
    names = [k for k in named]
    print("  " + "gradient".ljust(12) + "libbnn".rjust(9) + "".join(m.rjust(12) for m in CALIB))
    for k in names:
        print("  " + k.ljust(12) + f"{errs[k]:9.1e}" + "".join(f"{calib[m][k]:12.1e}" for m in CALIB))
    assert ez1 <= 1e-6, ez1
    assert dloss <= TOL, (loss_gpu, loss_ref)
    assert eout <= TOL, eout
    for i, (chg, outside) in enumerate(anchored):
        assert outside == 0, (i, anchored)               # the anchor decides only inside the window
    for k, v in errs.items():
        bar = max(TOL, calib["fp32"][k])
        assert v <= bar, (k, v, f"bar {bar:.2e}: 1e-5, or the fp32-GEMM calibration {calib['fp32'][k]:.2e} "
                          "where that exceeds it")
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


def test_wide_bench_loss_same_masks():
    """The bench workload against the reference semantics (torch fp32 RefMLP, the reference's .org
    protocol) driven by libbnn's OWN dropout masks: the seeds the fused head draws are recorded and
    the reference's dropout multiplies by bnn_dropout_mask of the same seed, so the runs differ only
    in arithmetic (FP6 digit planes and fixed-order sums against torch's fp32 GEMMs and BatchNorm).
    Calibration: the same reference run on the batch in another row order (masks permuted with it)
    -- the same math in another fp32 summation order.  Bars: step 0 within 1e-4; steps 1-2 (before
    the Adam steps at lr 0.01 have inflated the logits -- mnist-dist2.py's own dynamics, after which
    fp32 rounding differences grow chaotically) within 2e-3 relative; the mean of the last 10 steps
    within 1.5 x the calibration spread -- the largest gap between the tail means of the reference
    run and two row-permuted copies of it (three arithmetic orders of the same math).  (Round 5 held
    it to 3 x one permutation's gap; the differing-mask comparison this test superseded allowed 28 %.)"""
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    from bnn_amd import _lib as L
    from bnn_amd import functional as BF
    from bnn_amd.nets import binary_params
    from bnn_amd.optim import LatentAdam
    from oracle.bnn_torch import RefMLP, train_step
    model, x, y = _bench_setup()
    state = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    seeds = []
    orig = BF.dropout_seed

    def recording_seed():
        s = orig()
        seeds.append(int(s))
        return s

    BF.dropout_seed = recording_seed
    try:
        opt = LatentAdam(model.parameters(), lr=LR, clamp_params=binary_params(model))
        crit = torch.nn.CrossEntropyLoss()
        Lb = []
        for _ in range(STEPS):
            for p in model.parameters():
                p.grad = None
            loss = crit(model(x), y)
            loss.backward()
            opt.step()
            Lb.append(loss.detach())
    finally:
        BF.dropout_seed = orig
    Lb = np.array([float(v) for v in Lb])
    assert len(seeds) == STEPS, "the fused head drew one dropout seed per step"
    p_drop = model.drop.p
    del model, opt
    torch.cuda.empty_cache()

    class SeedDrop(torch.nn.Module):
        """x * bnn_dropout_mask(seed) (kept values x / (1 - p), as torch), rows in `order`."""

        def __init__(self, order):
            super().__init__()
            self.i, self.order = 0, order

        def forward(self, z):
            m = torch.empty(z.numel(), device=z.device)
            L.call("bnn_dropout_mask", z.numel(), float(p_drop), seeds[self.i], L.ptr(m), L.stream())
            self.i += 1
            m = m.view_as(z)
            return z * (m if self.order is None else m[self.order])

    def reference(order):
        ref = RefMLP(8192, 8192, 8192, p_drop=p_drop)
        ref.load_state_dict(state)
        ref = ref.cuda().train()
        ref.drop = SeedDrop(order)
        ropt = torch.optim.Adam(ref.parameters(), lr=LR)
        xf = x.float().div(255.0)
        yy = y
        if order is not None:
            xf, yy = xf[order], y[order]
        out = np.array([train_step(ref, ropt, xf.clone(), yy, True) for _ in range(STEPS)])
        del ref, ropt
        torch.cuda.empty_cache()
        return out

    T = reference(None)
    Tp = reference(torch.randperm(x.shape[0], generator=torch.Generator().manual_seed(5)).cuda())
    Tq = reference(torch.randperm(x.shape[0], generator=torch.Generator().manual_seed(6)).cuda())
    tail = lambda a: float(a[-10:].mean())   # noqa: E731
    rel = np.abs(Lb - T) / np.abs(T)
    calib = max(abs(tail(T) - tail(Tp)), abs(tail(T) - tail(Tq)), abs(tail(Tp) - tail(Tq)))
    bar = 1.5 * calib
    print("\nwide bench workload, same dropout masks: libbnn", " ".join(f"{v:.4f}" for v in Lb))
    print("reference semantics torch fp32, libbnn's masks  ", " ".join(f"{v:.4f}" for v in T))
    print("the same, batch rows permuted (calibration)     ", " ".join(f"{v:.4f}" for v in Tp))
    print("the same, another row permutation (calibration) ", " ".join(f"{v:.4f}" for v in Tq))
    print(f"relative gap per step: {' '.join(f'{v:.1e}' for v in rel)}")
    print(f"tail means: libbnn {tail(Lb):.4f}, torch {tail(T):.4f}, permuted {tail(Tp):.4f} / {tail(Tq):.4f}; "
          f"|libbnn - torch| {abs(tail(Lb) - tail(T)):.4f} against bar {bar:.4f} (calibration spread {calib:.4f})")
    assert abs(Lb[0] - T[0]) <= 1e-4
    assert np.all(rel[1:3] <= 2e-3)
    assert abs(tail(Lb) - tail(T)) <= bar

"""Loss curves on real MNIST: the build's fused training path against the reference's semantics.

Data: the MNIST t10k images / labels the reference ships (tests/golden/t10k-*-idx1/3-ubyte.gz),
10,000 samples in the DistributedSampler order the reference trains in (seed 0, no set_epoch:
every epoch repeats it, mnist-dist2.py:100-108), batch 100, 3 epochs = 300 steps, Adam lr 0.01,
the mnist-dist2.py:46-76 Net at infl_ratio 1 (784-1024-512-256-10), dropout 0 (every
implementation draws its own dropout masks), same initial weights.

Runs, on this GPU:
* L -- the build's fused trainer path (u8 pixels, libbnn layers, LatentAdam);
* T -- the reference's semantics on torch fp32 (oracle/bnn_torch.py: sign() + F.linear,
  BatchNorm1d, Hardtanh, Adam + the .org protocol), fp32 input u/255;
* T1 -- T with ONE fc2 latent weight (the one nearest 0) negated at start: the calibration.  A
  binarized network's trajectory is chaotic in its binarized weights -- one sign that differs
  (which a last-bit difference in a near-zero gradient produces, see test_gpu_wide_trace.py)
  decorrelates the per-step losses -- so "the same loss curve" means agreeing as closely as the
  reference agrees with itself after one flipped weight.

Bars: over 25-step windows, the mean loss of L is within max(2 x the largest
window gap |T1 - T|, 0.02) of T's; both learn (last window's mean loss below half of the
first's); training-set accuracy after the 300 steps within 1.5 points of T's.

With dropout on (p = 0.3 before bn3, mnist-dist2.py:69; test_mnist_loss_curve_dropout): L draws
its keep masks from the build's hash, T from torch's Philox stream, so no two runs
share a mask; both are sampled over several dropout seeds and their means compared, the bands set
by the spread of torch's own seeds (accuracy measured in eval mode, dropout off).
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

WIDTHS = (1024, 512, 256)
BATCH, EPOCHS, LR, WIN = 100, 3, 0.01, 25


def _data():
    from bnn_amd.data import load_idx_dataset, shard_indices
    x, y = load_idx_dataset(os.path.join(GOLDEN, "t10k-images-idx3-ubyte.gz"),
                            os.path.join(GOLDEN, "t10k-labels-idx1-ubyte.gz"), "cuda")
    order = torch.tensor(shard_indices(len(x), 1, 0), device="cuda")
    return x.view(len(x), 784), y, order


def _batches(order):
    nb = len(order) // BATCH
    for _ in range(EPOCHS):
        for b in range(nb):
            yield order[b * BATCH:(b + 1) * BATCH]


def _accuracy(model, x, y, fp32):
    model.eval()
    with torch.no_grad():
        correct = 0
        for i in range(0, len(x), 1000):
            xb = x[i:i + 1000]
            out = model(xb.float() / 255.0 if fp32 else xb)
            correct += int((out.argmax(1) == y[i:i + 1000]).sum())
    model.train()
    return correct / len(x)


def _run_libbnn(state, x, y, order, p_drop=0.0, seed=0):
    from bnn_amd import nets
    from bnn_amd.optim import LatentAdam
    torch.manual_seed(seed)                 # the fused dropout draws its seeds from torch's CPU RNG
    m = nets.MLP(*WIDTHS, p_drop=p_drop, org_protocol=False, mutate_input=False, fused_bn=True)
    m.load_state_dict(state)
    m = m.cuda().train()
    opt = LatentAdam(m.parameters(), lr=LR, clamp_params=nets.binary_params(m))
    losses = []
    for sel in _batches(order):
        for p in m.parameters():
            p.grad = None
        loss = torch.nn.functional.cross_entropy(m(x[sel]), y[sel])
        loss.backward()
        opt.step()
        losses.append(loss.detach())
    return np.array([float(v) for v in losses]), _accuracy(m, x, y, fp32=False)


def _run_torch(state, x, y, order, flip=False, p_drop=0.0, seed=0):
    from oracle.bnn_torch import RefMLP, train_step
    torch.manual_seed(seed)                 # torch's dropout masks (the CUDA generator)
    m = RefMLP(*WIDTHS, p_drop=p_drop)
    m.load_state_dict(state)
    if flip:
        with torch.no_grad():
            w = m.fc2.weight.view(-1)
            i = int(torch.argmin(w.abs()))
            w[i] = -w[i]
    m = m.cuda().train()
    opt = torch.optim.Adam(m.parameters(), lr=LR)
    losses = [train_step(m, opt, x[sel].float() / 255.0, y[sel], True) for sel in _batches(order)]
    return np.array(losses), _accuracy(m, x, y, fp32=True)


def _windows(a):
    return a[: len(a) // WIN * WIN].reshape(-1, WIN).mean(1)


def test_mnist_loss_curve_matches_reference_semantics():
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    from bnn_amd import nets
    torch.manual_seed(5)
    state = {k: v.clone() for k, v in nets.MLP(*WIDTHS, p_drop=0.0).state_dict().items()}
    x, y, order = _data()
    L, accL = _run_libbnn(state, x, y, order)
    T, accT = _run_torch(state, x, y, order)
    T1, accT1 = _run_torch(state, x, y, order, flip=True)
    w = _windows
    wl, wt, wt1 = w(L), w(T), w(T1)
    band = max(2 * float(np.abs(wt1 - wt).max()), 0.02)
    print("\nwindow mean loss  libbnn:", " ".join(f"{v:.3f}" for v in wl))
    print("window mean loss  torch :", " ".join(f"{v:.3f}" for v in wt))
    print("window mean loss  torch1:", " ".join(f"{v:.3f}" for v in wt1))
    print(f"first exact split: libbnn step {int(np.argmax(np.abs(L - T) > 1e-5))}, torch1 step "
          f"{int(np.argmax(np.abs(T1 - T) > 1e-5))}; max window gap libbnn {np.abs(wl - wt).max():.4f}, "
          f"torch1 {np.abs(wt1 - wt).max():.4f} (band {band:.4f}); accuracy libbnn {accL:.4f}, torch {accT:.4f}, "
          f"torch1 {accT1:.4f}")
    assert np.abs(wl - wt).max() <= band
    assert wl[-1] < 0.5 * wl[0] and wt[-1] < 0.5 * wt[0]
    assert abs(accL - accT) <= 0.015


LIBBNN_SEEDS = tuple(range(100, 108))
TORCH_SEEDS = tuple(range(200, 208))


def test_mnist_loss_curve_dropout():
    """p = 0.3 (mnist-dist2.py:69), the bench's dropout: the fused path's hash masks against torch's
    dropout.  No two runs share a mask, so both sides are sampled over 8 dropout seeds each and
    their MEANS are compared: window losses of the mean curves within max(2 x the largest window gap
    between the mean curves of torch's two seed halves, 0.02); mean training accuracy within 3
    standard errors of the difference of the two means (the seed-to-seed spread, estimated from all
    16 runs, so one outlying seed cannot set the bar), at least 0.5 points.
    History: round 5's single-seed form failed once at 1.54 points (94.21 % against 95.75 / 95.30 %,
    a sample of one), and its replacement's bar -- the range of 4 torch seeds -- let one outlier set
    it.  With 8 seeds per side (profiles/r06_a_dropout_spread.log): libbnn 95.13 % +- 0.29 (s.e.),
    BNN_FP6_RES=0 95.35 +- 0.32, BNN_KEEP_BITS=0 95.13 (bit-identical masks), torch 94.57 +- 0.45:
    neither round-5 change moved the accuracy beyond seed noise."""
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    from bnn_amd import nets
    torch.manual_seed(5)
    state = {k: v.clone() for k, v in nets.MLP(*WIDTHS, p_drop=0.3).state_dict().items()}
    x, y, order = _data()
    runs_l = [_run_libbnn(state, x, y, order, p_drop=0.3, seed=s) for s in LIBBNN_SEEDS]
    runs_t = [_run_torch(state, x, y, order, p_drop=0.3, seed=s) for s in TORCH_SEEDS]
    wl = np.mean([_windows(r[0]) for r in runs_l], axis=0)
    wts = [_windows(r[0]) for r in runs_t]
    wt = np.mean(wts, axis=0)
    h = len(wts) // 2
    half = np.abs(np.mean(wts[:h], axis=0) - np.mean(wts[h:], axis=0))
    band = max(2 * float(half.max()), 0.02)
    acc_l, acc_t = np.array([r[1] for r in runs_l]), np.array([r[1] for r in runs_t])
    se = float(np.hypot(acc_l.std(ddof=1) / np.sqrt(len(acc_l)), acc_t.std(ddof=1) / np.sqrt(len(acc_t))))
    abar = max(3 * se, 0.005)
    print("\nwindow mean loss, p=0.3  libbnn (mean of 8):", " ".join(f"{v:.3f}" for v in wl))
    print("window mean loss, p=0.3  torch  (mean of 8):", " ".join(f"{v:.3f}" for v in wt))
    print(f"max window gap {np.abs(wl - wt).max():.4f} (band {band:.4f}: torch halves {half.max():.4f}); "
          f"accuracy libbnn {np.round(acc_l, 4).tolist()} mean {acc_l.mean():.4f}, torch {np.round(acc_t, 4).tolist()} "
          f"mean {acc_t.mean():.4f}; |difference| {abs(acc_l.mean() - acc_t.mean()):.4f} against 3 s.e. = {3 * se:.4f} "
          f"(bar {abar:.4f})")
    assert np.abs(wl - wt).max() <= band
    assert all(_windows(r[0])[-1] < 0.5 * _windows(r[0])[0] for r in runs_l + runs_t)
    assert abs(acc_l.mean() - acc_t.mean()) <= abar

"""Float64 torch restatement of the reference's training step -- TEST INFRASTRUCTURE ONLY.

Only ``tests/`` may import this module, and only as the checker.  It is the algorithm of
``oracle/bnn_np.py`` (``MLPOracle``, itself pinned to the reference's own traces) written with
torch float64 ops so that it runs on any device: on the GPU box it checks whole training steps at
the benched sizes (BASELINE config 5: 65,536 x 8192 activations, 4.3 GB each in float64), where
numpy on the host would take hours.  ``CNNOracle`` adds the build-defined BinCNN of config 4.

Restated from:
* models/binarized_modules.py:11-13 (Binarize = sign, ternary), :73-85 (BinarizeLinear: first-layer
  rule, ``F.linear(input, sign(org))`` in fp32 then ``out += bias`` in fp32), :93-107
  (BinarizeConv2d: input binarised unless C == 3, ``F.conv2d`` with zero padding, + bias);
* autograd of both (STE = identity: binarisation goes through ``.data``);
* mnist-dist2.py:46-76 (Net: fc -> BatchNorm1d -> Hardtanh x3, Dropout(0.3) before bn3, fc4,
  LogSoftmax) and :118-137 (CrossEntropy on the log-probs, org restore -> Adam -> clamp);
* mnist-dist.py:31-51 (the ConvNet template of the BinCNN: conv5x5 p2 -> BN2d -> Hardtanh ->
  MaxPool2d(2), twice, Linear(1568, 10)).

Pinned by tests/test_oracle_golden.py (``test_t64_*``): the reference's trace_org / trace_wide
(MLP) and trace_cnn (BinCNN) fixtures, and the numpy oracle on the same inputs.

Every product of ternary operands is an integer sum, exact in float64; every pre-activation is
rounded to fp32 and gets its bias added in fp32 (binarized_modules.py:80-83) before the float64
BatchNorm -- the rounding that decides BatchNorm near-ties the way the reference does.
"""
import math

import torch
import torch.nn.functional as tF

F64 = torch.float64
F32 = torch.float32


def rel_err(a, b):
    """||a - b|| / ||b|| in float64 on the tensors' device (no host copy of large tensors)."""
    a = torch.as_tensor(a).to(F64)
    b = torch.as_tensor(b).to(device=a.device, dtype=F64)
    nb = float(torch.linalg.vector_norm(b))
    return float(torch.linalg.vector_norm(a - b)) / (nb if nb > 0 else 1.0)


# --------------------------------------------------------------------------- layers
# Hardtanh-boundary window: an element whose BatchNorm output lies within TAU of +-1 gets the
# strict mask 1[-1 < y < 1] (hardtanh backward) from whichever rounding its implementation applies
# -- fp32 arithmetic (the reference's, libbnn's) and float64 can decide it differently, as they do a
# BatchNorm near-tie's sign.  TAU = 2^-20: 8 fp32 ulps at 1.0, well above the fp32 rounding of
# y = (x - mean) * invstd * gamma + beta.  Such elements are recorded per column (MLPOracle.boundary).
TAU = 2.0 ** -20


def batchnorm_train(z, gamma, beta, rmean, rvar, dims, momentum=0.1, eps=1e-5, boundary=None, impl_y=None,
                    anchored=None):
    """nn.BatchNorm1d / 2d in training mode followed by nn.Hardtanh (mnist-dist2.py:52-53): batch
    statistics over ``dims`` (biased variance normalises, the unbiased one feeds the running
    estimate).  Returns (hardtanh output, cache, new running mean, new running var); z is
    consumed (overwritten by x_hat).  ``boundary`` (a list): the per-column count of elements
    within TAU of the Hardtanh boundary is appended.

    ``impl_y``: the BatchNorm output as the implementation under test rounds it (fp32, same shape).
    Elements within TAU of +-1 then take the backward mask 1[-1 < y < 1] from it -- the Hardtanh
    decision is anchored on the implementation's rounding there, as BatchNorm near-ties are anchored
    on its z1 -- and ``anchored`` (a list) receives (window elements whose mask changed, elements
    OUTSIDE the window whose impl_y mask differs from float64's: 0 unless impl_y is not a rounding
    of this y)."""
    m = z.numel() // z.shape[1]
    shape = [1] * z.dim()
    shape[1] = -1
    mu = z.mean(dims)
    var = z.var(dims, unbiased=False)
    inv = 1.0 / torch.sqrt(var + eps)
    xhat = z.sub_(mu.view(shape)).mul_(inv.view(shape))
    y = xhat * gamma.view(shape) + beta.view(shape)
    mask = (y > -1.0) & (y < 1.0)              # Hardtanh backward: strict
    win = (y.abs() - 1.0).abs() < TAU
    if boundary is not None:
        boundary.append(win.sum(dims))
    if impl_y is not None:
        imask = (impl_y > -1.0) & (impl_y < 1.0)
        diff = imask != mask
        if anchored is not None:
            anchored.append((int((diff & win).sum()), int((diff & ~win).sum())))
        mask = torch.where(win, imask, mask)
        del imask, diff
    del win
    y.clamp_(-1.0, 1.0)
    new_rm = (1 - momentum) * rmean + momentum * mu
    new_rv = (1 - momentum) * rvar + momentum * var * (m / max(m - 1, 1))
    return y, (xhat, inv, gamma, mask, dims, shape), new_rm, new_rv


def batchnorm_backward(cache, g):
    """Hardtanh mask, then BatchNorm's backward; returns (dz, dgamma, dbeta)."""
    xhat, inv, gamma, mask, dims, shape = cache
    g = g * mask
    m = g.numel() // g.shape[1]
    dgamma = (g * xhat).sum(dims)
    dbeta = g.sum(dims)
    dxhat = g.mul_(gamma.view(shape))
    s1 = dxhat.sum(dims).view(shape)
    s2 = (dxhat * xhat).sum(dims).view(shape)
    dz = dxhat.mul_(m).sub_(s1).sub_(xhat * s2).mul_(inv.view(shape) / m)
    return dz, dgamma, dbeta


def nll_of_log_softmax(out_logp, target):
    """CrossEntropyLoss on the LogSoftmax output (mnist-dist2.py:90,124): log_softmax is
    idempotent, so loss = NLL(log_softmax(out)), d loss / d out = (softmax - onehot) / B."""
    lp = torch.log_softmax(out_logp, 1)
    b = lp.shape[0]
    idx = torch.arange(b, device=lp.device)
    loss = -lp[idx, target].mean()
    p = lp.exp()
    p[idx, target] -= 1.0
    return float(loss), p / b


class Adam:
    """torch.optim.Adam defaults (mnist-dist2.py:91) in float64: betas (0.9, 0.999), eps 1e-8,
    bias-corrected as torch's single-tensor step."""

    def __init__(self, lr, betas=(0.9, 0.999), eps=1e-8):
        self.lr, self.b1, self.b2, self.eps = lr, betas[0], betas[1], eps
        self.state = {}

    def step(self, name, p, g):
        st = self.state.setdefault(name, {"t": 0, "m": torch.zeros_like(p), "v": torch.zeros_like(p)})
        st["t"] += 1
        t = st["t"]
        st["m"] = self.b1 * st["m"] + (1 - self.b1) * g
        st["v"] = self.b2 * st["v"] + (1 - self.b2) * g * g
        denom = torch.sqrt(st["v"]) / math.sqrt(1 - self.b2 ** t) + self.eps
        return p - (self.lr / (1 - self.b1 ** t)) * st["m"] / denom


def _z_fp32(sums, bias, shape):
    """F.linear / F.conv2d output (fp32; exact when the sums are integers) then ``out += bias`` in
    fp32 (binarized_modules.py:80-83, :100-105), returned in float64."""
    z = sums.to(F32)
    if bias is not None:
        z += bias.to(F32).view(shape)
    return z.to(F64)


# --------------------------------------------------------------------------- MLP (mnist-dist2.py Net)
BINARY = ("fc1", "fc2", "fc3")


class MLPOracle:
    """``Net`` (mnist-dist2.py:46-76) + one training step (:118-137), float64 torch, any device.

    ``state``: the model's state_dict (latent weights = ``weight.org``).  ``step`` options:
    ``z1`` -- fc1's output as the implementation under test computed it (the rest of the step then
    runs from it: fc1's input is continuous, see bnn_np.MLPOracle.step); ``drop`` -- the scaled keep
    mask (1/(1-p) or 0, fp32 [B, h3]) of the Dropout before bn3 (torch's dropout multiplies the
    fp32 pre-activation by it); ``update`` -- run the latent-weight protocol (restore -> Adam ->
    clamp).  After a step, ``boundary[i]`` counts per column the elements of hidden layer i's
    BatchNorm output within TAU of the Hardtanh boundary."""

    def __init__(self, state, lr=0.01, org_protocol=True, device="cpu"):
        self.dev = torch.device(device)
        self.p = {k: torch.as_tensor(v).to(self.dev, F64) for k, v in state.items() if "num_batches" not in k}
        self.org = {f"{l}.weight": self.p[f"{l}.weight"].clone() for l in BINARY}
        self.opt = Adam(lr)
        self.org_protocol = org_protocol

    def step(self, x, target, z1=None, drop=None, update=True, anchor=None, bwd=None):
        """``anchor``: callable (layer index i, fp32 BatchNorm input z as float64) -> the
        implementation's fp32 BatchNorm output, whose Hardtanh decision is taken for elements within
        TAU of +-1 (batchnorm_train ``impl_y``; ``self.anchored`` records what it changed).
        ``bwd``: callable (kind "dw" | "dx", layer index i, g, other operand) -> float64 product, to
        run the backward GEMMs in another arithmetic (calibration runs); default exact float64
        ``g.T @ x`` / ``g @ W_b``."""
        p = self.p
        self.boundary = []         # per hidden layer: [h_i] counts of elements within TAU of +-1
        self.anchored = []         # per hidden layer (with anchor): (changed in window, differing outside)
        x = torch.as_tensor(x).to(self.dev)
        target = torch.as_tensor(target).to(self.dev, torch.int64)
        a = x.reshape(x.shape[0], -1).to(F64)
        caches = []
        for i, l in enumerate(BINARY):
            wb = torch.sign(self.org[f"{l}.weight"])
            # the binarised input the GEMM multiplies (first layer: the pixels, :75), kept as int8
            xu = a if i == 0 else torch.sign(a).to(torch.int8)
            if i == 0 and z1 is not None:
                z = torch.as_tensor(z1).to(self.dev, F32).to(F64)
            else:
                z = _z_fp32(a @ wb.T if i == 0 else xu.to(F64) @ wb.T, p[f"{l}.bias"], (1, -1))
            del a
            if i == 2 and drop is not None:        # nn.Dropout(p) on fc3's fp32 output (:69)
                z = (z.to(F32) * torch.as_tensor(drop).to(self.dev, F32)).to(F64)
            bn = f"bn{i + 1}"
            iy = anchor(i, z) if anchor is not None else None
            a, cache, rm, rv = batchnorm_train(z, p[f"{bn}.weight"], p[f"{bn}.bias"],
                                               p[f"{bn}.running_mean"], p[f"{bn}.running_var"], (0,),
                                               boundary=self.boundary, impl_y=iy, anchored=self.anchored)
            del iy
            p[f"{bn}.running_mean"], p[f"{bn}.running_var"] = rm, rv
            caches.append((xu, wb, cache))
        logits = a @ p["fc4.weight"].T + p["fc4.bias"]
        out = torch.log_softmax(logits, 1)
        loss, dz = nll_of_log_softmax(out, target)
        grads = {"fc4.weight": dz.T @ a, "fc4.bias": dz.sum(0)}
        g = dz @ p["fc4.weight"]
        del a
        for i in (2, 1, 0):
            l, bn = BINARY[i], f"bn{i + 1}"
            xu, wb, cache = caches[i]
            g, grads[f"{bn}.weight"], grads[f"{bn}.bias"] = batchnorm_backward(cache, g)
            caches[i] = None
            if i == 2 and drop is not None:        # dropout backward: the same scaled mask
                g.mul_(torch.as_tensor(drop).to(self.dev, F32).to(F64))
            xo = xu if i == 0 else xu.to(F64)
            grads[f"{l}.weight"] = g.T @ xo if bwd is None else bwd("dw", i, g, xo)
            del xo
            grads[f"{l}.bias"] = g.sum(0)
            if i > 0:
                g = g @ wb if bwd is None else bwd("dx", i, g, wb)
            else:
                g = None
        if update:
            self._update(grads)
        return loss, out, grads

    def _update(self, grads):
        """mnist-dist2.py:131-137 (or mnist-dist3.py:113-119 without the protocol)."""
        p = self.p
        for k, gk in grads.items():
            layer = k.split(".")[0]
            if k.endswith(".weight") and layer in BINARY:
                if self.org_protocol:
                    self.org[k] = self.opt.step(k, self.org[k], gk).clamp_(-1, 1)
                    p[k] = self.org[k]
                else:
                    p[k] = self.opt.step(k, torch.sign(self.org[k]), gk)
            elif k.endswith(".bias") and layer in BINARY:
                new = self.opt.step(k, p[k], gk)
                p[k] = new.clamp_(-1, 1) if self.org_protocol else new
            else:
                p[k] = self.opt.step(k, p[k], gk)


# --------------------------------------------------------------------------- BinCNN (BASELINE config 4)
CONV = ("layer1", "layer2")


def _unfold(x, k, pad):
    """im2col: [N, C, H, W] -> [N, C*k*k, H*W] (stride 1, zero padding counts as 0)."""
    return tF.unfold(x, k, padding=pad)


def conv2d_sums(xu, wb, pad):
    """F.conv2d(xu, wb, padding=pad) (stride 1) in float64: exact for ternary operands."""
    n, c, h, w = xu.shape
    co, _, k, _ = wb.shape
    oh, ow = h + 2 * pad - k + 1, w + 2 * pad - k + 1
    return (wb.reshape(co, -1) @ _unfold(xu, k, pad)).view(n, co, oh, ow)


class CNNOracle:
    """The BinCNN (``nets.BinCNN``, ``oracle.bnn_torch.RefCNN``): two blocks of BinarizeConv2d 5x5 p2
    (binarized_modules.py:93-107; both binarise their input since C != 3 -- conv1's pixels become
    {0, 1}) -> BatchNorm2d -> Hardtanh -> MaxPool2d(2) (torch's first-maximum rule), then
    Linear(1568, 10) and LogSoftmax; one training step with the .org protocol (mnist-dist2.py:
    118-137).  Keys follow nets.BinCNN's state_dict (layer1.0 = conv, layer1.1 = BatchNorm2d)."""

    def __init__(self, state, lr=0.01, device="cpu"):
        self.dev = torch.device(device)
        self.p = {k: torch.as_tensor(v).to(self.dev, F64) for k, v in state.items() if "num_batches" not in k}
        self.org = {f"{l}.0.weight": self.p[f"{l}.0.weight"].clone() for l in CONV}
        self.opt = Adam(lr)

    def step(self, x, target, update=True, bwd=None):
        """``bwd``: callable (kind "dw" | "dx", layer index j, gradient [N, Co, H*W], im2col columns
        [N, C*k*k, H*W] | the binarised weight [Co, C*k*k]) -> the float64 contraction (dW [Co, C*k*k]
        | dcols [N, C*k*k, H*W]) in another arithmetic (calibration runs); default exact float64."""
        p = self.p
        x = torch.as_tensor(x).to(self.dev)
        target = torch.as_tensor(target).to(self.dev, torch.int64)
        a = x.to(F64)
        caches = []
        for l in CONV:
            wb = torch.sign(self.org[f"{l}.0.weight"])
            xu = torch.sign(a)                                    # C != 3: binarised (:94-95)
            pad = 2
            z = _z_fp32(conv2d_sums(xu, wb, pad), p.get(f"{l}.0.bias"), (1, -1, 1, 1))
            h, cache, rm, rv = batchnorm_train(z, p[f"{l}.1.weight"], p[f"{l}.1.bias"],
                                               p[f"{l}.1.running_mean"], p[f"{l}.1.running_var"], (0, 2, 3))
            p[f"{l}.1.running_mean"], p[f"{l}.1.running_var"] = rm, rv
            a, idx = tF.max_pool2d(h, 2, 2, return_indices=True)
            caches.append((xu, wb, pad, cache, idx, h.shape))
            del h
        flat = a.reshape(a.shape[0], -1)
        out = torch.log_softmax(flat @ p["fc.weight"].T + p["fc.bias"], 1)
        loss, dz = nll_of_log_softmax(out, target)
        grads = {"fc.weight": dz.T @ flat, "fc.bias": dz.sum(0)}
        g = (dz @ p["fc.weight"]).view(a.shape)
        for j in (1, 0):
            l = CONV[j]
            xu, wb, pad, cache, idx, hshape = caches[j]
            n, c = g.shape[:2]
            # MaxPool2d backward: each window's gradient goes to its (first) maximum
            gh = torch.zeros(hshape, dtype=F64, device=self.dev).view(n, c, -1)
            gh.scatter_(2, idx.view(n, c, -1), g.reshape(n, c, -1))
            g, grads[f"{l}.1.weight"], grads[f"{l}.1.bias"] = batchnorm_backward(cache, gh.view(hshape))
            co, ci, k, _ = wb.shape
            cols = _unfold(xu, k, pad)                             # [N, C*k*k, H*W]
            gf = g.reshape(n, co, -1)
            dw = torch.einsum("nol,nkl->ok", gf, cols) if bwd is None else bwd("dw", j, gf, cols)
            grads[f"{l}.0.weight"] = dw.reshape(wb.shape)
            grads[f"{l}.0.bias"] = g.sum((0, 2, 3))
            if j > 0:                                             # conv1's input needs no gradient
                w2 = wb.reshape(co, -1)
                dcols = w2.T @ gf if bwd is None else bwd("dx", j, gf, w2)   # [N, C*k*k, H*W]
                g = tF.fold(dcols, xu.shape[-2:], k, padding=pad)
        if update:
            self._update(grads)
        return loss, out, grads

    def _update(self, grads):
        """Adam on every parameter; the conv weights (latent: restore -> step -> clamp) and conv
        biases (.org too, binarized_modules.py:104) are clamped to [-1, 1] (mnist-dist2.py:131-137)."""
        p = self.p
        for k, gk in grads.items():
            if k.endswith(".0.weight"):
                self.org[k] = self.opt.step(k, self.org[k], gk).clamp_(-1, 1)
                p[k] = self.org[k]
            elif k.endswith(".0.bias"):
                p[k] = self.opt.step(k, p[k], gk).clamp_(-1, 1)
            else:
                p[k] = self.opt.step(k, p[k], gk)

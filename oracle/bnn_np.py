"""CPU oracle (numpy) for the binarized-network training hot path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module, and only as the checker.  The product path
(``distributed-mnist-bnns_amd/``) never imports it and has no CPU fallback.

It restates, in plain numpy, what the reference computes for this path:

* ``models/binarized_modules.py:11-13``  ``Binarize(t,'det') = t.sign()`` (ternary: sign(0)=0)
* ``models/binarized_modules.py:73-85``  ``BinarizeLinear.forward``
* ``models/binarized_modules.py:93-107`` ``BinarizeConv2d.forward``
* autograd of the two (STE = identity because binarisation goes through ``.data``)
* the caller protocol of ``mnist-dist2.py:118-137`` (org restore -> Adam -> clamp) and
  ``mnist-dist3.py:113-119`` (no protocol: binary weights frozen at their first sign)
* torch's ``BatchNorm1d`` (train), ``Hardtanh``, ``LogSoftmax`` + ``CrossEntropyLoss`` and
  ``Adam`` as the reference scripts use them (``mnist-dist2.py:46-76, 90-91``).

Integer-valued products (+-1/0 x +-1/0) are computed exactly (float64 BLAS on small integers
is exact), so the binarised forward is bit-exact against the reference's fp32 ``F.linear``
followed by one fp32 bias add.  Everything else is computed in float64; comparisons against
fp32 results use the tolerances written in the tests.

Pinned by ``tests/golden/*.npz``: outputs of the reference module itself, generated in the
build container by ``tests/golden/make_golden.py`` (see tests/test_oracle_golden.py).
"""
import numpy as np

F32 = np.float32
F64 = np.float64


# --------------------------------------------------------------------------- binarize
def to_tensor(u, normalize=None):
    """The reference loader's transform on u8 pixels (mnist-dist2.py:96-99
    ``transforms.ToTensor()`` = ``u.float().div(255)`` in fp32; mnist-distributed-BNNS2.py:82 adds
    ``Normalize((m,), (s,))`` = ``(x - m) / s`` in fp32)."""
    x = (np.asarray(u).astype(F32) / F32(255.0)).astype(F32)
    if normalize is not None:
        m, sd = normalize
        x = ((x - F32(m)) / F32(sd)).astype(F32)
    return x


def binarize(x):
    """``Binarize(tensor, 'det')`` -- models/binarized_modules.py:11-13.  sign(0) = 0."""
    return np.sign(x).astype(x.dtype, copy=False)


def first_layer(x, in_features_marker=784):
    """BinarizeLinear skips input binarisation iff ``input.size(1) == 784``
    (models/binarized_modules.py:75)."""
    return x.shape[1] == in_features_marker


# --------------------------------------------------------------------------- linear
def linear_forward(x, w_latent, bias=None):
    """``BinarizeLinear.forward`` -- models/binarized_modules.py:73-85.

    Returns ``(y, x_used)``; ``x_used`` is what the reference leaves in ``input.data``
    (``sign(x)`` unless the first-layer rule applies, :75-76).
    ``y = F.linear(x_used, sign(w_latent))`` (:79-80) then ``y += bias`` in fp32 (:81-83).
    """
    x = np.asarray(x, F32)
    wb = binarize(np.asarray(w_latent, F32))
    xu = x if first_layer(x) else binarize(x)
    y = (xu.astype(F64) @ wb.astype(F64).T).astype(F32)   # exact when xu is ternary
    if bias is not None and np.size(bias):
        y = (y + np.asarray(bias, F32)[None, :]).astype(F32)
    return y, xu


def linear_backward(x_used, w_latent, dy, need_dx=True):
    """Autograd of ``F.linear(x_used, W_b)`` (binarized_modules.py:80): the STE is the identity
    (binarisation happens through ``.data``), so dX = dY.W_b, dW = dY^T.x_used, dB = sum_B dY."""
    dy64 = np.asarray(dy, F64)
    wb = binarize(np.asarray(w_latent, F32)).astype(F64)
    dx = (dy64 @ wb).astype(F32) if need_dx else None
    dw = (dy64.T @ np.asarray(x_used, F64)).astype(F32)
    db = dy64.sum(0).astype(F32)
    return dx, dw, db


# --------------------------------------------------------------------------- conv2d
def _out_hw(h, w, kh, kw, stride, pad, dil):
    oh = (h + 2 * pad - dil * (kh - 1) - 1) // stride + 1
    ow = (w + 2 * pad - dil * (kw - 1) - 1) // stride + 1
    return oh, ow


def im2col(x, kh, kw, stride, pad, dil):
    """[N,C,H,W] -> [N, C*kh*kw, OH*OW] with zero padding (padding contributes 0)."""
    n, c, h, w = x.shape
    oh, ow = _out_hw(h, w, kh, kw, stride, pad, dil)
    xp = np.zeros((n, c, h + 2 * pad, w + 2 * pad), x.dtype)
    xp[:, :, pad:pad + h, pad:pad + w] = x
    cols = np.empty((n, c, kh, kw, oh, ow), x.dtype)
    for i in range(kh):
        for j in range(kw):
            hs, ws = i * dil, j * dil
            cols[:, :, i, j] = xp[:, :, hs:hs + stride * (oh - 1) + 1:stride,
                                  ws:ws + stride * (ow - 1) + 1:stride]
    return cols.reshape(n, c * kh * kw, oh * ow), (oh, ow)


def col2im(cols, shape, kh, kw, stride, pad, dil):
    n, c, h, w = shape
    oh, ow = _out_hw(h, w, kh, kw, stride, pad, dil)
    cols = cols.reshape(n, c, kh, kw, oh, ow)
    xp = np.zeros((n, c, h + 2 * pad, w + 2 * pad), cols.dtype)
    for i in range(kh):
        for j in range(kw):
            hs, ws = i * dil, j * dil
            xp[:, :, hs:hs + stride * (oh - 1) + 1:stride,
               ws:ws + stride * (ow - 1) + 1:stride] += cols[:, :, i, j]
    return xp[:, :, pad:pad + h, pad:pad + w]


def conv_binarizes_input(x):
    """BinarizeConv2d binarises its input unless ``input.size(1) == 3``
    (models/binarized_modules.py:94)."""
    return x.shape[1] != 3


def conv2d_forward(x, w_latent, bias=None, stride=1, padding=0, dilation=1, groups=1):
    """``BinarizeConv2d.forward`` -- models/binarized_modules.py:93-107.
    Returns ``(y, x_used)``."""
    x = np.asarray(x, F32)
    wb = binarize(np.asarray(w_latent, F32))
    xu = binarize(x) if conv_binarizes_input(x) else x
    n, c, h, w = xu.shape
    co, cig, kh, kw = wb.shape
    cols, (oh, ow) = im2col(xu.astype(F64), kh, kw, stride, padding, dilation)
    cog = co // groups
    y = np.empty((n, co, oh * ow), F64)
    kg = cig * kh * kw
    for g in range(groups):
        wg = wb[g * cog:(g + 1) * cog].reshape(cog, kg).astype(F64)
        y[:, g * cog:(g + 1) * cog] = np.einsum("ok,nkp->nop", wg, cols[:, g * kg:(g + 1) * kg])
    y = y.reshape(n, co, oh, ow).astype(F32)
    if bias is not None and np.size(bias):
        y = (y + np.asarray(bias, F32)[None, :, None, None]).astype(F32)
    return y, xu


def conv2d_backward(x_used, w_latent, dy, stride=1, padding=0, dilation=1, groups=1):
    """Autograd of ``F.conv2d(x_used, W_b, ...)`` (binarized_modules.py:100-101), STE identity."""
    wb = binarize(np.asarray(w_latent, F32)).astype(F64)
    xu = np.asarray(x_used, F64)
    dy = np.asarray(dy, F64)
    n, c, h, w = xu.shape
    co, cig, kh, kw = wb.shape
    cols, (oh, ow) = im2col(xu, kh, kw, stride, padding, dilation)
    dyc = dy.reshape(n, co, oh * ow)
    cog, kg = co // groups, cig * kh * kw
    dw = np.empty((co, kg), F64)
    dcols = np.empty_like(cols)
    for g in range(groups):
        dyg = dyc[:, g * cog:(g + 1) * cog]
        dw[g * cog:(g + 1) * cog] = np.einsum("nop,nkp->ok", dyg, cols[:, g * kg:(g + 1) * kg])
        wg = wb[g * cog:(g + 1) * cog].reshape(cog, kg)
        dcols[:, g * kg:(g + 1) * kg] = np.einsum("ok,nop->nkp", wg, dyg)
    dx = col2im(dcols, xu.shape, kh, kw, stride, padding, dilation)
    db = dy.sum((0, 2, 3))
    return dx.astype(F32), dw.reshape(wb.shape).astype(F32), db.astype(F32)


# --------------------------------------------------------------------------- torch layers used by the scripts
def hardtanh(x):
    """nn.Hardtanh() (mnist-dist2.py:51): clip to [-1, 1]."""
    return np.clip(x, -1.0, 1.0)


def hardtanh_backward(x, g):
    """Hardtanh backward passes the gradient only where -1 < x < 1 (strict)."""
    return g * ((x > -1.0) & (x < 1.0))


def batchnorm_train(x, gamma, beta, rmean, rvar, momentum=0.1, eps=1e-5):
    """nn.BatchNorm1d in train mode (mnist-dist2.py:52): batch stats, biased var for the
    normalisation, unbiased var for the running estimate."""
    x = np.asarray(x, F64)
    m = x.shape[0]
    mu = x.mean(0)
    var = x.var(0)
    inv = 1.0 / np.sqrt(var + eps)
    xhat = (x - mu) * inv
    y = xhat * gamma + beta
    new_rm = (1 - momentum) * rmean + momentum * mu
    new_rv = (1 - momentum) * rvar + momentum * var * m / max(m - 1, 1)
    return y, (xhat, inv, gamma), new_rm, new_rv


def batchnorm_backward(cache, g):
    xhat, inv, gamma = cache
    g = np.asarray(g, F64)
    m = g.shape[0]
    dgamma = (g * xhat).sum(0)
    dbeta = g.sum(0)
    dxhat = g * gamma
    dx = inv / m * (m * dxhat - dxhat.sum(0) - xhat * (dxhat * xhat).sum(0))
    return dx, dgamma, dbeta


def batchnorm2d_train(x, gamma, beta, rmean, rvar, momentum=0.1, eps=1e-5):
    """nn.BatchNorm2d in train mode (the block after each conv of the BinCNN; mnist-dist.py:33,39
    template): per-channel statistics over (N, H, W) -- BatchNorm1d on the [N*H*W, C] view."""
    x = np.asarray(x, F64)
    n, c, h, w = x.shape
    flat = x.transpose(0, 2, 3, 1).reshape(-1, c)
    y, cache, rm, rv = batchnorm_train(flat, gamma, beta, rmean, rvar, momentum, eps)
    return y.reshape(n, h, w, c).transpose(0, 3, 1, 2), cache, rm, rv


def batchnorm2d_backward(cache, g):
    g = np.asarray(g, F64)
    n, c, h, w = g.shape
    dx, dgamma, dbeta = batchnorm_backward(cache, g.transpose(0, 2, 3, 1).reshape(-1, c))
    return dx.reshape(n, h, w, c).transpose(0, 3, 1, 2), dgamma, dbeta


def maxpool2_forward(y):
    """nn.MaxPool2d(kernel_size=2, stride=2) (mnist-dist.py:35,41 template) with torch's argmax
    rule: the first strictly greater value in (h, w) scan order wins ties.  Returns the pooled
    map and the window slot (0..3) of each maximum."""
    y = np.asarray(y)
    n, c, h, w = y.shape
    win = y[:, :, :h - h % 2, :w - w % 2].reshape(n, c, h // 2, 2, w // 2, 2)
    win = win.transpose(0, 1, 2, 4, 3, 5).reshape(n, c, h // 2, w // 2, 4)
    arg = np.argmax(win, axis=-1)          # numpy's argmax also returns the first maximum
    return np.take_along_axis(win, arg[..., None], -1)[..., 0], arg


def maxpool2_backward(g, arg, shape):
    n, c, h, w = shape
    out = np.zeros((n, c, h // 2, w // 2, 4), F64)
    np.put_along_axis(out, arg[..., None], np.asarray(g, F64)[..., None], -1)
    out = out.reshape(n, c, h // 2, w // 2, 2, 2).transpose(0, 1, 2, 4, 3, 5).reshape(n, c, h, w)
    return out


def log_softmax(z):
    z = np.asarray(z, F64)
    zm = z - z.max(1, keepdims=True)
    return zm - np.log(np.exp(zm).sum(1, keepdims=True))


def nll_loss_and_grad(logp_out, target):
    """CrossEntropyLoss applied to the LogSoftmax output (mnist-dist2.py:90,124).
    log_softmax is idempotent, so the loss is NLL(log_softmax(z)); dL/dz = (p - onehot)/B."""
    lp = log_softmax(logp_out)  # CrossEntropy re-applies log_softmax
    b = lp.shape[0]
    loss = -lp[np.arange(b), target].mean()
    p = np.exp(lp)
    p[np.arange(b), target] -= 1.0
    return loss, p / b


class Adam:
    """torch.optim.Adam defaults (mnist-dist2.py:91): betas (0.9, 0.999), eps 1e-8,
    no weight decay, bias-corrected (torch's single-tensor formula)."""

    def __init__(self, lr, betas=(0.9, 0.999), eps=1e-8):
        self.lr, self.b1, self.b2, self.eps = lr, betas[0], betas[1], eps
        self.state = {}

    def step(self, name, p, g):
        st = self.state.setdefault(name, {"t": 0, "m": np.zeros_like(p, F64), "v": np.zeros_like(p, F64)})
        st["t"] += 1
        t = st["t"]
        g = np.asarray(g, F64)
        st["m"] = self.b1 * st["m"] + (1 - self.b1) * g
        st["v"] = self.b2 * st["v"] + (1 - self.b2) * g * g
        bc1 = 1 - self.b1 ** t
        bc2s = np.sqrt(1 - self.b2 ** t)
        denom = np.sqrt(st["v"]) / bc2s + self.eps
        return np.asarray(p, F64) - (self.lr / bc1) * st["m"] / denom


# --------------------------------------------------------------------------- MLP trainer (mnist-dist2.py)
BINARY = ("fc1", "fc2", "fc3")


class MLPOracle:
    """Restatement of ``Net`` (mnist-dist2.py:46-76) + one train step (:118-137) in numpy.

    ``params`` holds the *latent* weights (``weight.org``) and biases; the binarised copy is
    recomputed each forward from ``org`` exactly as binarized_modules.py:77-79 does.
    ``org_protocol=False`` reproduces mnist-dist3.py:113-119 where Adam updates the binarised
    copy that the next forward overwrites (binary weights stay frozen)."""

    def __init__(self, state, lr=0.01, org_protocol=True):
        self.p = {k: np.asarray(v, F64) for k, v in state.items()}
        self.org = {f"{l}.weight": np.asarray(state[f"{l}.weight"], F64) for l in BINARY}
        self.opt = Adam(lr)
        self.org_protocol = org_protocol

    def step(self, x, target, z1=None):
        """One training step.  ``z1``: fc1's output as an implementation under test computed it
        (fp32 [B, h1]); the rest of the step then runs from it.  fc1's input is continuous (the
        pixels), so z1 carries fp32 rounding that differs between implementations (the reference's
        own sgemm included), and its BatchNorm near-ties -- elements within an ulp-scale window of
        the batch mean -- take whichever sign that rounding gives them; the checker compares
        everything downstream of z1 given the same z1, and z1 itself separately."""
        p = self.p
        a = np.asarray(x, F64).reshape(x.shape[0], -1)
        caches = []
        for i, l in enumerate(BINARY):
            wb = np.sign(self.org[f"{l}.weight"])
            xu = a if i == 0 else np.sign(a)
            # F.linear output is fp32 (exact for +-1 inputs) and ``out += bias`` rounds in fp32
            # (binarized_modules.py:80-83).  Keeping z in fp32 matters: integer-valued
            # pre-activations make BatchNorm ties (z_i == mean) common, and the reference's
            # fp32 rounding of the bias add is what breaks them.
            if i == 0 and z1 is not None:
                z = np.asarray(z1, F32).astype(F64)
            else:
                z = ((xu @ wb.T).astype(F32) + p[f"{l}.bias"].astype(F32)).astype(F64)
            bn = f"bn{i + 1}"
            y, cache, rm, rv = batchnorm_train(z, p[f"{bn}.weight"], p[f"{bn}.bias"],
                                               p[f"{bn}.running_mean"], p[f"{bn}.running_var"])
            p[f"{bn}.running_mean"], p[f"{bn}.running_var"] = rm, rv
            h = hardtanh(y)
            caches.append((xu, wb, cache, y))
            a = h
        logits = a @ p["fc4.weight"].T + p["fc4.bias"]
        out = log_softmax(logits)
        loss, dz = nll_loss_and_grad(out, target)
        grads = {"fc4.weight": dz.T @ a, "fc4.bias": dz.sum(0)}
        g = dz @ p["fc4.weight"]
        for i in (2, 1, 0):
            l, bn = BINARY[i], f"bn{i + 1}"
            xu, wb, cache, y = caches[i]
            g = hardtanh_backward(y, g)
            g, grads[f"{bn}.weight"], grads[f"{bn}.bias"] = batchnorm_backward(cache, g)
            grads[f"{l}.weight"] = g.T @ xu
            grads[f"{l}.bias"] = g.sum(0)
            g = g @ wb
        # latent-weight protocol (mnist-dist2.py:131-137)
        for k, gk in grads.items():
            if k.endswith(".weight") and k.split(".")[0] in BINARY:
                if self.org_protocol:
                    new = self.opt.step(k, self.org[k], gk)
                    self.org[k] = np.clip(new, -1, 1)
                    p[k] = self.org[k]
                else:
                    p[k] = self.opt.step(k, np.sign(self.org[k]), gk)  # overwritten next forward
            elif k.endswith(".bias") and k.split(".")[0] in BINARY:
                new = self.opt.step(k, p[k], gk)
                p[k] = np.clip(new, -1, 1) if self.org_protocol else new
            else:
                p[k] = self.opt.step(k, p[k], gk)
        return loss, out, grads

"""Generate the golden fixtures that pin the oracle (test infrastructure only).

Run in the build container (NOT on the GPU box -- /root/reference does not exist there):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

It imports the reference operator module ``/root/reference/models/binarized_modules.py``
(``Binarize`` :11-15, ``HingeLoss`` :20-32, ``BinarizeLinear`` :68-85, ``BinarizeConv2d``
:87-107) and records inputs + outputs of the reference itself on CPU.  The caller-side
protocol is restated from ``mnist-dist2.py:118-137`` (org restore -> Adam -> clamp) and
``mnist-dist3.py:113-119`` (no org protocol: binary weights stay frozen), and the Net
topology from ``mnist-dist2.py:46-76`` at reduced widths so the fixtures stay small.

Everything is written with ``numpy.savez`` (no pickles) into ``tests/golden/*.npz``.
Only data is committed: inputs and expected outputs.
"""
import os
import sys

import numpy as np
import torch
import torch.nn as nn

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
sys.path.insert(0, REF)
from models.binarized_modules import (Binarize, BinarizeConv2d,  # noqa: E402
                                      BinarizeLinear, HingeLoss)


def mnist_like(gen, shape):
    """Synthetic MNIST-shaped pixels: 80.7% exact zeros, rest u8/255."""
    u = torch.rand(shape, generator=gen)
    v = torch.randint(1, 256, shape, generator=gen).float()
    return torch.where(u < 0.807, torch.zeros_like(v), v) / 255.0


def np32(t):
    return t.detach().cpu().numpy().astype(np.float32)


def save(name, **arrs):
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **arrs)
    print("wrote", path, sum(a.size for a in arrs.values()), "elements")


def linear_case(name, gen, fin, fout, batch, x, bias=True, zero_w=0):
    torch.manual_seed(1000 + fin + fout)
    layer = BinarizeLinear(fin, fout, bias=bias)
    if zero_w:
        with torch.no_grad():
            flat = layer.weight.view(-1)
            idx = torch.randperm(flat.numel(), generator=gen)[:zero_w]
            flat[idx] = 0.0
    w0 = layer.weight.detach().clone()
    b0 = layer.bias.detach().clone() if bias else torch.zeros(0)
    xin = x.clone().requires_grad_(True)
    y = layer(xin)
    dy = torch.randn(y.shape, generator=gen)
    y.backward(dy)
    save(name, x=np32(x), w_latent=np32(w0), bias=np32(b0), y=np32(y),
         x_after=np32(xin), w_data_after=np32(layer.weight), dy=np32(dy),
         dx=np32(xin.grad), dw=np32(layer.weight.grad),
         db=np32(layer.bias.grad) if bias else np.zeros(0, np.float32),
         has_bias=np.array(bias))


def conv_case(name, gen, x, cin, cout, k, stride=1, padding=0, dilation=1, groups=1, bias=True):
    torch.manual_seed(2000 + cin * 7 + cout)
    layer = BinarizeConv2d(cin, cout, k, stride=stride, padding=padding,
                           dilation=dilation, groups=groups, bias=bias)
    w0 = layer.weight.detach().clone()
    b0 = layer.bias.detach().clone() if bias else torch.zeros(0)
    xin = x.clone().requires_grad_(True)
    y = layer(xin)
    dy = torch.randn(y.shape, generator=gen)
    y.backward(dy)
    save(name, x=np32(x), w_latent=np32(w0), bias=np32(b0), y=np32(y),
         x_after=np32(xin), dy=np32(dy), dx=np32(xin.grad), dw=np32(layer.weight.grad),
         db=np32(layer.bias.grad) if bias else np.zeros(0, np.float32),
         conv=np.array([stride, padding, dilation, groups], np.int64),
         has_bias=np.array(bias))


class TraceNet(nn.Module):
    """mnist-dist2.py:46-76 topology (fc-bn-htanh x3, dropout before bn3, fc4, LogSoftmax)."""

    def __init__(self, h1, h2, h3, p_drop):
        super().__init__()
        self.fc1 = BinarizeLinear(784, h1)
        self.htanh1 = nn.Hardtanh()
        self.bn1 = nn.BatchNorm1d(h1)
        self.fc2 = BinarizeLinear(h1, h2)
        self.htanh2 = nn.Hardtanh()
        self.bn2 = nn.BatchNorm1d(h2)
        self.fc3 = BinarizeLinear(h2, h3)
        self.htanh3 = nn.Hardtanh()
        self.bn3 = nn.BatchNorm1d(h3)
        self.fc4 = nn.Linear(h3, 10)
        self.logsoftmax = nn.LogSoftmax(dim=1)
        self.drop = nn.Dropout(p_drop)

    def forward(self, x):
        x = x.view(-1, 28 * 28)
        x = self.htanh1(self.bn1(self.fc1(x)))
        x = self.htanh2(self.bn2(self.fc2(x)))
        x = self.fc3(x)
        x = self.drop(x)
        x = self.htanh3(self.bn3(x))
        x = self.fc4(x)
        return self.logsoftmax(x)


PARAM_NAMES = ["fc1.weight", "fc1.bias", "bn1.weight", "bn1.bias", "fc2.weight", "fc2.bias",
               "bn2.weight", "bn2.bias", "fc3.weight", "fc3.bias", "bn3.weight", "bn3.bias",
               "fc4.weight", "fc4.bias"]


def trace_case(name, gen, org_protocol, steps=3, batch=16, widths=(48, 32, 24), lr=0.01):
    torch.manual_seed(7)
    net = TraceNet(*widths, p_drop=0.0)
    init = {k: np32(v) for k, v in net.state_dict().items()}
    opt = torch.optim.Adam(net.parameters(), lr=lr)
    crit = nn.CrossEntropyLoss()
    rec = {"init/" + k: v for k, v in init.items()}
    # the reference's binarized hidden activations: BinarizeLinear leaves sign(input) in the
    # caller's tensor (binarized_modules.py:75-76), recorded from fc2 / fc3 after each call, so a
    # replay can tell BatchNorm near-tie resolutions (implementation rounding) from real errors
    acts = {}

    def keep(name):
        def hook(mod, inp, out):
            acts[name] = np32(inp[0]).astype(np.int8)
        return hook

    net.fc2.register_forward_hook(keep("fc2_in"))
    net.fc3.register_forward_hook(keep("fc3_in"))
    net.train()
    for s in range(steps):
        x = mnist_like(gen, (batch, 1, 28, 28))
        t = torch.randint(0, 10, (batch,), generator=gen)
        rec[f"s{s}/x"] = np32(x)
        rec[f"s{s}/target"] = t.numpy().astype(np.int64)
        opt.zero_grad()
        out = net(x)
        loss = crit(out, t)
        loss.backward()
        rec[f"s{s}/out"] = np32(out)
        rec[f"s{s}/loss"] = np.array(loss.item(), np.float64)
        for k, v in acts.items():
            rec[f"s{s}/act/{k}"] = v
        named = dict(net.named_parameters())
        for k in PARAM_NAMES:
            rec[f"s{s}/grad/{k}"] = np32(named[k].grad)
        if org_protocol:          # mnist-dist2.py:131-137
            for p in net.parameters():
                if hasattr(p, "org"):
                    p.data.copy_(p.org)
            opt.step()
            for p in net.parameters():
                if hasattr(p, "org"):
                    p.org.copy_(p.data.clamp_(-1, 1))
        else:                     # mnist-dist3.py:116-119
            opt.step()
        for k in PARAM_NAMES:
            p = named[k]
            rec[f"s{s}/data/{k}"] = np32(p)
            if hasattr(p, "org"):
                rec[f"s{s}/org/{k}"] = np32(p.org)
        for k, v in net.state_dict().items():
            if "running" in k:
                rec[f"s{s}/buf/{k}"] = np32(v)
    rec["meta/widths"] = np.array(widths, np.int64)
    rec["meta/lr"] = np.array(lr, np.float64)
    rec["meta/org_protocol"] = np.array(org_protocol)
    save(name, **rec)


def mnist_u8(gen, shape):
    """The same synthetic MNIST-shaped pixels as bytes (80.7% exact zeros, rest 1..255)."""
    u = torch.rand(shape, generator=gen)
    v = torch.randint(1, 256, shape, generator=gen, dtype=torch.int64)
    return torch.where(u < 0.807, torch.zeros_like(v), v).to(torch.uint8)


def _bits(a):
    """Sign pattern of a float array as packed bits (1 = positive), plus the count of zeros."""
    a = np.asarray(a)
    return np.packbits((a > 0).reshape(-1)), np.array(int((a == 0).sum()), np.int64)


def trace_wide_case(name, steps=10, batch=256, widths=(256, 256, 256), lr=0.01):
    """mnist-dist2.py:118-137 (org protocol, p = 0) at widths where every fusion of the build's
    benched path applies (C % 256 for the fused head and the FP4 tiles, C % 64 for the FP6
    hand-offs), input given as u8 pixels through ToTensor (x = u/255, mnist-dist2.py:96-99) so the
    u8 pixel path reproduces it exactly.  Recorded: the loss and log-probs of every step, the
    step-0 gradients of every parameter, the per-step gradients of the small (non-binarized)
    parameters, the sign pattern and a float64 digest (sum, sum |.|, sum of squares) of every
    latent weight after each step, the binarized activations of fc2 / fc3 (sign bits) per step,
    and the final latent weights, parameters and running statistics."""
    gen = torch.Generator().manual_seed(4321)
    torch.manual_seed(11)
    net = TraceNet(*widths, p_drop=0.0)
    rec = {"init/" + k: np32(v) for k, v in net.state_dict().items()}
    opt = torch.optim.Adam(net.parameters(), lr=lr)
    crit = nn.CrossEntropyLoss()
    acts = {}

    def keep(nm):
        def hook(mod, inp, out):
            acts[nm] = np32(inp[0])
        return hook

    net.fc2.register_forward_hook(keep("fc2_in"))
    net.fc3.register_forward_hook(keep("fc3_in"))
    net.train()
    named = dict(net.named_parameters())
    small = [k for k in PARAM_NAMES if k not in ("fc1.weight", "fc2.weight", "fc3.weight")]
    for s in range(steps):
        u = mnist_u8(gen, (batch, 1, 28, 28))
        t = torch.randint(0, 10, (batch,), generator=gen)
        x = u.float().div(255.0)                   # transforms.ToTensor()
        rec[f"s{s}/u8"] = u.numpy().reshape(batch, 784)
        rec[f"s{s}/target"] = t.numpy().astype(np.int64)
        opt.zero_grad()
        out = net(x)
        loss = crit(out, t)
        loss.backward()
        rec[f"s{s}/out"] = np32(out)
        rec[f"s{s}/loss"] = np.array(loss.item(), np.float64)
        for k, v in acts.items():
            rec[f"s{s}/act/{k}"], rec[f"s{s}/act0/{k}"] = _bits(v)
        for k in (PARAM_NAMES if s == 0 else small):
            rec[f"s{s}/grad/{k}"] = np32(named[k].grad)
        for p in net.parameters():                 # mnist-dist2.py:131-137
            if hasattr(p, "org"):
                p.data.copy_(p.org)
        opt.step()
        for p in net.parameters():
            if hasattr(p, "org"):
                p.org.copy_(p.data.clamp_(-1, 1))
        for k in ("fc1.weight", "fc2.weight", "fc3.weight"):
            o = named[k].org.double().numpy()
            rec[f"s{s}/orgsign/{k}"], rec[f"s{s}/orgzero/{k}"] = _bits(o)
            rec[f"s{s}/orgdigest/{k}"] = np.array([o.sum(), np.abs(o).sum(), (o * o).sum()], np.float64)
    for k in PARAM_NAMES:
        p = named[k]
        rec[f"final/data/{k}"] = np32(p.org if hasattr(p, "org") else p)
    for k, v in net.state_dict().items():
        if "running" in k:
            rec[f"final/buf/{k}"] = np32(v)
    rec["meta/widths"] = np.array(widths, np.int64)
    rec["meta/lr"] = np.array(lr, np.float64)
    rec["meta/steps"] = np.array(steps, np.int64)
    save(name, **rec)


class TraceCNN(nn.Module):
    """The build's BinCNN (BASELINE config 4) with the reference's own BinarizeConv2d
    (binarized_modules.py:87-107), on the ConvNet template of mnist-dist.py:31-51 (conv5x5 p2 ->
    BatchNorm2d -> MaxPool2d(2), twice, then Linear(7*7*32, 10)) with Hardtanh in place of ReLU,
    as in mnist-dist2.py's Net.  Module names follow nets.BinCNN so the state_dicts match."""

    def __init__(self):
        super().__init__()
        self.layer1 = nn.Sequential(BinarizeConv2d(1, 16, kernel_size=5, stride=1, padding=2),
                                    nn.BatchNorm2d(16), nn.Hardtanh(), nn.MaxPool2d(kernel_size=2, stride=2))
        self.layer2 = nn.Sequential(BinarizeConv2d(16, 32, kernel_size=5, stride=1, padding=2),
                                    nn.BatchNorm2d(32), nn.Hardtanh(), nn.MaxPool2d(kernel_size=2, stride=2))
        self.fc = nn.Linear(7 * 7 * 32, 10)
        self.logsoftmax = nn.LogSoftmax(dim=1)

    def forward(self, x):
        out = self.layer2(self.layer1(x))
        return self.logsoftmax(self.fc(out.reshape(out.size(0), -1)))


CNN_PARAMS = ["layer1.0.weight", "layer1.0.bias", "layer1.1.weight", "layer1.1.bias", "layer2.0.weight",
              "layer2.0.bias", "layer2.1.weight", "layer2.1.bias", "fc.weight", "fc.bias"]


def trace_cnn_case(name, steps=8, batch=256, lr=0.01):
    """The BinCNN trained by the reference loop (mnist-dist2.py:118-137: CrossEntropy on the
    log-probs, org restore -> Adam -> clamp), input = ToTensor of u8 pixels (conv1 binarises it:
    C = 1 != 3, binarized_modules.py:94-95).  Recorded per step: the u8 batch and targets, loss,
    log-probs, every gradient, the latent conv weights (.org) and their sign bits after the
    update, the binarized input of conv2 (sign bits + zero count), every parameter after the
    update and the running statistics."""
    gen = torch.Generator().manual_seed(8642)
    torch.manual_seed(13)
    net = TraceCNN()
    rec = {"init/" + k: np32(v) for k, v in net.state_dict().items()}
    opt = torch.optim.Adam(net.parameters(), lr=lr)
    crit = nn.CrossEntropyLoss()
    acts = {}
    net.layer2[0].register_forward_hook(lambda mod, inp, out: acts.__setitem__("conv2_in", np32(inp[0])))
    net.train()
    named = dict(net.named_parameters())
    for s in range(steps):
        u = mnist_u8(gen, (batch, 1, 28, 28))
        t = torch.randint(0, 10, (batch,), generator=gen)
        x = u.float().div(255.0)                   # transforms.ToTensor()
        rec[f"s{s}/u8"] = u.numpy().reshape(batch, 784)
        rec[f"s{s}/target"] = t.numpy().astype(np.int64)
        opt.zero_grad()
        out = net(x)
        loss = crit(out, t)
        loss.backward()
        rec[f"s{s}/out"] = np32(out)
        rec[f"s{s}/loss"] = np.array(loss.item(), np.float64)
        rec[f"s{s}/act/conv2_in"], rec[f"s{s}/act0/conv2_in"] = _bits(acts["conv2_in"])
        for k in CNN_PARAMS:
            rec[f"s{s}/grad/{k}"] = np32(named[k].grad)
        for p in net.parameters():                 # mnist-dist2.py:131-137
            if hasattr(p, "org"):
                p.data.copy_(p.org)
        opt.step()
        for p in net.parameters():
            if hasattr(p, "org"):
                p.org.copy_(p.data.clamp_(-1, 1))
        for k in CNN_PARAMS:
            p = named[k]
            rec[f"s{s}/data/{k}"] = np32(p.org if hasattr(p, "org") else p)
        for k in ("layer1.0.weight", "layer2.0.weight"):
            rec[f"s{s}/orgsign/{k}"], rec[f"s{s}/orgzero/{k}"] = _bits(named[k].org.numpy())
        for k, v in net.state_dict().items():
            if "running" in k:
                rec[f"s{s}/buf/{k}"] = np32(v)
    rec["meta/lr"] = np.array(lr, np.float64)
    rec["meta/steps"] = np.array(steps, np.int64)
    save(name, **rec)


def main():
    if sys.argv[1:] == ["trace_wide"]:        # regenerate only the wide trace
        trace_wide_case("trace_wide")
        return
    if sys.argv[1:] == ["trace_cnn"]:         # regenerate only the BinCNN trace
        trace_cnn_case("trace_cnn")
        return
    gen = torch.Generator().manual_seed(1234)
    # 1. first layer: input width 784 -> NOT binarised (binarized_modules.py:75)
    x = mnist_like(gen, (8, 784))
    linear_case("linear_first", gen, 784, 64, 8, x)
    # 2. hidden layer with exact zeros in the input (sign(0)=0: ternary)
    x = torch.randn(8, 256, generator=gen)
    x[torch.rand(x.shape, generator=gen) < 0.1] = 0.0
    linear_case("linear_hidden", gen, 256, 128, 8, x)
    # 3. no bias, zeros in the latent weight, ragged sizes
    x = torch.randn(5, 100, generator=gen)
    linear_case("linear_nobias_zw", gen, 100, 37, 5, x, bias=False, zero_w=50)
    # 4. conv, C=1 (!=3 so the pixels ARE binarised: binarized_modules.py:94-95), pad 2
    x = mnist_like(gen, (4, 1, 28, 28))
    conv_case("conv_c1", gen, x, 1, 16, 5, padding=2)
    # 5. conv C=16 -> 32, k5 p2 (build CNN conv2 shape)
    x = torch.randn(4, 16, 14, 14, generator=gen)
    x[torch.rand(x.shape, generator=gen) < 0.05] = 0.0
    conv_case("conv_c16", gen, x, 16, 32, 5, padding=2)
    # 6. conv C=3 -> input NOT binarised (fp32 conv)
    x = torch.randn(2, 3, 9, 9, generator=gen)
    conv_case("conv_c3", gen, x, 3, 8, 3, padding=1)
    # 7. stride/dilation/groups, no bias
    x = torch.randn(2, 4, 11, 11, generator=gen)
    conv_case("conv_sdg", gen, x, 4, 6, 3, stride=2, padding=2, dilation=2, groups=2, bias=False)
    # 8. Binarize / HingeLoss
    x = torch.randn(64, generator=gen)
    x[::7] = 0.0
    inp = torch.randn(16, 10, generator=gen)
    tgt = torch.where(torch.rand(16, 10, generator=gen) < 0.5, -1.0, 1.0)
    save("misc", binarize_in=np32(x), binarize_out=np32(Binarize(x.clone())),
         hinge_in=np32(inp), hinge_tgt=np32(tgt), hinge_out=np.array(HingeLoss()(inp, tgt).item()))
    # 9. training traces (dropout p=0): with the org protocol, and without it
    trace_case("trace_org", gen, org_protocol=True)
    trace_case("trace_frozen", gen, org_protocol=False)
    # 10. DistributedSampler order the reference relies on (mnist-dist2.py:100-102):
    from torch.utils.data.distributed import DistributedSampler
    rec = {}
    for n, ws in ((100, 2), (101, 3), (60000, 8)):
        for r in range(ws):
            s = DistributedSampler(range(n), num_replicas=ws, rank=r)
            idx = np.array(list(iter(s)), np.int64)
            rec[f"n{n}_ws{ws}_r{r}"] = idx if n < 1000 else idx[:64]
    save("sampler", **rec)
    # 11. the wide trace (every fusion of the benched path applies)
    trace_wide_case("trace_wide")
    # 12. the BinCNN (config 4) trace on the reference's BinarizeConv2d
    trace_cnn_case("trace_cnn")


if __name__ == "__main__":
    main()

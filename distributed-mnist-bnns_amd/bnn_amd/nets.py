"""Networks of the reference's training scripts, built on the libbnn layers.

* ``Net`` -- mnist-dist2.py:46-76: 784-(1024r)-(512r)-(256r)-10, r = infl_ratio = 3,
  fc -> BatchNorm1d -> Hardtanh per hidden layer, Dropout(0.3) between fc3 and bn3,
  fc4 = nn.Linear, LogSoftmax.
* ``SmallNet`` -- mnist-dist3.py:40-70 (64r = 192 wide; the source of the published CSVs).
* ``WideNet`` -- BASELINE config 5: 784-8192x3-10, same topology.
* Inputs: fp32 images (what the reference's transform yields) or the uint8 pixels themselves
  (``data.synthetic_mnist(..., as_u8=True)``, ``data.U8Dataset``): fc1 then works on the bytes.
* ``BinCNN`` -- BASELINE config 4 (build-defined; the reference never instantiates
  BinarizeConv2d): the ConvNet template of mnist-dist.py:31-51 with binarised convolutions and
  Hardtanh in place of ReLU: conv5x5(1->16,p2)-BN-Hardtanh-MaxPool2, conv5x5(16->32,p2)-BN-
  Hardtanh-MaxPool2, Linear(1568->10), LogSoftmax.
"""
import torch
import torch.nn as nn

from . import functional as BF
from .nn import BatchNorm1d, BinarizeConv2d, BinarizeLinear


def _configure(module, org_protocol, mutate_input, backend=None):
    for m in module.modules():
        if isinstance(m, (BinarizeLinear, BinarizeConv2d)):
            m.org_protocol = org_protocol
            m.mutate_input = mutate_input
            if backend is not None and isinstance(m, BinarizeLinear):
                m.backend = backend
    return module


class MLP(nn.Module):
    """mnist-dist2.py:46-76 with explicit widths."""

    def __init__(self, h1, h2, h3, p_drop=0.3, org_protocol=True, mutate_input=True, backend=None,
                 fused_bn=False, normalize=None, dropin_bn=False):
        super().__init__()
        # dropin_bn: bn1..bn3 are bnn_amd.nn.BatchNorm1d (torch's module on libbnn's passes), the
        # drop-in a user of the reference swaps for nn.BatchNorm1d; the modules and state_dict keep
        # their names and shapes either way
        BN = BatchNorm1d if dropin_bn else nn.BatchNorm1d
        # fused_bn: bn_i -> htanh_i run as one libbnn BatchNorm+Hardtanh pass (same parameters,
        # buffers and math; replaces torch's BatchNorm1d kernels)
        self.fused_bn = fused_bn
        self.fused_head = True     # with fused_bn: drop -> bn3 -> htanh3 -> fc4 as one libbnn op
        self.fc1 = BinarizeLinear(784, h1)
        self.htanh1 = nn.Hardtanh()
        self.bn1 = BN(h1)
        self.fc2 = BinarizeLinear(h1, h2)
        self.htanh2 = nn.Hardtanh()
        self.bn2 = BN(h2)
        self.fc3 = BinarizeLinear(h2, h3)
        self.htanh3 = nn.Hardtanh()
        self.bn3 = BN(h3)
        self.fc4 = nn.Linear(h3, 10)
        self.logsoftmax = nn.LogSoftmax(dim=1)
        self.drop = nn.Dropout(p_drop)
        # uint8 pixel batches: fc1 applies ToTensor (+ Normalize(*normalize)) on the bytes
        self.fc1.pixel_normalize = normalize
        _configure(self, org_protocol, mutate_input, backend)

    def _bnh(self, bn, ht, x):
        if self.fused_bn and x.is_cuda and x.dim() == 2 and x.shape[1] % 4 == 0:
            return BF.batch_norm_hardtanh(x, bn)
        return ht(bn(x))

    def _fusable(self, fc, z):
        return (self.fused_bn and z.is_cuda and z.dim() == 2 and z.shape[1] % 4 == 0 and not fc.org_protocol
                and fc.backend in ("fp4", "mfma"))

    def _bnh_fc(self, bn, ht, fc, z, emit_z16=False, emit_stats=False):
        """fc(ht(bn(z))); fused into one libbnn op (no fp32 hardtanh output) when the fc keeps
        its latent weight in the Parameter and runs an MFMA backend.  emit_stats: fc's FP4 forward
        also forms the next (training-mode, fused) BatchNorm's forward statistics."""
        if self._fusable(fc, z):
            return BF.bn_hardtanh_binary_linear(z, bn, fc, fc.backend, emit_z16=emit_z16, emit_stats=emit_stats)
        return fc(self._bnh(bn, ht, z))

    def _z16(self, fc, M, consumer):
        """fc's output may travel as int16 dot products + bias (functional.z16_ok): it is produced by
        the fused FP4 path and its consumer is a z16-aware libbnn BatchNorm pass."""
        return (consumer and self.training and fc.backend == "fp4" and not fc.org_protocol
                and BF.z16_ok(M, fc.out_features, fc.in_features))

    def _head_fused(self, x_width):
        return (self.fused_bn and self.fused_head and self.training and self.bn3.training
                and x_width % 256 == 0 and self.fc4.out_features == BF.HEAD_NOUT and self.bn3.track_running_stats
                and self.bn3.momentum is not None)

    def _s20(self, x):
        """fc1 (on u8 pixels) may hand z1 on as its exact integer sums (functional S20): its consumer
        is the training-mode fused bn1 -> fc2 op on the FP4/FP6 backend."""
        return (x.dtype == torch.uint8 and x.is_cuda and self.fused_bn and self.training and self.bn1.training
                and self.bn1.track_running_stats and self.fc2.backend == "fp4" and BF.DIGIT_GEMM == "fp6"
                and not self.fc2.org_protocol and self.fc1.out_features % 256 == 0)

    def forward(self, x):
        with BF.bn_counter_batch():          # the BatchNorms' num_batches_tracked += 1 in one launch
            return self._forward(x)

    def _forward(self, x):
        x = x.view(-1, 28 * 28)
        z1 = self.fc1(x, emit_compact=True) if self._s20(x) else self.fc1(x)
        M = z1.shape[0]
        fuse2 = self._fusable(self.fc2, z1)
        # fc2's output feeds the fused bn2 -> fc3 op; fc3's the fused head
        z16_2 = fuse2 and self._z16(self.fc2, M, self._fusable(self.fc3, z1) and self.fc3.backend == "fp4"
                                    and self.bn2.training)
        # bn2 (no dropout ahead of it) takes its forward statistics from fc2's epilogue
        st2 = fuse2 and self._fusable(self.fc3, z1) and self.bn2.training and self.training
        x = self._bnh_fc(self.bn1, self.htanh1, self.fc2, z1, emit_z16=z16_2, emit_stats=st2)
        z16_3 = (self._fusable(self.fc3, x) and self._z16(self.fc3, M, self._head_fused(self.fc3.out_features))
                 and x.is_cuda)
        # (bn3's statistics of drop(z3) could come from fc3's epilogue too -- emit_stats=(p, seed) with
        # the head's seed drawn first -- but the mask hash in the epilogue costs more than the pass:
        # DESIGN §5)
        x = self._bnh_fc(self.bn2, self.htanh2, self.fc3, x, emit_z16=z16_3)
        if (self.fused_bn and self.fused_head and self.training and self.bn3.training
                and BF.head_fusable(x, self.bn3, self.fc4)):
            # drop -> bn3 -> htanh3 -> fc4 as one libbnn head: h3 is never written
            return self.logsoftmax(BF.dropout_bn_hardtanh_linear(x, self.drop.p, self.bn3, self.fc4))
        if (self.fused_bn and self.training and self.drop.p > 0 and self.bn3.training and x.is_cuda
                and x.dim() == 2 and x.shape[1] % 4 == 0):
            # drop -> bn3 -> htanh3 as one libbnn op (mask regenerated in every pass, never stored)
            x = BF.dropout_batch_norm_hardtanh(x, self.drop.p, self.bn3)
        else:
            x = self.drop(x)
            x = self._bnh(self.bn3, self.htanh3, x)
        x = self.fc4(x)
        return self.logsoftmax(x)


def Net(infl_ratio=3, **kw):
    """mnist-dist2.py Net: 784-3072-1536-768-10 at infl_ratio 3."""
    return MLP(1024 * infl_ratio, 512 * infl_ratio, 256 * infl_ratio, **kw)


def SmallNet(infl_ratio=3, **kw):
    """mnist-dist3.py Net: 784-192-192-192-10."""
    return MLP(64 * infl_ratio, 64 * infl_ratio, 64 * infl_ratio, **kw)


def WideNet(width=8192, **kw):
    """BASELINE config 5: 784-8192x3-10."""
    return MLP(width, width, width, **kw)


class BinCNN(nn.Module):
    def __init__(self, num_classes=10, org_protocol=True, mutate_input=True, fused_bn=False):
        super().__init__()
        # fused_bn: BatchNorm2d -> Hardtanh -> MaxPool2d of each layer run as one libbnn op (same
        # parameters, buffers and math; the Sequential modules and state_dict are unchanged)
        self.fused_bn = fused_bn
        self.layer1 = nn.Sequential(BinarizeConv2d(1, 16, kernel_size=5, stride=1, padding=2),
                                    nn.BatchNorm2d(16), nn.Hardtanh(), nn.MaxPool2d(kernel_size=2, stride=2))
        self.layer2 = nn.Sequential(BinarizeConv2d(16, 32, kernel_size=5, stride=1, padding=2),
                                    nn.BatchNorm2d(32), nn.Hardtanh(), nn.MaxPool2d(kernel_size=2, stride=2))
        self.fc = nn.Linear(7 * 7 * 32, num_classes)
        self.logsoftmax = nn.LogSoftmax(dim=1)
        _configure(self, org_protocol, mutate_input)

    def _layer(self, seq, x):
        conv, bn, ht, pool = seq
        fuse = (self.fused_bn and isinstance(bn, nn.BatchNorm2d) and pool.kernel_size == 2 and pool.stride == 2
                and pool.padding == 0 and not pool.ceil_mode and ht.min_val == -1.0 and ht.max_val == 1.0)
        # training-mode fused layers take the conv output as its exact integer sums (int8 / int16 +
        # bias: 1/4 or 1/2 the bytes of every BatchNorm2d pass over it)
        z = conv(x, emit_compact=fuse and bn.training)
        if fuse and BF.bn2d_fusable(z, 2):
            return BF.batch_norm2d_hardtanh_pool(z, bn, hardtanh=True, pool=2)
        return pool(ht(bn(z)))

    def forward(self, x):
        with BF.bn_counter_batch():          # the BatchNorms' num_batches_tracked += 1 in one launch
            return self._forward(x)

    def _forward(self, x):
        out = self._layer(self.layer2, self._layer(self.layer1, x))
        out = out.reshape(out.size(0), -1)
        if self.fused_bn and BF.linear_nsmall_ok(out, self.fc.weight):
            # the fp32 classifier through libbnn's narrow-Linear kernels (same parameters and math)
            return self.logsoftmax(BF.linear_nsmall(out, self.fc.weight, self.fc.bias))
        return self.logsoftmax(self.fc(out))


MODELS = {"mlp": Net, "small": SmallNet, "wide": WideNet, "cnn": BinCNN}


def binary_params(model):
    """Parameters the reference clamps: weights and biases of BinarizeLinear/BinarizeConv2d
    (they carry ``.org``, mnist-dist2.py:131-137)."""
    out = []
    for m in model.modules():
        if isinstance(m, (BinarizeLinear, BinarizeConv2d)):
            out.append(m.weight)
            if m.bias is not None:
                out.append(m.bias)
    return out

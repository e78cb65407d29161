"""The reference operator API (models/binarized_modules.py) on libbnn.

Names, constructor signatures and side effects follow the reference:

* ``Binarize(tensor, quant_mode='det')``                   -- :11-15
* ``HingeLoss``                                            -- :20-32
* ``SqrtHingeLossFunction`` (stub: the reference's is a pre-0.4 autograd Function with a
  ``pdb.set_trace()`` in backward, :34-54)
* ``Quantize(tensor, quant_mode='det', params=None, numBits=8)`` -- :56-63
* ``BinarizeLinear(*kargs, **kwargs)`` (an ``nn.Linear``)   -- :68-85
* ``BinarizeConv2d(*kargs, **kwargs)`` (an ``nn.Conv2d``)   -- :87-107

and the training loop's criterion, ``CrossEntropyLoss`` (mnist-dist2.py:118-137), on libbnn.

Side effects kept (the caller loop of mnist-dist2.py:131-137 depends on them):
  ``weight.org`` is created once on the first forward from ``weight.data`` (:77-78),
  ``weight.data`` is replaced by ``sign(weight.org)`` every forward (:79),
  ``bias.org`` is re-cloned every forward (:82, :104), and the caller's input tensor is
  replaced by its sign unless the first-layer rule applies (:75-76, :94-95).

Two class attributes switch behaviour for the build's own trainer:
  ``org_protocol = False`` keeps the latent weight in the Parameter itself (no ``.org``,
  binarised on the fly inside the kernel; pair it with ``bnn_amd.optim.LatentAdam``), and
  ``mutate_input = False`` skips materialising ``sign(input)`` in fp32 (nothing reads it).

A ``uint8`` input to a 784-input ``BinarizeLinear`` is taken as the raw pixels the reference's
loader would turn into ``ToTensor()`` (``u/255``), followed by ``Normalize(*pixel_normalize)``
when that attribute is set: the layer then runs on the bytes (functional.binary_linear_pixels),
with the same output as on the fp32 tensor the transform would have produced.
"""
import torch
import torch.nn as nn

from . import functional as BF

__all__ = ["Binarize", "HingeLoss", "SqrtHingeLossFunction", "Quantize", "BinarizeLinear", "BatchNorm1d",
           "BinarizeConv2d", "CrossEntropyLoss"]


def Binarize(tensor, quant_mode="det"):
    """Deterministic: ``tensor.sign()`` as a new tensor (libbnn).  Stochastic (reference :15, never
    used by the reference modules): in place, ``round(clamp((x+1)/2 + U(-.5,.5), 0, 1))*2 - 1``."""
    if quant_mode == "det":
        return BF.sign(tensor)
    noise = torch.rand(tensor.size(), device=tensor.device, dtype=tensor.dtype) - 0.5
    prob = tensor.add_(1.0).div_(2.0).add_(noise).clamp_(0.0, 1.0)
    return prob.round().mul_(2.0).sub_(1.0)


class HingeLoss(nn.Module):
    """mean(max(0, margin - input*target)), margin = 1 (reference :20-32)."""

    def __init__(self):
        super().__init__()
        self.margin = 1.0

    def hinge_loss(self, input, target):
        # output[output.le(0)] = 0 (:27-29): relu zeroes the gradient where margin - x*t <= 0,
        # ties included, and keeps NaN, as the masked assignment does
        return torch.relu(self.margin - input * target).mean()

    def forward(self, input, target):
        return self.hinge_loss(input, target)


class CrossEntropyLoss(nn.CrossEntropyLoss):
    """The training loop's criterion (mnist-dist2.py:118-137: ``nn.CrossEntropyLoss()`` on the nets'
    LogSoftmax output) on libbnn (functional.cross_entropy: one row-loss + one fold launch forward,
    one backward, no host synchronisation) for CUDA fp32 [M, C] rows with C in {2, 10, 16, 32, 64},
    int64 class-index targets, no class weights, reduction 'mean' and no label smoothing; anything
    else goes to torch.  Rows whose target is ``ignore_index`` are skipped on the device as torch
    skips them (the mean is over the other rows)."""

    def forward(self, input, target):
        if (self.weight is None and self.reduction == "mean" and self.label_smoothing == 0.0
                and BF.cross_entropy_ok(input, target)):
            return BF.cross_entropy(input, target, self.ignore_index)
        return super().forward(input, target)


class SqrtHingeLossFunction(torch.autograd.Function):
    """Exported for import compatibility only.  The reference version (:34-54) is a legacy
    non-static autograd.Function that drops into pdb in backward; no reference script uses it."""

    @staticmethod
    def forward(ctx, input, target):
        raise NotImplementedError("SqrtHingeLossFunction is not part of the BNN hot path "
                                  "(the reference implementation is non-functional)")


def Quantize(tensor, quant_mode="det", params=None, numBits=8):
    """Reference :56-63.  Deterministic mode clamps in place then rounds to numBits-1 fractional
    bits; the stochastic mode calls an undefined ``quant_fixed`` in the reference (NameError)."""
    lim = 2.0 ** (numBits - 1)
    tensor.clamp_(-lim, lim)
    if quant_mode == "det":
        return tensor.mul(lim).round().div(lim)
    raise NotImplementedError("Quantize(quant_mode!='det') calls an undefined quant_fixed in the reference")


def _apply_org_protocol(p):
    """binarized_modules.py:77-79: lazily keep the latent copy, expose its sign in .data."""
    if not hasattr(p, "org"):
        p.org = p.data.clone()
    p.data = BF.sign(p.org)


class BinarizeLinear(nn.Linear):
    org_protocol = True
    mutate_input = True
    backend = "fp4"        # ternary GEMM engine: "fp4" (FP4 MFMA), "mfma" (int8 MFMA), "xnor" (VALU)

    def __init__(self, *kargs, **kwargs):
        super().__init__(*kargs, **kwargs)

    pixel_normalize = None   # (mean, std) of a Normalize after ToTensor, for uint8 inputs
    # the 784-input layer recognises fp32 ToTensor images (exact multiples fl(u / 255) of bytes) and
    # runs its u8-pixel GEMMs on them (BF.unit_to_pixels); False keeps the fp32-digit GEMMs
    detect_pixels = True

    def forward(self, input, emit_compact=False):
        # emit_compact (the build's fused MLP only): a u8-pixel layer's output may travel as its
        # exact integer sums (functional.binary_linear_pixels, s20)
        binarize = input.size(1) != 784                       # :75
        if input.dtype == torch.uint8:
            if binarize:
                raise TypeError("BinarizeLinear: uint8 (pixel) input is only defined for the 784-input layer")
            if self.org_protocol:
                _apply_org_protocol(self.weight)
                if self.bias is not None:
                    self.bias.org = self.bias.data.clone()
            return BF.binary_linear_pixels(input, self.weight, self.bias, self.pixel_normalize,
                                           cache=not self.org_protocol, emit_compact=emit_compact)
        if (not binarize and self.detect_pixels and self.pixel_normalize is None and input.dtype == torch.float32
                and input.dim() == 2 and input.is_cuda and not input.requires_grad):
            # fp32 images straight from ToTensor (mnist-dist2.py:96-99): exactly fl(u / 255) for bytes
            # u, so fc1 runs on the bytes -- the same F.linear value within fp32 rounding (the u8
            # path's integer sums are exact), one int8 pass instead of three digit planes each way
            # under graph capture the recognition is replayed only if this layer's eager calls made
            # it (the warm-up of graph.GraphedStep does), guarded by a device flag the replays check
            if torch.cuda.is_current_stream_capturing():
                guard = self.__dict__.get("_pixel_guard") if self.__dict__.get("_pixel_mode") else None
                u = BF.unit_to_pixels(input, guard=guard) if guard is not None else None
            else:
                u = BF.unit_to_pixels(input)
                self._pixel_mode = u is not None
                if u is not None:
                    # a fresh (zero) guard for the next capture; an eager warm-up precedes every one
                    g = self.__dict__.get("_pixel_guard")
                    if g is None or g.device != input.device:
                        self._pixel_guard = torch.zeros((1,), dtype=torch.int32, device=input.device)
                    else:
                        g.zero_()
            if u is not None:
                if self.org_protocol:
                    _apply_org_protocol(self.weight)
                    if self.bias is not None:
                        self.bias.org = self.bias.data.clone()
                return BF.binary_linear_pixels(u, self.weight, self.bias, None, cache=not self.org_protocol)
        xpack = None
        if binarize and self.mutate_input:
            if (self.backend == "fp4" and BF.DIGIT_GEMM == "fp6" and input.dim() == 2 and input.dtype == torch.float32
                    and input.is_cuda):
                # the write-back and the GEMM operands of sign(input) from one read of the input
                need_dw = self.weight.requires_grad and torch.is_grad_enabled()
                s, x4, xqt = BF.sign_pack_fp4_writeback(input.data, want_qt=need_dw)
                input.data = s                                  # :76
                xpack = (x4, xqt)
            else:
                input.data = BF.sign(input.data)                # :76
        if self.org_protocol:
            _apply_org_protocol(self.weight)                    # :77-79
            if self.bias is not None:
                self.bias.org = self.bias.data.clone()          # :82
        return BF.binary_linear(input, self.weight, self.bias, binarize, self.backend,
                                cache=not self.org_protocol, xpack=xpack)


class BatchNorm1d(nn.BatchNorm1d):
    """torch.nn.BatchNorm1d on libbnn's BatchNorm passes, for the reference Nets' bn1..bn3
    (mnist-dist2.py:52-57: nn.BatchNorm1d(3072 * r) etc. between BinarizeLinear and Hardtanh).
    Same constructor, parameters, buffers and state_dict as torch's; torch's _BatchNorm.forward
    semantics (batch statistics with the biased variance in training, the unbiased one into the
    running variance, momentum or the cumulative average for momentum=None, num_batches_tracked,
    track_running_stats=False, affine=False, eval mode) through functional.batch_norm_hardtanh
    with the Hardtanh off.  The statistics are fixed-order double sums (deterministic).  Inputs:
    [M, C] fp32 on the GPU; anything else raises (no silent torch fallback).

    Not in the reference's models/binarized_modules.py: a user of the drop-in swaps
    nn.BatchNorm1d for it to take torch's channels_last BatchNorm kernels (121 of the 182 ms of the
    wide drop-in step) off the path."""

    def forward(self, input):
        if input.dim() != 2 or not input.is_cuda or input.dtype != torch.float32:
            raise TypeError(f"bnn_amd.nn.BatchNorm1d: needs a [M, C] float32 CUDA input (got {tuple(input.shape)} "
                            f"{input.dtype} on {input.device}); use torch.nn.BatchNorm1d for other inputs")
        if input.shape[1] != self.num_features:
            raise ValueError(f"bnn_amd.nn.BatchNorm1d: expected {self.num_features} features, got {input.shape[1]}")
        if self.training and input.shape[0] <= 1:
            raise ValueError("Expected more than 1 value per channel when training")   # torch's message
        # the FP6 digit hand-off stays on: dx is written in full as well and the digits are keyed to
        # that tensor, so a producing BinarizeLinear takes them only when it receives exactly this
        # gradient (a gradient summed with another consumer's is quantised afresh)
        return BF.batch_norm_hardtanh(input, self, hardtanh=False)


class BinarizeConv2d(nn.Conv2d):
    org_protocol = True
    mutate_input = True

    def __init__(self, *kargs, **kwargs):
        super().__init__(*kargs, **kwargs)
        if self.padding_mode != "zeros":
            raise NotImplementedError("BinarizeConv2d: only zero padding (F.conv2d default, :100)")
        if isinstance(self.padding, str):
            raise NotImplementedError("BinarizeConv2d: string padding is not supported")

    def forward(self, input, emit_compact=False):
        # emit_compact (the build's fused BinCNN only): the output may travel as its exact int8 /
        # int16 sums + bias to a libbnn BatchNorm2d (functional.binary_conv2d)
        binarize = input.size(1) != 3                         # :94
        if binarize and self.mutate_input:
            input.data = BF.sign(input.data)                    # :95
        if self.org_protocol:
            _apply_org_protocol(self.weight)                    # :96-98
            if self.bias is not None:
                self.bias.org = self.bias.data.clone()          # :104
        return BF.binary_conv2d(input, self.weight, self.bias, binarize, self.stride, self.padding,
                                self.dilation, self.groups, emit_compact=emit_compact)

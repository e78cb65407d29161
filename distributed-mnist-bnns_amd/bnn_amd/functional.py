"""Tensor-level wrappers of libbnn and the autograd Functions of the binarized layers.

Semantics restated from the reference operator module (models/binarized_modules.py):

* ``Binarize(t, 'det') = t.sign()`` (:11-13) -- ternary, sign(0) = 0.
* ``BinarizeLinear.forward`` (:73-85): input binarised unless ``input.size(1) == 784`` (:75),
  ``F.linear(input, sign(w))`` (:80), then ``out += bias`` in fp32 (:81-83).
* ``BinarizeConv2d.forward`` (:93-107): input binarised unless ``input.size(1) == 3`` (:94).
* autograd: binarisation goes through ``.data`` so the straight-through estimator is the
  identity: dX = dY.W_b, dW = dY^T.X_b, dB = sum dY.

Every op here runs on ROCm tensors through libbnn.so; there is no CPU fallback.
"""
import contextlib

import itertools
import os

import torch

from . import _lib as L

__all__ = [
    "KernelTimer", "timing", "sign", "sign_pack", "sign_pack_bits", "quant_rows", "quant_cols_t", "gemm_i8", "gemm_xnor",
    "quant6_rows", "quant6_cols_t", "gemm_fp6", "set_digit_gemm",
    "binary_linear", "binary_conv2d", "hardtanh_backward", "adam_clamp_", "adam_clamp_pack_", "packed_weight",
    "invalidate_packed", "batch_norm_hardtanh",
    "bn_hardtanh_binary_linear", "batch_norm2d_hardtanh_pool", "dropout_batch_norm_hardtanh", "dropout_mask",
    "BinaryLinearFunction", "BinaryConv2dFunction",
]

ALIGN = 64


# ----------------------------------------------------------------------------- kernel timing
class KernelTimer:
    """HIP-event timing of libbnn launches on the stream they run on (bench.py's roofline).

    Records (kernel, start, end, algorithmic ops, algorithmic bytes) per launch while installed
    with ``timing(timer)``; ``summary()`` synchronises and aggregates per kernel."""

    def __init__(self):
        self.records = []

    def summary(self):
        torch.cuda.synchronize()
        out = {}
        for name, s, e, ops, nbytes in self.records:
            d = out.setdefault(name, {"launches": 0, "ms": 0.0, "ops": 0.0, "bytes": 0.0})
            d["launches"] += 1
            d["ms"] += s.elapsed_time(e)
            d["ops"] += ops
            d["bytes"] += nbytes
        for d in out.values():
            n = d["launches"]
            d["avg_ms"] = d["ms"] / n
            d["avg_ops"] = d["ops"] / n
            d["avg_bytes"] = d["bytes"] / n
        return out


_TIMER = None


@contextlib.contextmanager
def timing(timer):
    global _TIMER
    prev, _TIMER = _TIMER, timer
    try:
        yield timer
    finally:
        _TIMER = prev


@contextlib.contextmanager
def _timed(name, ops=0.0, nbytes=0.0):
    if _TIMER is None:
        yield
        return
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    yield
    e.record()
    _TIMER.records.append((name, s, e, float(ops), float(nbytes)))


GEMM_PAIRS = {(1, 1): 1, (3, 1): 3, (3, 3): 6}


def gemm_kernel_name(a_digits, b_digits, M, N, K):
    """The kernel instance libbnn launches for this GEMM (rocprofv3's name for it)."""
    return L.lib().bnn_gemm_i8_kernel(a_digits, b_digits, M, N, K).decode()


def round_up(x, m=ALIGN):
    return (x + m - 1) // m * m


def _check(*ts, dtype=torch.float32):
    for t in ts:
        if t is None:
            continue
        if not t.is_cuda:
            raise RuntimeError("bnn_amd: libbnn runs on ROCm (cuda) tensors only; "
                               f"got a {t.device} tensor (there is no CPU fallback)")
        if t.dtype != dtype:
            raise TypeError(f"bnn_amd: expected {dtype}, got {t.dtype}")


def _c2d(x):
    """Contiguous fp32 2-D view."""
    if getattr(x, "_bnn_z16", None) is not None or getattr(x, "_bnn_s20", None) is not None:
        raise RuntimeError("a compact pre-activation placeholder reached an op that reads fp32 values")
    return x if x.is_contiguous() else x.contiguous()


# ----------------------------------------------------------------------------- (1) sign / pack
def sign(x, out=None):
    """``Binarize(x, 'det')`` as a new fp32 tensor (models/binarized_modules.py:13)."""
    _check(x)
    x = _c2d(x)
    y = torch.empty_like(x) if out is None else out
    if x.numel() == 0:            # empty tensors have no device pointer; nothing to compute
        return y
    L.call("bnn_sign_f32", L.ptr(x), L.ptr(y), x.numel(), L.stream())
    return y


def sign_pack(x, want_q=True, want_qt=False):
    """fp32 [M,K] -> (q int8 [M, ldq] ternary, qt int8 [K, ldqt] transposed); padding zeroed."""
    _check(x)
    x = _c2d(x)
    M, K = x.shape
    q = qt = None
    if want_q:
        q = torch.empty((M, round_up(K)), dtype=torch.int8, device=x.device)
    if want_qt:
        qt = torch.empty((K, round_up(M)), dtype=torch.int8, device=x.device)
    nbytes = 4 * M * K + (q.numel() if q is not None else 0) + (qt.numel() if qt is not None else 0)
    with _timed("sign_pack_tile_k", 0, nbytes):
        L.call("bnn_sign_pack_i8", L.ptr(x), M, K, K, L.ptr(q), q.shape[1] if q is not None else 0,
               L.ptr(qt), qt.shape[1] if qt is not None else 0, L.stream())
    return q, qt


_QT_CODE = {"i8": 0, "fp4": 1, "fp4p": 2}


def _qt_buffer(K, M, qt_fmt, device):
    """The transposed ternary operand [K, .] of an [M, K] matrix: int8 (qt_fmt "i8"), FP4
    nibbles (qt_fmt "fp4": round_up(M, 256) / 2 bytes per row, the B operand of gemm_fp6), or those
    nibbles in gemm_fp6's panel layout (qt_fmt "fp4p": the rows rounded up to 512, panel_ks =
    shape[1] // 32; see fp4_panels)."""
    if qt_fmt == "fp4":
        return torch.empty((K, round_up(M, 256) // 2), dtype=torch.uint8, device=device)
    if qt_fmt == "fp4p":
        buf = torch.empty(((K + 511) // 512 * 512, round_up(M, 256) // 2), dtype=torch.uint8, device=device)
        if buf.shape[0] > K:
            # the packing kernels write rows < K only; the panel GEMM stages whole 512-row panels,
            # so the pad rows are zeroed here (e2m1 zeros: they add nothing to any column)
            buf[K:].zero_()
        return buf
    return torch.empty((K, round_up(M)), dtype=torch.int8, device=device)


def sign_pack_fp4(x, want_qt=False, qt_fmt="i8", want_q=True):
    """fp32 [M,K] -> (q4 uint8 [M, ldq4] FP4 e2m1 ternary nibbles, qt [K, ldqt] or None).
    ldq4 = round_up(K, 256) / 2 bytes (zero nibbles beyond K); qt as _qt_buffer."""
    _check(x)
    x = _c2d(x)
    M, K = x.shape
    q4 = torch.empty((M, round_up(K, 256) // 2), dtype=torch.uint8, device=x.device) if want_q else None
    qt = _qt_buffer(K, M, qt_fmt, x.device) if want_qt else None
    nbytes = 4 * M * K + (q4.numel() if q4 is not None else 0) + (qt.numel() if qt is not None else 0)
    with _timed("sign_pack_tile_k<1>", 0, nbytes):
        L.call("bnn_sign_pack_fp4", L.ptr(x), M, K, K, L.ptr(q4), q4.shape[1] if q4 is not None else 0,
               L.ptr(qt), qt.shape[1] if qt is not None else 0, _QT_CODE[qt_fmt], L.stream())
    return q4, qt


def sign_pack_fp4_writeback(x, want_qt=False):
    """The drop-in BinarizeLinear's input side effect and its GEMM operands from one read of x:
    (sign(x) fp32 -- the new ``input.data`` of binarized_modules.py:76 -- FP4 rows, FP4 transpose in
    the FP6 GEMM's panel layout or None)."""
    _check(x)
    x = _c2d(x)
    M, K = x.shape
    s = torch.empty_like(x)
    q4 = torch.empty((M, round_up(K, 256) // 2), dtype=torch.uint8, device=x.device)
    qt = _qt_buffer(K, M, "fp4p", x.device) if want_qt else None
    if M == 0:
        return s, q4, qt
    if qt is None:
        sign(x, out=s)
        return (s,) + sign_pack_fp4(s, want_qt=False)[:1] + (None,)
    with _timed("sign_pack_fp4_out", 0, 8 * M * K + q4.numel() + qt.numel()):
        L.call("bnn_sign_pack_fp4_out", L.ptr(x), M, K, L.ptr(q4), q4.shape[1], L.ptr(qt), qt.shape[1],
               _QT_CODE["fp4p"], L.ptr(s), L.stream())
    return s, q4, qt


def sign_pack_bits(x, words=None):
    """fp32 [M,K] -> (sign bits, nonzero bits) int32 [M, words], words >= ceil(K/32)."""
    _check(x)
    x = _c2d(x)
    M, K = x.shape
    kw = words if words is not None else round_up((K + 31) // 32, 32)
    sb = torch.empty((M, kw), dtype=torch.int32, device=x.device)
    nz = torch.empty((M, kw), dtype=torch.int32, device=x.device)
    L.call("bnn_sign_pack_bits", L.ptr(x), M, K, K, L.ptr(sb), L.ptr(nz), kw, L.stream())
    return sb, nz


def quant_rows(x):
    """fp32 [M,K] -> (digits int8 [3, M, ldq], scale fp32 [M]) with x ~= scale*(d2*2^16+d1*2^8+d0)."""
    _check(x)
    x = _c2d(x)
    M, K = x.shape
    ldq = round_up(K)
    dg = torch.empty((3, M, ldq), dtype=torch.int8, device=x.device)
    sc = torch.empty((M,), dtype=torch.float32, device=x.device)
    with _timed("quant_rows_k", 0, 4 * M * K + dg.numel() + 4 * M):
        L.call("bnn_quant_rows", L.ptr(x), M, K, K, L.ptr(dg), ldq, M * ldq, L.ptr(sc), L.stream())
    return dg, sc


def quant_cols_t(x, want_colsum=False, want_dsum=False):
    """fp32 [M,N] -> (digits_t int8 [3, N, ldqt], scale [N], colsum [N] or None), plus the exact
    int64 digit column sums [N] when ``want_dsum`` (bnn_quant_cols_t_dsum)."""
    _check(x)
    x = _c2d(x)
    M, N = x.shape
    ldqt = round_up(M)
    dg = torch.empty((3, N, ldqt), dtype=torch.int8, device=x.device)
    sc = torch.empty((N,), dtype=torch.float32, device=x.device)
    cs = torch.empty((N,), dtype=torch.float32, device=x.device) if want_colsum else None
    ds = torch.empty((N,), dtype=torch.int64, device=x.device) if want_dsum else None
    ws = torch.empty((L.lib().bnn_quant_cols_workspace(M, N),), dtype=torch.uint8, device=x.device)
    with _timed("quant_cols_t", 0, 4 * M * N + dg.numel() + 8 * N):
        L.call("bnn_quant_cols_t_dsum", L.ptr(x), M, N, N, L.ptr(dg), ldqt, N * ldqt, L.ptr(sc), L.ptr(cs),
               L.ptr(ds), L.ptr(ws), L.stream())
    return (dg, sc, cs, ds) if want_dsum else (dg, sc, cs)


# ----------------------------------------------------------------------------- packed latent weights
# The next forward's ternary weight operands, cached on the latent-weight Parameter of a layer
# that keeps its latent weight in the Parameter (``org_protocol = False``).  The fused latent
# update (``optim.LatentAdam`` -> bnn_adam_clamp_pack) rewrites them in place in the same pass
# that updates the weight, so no forward re-packs the weight.  The cache is keyed
# on (data_ptr, _version): torch in-place ops and load_state_dict bump the version; raw writes
# through ``p.data`` do not -- code doing those calls ``invalidate_packed(p)``.
def _pack_key(w):
    return (w.data_ptr(), w._version)


def invalidate_packed(w):
    if hasattr(w, "_bnn_pack"):
        del w._bnn_pack


def packed_weight(weight, fmt, want_q, want_qt, cache=True, qt_fmt="i8"):
    """(q, qt) of sign(weight) [N,K]: q = FP4 rows (fmt "fp4") or int8 rows (fmt "i8"), qt = the
    transpose [K, .] in qt_fmt ("i8" or "fp4", _qt_buffer).  With ``cache`` the operands are kept
    on the Parameter."""
    ent = getattr(weight, "_bnn_pack", None) if cache else None
    same = ent is not None and ent["fmt"] == fmt and ent["qt_fmt"] == qt_fmt
    if same and ent["key"] == _pack_key(weight) \
            and (ent["q"] is not None or not want_q) and (ent["qt"] is not None or not want_qt):
        return ent["q"], ent["qt"]
    if same:                                    # keep producing what earlier forwards needed
        want_q = want_q or ent["q"] is not None
        want_qt = want_qt or ent["qt"] is not None
    if fmt == "fp4" or qt_fmt in ("fp4", "fp4p"):
        assert fmt == "fp4" or not want_q, "int8 rows with an FP4 transpose are not a supported pairing"
        q, qt = sign_pack_fp4(weight, want_qt=want_qt, qt_fmt=qt_fmt, want_q=want_q)
    else:
        q, qt = sign_pack(weight, want_q=want_q, want_qt=want_qt)
    if cache:
        weight._bnn_pack = {"key": _pack_key(weight), "fmt": fmt, "qt_fmt": qt_fmt, "q": q, "qt": qt}
    return q, qt


_DEVICE_STEP = None


class DeviceStep:
    """A device-resident training-step counter, for steps captured in a HIP graph (a replay keeps
    every kernel argument of the capture): while active, dropout masks are drawn from
    seed + ctr * golden (bnn_set_seed_counter) and Adam reads its bias corrections from a host-built
    table at index ctr (bnn_adam_schedule / *_sched); the optimizer advances ctr by one at the end
    of each step, on the device."""

    def __init__(self, device="cuda"):
        self.ctr = torch.zeros((1,), dtype=torch.int64, device=device)
        self.active = False
        self.steps = 0          # host shadow of ctr: advance() in eager steps, note_replays() for graphs

    def activate(self):
        """Make this the process's device step: dropout then uses one base seed (drawn here from
        torch's CPU generator) + the device counter, in eager and captured steps alike."""
        global _DEVICE_STEP
        self.base_seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        L.call("bnn_set_seed_counter", L.ptr(self.ctr))
        self.active = True
        _DEVICE_STEP = self
        return self

    def deactivate(self):
        global _DEVICE_STEP
        L.call("bnn_set_seed_counter", None)
        self.active = False
        if _DEVICE_STEP is self:
            _DEVICE_STEP = None

    def advance(self):
        L.call("bnn_counter_add", L.ptr(self.ctr), 1, L.stream())
        self.steps += 1

    def note_replays(self, n):
        """A captured step that contains one advance() was replayed n times."""
        self.steps += int(n)


def adam_schedule(lr, beta1, beta2, step0, n, device):
    """[n, 2] fp32 (step_size, sqrt(bias_correction2)) for Adam steps step0 .. step0+n-1, computed
    by libbnn's host code exactly as the per-launch form does, copied to ``device``."""
    host = torch.empty((n, 2), dtype=torch.float32)
    L.call("bnn_adam_schedule", float(lr), float(beta1), float(beta2), int(step0), int(n), L.ptr(host))
    return host.to(device)


# BNN_ADAM_TILE256=1 / 0: the 256 x 256-tile form of bnn_adam_clamp_pack on / off (A/B timing);
# unset: the library's default
_ADAM_TILE256 = [os.environ.get("BNN_ADAM_TILE256")]


def adam_clamp_pack_(p, grad, exp_avg, exp_avg_sq, step, lr, beta1=0.9, beta2=0.999, eps=1e-8,
                     grad_scale=1.0, clamp=True, sched=None, ctr=None):
    """bnn_adam_clamp on a 2-D latent weight that also rewrites its cached packed operands (see
    packed_weight).  Returns False (nothing done) when ``p`` has no valid cache."""
    if _ADAM_TILE256[0] is not None:
        L.call("bnn_adam_pack_set_tile256", int(_ADAM_TILE256[0] != "0"))
        _ADAM_TILE256[0] = None
    ent = getattr(p, "_bnn_pack", None)
    if ent is None or ent["key"] != _pack_key(p) or p.dim() != 2:
        return False
    _check(p, grad, exp_avg, exp_avg_sq)
    for t in (p, grad, exp_avg, exp_avg_sq):
        if not t.is_contiguous():
            raise ValueError("adam_clamp_pack_: tensors must be contiguous")
    N, K = p.shape
    q, qt = ent["q"], ent["qt"]
    nbytes = 28 * N * K + (q.numel() if q is not None else 0) + (qt.numel() if qt is not None else 0)
    tail = (1 if ent["fmt"] == "fp4" else 0, L.ptr(q), q.shape[1] if q is not None else 0,
            L.ptr(qt), qt.shape[1] if qt is not None else 0, _QT_CODE[ent["qt_fmt"]], L.stream())
    with _timed("sign_pack_tile_k<adam>", 0, nbytes):
        if sched is not None:
            L.call("bnn_adam_clamp_pack_sched", L.ptr(p), L.ptr(grad), L.ptr(exp_avg), L.ptr(exp_avg_sq), N, K,
                   float(beta1), float(beta2), float(eps), L.ptr(sched), L.ptr(ctr), float(grad_scale),
                   int(bool(clamp)), *tail)
        else:
            L.call("bnn_adam_clamp_pack", L.ptr(p), L.ptr(grad), L.ptr(exp_avg), L.ptr(exp_avg_sq), N, K,
                   float(lr), float(beta1), float(beta2), float(eps), int(step), float(grad_scale),
                   int(bool(clamp)), *tail)
    _bump(p)
    ent["key"] = _pack_key(p)           # the operands just written match the bumped version
    return True


# ----------------------------------------------------------------------------- (2) GEMMs
def gemm_i8(A, a_digits, B, b_digits, M, N, a_scale=None, b_scale=None, bias=None, out=None,
            k_true=None):
    """C[M,N] = combine(sum_k A[.,m,k] B[.,n,k]) * a_scale[m] * b_scale[n] + bias[n].

    A: int8 [M, K] (a_digits=1) or [3, M, K]; B: int8 [N, K] or [3, N, K]; K = padded length
    (multiple of 64, zero padding)."""
    K = A.shape[-1]
    assert B.shape[-1] == K and K % ALIGN == 0
    lda, ldb = A.shape[-1], B.shape[-1]
    a_plane = A.shape[-2] * lda if a_digits > 1 else 0
    b_plane = B.shape[-2] * ldb if b_digits > 1 else 0
    C = torch.empty((M, N), dtype=torch.float32, device=A.device) if out is None else out
    if M == 0 or N == 0:
        return C
    if K == 0:
        C.zero_()
        if bias is not None:
            C += bias
        return C
    k_true = K if k_true is None else k_true
    ops = 2.0 * M * N * k_true          # algorithmic work; digit passes are not work
    name = gemm_kernel_name(a_digits, b_digits, M, N, K) if _TIMER is not None else ""
    with _timed(name, ops, a_digits * M * K + b_digits * N * K + 4 * M * N):
        L.call("bnn_gemm_i8", L.ptr(A), lda, a_plane, a_digits, L.ptr(B), ldb, b_plane, b_digits,
               L.ptr(a_scale), L.ptr(b_scale), L.ptr(bias), L.ptr(C), C.stride(0), M, N, K, L.stream())
    return C


def gemm_i8_affine(A, a_digits, B, b_digits, M, N, a_scale=None, b_scale=None, bias=None, row_off=None,
                   col_off=None, off_mul=0.0, k_true=None, label=None):
    """gemm_i8 with exact integer offsets: C = (sums + off_mul*(row_off[m] + col_off[n])) * a_scale[m]
    * b_scale[n] + bias[n] (bnn_gemm_i8_affine; row_off / col_off int64)."""
    K = A.shape[-1]
    assert B.shape[-1] == K and K % ALIGN == 0
    for o in (row_off, col_off):
        assert o is None or o.dtype == torch.int64
    lda, ldb = A.shape[-1], B.shape[-1]
    a_plane = A.shape[-2] * lda if a_digits > 1 else 0
    b_plane = B.shape[-2] * ldb if b_digits > 1 else 0
    C = torch.empty((M, N), dtype=torch.float32, device=A.device)
    if M == 0 or N == 0:
        return C
    k_true = K if k_true is None else k_true
    name = gemm_kernel_name(a_digits, b_digits, M, N, K) if _TIMER is not None else ""
    if label and name:
        name = f"{name} [{label}]"
    with _timed(name, 2.0 * M * N * k_true, a_digits * M * K + b_digits * N * K + 4 * M * N):
        L.call("bnn_gemm_i8_affine", L.ptr(A), lda, a_plane, a_digits, L.ptr(B), ldb, b_plane, b_digits,
               L.ptr(a_scale), L.ptr(b_scale), L.ptr(bias), L.ptr(row_off), L.ptr(col_off), float(off_mul),
               L.ptr(C), C.stride(0), M, N, K, L.stream())
    return C


def gemm_fp4(A4, B4, M, N, bias=None, k_true=None):
    """Ternary x ternary GEMM on FP4-packed operands (2 elements per byte): C = A.B^T + bias."""
    Kb = A4.shape[-1]
    assert B4.shape[-1] == Kb and Kb % ALIGN == 0
    C = torch.empty((M, N), dtype=torch.float32, device=A4.device)
    if M == 0 or N == 0:
        return C
    k_true = 2 * Kb if k_true is None else k_true
    name = gemm_kernel_name(0, 0, M, N, Kb) if _TIMER is not None else ""
    with _timed(name, 2.0 * M * N * k_true, (M + N) * Kb + 4 * M * N):
        L.call("bnn_gemm_fp4", L.ptr(A4), Kb, L.ptr(B4), Kb, L.ptr(bias), L.ptr(C), N, M, N, Kb, L.stream())
    return C


def gemm_fp4_i16(A4, B4, M, N, k_true=None):
    """gemm_fp4 without bias, the exact dot products as int16 [M, N] (bnn_gemm_fp4_i16)."""
    Kb = A4.shape[-1]
    assert B4.shape[-1] == Kb and Kb % ALIGN == 0 and 2 * Kb <= 32767 and N % 4 == 0
    C = torch.empty((M, N), dtype=torch.int16, device=A4.device)
    if M == 0 or N == 0:
        return C
    k_true = 2 * Kb if k_true is None else k_true
    name = (gemm_kernel_name(0, 0, M, N, Kb) + " [i16]") if _TIMER is not None else ""
    with _timed(name, 2.0 * M * N * k_true, (M + N) * Kb + 2 * M * N):
        L.call("bnn_gemm_fp4_i16", L.ptr(A4), Kb, L.ptr(B4), Kb, L.ptr(C), N, M, N, Kb, L.stream())
    return C


# Compact pre-activations (z16): the output z = F.linear(sign(h), W_b) + bias of a hidden
# BinarizeLinear (binarized_modules.py:80-83) is an integer plus a per-column bias, so when its only
# consumer is a libbnn BatchNorm pass it travels as int16 dot products + the bias
# (bnn_gemm_fp4_i16; the *_i16 BatchNorm entries form fl(I + bias), bit-identical to the fp32 z)
# at half the bytes of every pass over it.  Autograd sees a stride-0 float placeholder of z's
# shape carrying (int16, bias) in _Z16_ATTR; only the z16-aware functions below read it, and its
# gradient is an ordinary fp32 tensor.
Z16 = True
_Z16_ATTR = "_bnn_z16"


Z16_MIN_TILES = 512      # below this many 256x256 output tiles the fp32 epilogue is as cheap


def z16_ok(M, N, K):
    """Whether a hidden BinarizeLinear [K -> N] over M rows may hand its output on as z16."""
    return (Z16 and Q6_HANDOFF and DIGIT_GEMM == "fp6" and N % 256 == 0 and round_up(K, 256) <= 32767
            and (N // 256) * ((M + 255) // 256) >= Z16_MIN_TILES)


Z16_HANDOFFS = 0          # z16 placeholders produced (tests check the hand-off actually ran)


_ZERO1 = {}


_TOKENS = itertools.count(1)


def _placeholder(shape, device):
    """A stride-0 fp32 tensor of `shape` (the carrier of a hand-off attribute) viewing one cached zero
    per device: no fill kernel per placeholder.  In-place writes through it are refused by torch
    (every element aliases one location).  Placeholders share data_ptr and version counter, so each
    carries a unique token that _q6_key includes (the hand-offs' staleness checks tell them apart)."""
    key = str(device)
    z = _ZERO1.get(key)
    if z is None:
        z = torch.zeros((1,), dtype=torch.float32, device=device)
        if z.device.type != "cuda" or not torch.cuda.is_current_stream_capturing():
            _ZERO1[key] = z
        _ZERO_PTRS.add(z.data_ptr())          # capture-time zeros too: the graph's pool keeps them
    ph = z.as_strided(tuple(shape), (0,) * len(shape))
    ph._bnn_token = next(_TOKENS)
    return ph


_ZERO_PTRS = set()


def _is_placeholder(t):
    """t is a hand-off placeholder: it carries a placeholder token, or (an object torch re-wrapped
    without the Python attributes) views one of the zeros placeholders are made of -- in graph
    capture each placeholder gets a fresh zero from the graph's pool, so the cached one is not
    enough.  A stride-0 gradient that is NOT a placeholder (e.g. sum()'s expanded ones) is a
    legitimate dense-valued gradient."""
    return getattr(t, "_bnn_token", None) is not None or t.data_ptr() in _ZERO_PTRS


def _z16_carrier(y16, bias):
    global Z16_HANDOFFS
    Z16_HANDOFFS += 1
    ph = _placeholder(y16.shape, y16.device)
    setattr(ph, _Z16_ATTR, (y16, bias))
    return ph


def _z16_of(x):
    """(int16 [M, C], bias [C] or None) carried by a z16 placeholder, or None."""
    return getattr(x, _Z16_ATTR, None)


def _grad_sink(w):
    """(view, exchange) when a GradExchange lets this weight's gradient be written straight into
    its bucket view (parallel.GradExchange direct_write), else (None, None)."""
    ex = getattr(w, "_bnn_grad_sink", None)
    if ex is None:
        return None, None
    v = ex.grad_sink(w)
    return (v, ex) if v is not None and v.is_contiguous() and v.shape == w.shape else (None, None)


def gemm_xnor(a_bits, b_bits, M, N, bias=None):
    """XNOR-popcount GEMM on (sign, nonzero) bit-plane pairs; same result as the (1,1) int8 form."""
    (As, An), (Bs, Bn) = a_bits, b_bits
    kw = As.shape[1]
    C = torch.empty((M, N), dtype=torch.float32, device=As.device)
    if M == 0 or N == 0:
        return C
    with _timed("gemm_xnor_k", 2.0 * M * N * kw * 32, 8 * (M + N) * kw + 4 * M * N):
        L.call("bnn_gemm_xnor", L.ptr(As), L.ptr(An), kw, L.ptr(Bs), L.ptr(Bn), Bs.shape[1], L.ptr(bias),
               L.ptr(C), N, M, N, kw, L.stream())
    return C


# ----------------------------------------------------------------------------- fp32 x ternary on the FP6 MFMA
# The fp32 operand (dY in both backward GEMMs, the pixels of the first layer) as 4 FP6 digit
# planes with per-32-element block scales (bnn_gemm6.hip); the ternary operand as FP4.  "i8"
# selects the int8 3-digit-plane form (bnn_gemm.hip) instead -- kept for cross-checks.
DIGIT_GEMM = "fp6"


def set_digit_gemm(kind):
    global DIGIT_GEMM
    if kind not in ("fp6", "i8"):
        raise ValueError(kind)
    DIGIT_GEMM = kind


class Fp6Operand:
    """4 FP6 digit planes of an fp32 matrix [rows, K] (blocks of 32 along K, padded to Kp), and
    optionally the residual FP4 plane (``res``: 3 more bits, a fifth MFMA pass; bnn.h)."""
    __slots__ = ("lo", "hi", "sc", "rows", "Kp", "res")

    def __init__(self, lo, hi, sc, rows, Kp, res=None):
        self.lo, self.hi, self.sc, self.rows, self.Kp, self.res = lo, hi, sc, rows, Kp, res


# The residual plane on the row operands of the dX GEMMs (dY rows): the hidden BatchNorms' bias
# gradients sum dX over the batch, where it nearly cancels, and need fp32-grade dX (4 planes: 1.5e-5
# norm-wise on config 5's bn1/bn2 biases, fp32 GEMMs 7e-6 / 4e-6; tests/test_gpu_wide_step.py).
# BNN_FP6_RES=0 drops it (A/B timing only).
FP6_RES = os.environ.get("BNN_FP6_RES", "1") != "0"
# ... on operands of at least this many rows.  dbeta sums dX over the batch, and the 4-plane
# operand's rounding there grows with it (~sqrt(rows) against a sum that cancels): at B = 65,536
# the 4-plane dX put bn1/bn2's bias gradients at 1.6e-5 / 1.5e-5 (profiles/r05_d_wide_step_parity_
# residual.log), at B = 4,096 (config 3) every gradient stays <= 1e-5 without the fifth pass
# (tests/test_gpu_net_configs.py, profiles/r06_*), so the smaller batches skip its MFMA pass and stores.
FP6_RES_MIN_ROWS = int(os.environ.get("BNN_FP6_RES_MIN_ROWS", "8192"))


def _res_buffer(rows, Kp, device):
    return (torch.empty((rows, Kp // 32 * 16), dtype=torch.uint8, device=device)
            if FP6_RES and rows >= FP6_RES_MIN_ROWS else None)


def _fp6_buffers(rows, Kp, device):
    nb = Kp // 32
    lo = torch.empty((rows, nb * 64), dtype=torch.uint8, device=device)
    hi = torch.empty((rows, nb * 32), dtype=torch.uint8, device=device)
    # every producer writes the scale bytes of all `rows` rows; the slab's padding rows are read only
    # by the GEMM's 512-row scale pieces and scale only accumulator rows >= rows, which are never
    # stored or reduced (gemm_fp6_k clamps its digit rows, the split-K fold and the statistics
    # epilogue stop at M): left unwritten (a zero fill cost ~5-7 us per operand on the wide step)
    sc = torch.empty((Kp // 64, L.lib().bnn_quant6_scale_rows(rows), 2), dtype=torch.uint8, device=device)
    return lo, hi, sc


def quant6_rows(x):
    """fp32 [M,K] -> Fp6Operand of its rows (Kp = round_up(K, 64))."""
    _check(x)
    x = _c2d(x)
    M, K = x.shape
    Kp = round_up(K)
    lo, hi, sc = _fp6_buffers(M, Kp, x.device)
    res = _res_buffer(M, Kp, x.device)
    with _timed("quant6_rows_k", 0, 4 * M * K + (3.5 if res is not None else 3) * M * Kp + M * Kp // 32):
        L.call("bnn_quant6_rows", L.ptr(x), M, K, K, Kp, L.ptr(lo), L.ptr(hi), L.ptr(sc), L.ptr(res), L.stream())
    return Fp6Operand(lo, hi, sc, M, Kp, res)


def quant6_cols_t(x, want_colsum=False):
    """fp32 [M,N] -> (Fp6Operand of x^T [N, Mp], colsum [N] or None)."""
    _check(x)
    x = _c2d(x)
    M, N = x.shape
    Mp = round_up(M)
    lo, hi, sc = _fp6_buffers(N, Mp, x.device)
    cs = ws = None
    if want_colsum:
        cs = torch.empty((N,), dtype=torch.float32, device=x.device)
        ws = torch.empty((L.lib().bnn_quant6_cols_workspace(M, N),), dtype=torch.uint8, device=x.device)
    with _timed("quant6_cols_t_k", 0, 4 * M * N + 3 * N * Mp + N * Mp // 32):
        L.call("bnn_quant6_cols_t", L.ptr(x), M, N, N, Mp, L.ptr(lo), L.ptr(hi), L.ptr(sc), L.ptr(cs), L.ptr(ws),
               L.stream())
    return Fp6Operand(lo, hi, sc, N, Mp), cs


# B operands of at least this many MACs are staged from FP4 panels (bnn_fp4_panelize): the panel
# pass costs one read + write of B, the GEMM ~29 % less (profiles/r03_fp6_staging_diag.log)
PANEL_MIN_MACS = 1 << 30


def fp4_panels(B4, N, Kp):
    """FP4 rows [N, >= Kp/2 bytes] -> the panel layout [ceil(N/512), Kp/64, 512, 32 B] (flat uint8)."""
    P = torch.empty((L.lib().bnn_fp4_panel_bytes(N, Kp),), dtype=torch.uint8, device=B4.device)
    with _timed("fp4_panelize_k", 0, 2 * N * Kp // 2):
        L.call("bnn_fp4_panelize", L.ptr(B4), N, B4.shape[1], Kp, L.ptr(P), L.stream())
    return P


def gemm_fp6(A, B4, N, bias=None, k_true=None, out=None, panels=None, panel_ks=None):
    """C[A.rows, N] = A . B4^T (+ bias): A an Fp6Operand, B4 FP4 nibbles [N, >= A.Kp/2 bytes], or
    B4 = None and panels = the same operand in the panel layout with panel_ks 64-k steps per panel
    (fp4_panels, or a panel transpose from bn_apply_pack); large products panelize B4 themselves."""
    M, K = A.rows, A.Kp
    if B4 is None:
        assert panels is not None and panel_ks is not None and panel_ks * 64 >= K
        dev = panels.device
    else:
        assert B4.dtype == torch.uint8 and B4.shape[0] == N and 2 * B4.shape[1] >= K
        dev = B4.device
        if panel_ks is None:
            panel_ks = K // 64
    C = torch.empty((M, N), dtype=torch.float32, device=dev) if out is None else out
    if M == 0 or N == 0:
        return C
    k_true = K if k_true is None else k_true
    if panels is None and M * N * K >= PANEL_MIN_MACS:
        panels = fp4_panels(B4, N, K)
    name = _fp6_name(M, N, K, A) if _TIMER is not None else ""
    wsb = L.lib().bnn_gemm_fp6_workspace(M, N, K)    # split-K partials (small grids), else 0
    ws = torch.empty((wsb,), dtype=torch.uint8, device=dev) if wsb > 0 else None
    with _timed(name, 2.0 * M * N * k_true, (3.5 if A.res is not None else 3) * M * K + N * K // 2 + 4 * M * N):
        if panels is not None:
            L.call("bnn_gemm_fp6_panel_ws", L.ptr(A.lo), L.ptr(A.hi), L.ptr(A.sc), A.sc.shape[1], L.ptr(A.res),
                   L.ptr(panels), panel_ks, L.ptr(bias), L.ptr(C), C.stride(0), M, N, K, L.ptr(ws), wsb, L.stream())
        else:
            L.call("bnn_gemm_fp6_ws", L.ptr(A.lo), L.ptr(A.hi), L.ptr(A.sc), A.sc.shape[1], L.ptr(A.res), L.ptr(B4),
                   B4.shape[1], L.ptr(bias), L.ptr(C), C.stride(0), M, N, K, L.ptr(ws), wsb, L.stream())
    return C


def _fp6_name(M, N, K, A):
    """Timer name of an FP6 GEMM launch: the library's kernel choice, + " +res" with the residual
    plane (a fifth MFMA pass: bench.py counts its passes)."""
    res = A.res is not None
    return L.lib().bnn_gemm_fp6_kernel_kr(M, N, K, int(res)).decode() + (" +res" if res else "")


# The BatchNorm-backward statistics in the dX GEMM's epilogue (bnn_gemm_fp6_bnstats): the fused
# BN -> linear layer's backward takes sum g, sum g*xhat (and the i8cols bound's maxima) from the
# GEMM that writes dy instead of a separate pass over (x, dy).  Off by default: on the wide step
# every CU reaches its tile epilogue in the same round, so the epilogue's x reads are not hidden
# behind MFMA work and cost as much as the pass they replace (BNN_BN_EPI=1 enables).
BN_EPI = os.environ.get("BNN_BN_EPI", "0") == "1"
BN_EPI_USES = 0           # epilogue-statistics backward passes run (tests check the path ran)


def gemm_fp6_bnstats(A, panels, panel_ks, N, x, xbias, x_i16, mean, mlo, invstd, gamma, beta, mode):
    """(C = A . B^T with B in panels, the per-128-row partials [2|4, R, N] of the BatchNorm-backward
    statistics of C over x [A.rows, N], R)."""
    global BN_EPI_USES
    M, K = A.rows, A.Kp
    dev = panels.device
    C = torch.empty((M, N), dtype=torch.float32, device=dev)
    R = L.lib().bnn_gemm_fp6_bnstats_rows(M)
    part = torch.empty(((4 if mode == 2 else 2) * R * N,), dtype=torch.float32, device=dev)
    name = _fp6_name(M, N, K, A) if _TIMER is not None else ""
    with _timed(name, 2.0 * M * N * K, 3 * M * K + N * K // 2 + 4 * M * N + (2 if x_i16 else 4) * M * N):
        L.call("bnn_gemm_fp6_bnstats", L.ptr(A.lo), L.ptr(A.hi), L.ptr(A.sc), A.sc.shape[1], L.ptr(A.res),
               L.ptr(panels), panel_ks,
               L.ptr(C), N, M, N, K, L.ptr(x), L.ptr(xbias), int(bool(x_i16)), L.ptr(mean), L.ptr(mlo), L.ptr(invstd),
               L.ptr(gamma), L.ptr(beta), 1, int(mode), L.ptr(part), L.stream())
    BN_EPI_USES += 1
    return C, part, R


def _bn_epi_ok(M, N, K):
    """Whether the dX GEMM of this shape can carry the statistics epilogue (the unsplit default)."""
    return BN_EPI and N % 4 == 0 and L.lib().bnn_gemm_fp6_workspace(M, N, K) == 0


# ----------------------------------------------------------------------------- linear
class BinaryLinearFunction(torch.autograd.Function):
    """y = F.linear(bin(x), sign(w)) + b with the reference's STE backward (see module doc)."""

    @staticmethod
    def forward(ctx, x, weight, bias, binarize_input, backend="fp4", cache=False, xpack=None):
        # xpack: (FP4 rows, FP4 panel transpose or None) of sign(x), made with the input write-back
        # (sign_pack_fp4_writeback); used instead of packing x again
        _check(x, weight, bias)
        M, K = x.shape
        N = weight.shape[0]
        ctx.dims = (M, K, N)
        ctx.has_bias = bias is not None
        if M == 0:                # empty batch: F.linear returns [0, N]; gradients are empty / zero
            ctx.empty = True
            return torch.empty((0, N), dtype=torch.float32, device=x.device)
        ctx.empty = False
        need_dx, need_dw = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        b = bias.detach() if bias is not None else None
        # the FP6 digit GEMMs carry 20-bit block-scaled operands: used for the backward GEMMs of a
        # layer with a ternary input (gradient bar 1e-5); the first layer's fp32-input forward
        # keeps the 24-bit int8 digit form (forward bar 1e-6)
        ctx.fp6 = backend == "fp4" and DIGIT_GEMM == "fp6" and binarize_input
        qf = "fp4" if ctx.fp6 else "i8"
        ctx.x_panels = False
        if binarize_input:
            if backend == "fp4" and xpack is not None and ctx.fp6 and (xpack[1] is not None or not need_dw):
                x4, xqt = xpack
                ctx.x_panels = xqt is not None
                w4, wqt = packed_weight(weight, "fp4", True, need_dx, cache, qt_fmt=qf)
                y = gemm_fp4(x4, w4, M, N, bias=b, k_true=K)
            elif backend == "fp4":
                x4, xqt = sign_pack_fp4(x, want_qt=need_dw, qt_fmt=qf)
                w4, wqt = packed_weight(weight, "fp4", True, need_dx, cache, qt_fmt=qf)
                y = gemm_fp4(x4, w4, M, N, bias=b, k_true=K)
            elif backend == "xnor":
                y = gemm_xnor(sign_pack_bits(x), sign_pack_bits(weight), M, N, bias=b)
                xqt = sign_pack(x, want_q=False, want_qt=True)[1] if need_dw else None
                wqt = packed_weight(weight, "i8", False, need_dx, cache)[1] if need_dx else None
            else:
                xq, xqt = sign_pack(x, want_q=True, want_qt=need_dw)
                wq, wqt = packed_weight(weight, "i8", True, need_dx, cache)
                y = gemm_i8(xq, 1, wq, 1, M, N, bias=b, k_true=K)
            ctx.save_for_backward(xqt, wqt)
        else:
            wq, wqt = packed_weight(weight, "i8", True, need_dx, cache)
            xd, sx = quant_rows(x)
            y = gemm_i8(xd, 3, wq, 1, M, N, a_scale=sx, bias=b, k_true=K)
            ctx.save_for_backward(x if need_dw else None, wqt)
        ctx.binarize_input = binarize_input
        if ctx.fp6:
            setattr(y, _Q6_WANT, True)
        return y

    @staticmethod
    def backward(ctx, dy):
        M, K, N = ctx.dims
        if ctx.empty:
            dev = dy.device
            return (torch.empty((0, K), dtype=torch.float32, device=dev) if ctx.needs_input_grad[0] else None,
                    torch.zeros((N, K), dtype=torch.float32, device=dev) if ctx.needs_input_grad[1] else None,
                    torch.zeros((N,), dtype=torch.float32, device=dev)
                    if ctx.has_bias and ctx.needs_input_grad[2] else None, None, None, None, None)
        xs, wqt = ctx.saved_tensors
        dy = _c2d(dy)
        dx = dw = db = None
        need_db = ctx.has_bias and ctx.needs_input_grad[2]
        if ctx.fp6:
            pre = _q6_take(dy)                      # digits of dy from the BatchNorm backward
            if ctx.needs_input_grad[0]:
                dx = gemm_fp6(pre[0] if pre is not None else quant6_rows(dy), wqt, K, k_true=N)   # dY . W_b
            if ctx.needs_input_grad[1] or need_db:
                dt, cs = (pre[1], pre[2]) if pre is not None else quant6_cols_t(dy, want_colsum=need_db)
                if ctx.needs_input_grad[1]:
                    if ctx.x_panels:                                           # dY^T . X_b
                        dw = gemm_fp6(dt, None, K, k_true=M, panels=xs, panel_ks=xs.shape[1] // 32)
                    else:
                        dw = gemm_fp6(dt, xs, K, k_true=M)
                db = cs if need_db else None
            return dx, dw, db, None, None, None, None
        if ctx.needs_input_grad[0]:
            d, s = quant_rows(dy)                                   # [3, M, ldN]
            dx = gemm_i8(d, 3, wqt, 1, M, K, a_scale=s, k_true=N)   # dY . W_b
        if ctx.needs_input_grad[1] or need_db:
            dt, sc, cs = quant_cols_t(dy, want_colsum=need_db)      # [3, N, ldM]
            if ctx.needs_input_grad[1]:
                if ctx.binarize_input:
                    dw = gemm_i8(dt, 3, xs, 1, N, K, a_scale=sc, k_true=M)  # dY^T . X_b
                else:
                    xt, sxc, _ = quant_cols_t(xs)
                    dw = gemm_i8(dt, 3, xt, 3, N, K, a_scale=sc, b_scale=sxc, k_true=M)
            db = cs
        return dx, dw, db, None, None, None, None


def binary_linear(x, weight, bias=None, binarize_input=True, backend="fp4", cache=False, xpack=None):
    """Functional BinarizeLinear core: 2-D or N-D input (leading dims flattened).  ``cache``: the
    weight is a latent weight whose packed operands are cached on it (packed_weight)."""
    if x.dim() == 2:
        # no reshape view: the output tensor itself carries the FP6 hand-off request (_Q6_WANT) to
        # the BatchNorm that consumes it, and its gradient comes back to this Function unchanged
        return BinaryLinearFunction.apply(x, weight, bias, binarize_input, backend, cache, xpack)
    lead = x.shape[:-1]
    y = BinaryLinearFunction.apply(x.reshape(-1, x.shape[-1]), weight, bias, binarize_input, backend, cache, xpack)
    return y.reshape(*lead, weight.shape[0])


# ----------------------------------------------------------------------------- u8 pixels (fc1)
# The reference's loader hands fc1 x = ToTensor(u8) = u/255, optionally Normalize((m,), (s,))
# (mnist-dist2.py:96-99, mnist-distributed-BNNS2.py:82).  Kept as bytes in HBM and fed to fc1 as
# v = u - 128 (int8): x = a*v + c exactly, so fc1 and its weight gradient are one-pass int8 MFMA
# sums with the offset folded back in as an integer (bnn_pixels.hip).
def pixel_affine(normalize=None):
    """(a, s0) with x = a * (v + s0), v = u - 128: ToTensor (s0 = 128) or ToTensor + Normalize."""
    m, sd = normalize if normalize is not None else (0.0, 1.0)
    return 1.0 / (255.0 * sd), 128.0 - 255.0 * m


def pixels_to_float(u, normalize=None):
    """The fp32 tensor the reference's transform produces from the same bytes (reference
    semantics; for the CPU/oracle paths and comparisons)."""
    x = u.float() / 255.0
    if normalize is not None:
        x = (x - normalize[0]) / normalize[1]
    return x


COL_SUMS = os.environ.get("BNN_COLSUM", "1") != "0"   # the head's db4 on bnn_col_sums_narrow (0: torch's sum)
UNIT_PIXELS = 0          # fp32 ToTensor images recognised as bytes (tests check the path ran)
CAPTURE_GUARDS = []      # mismatch flags of the recognitions captured into a graph (graph.GraphedStep)


def unit_to_pixels(x, guard=None):
    """fp32 images [.., K] that are exactly ToTensor's fl(u / 255) -> their bytes u (uint8, same
    shape), else None.  One pass (bnn_unit_to_pixels) and one host read of its mismatch flag.

    During graph capture the flag cannot be read: without a guard the call returns None (the
    caller keeps its fp32 path); with one (an int32 [1] zero tensor, owned by the caller, which
    passes it only when its eager calls recognised the images) the pass is captured with the guard
    as its sticky mismatch flag, the bytes are returned, and the guard joins CAPTURE_GUARDS, which
    GraphedStep reads before each replay -- a replay over inputs that are not ToTensor images makes
    the next call raise."""
    global UNIT_PIXELS
    _check(x)
    capturing = x.is_cuda and torch.cuda.is_current_stream_capturing()
    if x.numel() == 0 or (capturing and guard is None):
        return None
    x = x if x.is_contiguous() else x.contiguous()
    u = torch.empty(x.shape, dtype=torch.uint8, device=x.device)
    if capturing:
        _check(guard, dtype=torch.int32)
        bad = guard
    else:
        bad = torch.zeros((1,), dtype=torch.int32, device=x.device)
    with _timed("unit_to_pixels_k", 0, 5 * x.numel()):
        L.call("bnn_unit_to_pixels", L.ptr(x), x.numel(), L.ptr(u), L.ptr(bad), L.stream())
    if capturing:
        CAPTURE_GUARDS.append(guard)
    elif int(bad.item()) != 0:
        return None
    UNIT_PIXELS += 1
    return u


def pixels_pack(u, want_q=True, want_qt=False):
    """u8 [M, K] -> (int8 rows v [M, round_up(K)], int8 v^T [K, round_up(M)]) (either None)."""
    _check(u, dtype=torch.uint8)
    u = u if u.is_contiguous() else u.contiguous()
    M, K = u.shape
    q = torch.empty((M, round_up(K)), dtype=torch.int8, device=u.device) if want_q else None
    qt = torch.empty((K, round_up(M)), dtype=torch.int8, device=u.device) if want_qt else None
    if (q is None and qt is None) or M == 0:
        return q, qt
    with _timed("pixels_pack_k", 0, M * K + (q.numel() if q is not None else 0) + (qt.numel() if qt is not None else 0)):
        L.call("bnn_pixels_pack", L.ptr(u), M, K, K, L.ptr(q), q.shape[1] if q is not None else 0,
               L.ptr(qt), qt.shape[1] if qt is not None else 0, L.stream())
    return q, qt


def row_sums(q, K):
    """Exact int64 row sums of an int8 matrix's first K columns (bnn_row_sums)."""
    N = q.shape[0]
    out = torch.empty((N,), dtype=torch.int64, device=q.device)
    L.call("bnn_row_sums", L.ptr(q), N, K, q.shape[1], L.ptr(out), L.stream())
    return out


_CONST = {}


def _const_vec(val, n, device):
    key = (float(val), int(n), str(device))
    t = _CONST.get(key)
    if t is None:
        t = torch.full((n,), float(val), dtype=torch.float32, device=device)
        _CONST[key] = t
    return t


# fc1 -> bn1 (mnist-dist2.py:64-65): in training the pixel GEMM's epilogue also forms bn1's
# forward statistics (chunk sums and M2 of z from its exact integer sums,
# bnn_gemm_i8_affine_bnstats), carried on the output; the fused BatchNorm then runs only the final
# (bnn_bn_fwd_final_parts) instead of a statistics pass over z.
PIX_STATS = os.environ.get("BNN_PIX_STATS", "1") != "0"      # BNN_PIX_STATS=0: the statistics pass
_FSTATS_ATTR = "_bnn_fstats"
PIX_STATS_USES = 0


def _pixels_fwd_with_stats(q, wq, M, N, K, bscale, bias, R, s0):
    chunk = int(L.lib().bnn_gemm_i8_bnstats_chunk(M, N))
    rows = (M + chunk - 1) // chunk
    part = torch.empty((2, rows, N), dtype=torch.float64, device=q.device)
    y = torch.empty((M, N), dtype=torch.float32, device=q.device)
    Kp = q.shape[1]
    assert wq.shape[1] == Kp and Kp % ALIGN == 0
    name = f"{gemm_kernel_name(1, 1, M, N, Kp)} [pixels]" if _TIMER is not None else ""
    with _timed(name, 2.0 * M * N * K, M * Kp + N * Kp + 4 * M * N):
        L.call("bnn_gemm_i8_affine_bnstats", L.ptr(q), Kp, L.ptr(wq), Kp, L.ptr(bscale), L.ptr(bias), L.ptr(R),
               float(s0), L.ptr(y), N, M, N, Kp, L.ptr(part), rows, L.stream())
    setattr(y, _FSTATS_ATTR, (part, rows, chunk, M, N, "pixels", 0.0, 0))
    return y


# fc1 -> bn1 in its compact form (s20): the pixel layer's output z1 = fl(fl(S * a) + b) is carried
# as the exact integer S = sum_k u_k sign(w_k) (|S| < 2^19 for ToTensor pixels at K = 784) in 20 bits
# -- an int16 plane and a nibble plane, 2.5 B per element instead of 4 -- when its only reader is the
# fused bn1 -> fc2 op in training (apply-pack forward, int8-column-digit backward), whose *_s20
# entries form the same fp32 z1 bit for bit.  The statistics still come from the GEMM epilogue.
# Autograd sees a stride-0 placeholder (as for z16); dense_preact() rebuilds the fp32 tensor.
S20 = os.environ.get("BNN_S20", "1") != "0"    # BNN_S20=0: fc1 writes the fp32 z1
_S20_ATTR = "_bnn_s20"
S20_HANDOFFS = 0          # s20 placeholders produced (tests check the hand-off ran)


def _s20_carrier(lo, hi, bias, scale):
    global S20_HANDOFFS
    S20_HANDOFFS += 1
    ph = _placeholder(lo.shape, lo.device)
    setattr(ph, _S20_ATTR, (lo, hi, bias, float(scale)))
    return ph


def _s20_of(x):
    """(int16 low bits [M, C], uint8 nibbles [M, C/2], bias [C] or None, scale) of an s20
    placeholder, or None."""
    return getattr(x, _S20_ATTR, None)


def dense_preact(z):
    """The fp32 tensor a compact pre-activation placeholder (s20 or z16) stands for, formed with
    the same fp32 roundings as the kernels that read it; any other tensor is returned as is (test
    and debugging aid -- the training path never materialises it)."""
    zs = _s20_of(z)
    if zs is not None:
        lo, hi, bias, scale = zs
        nib = torch.stack(((hi & 15), (hi >> 4) & 15), dim=-1).reshape(lo.shape).to(torch.int32)
        S = ((lo.to(torch.int32) & 0xFFFF) | (nib << 16))
        S = torch.where(S >= (1 << 19), S - (1 << 20), S)
        y = S.to(torch.float32) * torch.tensor(scale, dtype=torch.float32, device=lo.device)
        return y + bias if bias is not None else y
    zz = _z16_of(z)
    if zz is not None:
        y = zz[0].to(torch.float32)
        return y + zz[1] if zz[1] is not None else y
    return z


def _pixels_fwd_s20(q, wq, M, N, K, a, bias, R, s0):
    chunk = int(L.lib().bnn_gemm_i8_bnstats_chunk(M, N))
    rows = (M + chunk - 1) // chunk
    dev = q.device
    part = torch.empty((2, rows, N), dtype=torch.float64, device=dev)
    lo = torch.empty((M, N), dtype=torch.int16, device=dev)
    hi = torch.empty((M, N // 2), dtype=torch.uint8, device=dev)
    Kp = q.shape[1]
    assert wq.shape[1] == Kp and Kp % ALIGN == 0
    # the bias itself (a detached view sharing the Parameter's version counter): the consumer saves it
    # for backward, so torch refuses a backward after an in-place update of it -- no snapshot copy
    bs = bias
    name = f"{gemm_kernel_name(1, 1, M, N, Kp)} [pixels s20]" if _TIMER is not None else ""
    with _timed(name, 2.0 * M * N * K, M * Kp + N * Kp + 2.5 * M * N):
        L.call("bnn_gemm_i8_affine_bnstats_s20", L.ptr(q), Kp, L.ptr(wq), Kp, L.ptr(R), float(s0), K, L.ptr(lo),
               L.ptr(hi), N, M, N, Kp, L.ptr(part), rows, L.ptr(_const_vec(a, N, dev)), L.ptr(bias), L.stream())
    y = _s20_carrier(lo, hi, bs, a)
    setattr(y, _FSTATS_ATTR, (part, rows, chunk, M, N, "pixels", 0.0, 0))
    return y


def _fstats_of(z, M, C, drop=(0.0, 0)):
    """The forward-statistics partials a GEMM epilogue attached to z (None if absent, stale, or
    formed for another dropout (p, seed) than the consuming BatchNorm's)."""
    fs = getattr(z, _FSTATS_ATTR, None)
    if fs is None or fs[3] != M or fs[4] != C or z._version != 0:
        return None
    p, seed = float(drop[0]), int(drop[1])
    if fs[6] != p or (p > 0 and fs[7] != seed):
        return None
    return fs


# fc2 -> bn2 (mnist-dist2.py:66-67): the FP4 forward's epilogue forms bn2's forward statistics from
# the stored z = fl(sum + bias) (bnn_gemm_fp4_bnstats), carried on its output like fc1's.
FP4_STATS = os.environ.get("BNN_FP4_STATS", "1") != "0"      # BNN_FP4_STATS=0: the statistics pass
FP4_STATS_USES = 0


def _fp4_fwd_with_stats(q, wq, M, N, k_true, bias, zbias, chunk, i16, drop=(0.0, 0)):
    """(C [M, N] fp32 with bias, or int16 sums without; the statistics tuple for _FSTATS_ATTR).
    drop = (p, seed): the statistics of drop(z) for a fused dropout BatchNorm with that seed."""
    Kb = q.shape[1]
    assert wq.shape[1] == Kb and Kb % ALIGN == 0
    rows = (M + chunk - 1) // chunk
    part = torch.empty((2, rows, N), dtype=torch.float64, device=q.device)
    C = torch.empty((M, N), dtype=torch.int16 if i16 else torch.float32, device=q.device)
    name = (gemm_kernel_name(0, 0, M, N, Kb) + (" [i16]" if i16 else "")) if _TIMER is not None else ""
    with _timed(name, 2.0 * M * N * k_true, (M + N) * Kb + (2 if i16 else 4) * M * N):
        L.call("bnn_gemm_fp4_bnstats", L.ptr(q), Kb, L.ptr(wq), Kb, L.ptr(None if i16 else bias),
               None if i16 else L.ptr(C), L.ptr(C) if i16 else None, N, L.ptr(zbias), M, N, Kb, float(drop[0]),
               int(drop[1]), L.ptr(part), rows, L.stream())
    return C, (part, rows, chunk, M, N, "fp4", float(drop[0]), int(drop[1]))


class BinaryLinearPixelsFunction(torch.autograd.Function):
    """fc1 on u8 pixels: y = F.linear(x, sign(w)) + b with x = a*(u - 128 + s0), the reference's
    first BinarizeLinear (models/binarized_modules.py:68-85 with size(1) == 784: input not
    binarised) fed by ToTensor[/Normalize].  No gradient flows to the pixels."""

    @staticmethod
    def forward(ctx, u, weight, bias, a, s0, cache=False, emit_s20=False):
        _check(u, dtype=torch.uint8)
        _check(weight, bias)
        M, K = u.shape
        N = weight.shape[0]
        ctx.dims = (M, K, N)
        ctx.has_bias = bias is not None
        ctx.a, ctx.s0 = a, s0
        need_dw = ctx.needs_input_grad[1]
        q, qt = pixels_pack(u, want_q=M > 0, want_qt=need_dw and M > 0)
        if M == 0:
            ctx.save_for_backward(None)
            return torch.empty((0, N), dtype=torch.float32, device=u.device)
        wq, _ = packed_weight(weight, "i8", True, False, cache)
        R = row_sums(wq, K)
        bvec = bias.detach() if bias is not None else None
        stats_ok = (PIX_STATS and need_dw and K <= q.shape[1]
                    and L.lib().bnn_gemm_i8_bnstats_ok(M, N, q.shape[1], q.shape[1], wq.shape[1]))
        # (small grids keep the fp32 z1: the s20 apply-pack is the 256x256-tile kernel, slower than
        # the small-batch pass below Z16_MIN_TILES tiles -- config 3: 37.7 vs 20 us)
        if (stats_ok and emit_s20 and S20 and I8C_HANDOFF and N % 256 == 0
                and (N // 256) * ((M + 255) // 256) >= Z16_MIN_TILES
                and L.lib().bnn_gemm_i8_s20_ok(M, N, q.shape[1], K, float(s0))):
            y = _pixels_fwd_s20(q, wq, M, N, K, a, bvec, R, s0)
        elif stats_ok:
            y = _pixels_fwd_with_stats(q, wq, M, N, K, _const_vec(a, N, u.device), bvec, R, s0)
        else:
            y = gemm_i8_affine(q, 1, wq, 1, M, N, b_scale=_const_vec(a, N, u.device), bias=bvec, col_off=R,
                               off_mul=s0, k_true=K, label="pixels")
        ctx.save_for_backward(qt)
        if I8C_HANDOFF and need_dw:
            setattr(y, _I8C_WANT, True)
        return y

    @staticmethod
    def backward(ctx, dy):
        M, K, N = ctx.dims
        (qt,) = ctx.saved_tensors
        dev = dy.device
        need_db = ctx.has_bias and ctx.needs_input_grad[2]
        dw = db = None
        if M == 0:
            return (None, torch.zeros((N, K), dtype=torch.float32, device=dev) if ctx.needs_input_grad[1] else None,
                    torch.zeros((N,), dtype=torch.float32, device=dev) if need_db else None, None, None, None, None)
        pre = _i8c_take(dy)          # the digits straight from the BatchNorm backward, if it made them
        if pre is None:
            dy = _c2d(dy)
        if ctx.needs_input_grad[1] or need_db:
            if pre is not None:
                dt, sc, cs, ds = pre
            else:
                dt, sc, cs, ds = quant_cols_t(dy, want_colsum=need_db, want_dsum=True)   # dY^T digits, T[n]
            if ctx.needs_input_grad[1]:
                dw = gemm_i8_affine(dt, 3, qt, 1, N, K, a_scale=sc, b_scale=_const_vec(ctx.a, K, dev),
                                    row_off=ds, off_mul=ctx.s0, k_true=M, label="pixels")
            db = cs
        return None, dw, db, None, None, None, None


def binary_linear_pixels(u, weight, bias=None, normalize=None, cache=False, emit_compact=False):
    """fc1 on u8 pixels [.., K] (leading dims flattened); ``normalize`` = (mean, std) or None.
    emit_compact: the output may travel as an s20 placeholder (its consumer must be the
    training-mode fused bn_hardtanh_binary_linear with the FP4/FP6 backend; see nets.MLP)."""
    if u.dtype != torch.uint8:
        raise TypeError("binary_linear_pixels: expects uint8 pixels")
    a, s0 = pixel_affine(normalize)
    lead = u.shape[:-1]
    if emit_compact and len(lead) != 1:
        raise ValueError("binary_linear_pixels: a compact output needs a 2-D batch")
    y = BinaryLinearPixelsFunction.apply(u.reshape(-1, u.shape[-1]), weight, bias, a, s0, cache, bool(emit_compact))
    # a 2-D batch returns the Function's own output: it carries the int8 column-digit hand-off
    # marker (_I8C_WANT) a reshape view would drop
    return y if len(lead) == 1 else y.reshape(*lead, weight.shape[0])


# ----------------------------------------------------------------------------- narrow Linear
LINEAR_NSMALL = (1, 2, 4, 8, 10, 16)


class LinearNSmallFunction(torch.autograd.Function):
    """y = F.linear(x, w, b) for a narrow fp32 classifier (bnn_linear_nsmall_*): the BinCNN's
    nn.Linear(7*7*32, 10), which a library GEMM runs at ~16 us per product on this shape."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        _check(x, weight, bias)
        x = x.contiguous()
        w = weight.detach().contiguous()
        M, K = x.shape
        N = w.shape[0]
        y = torch.empty((M, N), dtype=torch.float32, device=x.device)
        with _timed("linear_nsmall_fwd", 2.0 * M * N * K, 4 * M * K):
            L.call("bnn_linear_nsmall_fwd", L.ptr(x), M, K, L.ptr(w), L.ptr(bias.detach() if bias is not None else None),
                   N, L.ptr(y), L.stream())
        ctx.save_for_backward(x, w)
        ctx.has_bias = bias is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        M, K = x.shape
        N = w.shape[0]
        dy = dy.contiguous()
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        dw = torch.empty_like(w) if ctx.needs_input_grad[1] else None
        db = torch.empty((N,), dtype=torch.float32, device=x.device) if ctx.has_bias and ctx.needs_input_grad[2] else None
        nb = int(L.lib().bnn_linear_nsmall_workspace(M, N, K)) if dw is not None or db is not None else 0
        work = torch.empty((nb,), dtype=torch.uint8, device=x.device) if nb else None
        with _timed("linear_nsmall_bwd", 4.0 * M * N * K, 8 * M * K):
            L.call("bnn_linear_nsmall_bwd", L.ptr(x), L.ptr(w), L.ptr(dy), M, K, N, L.ptr(dx), L.ptr(dw), L.ptr(db),
                   L.ptr(work), nb, L.stream())
        return dx, dw, db


def linear_nsmall_ok(x, weight):
    return (x.is_cuda and x.dim() == 2 and x.dtype == torch.float32 and weight.shape[0] in LINEAR_NSMALL
            and x.shape[1] % 4 == 0 and x.shape[1] == weight.shape[1] and weight.numel() <= 16384)


def linear_nsmall(x, weight, bias=None):
    return LinearNSmallFunction.apply(x, weight, bias)


# ----------------------------------------------------------------------------- loss
class CrossEntropyFunction(torch.autograd.Function):
    """torch.nn.CrossEntropyLoss() (reduction 'mean') on [M, C] fp32 rows with int64 targets
    (bnn_cross_entropy_*): the training loop's criterion applied to the nets' LogSoftmax output
    (mnist-dist2.py:118-137).  Two launches forward (row losses, fixed-order fold), one backward;
    the loss and its incoming gradient stay on the device (no host synchronisation).  Rows whose
    target equals ``ignore_index`` are skipped as torch skips them."""

    @staticmethod
    def forward(ctx, p, target, ignore_index=-100):
        _check(p)
        p = p.contiguous()
        target = target.contiguous()
        M, C = p.shape
        loss = torch.empty((), dtype=torch.float32, device=p.device)
        work = torch.empty((int(L.lib().bnn_cross_entropy_workspace(M)),), dtype=torch.uint8, device=p.device)
        with _timed("cross_entropy_fwd", 0, 4 * M * C + 8 * M):
            L.call("bnn_cross_entropy_fwd", L.ptr(p), L.ptr(target), M, C, int(ignore_index), L.ptr(loss),
                   L.ptr(work), work.numel(), L.stream())
        ctx.save_for_backward(p, target, work)
        ctx.ignore_index = int(ignore_index)
        return loss

    @staticmethod
    def backward(ctx, go):
        p, target, work = ctx.saved_tensors
        M, C = p.shape
        dp = torch.empty_like(p)
        go = go.to(torch.float32).contiguous()
        with _timed("cross_entropy_bwd", 0, 8 * M * C + 8 * M):
            L.call("bnn_cross_entropy_bwd", L.ptr(p), L.ptr(target), M, C, ctx.ignore_index, L.ptr(go),
                   L.ptr(work), L.ptr(dp), L.stream())
        return dp, None, None


def cross_entropy_ok(p, target):
    return (p.is_cuda and p.dim() == 2 and p.dtype == torch.float32 and p.shape[0] > 0
            and bool(L.lib().bnn_cross_entropy_ok(p.shape[1])) and target.dim() == 1
            and target.dtype == torch.int64 and target.shape[0] == p.shape[0] and target.device == p.device)


def cross_entropy(p, target, ignore_index=-100):
    """Mean cross-entropy of the rows of p against target (torch.nn.CrossEntropyLoss() semantics,
    ignore_index included)."""
    return CrossEntropyFunction.apply(p, target, int(ignore_index))


# ----------------------------------------------------------------------------- conv2d
def _pair_same(v, what):
    if isinstance(v, (tuple, list)):
        if len(set(v)) != 1:
            raise NotImplementedError(f"bnn_amd: asymmetric {what} {v} is not supported")
        return int(v[0])
    return int(v)


# conv1 -> BatchNorm2d backward hand-off (c1bn): when the BinCNN's first conv (one input channel,
# its input needing no gradient) emits its compact output into the fused BatchNorm2d + Hardtanh +
# MaxPool2d op, that op's backward computes only its statistics (bnn_bn2d_bwd_stats_q) and hands the
# conv the pooled gradient and those statistics; the conv's weight gradient then forms dY itself
# (bnn_conv2d_bwd_filter_bn) -- the fp32 dY of the layer is never written.
C1BN = os.environ.get("BNN_C1BN", "1") != "0"
_C1BN_WANT = "_bnn_c1bn_consumer"
_C1BN_ATTR = "_bnn_c1bn"
C1BN_HANDOFFS = 0


def _c1bn_take(dy):
    ent = getattr(dy, _C1BN_ATTR, None)
    if ent is None:
        return None
    delattr(dy, _C1BN_ATTR)
    if ent[0] != _q6_key(dy):
        raise RuntimeError("stale conv1 / BatchNorm2d hand-off")
    return ent[1:]


# BNN_CONV_C1F=1 / 0: the one-input-channel VALU filter-gradient kernel on / off (A/B timing);
# unset: the library's default.  Applied once, before the first conv forward (the forward decides
# whether conv1 takes the BatchNorm2d hand-off, whose kernel depends on the same switch).
_CONV_C1F = [os.environ.get("BNN_CONV_C1F")]
# BNN_FP6_PERS=1 / 0: the FP6 GEMM's persistent tile on / off (A/B timing); unset: the library's
# default (off)
if os.environ.get("BNN_FP6_PERS") is not None:
    L.call("bnn_gemm_fp6_set_persistent", int(os.environ["BNN_FP6_PERS"] != "0"))
# BNN_FP6_HALF=0 / 1 / 2: the FP6 GEMM's half-tile form off / on the residual-plane (dX) launches (the
# library's default) / on every launch (A/B timing; bnn_gemm_fp6_set_half)
if os.environ.get("BNN_FP6_HALF") is not None:
    L.call("bnn_gemm_fp6_set_half", int(os.environ["BNN_FP6_HALF"]), 0.0)
# BNN_PIX_TILE=1 / 2: the u8-pixel statistics GEMM's tile, 128 x 128 / 256 x 256 (A/B timing)
if os.environ.get("BNN_PIX_TILE") is not None:
    L.call("bnn_gemm_i8_bnstats_set_tile", int(os.environ["BNN_PIX_TILE"]))
# BNN_HEAD_RED_COLS=2 / 4: columns per thread of the head's statistics pass (A/B timing)
if os.environ.get("BNN_HEAD_RED_COLS") is not None:
    L.call("bnn_bn_set_head_reduce_cols", int(os.environ["BNN_HEAD_RED_COLS"]))


def _conv_env():
    if _CONV_C1F[0] is not None:
        L.call("bnn_conv_set_c1_filter", int(_CONV_C1F[0] != "0"))
        _CONV_C1F[0] = None


# Compact conv outputs (zq): a binary-input BinarizeConv2d computes exact integer sums I (|I| <=
# C*KH*KW: 25 for the BinCNN's first layer, 400 for its second) plus a per-channel bias, so when
# its only consumer is the fused BatchNorm2d it travels as int16 sums + the bias
# (bnn_conv2d_fwd_q; bnn_bn2d_*_q read fl(I + bias), bit-identical to the fp32 output) -- a stride-0
# placeholder of the output shape carries them, as the MLP's z16 does.
ZQ = True
_ZQ_ATTR = "_bnn_zq"
ZQ_HANDOFFS = 0


def _zq_of(x):
    """(int8 / int16 sums [N, C, H, W], bias [C] or None, fmt 1 / 2) carried by a zq placeholder."""
    return getattr(x, _ZQ_ATTR, None)


def _zq_fmt(x, binarize_input, stride, dilation, groups, C, KH, KW, H, W, pad, N, Co):
    """1 (int8) / 2 (int16) when bnn_conv2d_fwd_q takes the shape, else 0 (then the fp32 output is
    written: the library's own geometry check, bnn_conv2d_fwd_q_ok, has the last word)."""
    if not (ZQ and binarize_input and stride == 1 and dilation == 1 and groups == 1 and pad <= min(KH, KW) - 1):
        return 0
    if not (C == 1 and KW <= 8) and not (C % 16 == 0 and C <= 64):
        return 0
    # int16 even where int8 would hold the sums (the first layer's |I| <= 25): the pooled BatchNorm2d
    # passes read 2 elements per lane, and 2-byte loads made them slower than on fp32 (int8 conv1:
    # apply 33 -> 46 us, backward 115 -> 139 us; int16 conv2: backward 115 -> 78 us, tools/gpu_r03_q6b.sh)
    fmt = 2 if C * KH * KW <= 32767 else 0
    if fmt and not L.lib().bnn_conv2d_fwd_q_ok(fmt, N, C, H, W, Co, KH, KW, stride, pad, dilation, groups):
        return 0
    return fmt


class BinaryConv2dFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, binarize_input, stride, padding, dilation, groups, emit_compact=False):
        global ZQ_HANDOFFS
        _check(x, weight, bias)
        _conv_env()
        x = _c2d(x)
        w = _c2d(weight.detach())
        N, C, H, W = x.shape
        Co, _, KH, KW = w.shape
        OH = (H + 2 * padding - dilation * (KH - 1) - 1) // stride + 1
        OW = (W + 2 * padding - dilation * (KW - 1) - 1) // stride + 1
        b = bias.detach() if bias is not None else None
        ctx.empty = N == 0
        zf = _zq_fmt(x, binarize_input, stride, dilation, groups, C, KH, KW, H, W, padding, N, Co) if emit_compact else 0
        if zf and N > 0 and Co <= 64 and (OH * OW) % 4 == 0 and OH % 2 == 0 and OW % 2 == 0:
            yq = torch.empty((N, Co, OH, OW), dtype=torch.int8 if zf == 1 else torch.int16, device=x.device)
            macs = N * Co * OH * OW * C * KH * KW
            with _timed("conv2d_fwd", 2 * macs, 4 * x.numel() + yq.numel() * yq.element_size() + 4 * w.numel()):
                L.call("bnn_conv2d_fwd_q", L.ptr(x), L.ptr(w), L.ptr(yq), zf, N, C, H, W, Co, KH, KW, stride,
                       padding, dilation, groups, L.stream())
            ctx.save_for_backward(x, w)
            ctx.conf = (binarize_input, stride, padding, dilation, groups)
            ctx.has_bias = bias is not None
            ZQ_HANDOFFS += 1
            ph = _placeholder((N, Co, OH, OW), x.device)
            # the bias as a detached view (its consumer saves it for backward: an in-place update
            # before this step's backward is refused by torch's saved-tensor check, no copy needed)
            setattr(ph, _ZQ_ATTR, (yq, b, zf))
            if (C1BN and C == 1 and binarize_input and not ctx.needs_input_grad[0]
                    and L.lib().bnn_conv2d_bwd_filter_bn_ok(N, C, H, W, Co, KH, KW, stride, padding, dilation,
                                                            groups)):
                setattr(ph, _C1BN_WANT, True)
            return ph
        y = torch.empty((N, Co, OH, OW), dtype=torch.float32, device=x.device)
        if ctx.empty:             # empty batch: F.conv2d returns [0, Co, OH, OW]
            ctx.save_for_backward(x, w)
            ctx.conf = (binarize_input, stride, padding, dilation, groups)
            ctx.has_bias = bias is not None
            return y
        macs = N * Co * OH * OW * (C // groups) * KH * KW
        with _timed("conv2d_fwd", 2 * macs, 4 * (x.numel() + y.numel() + w.numel())):
            L.call("bnn_conv2d_fwd", L.ptr(x), int(binarize_input), L.ptr(w), L.ptr(b), L.ptr(y),
                   N, C, H, W, Co, KH, KW, stride, padding, dilation, groups, L.stream())
        ctx.save_for_backward(x, w)
        ctx.conf = (binarize_input, stride, padding, dilation, groups)
        ctx.has_bias = bias is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        binarize_input, stride, padding, dilation, groups = ctx.conf
        bn = _c1bn_take(dy)      # the BatchNorm2d backward's pooled gradient and statistics, if handed over
        if bn is None:
            if dy.dim() == 4 and dy.numel() > 1 and dy.stride() == (0, 0, 0, 0) and _is_placeholder(dy):
                raise RuntimeError("a conv gradient placeholder lost its BatchNorm2d hand-off")
            dy = _c2d(dy)
        N, C, H, W = x.shape
        Co, _, KH, KW = w.shape
        if ctx.empty:
            return (torch.empty_like(x) if ctx.needs_input_grad[0] else None,
                    torch.zeros_like(w) if ctx.needs_input_grad[1] else None,
                    torch.zeros((Co,), dtype=torch.float32, device=x.device)
                    if ctx.has_bias and ctx.needs_input_grad[2] else None, None, None, None, None, None, None)
        dx = dw = db = None
        if bn is not None and not L.lib().bnn_conv2d_bwd_filter_bn_ok(N, C, H, W, Co, KH, KW, stride, padding,
                                                                      dilation, groups):
            # the fused kernel was switched off since the forward (bnn_conv_set_c1_filter /
            # bnn_conv_set_mfma): form dy with the BatchNorm2d backward and take the regular path
            dy = _bn2d_dy_of_handoff(bn, dy.shape)
            bn = None
        macs = dy.numel() * (C // groups) * KH * KW
        if bn is not None:
            global C1BN_HANDOFFS
            need_db = ctx.has_bias and ctx.needs_input_grad[2]
            dw = torch.empty_like(w)
            db = torch.empty((Co,), dtype=torch.float32, device=x.device) if need_db else None
            ws = torch.empty((L.lib().bnn_conv2d_bwd_filter_workspace(N, C, Co, KH, KW, groups),),
                             dtype=torch.uint8, device=x.device)
            zq, zb, zf, dyp, mean, invstd, gw, gb, sg, sgx, inv_n, ht = bn
            with _timed("conv2d_bwd_filter_bn", 2 * macs, zq.numel() * zq.element_size() + 4 * dyp.numel()):
                L.call("bnn_conv2d_bwd_filter_bn", L.ptr(zq), L.ptr(zb), zf, L.ptr(dyp), L.ptr(mean), L.ptr(invstd),
                       L.ptr(gw), L.ptr(gb), L.ptr(sg), L.ptr(sgx), float(inv_n), int(ht), L.ptr(x),
                       int(binarize_input), L.ptr(dw), L.ptr(db), L.ptr(ws), N, C, H, W, Co, KH, KW, stride,
                       padding, dilation, groups, L.stream())
            C1BN_HANDOFFS += 1
            return (None, dw if ctx.needs_input_grad[1] else None, db, None, None, None, None, None, None)
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            with _timed("conv2d_bwd_data", 2 * macs, 4 * (dy.numel() + dx.numel() + w.numel())):
                L.call("bnn_conv2d_bwd_data", L.ptr(dy), L.ptr(w), L.ptr(dx), N, C, H, W, Co, KH, KW,
                       stride, padding, dilation, groups, L.stream())
        need_db = ctx.has_bias and ctx.needs_input_grad[2]
        if ctx.needs_input_grad[1] or need_db:
            dw = torch.empty_like(w)
            db = torch.empty((Co,), dtype=torch.float32, device=x.device) if need_db else None
            ws = torch.empty((L.lib().bnn_conv2d_bwd_filter_workspace(N, C, Co, KH, KW, groups),),
                             dtype=torch.uint8, device=x.device)
            with _timed("conv2d_bwd_filter", 2 * macs, 4 * (dy.numel() + x.numel() + w.numel())):
                L.call("bnn_conv2d_bwd_filter", L.ptr(dy), L.ptr(x), int(binarize_input), L.ptr(dw),
                       L.ptr(db), L.ptr(ws), N, C, H, W, Co, KH, KW, stride, padding, dilation, groups,
                       L.stream())
            if not ctx.needs_input_grad[1]:
                dw = None
        return dx, dw, db, None, None, None, None, None, None


def _bn2d_dy_of_handoff(bn, shape):
    """The fp32 gradient of the conv output a conv1 / BatchNorm2d hand-off stands for: the pooled
    BatchNorm2d(+Hardtanh) backward written out by bnn_bn2d_bwd_q (its dgamma / dbeta, already
    delivered by the BatchNorm's own backward, go to scratch)."""
    zq, zb, zf, dyp, mean, invstd, gw, gb, sg, sgx, inv_n, ht = bn
    N, C, H, W = shape
    dev = dyp.device
    dz = torch.empty((N, C, H, W), dtype=torch.float32, device=dev)
    scratch = torch.empty((2, C), dtype=torch.float32, device=dev)
    ws = torch.empty((L.lib().bnn_bn2d_workspace(N, C),), dtype=torch.uint8, device=dev)
    L.call("bnn_bn2d_bwd_q", L.ptr(zq), L.ptr(zb), zf, L.ptr(dyp), N, C, H, W, L.ptr(gw), L.ptr(gb), L.ptr(mean),
           L.ptr(invstd), int(ht), 2, L.ptr(dz), L.ptr(scratch[0]), L.ptr(scratch[1]), L.ptr(ws), L.stream())
    return dz


def binary_conv2d(x, weight, bias=None, binarize_input=True, stride=1, padding=0, dilation=1, groups=1,
                  emit_compact=False):
    """emit_compact: return the output as a zq placeholder when the shape allows (its consumer
    must be batch_norm2d_hardtanh_pool in training mode)."""
    return BinaryConv2dFunction.apply(x, weight, bias, binarize_input, _pair_same(stride, "stride"),
                                      _pair_same(padding, "padding"), _pair_same(dilation, "dilation"),
                                      int(groups), bool(emit_compact))


# ----------------------------------------------------------------------------- (3) STE helpers
def hardtanh_backward(x, g):
    _check(x, g)
    x, g = _c2d(x), _c2d(g)
    out = torch.empty_like(g)
    L.call("bnn_hardtanh_bwd", L.ptr(x), L.ptr(g), L.ptr(out), g.numel(), L.stream())
    return out


def _bump(p):
    """A raw in-place write through the data pointer: bump the tensor's version as a torch in-place
    op would, so a backward that saved it (the z16 / s20 / conv bias carriers) refuses to run on
    the updated value instead of silently using it."""
    torch.autograd.graph.increment_version(p)


def adam_clamp_(p, grad, exp_avg, exp_avg_sq, step, lr, beta1=0.9, beta2=0.999, eps=1e-8,
                grad_scale=1.0, clamp=True, sched=None, ctr=None):
    """In-place fused Adam (torch formula) + clamp to [-1, 1] on a latent weight."""
    _check(p, grad, exp_avg, exp_avg_sq)
    invalidate_packed(p)        # a raw in-place write: cached packed operands would go stale
    for t in (p, grad, exp_avg, exp_avg_sq):
        if not t.is_contiguous():
            raise ValueError("adam_clamp_: tensors must be contiguous")
    _bump(p)
    if sched is not None:
        L.call("bnn_adam_clamp_sched", L.ptr(p), L.ptr(grad), L.ptr(exp_avg), L.ptr(exp_avg_sq), p.numel(),
               float(beta1), float(beta2), float(eps), L.ptr(sched), L.ptr(ctr), float(grad_scale),
               int(bool(clamp)), L.stream())
        return
    L.call("bnn_adam_clamp", L.ptr(p), L.ptr(grad), L.ptr(exp_avg), L.ptr(exp_avg_sq), p.numel(),
           float(lr), float(beta1), float(beta2), float(eps), int(step), float(grad_scale),
           int(bool(clamp)), L.stream())


ADAM_MULTI_MAX = 16     # tensors per bnn_adam_clamp_multi launch


def adam_clamp_multi_(items, lr, beta1=0.9, beta2=0.999, eps=1e-8, grad_scale=1.0, sched=None, ctr=None):
    """adam_clamp_ on several tensors in one launch per ADAM_MULTI_MAX: items = [(p, grad, exp_avg,
    exp_avg_sq, step, clamp)], bit-identical per tensor to adam_clamp_ (bnn_adam_clamp_multi)."""
    import ctypes
    for i in range(0, len(items), ADAM_MULTI_MAX):
        chunk = items[i:i + ADAM_MULTI_MAX]
        for p, g, m, v, _, _ in chunk:
            _check(p, g, m, v)
            invalidate_packed(p)
            for t in (p, g, m, v):
                if not t.is_contiguous():
                    raise ValueError("adam_clamp_multi_: tensors must be contiguous")
            _bump(p)
        k = len(chunk)
        arr = [(ctypes.c_void_p * k)(*[it[j].data_ptr() for it in chunk]) for j in range(4)]
        nn_ = (ctypes.c_int64 * k)(*[it[0].numel() for it in chunk])
        st = (ctypes.c_int64 * k)(*[int(it[4]) for it in chunk])
        cl = (ctypes.c_int32 * k)(*[int(bool(it[5])) for it in chunk])
        vp = [ctypes.cast(a, ctypes.c_void_p) for a in arr + [nn_, st, cl]]
        L.call("bnn_adam_clamp_multi", k, *vp, float(lr), float(beta1), float(beta2), float(eps), L.ptr(sched),
               L.ptr(ctr), float(grad_scale), L.stream())


# ----------------------------------------------------------------------------- BatchNorm1d (+ Hardtanh)
def _bn_ws(M, C, device):
    return torch.empty((L.lib().bnn_bn_workspace(M, C),), dtype=torch.uint8, device=device)


STATS_TAP = None   # tests: a list that receives the [3, C] (save_mean, save_invstd, save_mean_lo) of
                   # every training-mode BatchNorm1d forward, in call order


def _bn_stat_buffers(C, device):
    """save_mean, save_invstd, save_mean_lo of a training-mode BatchNorm forward (bnn.h)."""
    st = torch.empty((3, C), dtype=torch.float32, device=device)
    if STATS_TAP is not None:
        STATS_TAP.append(st)
    return st[0], st[1], st[2]


def _bn_bwd_call(training, x, dy, M, C, w, b, mean, invstd, mlo, hardtanh, dx, dw, db, ws):
    # eval mode: the running statistics are constants (dx = gamma*invstd*g)
    if training:
        L.call("bnn_bn_bwd", L.ptr(x), L.ptr(dy), M, C, L.ptr(w), L.ptr(b), L.ptr(mean), L.ptr(invstd), L.ptr(mlo),
               int(hardtanh), L.ptr(dx), L.ptr(dw), L.ptr(db), L.ptr(ws), L.stream())
    else:
        L.call("bnn_bn_bwd_eval", L.ptr(x), L.ptr(dy), M, C, L.ptr(w), L.ptr(b), L.ptr(mean), L.ptr(invstd),
               int(hardtanh), L.ptr(dx), L.ptr(dw), L.ptr(db), L.ptr(ws), L.stream())


# FP6 digits of a gradient, handed from the BatchNorm backward that produces it to the
# BinarizeLinear backward that consumes it (bnn_bn_bwd_q6: dz is quantised in the pass that
# computes it, never re-read).  A forward output whose gradient an FP6-backward linear will
# quantise carries _Q6_WANT; the BatchNorm function that takes it as input then emits the digits
# on its gradient (_Q6_ATTR, keyed on the tensor's storage / version / shape, taken once).
_Q6_ATTR = "_bnn_q6"
_Q6_WANT = "_bnn_q6_consumer"


def _q6_key(t):
    return (t.data_ptr(), t._version, tuple(t.shape), getattr(t, "_bnn_token", None))


Q6_HANDOFF = True        # False: every FP6 linear backward quantises its dy itself (cross-checks)


def _q6_wanted(x, C, training=True):
    return (Q6_HANDOFF and bool(getattr(x, _Q6_WANT, False)) and training and DIGIT_GEMM == "fp6"
            and C % 64 == 0)


Q6_HANDOFFS = 0           # FP6 digit hand-offs consumed by a linear backward (tests check they ran)


def _q6_take(dy):
    """(rows Fp6Operand, cols Fp6Operand, colsum) attached to ``dy`` by bnn_bn_bwd_q6, or None."""
    global Q6_HANDOFFS
    ent = getattr(dy, _Q6_ATTR, None)
    if ent is None:
        return None
    delattr(dy, _Q6_ATTR)
    if ent[0] != _q6_key(dy):
        return None
    Q6_HANDOFFS += 1
    return ent[1:]


def _dz_placeholder(M, C, device):
    """The gradient of a z16 pre-activation: its only reader is the producing linear's backward,
    which takes the FP6 digits handed to it, so dz itself is never written (a stride-0 tensor of
    the right shape carries the hand-off)."""
    return _placeholder((M, C), device)


def _q6_take_required(dy):
    pre = _q6_take(dy)
    if pre is None and dy.dim() == 2 and dy.stride() == (0, 0) and _is_placeholder(dy):
        raise RuntimeError("a z16 gradient placeholder lost its FP6 hand-off (was the pre-activation consumed twice?)")
    return pre


def _bn_bwd_q6(x, dy, M, C, w, b, mean, invstd, mlo, hardtanh, p, seed, dw, db, ws, name, z16=None, pre=None):
    """BatchNorm(+Dropout) backward that also quantises dz (returned, with the digits attached).
    z16 = (int16, bias): the input in its compact form (x unused); dz is then not written (the
    returned gradient is a placeholder carrying only the digits, _dz_placeholder).  pre = (part, R):
    the statistics from the dX GEMM's epilogue (gemm_fp6_bnstats mode 1; p = 0)."""
    dev = dy.device
    dx = torch.empty((M, C), dtype=torch.float32, device=dev) if z16 is None else _dz_placeholder(M, C, dev)
    dx_ptr = L.ptr(dx) if z16 is None else None
    rows = Fp6Operand(*_fp6_buffers(M, C, dev), M, C, _res_buffer(M, C, dev))
    Mp = round_up(M)
    cols = Fp6Operand(*_fp6_buffers(C, Mp, dev), C, Mp)
    cs = torch.empty((C,), dtype=torch.float32, device=dev)
    xb, dzb = (8, 4) if z16 is None else (4, 0)   # bytes per element: two passes over x, the dz write
    if pre is not None:
        xb //= 2                                    # one pass over x and dy: the statistics came with dy
        L.call("bnn_bn_bwd_stats_pre", L.ptr(pre[0]), pre[1], M, C, 1, L.ptr(w), L.ptr(invstd), L.ptr(dw), L.ptr(db),
               None, None, L.ptr(ws), L.stream())
    sfx = "_pre" if pre is not None else ""
    rb = 0.5 if rows.res is not None else 0.0
    with _timed(name, 0, xb * M * C + (4 if pre is not None else 8) * M * C + dzb * M * C + (3 + rb) * M * C + 3 * C * Mp
                + M * C // 16):
        if z16 is None:
            L.call("bnn_bn_bwd_q6" + sfx, L.ptr(x), L.ptr(dy), M, C, L.ptr(w), L.ptr(b), L.ptr(mean), L.ptr(invstd),
                   L.ptr(mlo), int(hardtanh), float(p), int(seed), dx_ptr, L.ptr(dw), L.ptr(db), L.ptr(rows.lo),
                   L.ptr(rows.hi), L.ptr(rows.sc), L.ptr(rows.res), L.ptr(cols.lo), L.ptr(cols.hi), L.ptr(cols.sc),
                   L.ptr(cs), L.ptr(ws), L.stream())
        else:
            L.call("bnn_bn_bwd_q6_i16" + sfx, L.ptr(z16[0]), L.ptr(z16[1]), L.ptr(dy), M, C, L.ptr(w), L.ptr(b),
                   L.ptr(mean), L.ptr(invstd), L.ptr(mlo), int(hardtanh), float(p), int(seed), dx_ptr, L.ptr(dw),
                   L.ptr(db), L.ptr(rows.lo), L.ptr(rows.hi), L.ptr(rows.sc), L.ptr(rows.res), L.ptr(cols.lo),
                   L.ptr(cols.hi), L.ptr(cols.sc), L.ptr(cs), L.ptr(ws), L.stream())
    setattr(dx, _Q6_ATTR, (_q6_key(dx), rows, cols, cs))
    return dx


# int8 column digits of dz handed from the BatchNorm backward to the input layer's weight gradient
# (bnn_bn_bwd_i8cols -> BinaryLinearPixelsFunction.backward): the pixel layer needs dz only as the
# digit planes of dz^T (with scales, column sums and exact digit sums), so dz is never written.
_I8C_ATTR = "_bnn_i8c"
_I8C_WANT = "_bnn_i8c_consumer"
I8C_HANDOFF = True
I8C_HANDOFFS = 0          # hand-offs made (tests check the path actually ran)


def _bn_bwd_i8c(x, dy, M, C, w, b, mean, invstd, mlo, dw, db, pre=None, s20=None):
    """pre = (part, R): the statistics and the digit bound's maxima from the dX GEMM's epilogue
    (gemm_fp6_bnstats mode 2).  s20 = (low bits, nibbles, bias, scale): x in its compact form
    (x unused)."""
    dev = x.device
    ldqt = round_up(M)
    dg = torch.empty((3, C, ldqt), dtype=torch.int8, device=dev)
    sc = torch.empty((C,), dtype=torch.float32, device=dev)
    cs = torch.empty((C,), dtype=torch.float32, device=dev)
    ds = torch.empty((C,), dtype=torch.int64, device=dev)
    ws = torch.empty((L.lib().bnn_bn_bwd_i8cols_workspace(M, C),), dtype=torch.uint8, device=dev)
    if pre is not None:
        L.call("bnn_bn_bwd_stats_pre", L.ptr(pre[0]), pre[1], M, C, 2, L.ptr(w), L.ptr(invstd), L.ptr(dw), L.ptr(db),
               L.ptr(sc), L.ptr(ds), L.ptr(ws), L.stream())
    xb = 2.5 if s20 is not None else 4
    with _timed("bn_bwd_i8cols", 0, (xb + 4) * (1 if pre is not None else 2) * M * C + dg.numel()):
        sfx = "_pre" if pre is not None else ""
        if s20 is not None:
            L.call("bnn_bn_bwd_i8cols_s20" + sfx, L.ptr(s20[0]), L.ptr(s20[1]), L.ptr(s20[2]), s20[3], L.ptr(dy), M, C,
                   L.ptr(w), L.ptr(b), L.ptr(mean), L.ptr(invstd), L.ptr(mlo), 1, L.ptr(dw), L.ptr(db), L.ptr(dg), ldqt,
                   C * ldqt, L.ptr(sc), L.ptr(cs), L.ptr(ds), L.ptr(ws), L.stream())
        else:
            L.call("bnn_bn_bwd_i8cols" + sfx, L.ptr(x), L.ptr(dy), M, C, L.ptr(w), L.ptr(b), L.ptr(mean), L.ptr(invstd),
                   L.ptr(mlo), 1, L.ptr(dw), L.ptr(db), L.ptr(dg), ldqt, C * ldqt, L.ptr(sc), L.ptr(cs), L.ptr(ds),
                   L.ptr(ws), L.stream())
    dz = _dz_placeholder(M, C, dev)
    setattr(dz, _I8C_ATTR, (_q6_key(dz), dg, sc, cs, ds))
    global I8C_HANDOFFS
    I8C_HANDOFFS += 1
    return dz


def _i8c_take(dy):
    ent = getattr(dy, _I8C_ATTR, None)
    if ent is None:
        if dy.dim() == 2 and dy.stride() == (0, 0) and _is_placeholder(dy):
            raise RuntimeError("a gradient placeholder lost its int8 column-digit hand-off")
        return None
    delattr(dy, _I8C_ATTR)
    if ent[0] != _q6_key(dy):
        raise RuntimeError("stale int8 column-digit hand-off")
    return ent[1:]


class BatchNormHardtanhFunction(torch.autograd.Function):
    """nn.BatchNorm1d on [M, C] (train or eval) optionally followed by nn.Hardtanh, fused
    (mnist-dist2.py:52-74).  Running stats are updated in place in training mode."""

    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, training, momentum, eps, hardtanh, handoff=True):
        _check(x, weight, bias, running_mean, running_var)
        # handoff = False: no FP6 digits of dx for the producing linear (dx is a dense tensor either
        # way here: x is fp32, never a compact placeholder)
        ctx.q6 = handoff and _q6_wanted(x, x.shape[-1], training)
        x = _c2d(x)
        M, C = x.shape
        y = torch.empty_like(x)
        w = weight.detach() if weight is not None else None
        b = bias.detach() if bias is not None else None
        ws = _bn_ws(M, C, x.device)
        if training:
            mean, invstd, mlo = _bn_stat_buffers(C, x.device)
            with _timed("bn_fwd_train", 0, 12 * M * C):
                L.call("bnn_bn_fwd_train", L.ptr(x), M, C, L.ptr(w), L.ptr(b), L.ptr(running_mean),
                       L.ptr(running_var), float(momentum if momentum is not None else -1.0), float(eps),
                       L.ptr(mean), L.ptr(invstd), L.ptr(mlo), L.ptr(y), int(hardtanh), L.ptr(ws), L.stream())
        else:
            mean, mlo = running_mean, None
            invstd = (running_var + eps).rsqrt()
            with _timed("bn_fwd_eval", 0, 8 * M * C):
                L.call("bnn_bn_fwd_eval", L.ptr(x), M, C, L.ptr(w), L.ptr(b), L.ptr(running_mean),
                       L.ptr(running_var), float(eps), L.ptr(y), int(hardtanh), L.ptr(ws), L.stream())
        ctx.save_for_backward(x, w, b, mean, invstd, mlo)
        ctx.hardtanh = hardtanh
        ctx.training = training
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, b, mean, invstd, mlo = ctx.saved_tensors
        dy = _c2d(dy)
        M, C = x.shape
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        dw = torch.empty((C,), dtype=torch.float32, device=x.device) if w is not None else None
        db = torch.empty((C,), dtype=torch.float32, device=x.device) if b is not None else None
        ws = _bn_ws(M, C, x.device)
        if ctx.q6 and dx is not None:
            dx = _bn_bwd_q6(x, dy, M, C, w, b, mean, invstd, mlo, ctx.hardtanh, 0.0, 0, dw, db, ws, "bn_bwd_q6")
        else:
            with _timed("bn_bwd", 0, 16 * M * C):
                _bn_bwd_call(ctx.training, x, dy, M, C, w, b, mean, invstd, mlo, ctx.hardtanh, dx, dw, db, ws)
        return (dx, dw if ctx.needs_input_grad[1] else None, db if ctx.needs_input_grad[2] else None,
                None, None, None, None, None, None, None)


class DropoutBatchNormHardtanhFunction(torch.autograd.Function):
    """hardtanh(nn.BatchNorm1d(nn.Dropout(p)(x))) in training mode, fused (mnist-dist2.py:69-74:
    fc3 -> drop -> bn3 -> htanh3).  The dropout mask is regenerated from ``seed`` by every pass
    (bnn_bn_dropout_*), so neither the mask nor the dropped activation is written to HBM."""

    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, momentum, eps, p, seed):
        _check(x, weight, bias, running_mean, running_var)
        ctx.q6 = _q6_wanted(x, x.shape[-1])
        x = _c2d(x)
        M, C = x.shape
        y = torch.empty_like(x)
        w = weight.detach() if weight is not None else None
        b = bias.detach() if bias is not None else None
        ws = _bn_ws(M, C, x.device)
        mean, invstd, mlo = _bn_stat_buffers(C, x.device)
        with _timed("bn_dropout_fwd_train", 0, 12 * M * C):
            L.call("bnn_bn_dropout_fwd_train", L.ptr(x), M, C, L.ptr(w), L.ptr(b), L.ptr(running_mean),
                   L.ptr(running_var), float(momentum if momentum is not None else -1.0), float(eps),
                   L.ptr(mean), L.ptr(invstd), L.ptr(mlo), L.ptr(y), 1, float(p), int(seed), None, L.ptr(ws),
                   L.stream())
        ctx.save_for_backward(x, w, b, mean, invstd, mlo)
        ctx.p, ctx.seed = p, seed
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, b, mean, invstd, mlo = ctx.saved_tensors
        dy = _c2d(dy)
        M, C = x.shape
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        dw = torch.empty((C,), dtype=torch.float32, device=x.device) if w is not None else None
        db = torch.empty((C,), dtype=torch.float32, device=x.device) if b is not None else None
        ws = _bn_ws(M, C, x.device)
        if ctx.q6 and dx is not None:
            dx = _bn_bwd_q6(x, dy, M, C, w, b, mean, invstd, mlo, True, ctx.p, ctx.seed, dw, db, ws,
                            "bn_dropout_bwd_q6")
            return (dx, dw if ctx.needs_input_grad[1] else None, db if ctx.needs_input_grad[2] else None,
                    None, None, None, None, None, None)
        with _timed("bn_dropout_bwd", 0, 16 * M * C):
            L.call("bnn_bn_dropout_bwd", L.ptr(x), L.ptr(dy), M, C, L.ptr(w), L.ptr(b), L.ptr(mean), L.ptr(invstd),
                   L.ptr(mlo), 1, float(ctx.p), int(ctx.seed), L.ptr(dx), L.ptr(dw), L.ptr(db), L.ptr(ws),
                   L.stream())
        return (dx, dw if ctx.needs_input_grad[1] else None, db if ctx.needs_input_grad[2] else None,
                None, None, None, None, None, None)


HEAD_NOUT = 10
HEAD_CALLS = 0
# BNN_KEEP_BITS=0: the head passes evaluate the dropout hash themselves instead of reading the keep-bit
# plane the statistics pass writes (A/B; identical masks either way)
_KEEP_BITS = [os.environ.get("BNN_KEEP_BITS", "1") != "0"]            # fused drop->bn->htanh->fc heads run (tests check the path actually ran)


class DropoutBNHardtanhLinearFunction(torch.autograd.Function):
    """fc4(hardtanh(bn3(drop(z)))) in training mode, fused (mnist-dist2.py:69-76): the BatchNorm
    statistics pass, then ONE pass that forms h3 tile by tile and multiplies it into the head
    (bnn_bn_head_fwd) -- h3 [M, C] is never written.  Backward (bnn_bn_head_bwd_q6): dh3 = dY4 . W4
    is formed per element inside the BatchNorm passes, dW4 = dY4^T . h3 accumulated there, and dz
    comes out with its FP6 digits for the upstream linear (the _Q6_ATTR hand-off)."""

    @staticmethod
    def forward(ctx, z, weight, bias, running_mean, running_var, momentum, eps, p, seed, w4, b4):
        _check(z, weight, bias, running_mean, running_var, w4, b4)
        global HEAD_CALLS
        HEAD_CALLS += 1
        ctx.q6 = _q6_wanted(z, z.shape[-1])
        zz = _z16_of(z)                       # (int16, bias): the compact pre-activation
        if zz is None:
            z = _c2d(z)
        M, C = z.shape
        gw = weight.detach() if weight is not None else None
        gb = bias.detach() if bias is not None else None
        ws = _bn_ws(M, C, z.device)
        mean, invstd, mlo = _bn_stat_buffers(C, z.device)
        mom = float(momentum if momentum is not None else -1.0)
        fs = _fstats_of(z, M, C, (float(p), int(seed)))
        kb = None   # the dropout keep-bit plane: written by the statistics pass, read by the head passes
        if fs is not None and float(p) > 0:
            global FP4_STATS_USES
            FP4_STATS_USES += 1
            L.call("bnn_bn_fwd_final_parts", L.ptr(fs[0]), fs[1], fs[2], M, C, L.ptr(running_mean),
                   L.ptr(running_var), mom, float(eps), L.ptr(mean), L.ptr(invstd), L.ptr(mlo), L.stream())
        else:
            if float(p) > 0 and _KEEP_BITS[0]:
                kb = torch.empty((int(L.lib().bnn_dropout_keep_bits_bytes(M, C)) // 4,), dtype=torch.int32,
                                 device=z.device)
            with _timed("bn_dropout_fwd_stats", 0, (4 if zz is None else 2) * M * C):
                if zz is None:
                    L.call("bnn_bn_dropout_fwd_train", L.ptr(z), M, C, L.ptr(gw), L.ptr(gb), L.ptr(running_mean),
                           L.ptr(running_var), mom, float(eps), L.ptr(mean), L.ptr(invstd), L.ptr(mlo), None, 1,
                           float(p), int(seed), L.ptr(kb), L.ptr(ws), L.stream())
                else:
                    L.call("bnn_bn_fwd_train_i16", L.ptr(zz[0]), L.ptr(zz[1]), M, C, L.ptr(gw), L.ptr(gb),
                           L.ptr(running_mean), L.ptr(running_var), mom, float(eps), L.ptr(mean), L.ptr(invstd),
                           L.ptr(mlo), float(p), int(seed), L.ptr(kb), L.ptr(ws), L.stream())
        w4c = w4.detach().contiguous()
        y4 = torch.empty((M, HEAD_NOUT), dtype=torch.float32, device=z.device)
        b4d = b4.detach() if b4 is not None else None
        with _timed("bn_head_fwd", 0, (4 if zz is None else 2) * M * C + 4 * M * HEAD_NOUT):
            if zz is None:
                L.call("bnn_bn_head_fwd", L.ptr(z), M, C, L.ptr(mean), L.ptr(invstd), L.ptr(mlo), L.ptr(gw),
                       L.ptr(gb), float(p), int(seed), L.ptr(kb), L.ptr(w4c), HEAD_NOUT, L.ptr(b4d), L.ptr(y4),
                       L.stream())
            else:
                L.call("bnn_bn_head_fwd_i16", L.ptr(zz[0]), L.ptr(zz[1]), M, C, L.ptr(mean), L.ptr(invstd),
                       L.ptr(mlo), L.ptr(gw), L.ptr(gb), float(p), int(seed), L.ptr(kb), L.ptr(w4c), HEAD_NOUT,
                       L.ptr(b4d), L.ptr(y4), L.stream())
        if zz is None:
            ctx.save_for_backward(z, gw, gb, mean, invstd, mlo, w4c, None)
        else:
            ctx.save_for_backward(zz[0], gw, gb, mean, invstd, mlo, w4c, zz[1])
        ctx.z16 = zz is not None
        ctx.dims = (M, C)
        ctx.p, ctx.seed = p, seed
        ctx.kb = kb
        ctx.has_b4 = b4 is not None
        return y4

    @staticmethod
    def backward(ctx, dy4):
        z, gw, gb, mean, invstd, mlo, w4c, zb = ctx.saved_tensors
        dy4 = _c2d(dy4)
        M, C = ctx.dims
        dev = z.device
        # z16 input: its producer's backward takes the digits; dz itself is never written
        dx = _dz_placeholder(M, C, dev) if ctx.z16 else torch.empty((M, C), dtype=torch.float32, device=dev)
        dgw = torch.empty((C,), dtype=torch.float32, device=dev) if gw is not None else None
        dgb = torch.empty((C,), dtype=torch.float32, device=dev) if gb is not None else None
        dw4 = torch.empty((HEAD_NOUT, C), dtype=torch.float32, device=dev)
        rows = Fp6Operand(*_fp6_buffers(M, C, dev), M, C, _res_buffer(M, C, dev))
        Mp = round_up(M)
        cols = Fp6Operand(*_fp6_buffers(C, Mp, dev), C, Mp)
        cs = torch.empty((C,), dtype=torch.float32, device=dev)
        ws = torch.empty((L.lib().bnn_bn_head_workspace(M, C, HEAD_NOUT),), dtype=torch.uint8, device=dev)
        with _timed("bn_head_bwd_q6", 0, (8 if ctx.z16 else 16) * M * C + (0 if ctx.z16 else 4) * M * C + 6 * M * C):
            if not ctx.z16:
                L.call("bnn_bn_head_bwd_q6", L.ptr(z), L.ptr(dy4), L.ptr(w4c), HEAD_NOUT, M, C, L.ptr(gw),
                       L.ptr(gb), L.ptr(mean), L.ptr(invstd), L.ptr(mlo), float(ctx.p), int(ctx.seed),
                       L.ptr(ctx.kb), L.ptr(dx),
                       L.ptr(dgw), L.ptr(dgb), L.ptr(dw4), L.ptr(rows.lo), L.ptr(rows.hi), L.ptr(rows.sc),
                       L.ptr(rows.res), L.ptr(cols.lo), L.ptr(cols.hi), L.ptr(cols.sc), L.ptr(cs), L.ptr(ws), L.stream())
            else:
                L.call("bnn_bn_head_bwd_q6_i16", L.ptr(z), L.ptr(zb), L.ptr(dy4), L.ptr(w4c), HEAD_NOUT, M, C,
                       L.ptr(gw), L.ptr(gb), L.ptr(mean), L.ptr(invstd), L.ptr(mlo), float(ctx.p), int(ctx.seed),
                       L.ptr(ctx.kb), None, L.ptr(dgw), L.ptr(dgb), L.ptr(dw4), L.ptr(rows.lo), L.ptr(rows.hi),
                       L.ptr(rows.sc), L.ptr(rows.res), L.ptr(cols.lo), L.ptr(cols.hi), L.ptr(cols.sc), L.ptr(cs),
                       L.ptr(ws), L.stream())
        if ctx.q6 or ctx.z16:
            setattr(dx, _Q6_ATTR, (_q6_key(dx), rows, cols, cs))
        db4 = None
        if ctx.has_b4 and ctx.needs_input_grad[10]:
            if COL_SUMS and M <= 32768 and dy4.is_contiguous():   # one libbnn launch (fixed order)
                db4 = torch.empty((HEAD_NOUT,), dtype=torch.float32, device=dev)
                L.call("bnn_col_sums_narrow", L.ptr(dy4), M, HEAD_NOUT, HEAD_NOUT, L.ptr(db4), L.stream())
            else:
                db4 = dy4.sum(0)
        return (dx, dgw if ctx.needs_input_grad[1] else None, dgb if ctx.needs_input_grad[2] else None,
                None, None, None, None, None, None, dw4 if ctx.needs_input_grad[9] else None, db4)


def head_fusable(x, bn, fc):
    """drop -> bn -> htanh -> fc as one libbnn head (DropoutBNHardtanhLinearFunction): training-mode
    BatchNorm1d with batch statistics, a Linear(C, 10), C % 256 == 0."""
    return (x.is_cuda and x.dim() == 2 and x.shape[1] % 256 == 0 and x.shape[0] > 0 and bn.training
            and bn.track_running_stats and isinstance(fc, torch.nn.Linear) and fc.out_features == HEAD_NOUT
            and fc.in_features == x.shape[1] and bn.momentum is not None)


def dropout_seed():
    """The seed of a fused dropout: the graph step's base seed, else one draw of torch's CPU RNG."""
    return _DEVICE_STEP.base_seed if _DEVICE_STEP is not None else int(torch.randint(0, 2 ** 62, (1,)).item())


def dropout_bn_hardtanh_linear(x, p, bn, fc, seed=None):
    """fc(hardtanh(bn(nn.Dropout(p)(x)))) through libbnn (training mode; see head_fusable)."""
    if seed is None:
        seed = dropout_seed()
    rm, rv, bn_training, factor = _bn_module_args(bn)
    if not bn_training:
        raise ValueError("dropout_bn_hardtanh_linear is the training-mode fusion")
    return DropoutBNHardtanhLinearFunction.apply(x, bn.weight, bn.bias, rm, rv, factor, bn.eps, float(p), seed,
                                                 fc.weight, fc.bias)


def dropout_mask(n, p, seed, device="cuda"):
    """The keep mask (scaled: 1/(1-p) or 0) the fused dropout passes use for elements 0..n-1."""
    out = torch.empty((n,), dtype=torch.float32, device=device)
    L.call("bnn_dropout_mask", n, float(p), int(seed), L.ptr(out), L.stream())
    return out


def dropout_batch_norm_hardtanh(x, p, bn, seed=None):
    """nn.Dropout(p) -> nn.BatchNorm1d module (training mode) -> Hardtanh through libbnn.  The seed
    is drawn from torch's CPU generator (so torch.manual_seed makes runs repeatable) unless given."""
    if seed is None:
        # device-step mode: a fixed base seed, the kernels add the device step counter
        seed = _DEVICE_STEP.base_seed if _DEVICE_STEP is not None else int(torch.randint(0, 2 ** 62, (1,)).item())
    rm, rv, bn_training, factor = _bn_module_args(bn)
    if not bn_training:
        raise ValueError("dropout_batch_norm_hardtanh is the training-mode fusion")
    return DropoutBatchNormHardtanhFunction.apply(x, bn.weight, bn.bias, rm, rv, factor, bn.eps, float(p), seed)


_BN_DEFER = None   # while a bn_counter_batch is open: the num_batches_tracked buffers to increment


class bn_counter_batch:
    """Inside it, the fused BatchNorm ops defer torch's per-module ``num_batches_tracked += 1``
    (_BatchNorm.forward) and issue all of them as one multi-tensor launch on exit -- the nets'
    forward opens one (one launch instead of one per BatchNorm).  Modules with momentum=None
    (the cumulative average reads the counter) still increment at once."""

    def __enter__(self):
        global _BN_DEFER
        self._prev, _BN_DEFER = _BN_DEFER, []
        return self

    def __exit__(self, *exc):
        global _BN_DEFER
        todo, _BN_DEFER = _BN_DEFER, self._prev
        if len(todo) == 1:
            todo[0].add_(1)
        elif todo:
            torch._foreach_add_(todo, 1)
        return False


def _bn_module_args(bn):
    """torch _BatchNorm.forward bookkeeping: (running_mean, running_var, use_batch_stats, factor)."""
    factor = 0.0 if bn.momentum is None else bn.momentum
    if bn.training and bn.track_running_stats and bn.num_batches_tracked is not None:
        if bn.momentum is not None and _BN_DEFER is not None:
            _BN_DEFER.append(bn.num_batches_tracked)
        else:
            bn.num_batches_tracked.add_(1)
        if bn.momentum is None:               # cumulative moving average (host sync, rare)
            factor = 1.0 / float(bn.num_batches_tracked)
    bn_training = bn.training or (bn.running_mean is None and bn.running_var is None)
    pass_stats = (not bn.training) or bn.track_running_stats
    rm = bn.running_mean if pass_stats else None
    rv = bn.running_var if pass_stats else None
    return rm, rv, bn_training, factor


def batch_norm_hardtanh(x, bn, hardtanh=True, handoff=True):
    """Apply an ``nn.BatchNorm1d`` module (its parameters, buffers, momentum / eps /
    track_running_stats semantics as in torch's ``_BatchNorm.forward``) followed by Hardtanh,
    through libbnn.  handoff = False: never hand FP6 digits of dx to the producing linear."""
    rm, rv, bn_training, factor = _bn_module_args(bn)
    return BatchNormHardtanhFunction.apply(x, bn.weight, bn.bias, rm, rv, bn_training, factor, bn.eps,
                                           hardtanh, bool(handoff))


# ----------------------------------------------------------------------------- BatchNorm2d (+ Hardtanh + MaxPool2d)
class BatchNorm2dHardtanhPoolFunction(torch.autograd.Function):
    """maxpool2(hardtanh(nn.BatchNorm2d(x))) on NCHW, fused (the block after each BinarizeConv2d of
    the build's CNN; mnist-dist.py:31-51 template).  pool = 2 fuses MaxPool2d(2, 2) (argmax
    recomputed in backward), pool = 0 leaves it out.  Running stats updated in place (train)."""

    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, training, momentum, eps, hardtanh, pool):
        _check(x, weight, bias, running_mean, running_var)
        zq = _zq_of(x)                        # (int8/int16 sums, bias, fmt): x in its compact form
        if zq is not None and not training:
            raise RuntimeError("a compact conv output needs the training-mode BatchNorm2d")
        if zq is None:
            x = x if x.is_contiguous() else x.contiguous()
        N, C, H, W = x.shape
        oh, ow = (H // 2, W // 2) if pool else (H, W)
        y = torch.empty((N, C, oh, ow), dtype=torch.float32, device=x.device)
        w = weight.detach() if weight is not None else None
        b = bias.detach() if bias is not None else None
        ws = torch.empty((L.lib().bnn_bn2d_workspace(N, C),), dtype=torch.uint8, device=x.device)
        nel = N * C * H * W
        if training:
            mean = torch.empty((C,), dtype=torch.float32, device=x.device)
            invstd = torch.empty_like(mean)
            xb = 4 if zq is None else zq[0].element_size()
            with _timed("bn2d_fwd_train", 0, 2 * xb * nel + 4 * y.numel()):
                if zq is None:
                    L.call("bnn_bn2d_fwd_train", L.ptr(x), N, C, H, W, L.ptr(w), L.ptr(b), L.ptr(running_mean),
                           L.ptr(running_var), float(momentum if momentum is not None else -1.0), float(eps),
                           L.ptr(mean), L.ptr(invstd), L.ptr(y), int(hardtanh), int(pool), L.ptr(ws), L.stream())
                else:
                    L.call("bnn_bn2d_fwd_train_q", L.ptr(zq[0]), L.ptr(zq[1]), zq[2], N, C, H, W, L.ptr(w), L.ptr(b),
                           L.ptr(running_mean), L.ptr(running_var), float(momentum if momentum is not None else -1.0),
                           float(eps), L.ptr(mean), L.ptr(invstd), L.ptr(y), int(hardtanh), int(pool), L.ptr(ws),
                           L.stream())
        else:
            mean = running_mean
            invstd = (running_var + eps).rsqrt()
            with _timed("bn2d_fwd_eval", 0, 4 * nel + 4 * y.numel()):
                L.call("bnn_bn2d_fwd_eval", L.ptr(x), N, C, H, W, L.ptr(w), L.ptr(b), L.ptr(running_mean),
                       L.ptr(running_var), float(eps), L.ptr(y), int(hardtanh), int(pool), L.ptr(ws), L.stream())
        if zq is None:
            ctx.save_for_backward(x, w, b, mean, invstd, None, None)
        else:
            ctx.save_for_backward(zq[0], w, b, mean, invstd, zq[1], None)
        ctx.zq_fmt = 0 if zq is None else zq[2]
        ctx.c1bn = (zq is not None and training and pool == 2 and bool(getattr(x, _C1BN_WANT, False)))
        ctx.shape = (N, C, H, W)
        ctx.hardtanh, ctx.pool = hardtanh, pool
        ctx.training = training
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, b, mean, invstd, xbias, _ = ctx.saved_tensors
        dy = dy if dy.is_contiguous() else dy.contiguous()
        N, C, H, W = ctx.shape
        dx = torch.empty((N, C, H, W), dtype=torch.float32, device=dy.device) if ctx.needs_input_grad[0] else None
        dw = torch.empty((C,), dtype=torch.float32, device=dy.device) if w is not None else None
        db = torch.empty((C,), dtype=torch.float32, device=dy.device) if b is not None else None
        ws = torch.empty((L.lib().bnn_bn2d_workspace(N, C),), dtype=torch.uint8, device=dy.device)
        nel = N * C * H * W
        xb = 4 if ctx.zq_fmt == 0 else x.element_size()
        if ctx.c1bn and ctx.needs_input_grad[0]:
            # statistics only; the conv's filter gradient forms dx from them (bnn_conv2d_bwd_filter_bn)
            sg = torch.empty((C,), dtype=torch.float32, device=dy.device)
            sgx = torch.empty_like(sg)
            with _timed("bn2d_bwd_stats", 0, xb * nel + 4 * dy.numel()):
                L.call("bnn_bn2d_bwd_stats_q", L.ptr(x), L.ptr(xbias), ctx.zq_fmt, L.ptr(dy), N, C, H, W, L.ptr(w),
                       L.ptr(b), L.ptr(mean), L.ptr(invstd), int(ctx.hardtanh), int(ctx.pool), L.ptr(dw), L.ptr(db),
                       L.ptr(sg), L.ptr(sgx), L.ptr(ws), L.stream())
            dx = _placeholder((N, C, H, W), dy.device)
            setattr(dx, _C1BN_ATTR, (_q6_key(dx), x, xbias, ctx.zq_fmt, dy, mean, invstd, w, b, sg, sgx,
                                     1.0 / (N * H * W), int(ctx.hardtanh)))
            return (dx, dw if ctx.needs_input_grad[1] else None, db if ctx.needs_input_grad[2] else None,
                    None, None, None, None, None, None, None)
        with _timed("bn2d_bwd", 0, (2 * xb + 4) * nel + 8 * dy.numel()):
            if ctx.zq_fmt:
                L.call("bnn_bn2d_bwd_q", L.ptr(x), L.ptr(xbias), ctx.zq_fmt, L.ptr(dy), N, C, H, W, L.ptr(w), L.ptr(b),
                       L.ptr(mean), L.ptr(invstd), int(ctx.hardtanh), int(ctx.pool), L.ptr(dx), L.ptr(dw), L.ptr(db),
                       L.ptr(ws), L.stream())
            else:
                L.call("bnn_bn2d_bwd" if ctx.training else "bnn_bn2d_bwd_eval", L.ptr(x), L.ptr(dy), N, C, H, W,
                       L.ptr(w), L.ptr(b), L.ptr(mean), L.ptr(invstd), int(ctx.hardtanh), int(ctx.pool), L.ptr(dx),
                       L.ptr(dw), L.ptr(db), L.ptr(ws), L.stream())
        return (dx, dw if ctx.needs_input_grad[1] else None, db if ctx.needs_input_grad[2] else None,
                None, None, None, None, None, None, None)


def bn2d_fusable(x, pool):
    """Shapes the fused BatchNorm2d kernels take (else the caller runs the torch modules)."""
    if not (x.is_cuda and x.dim() == 4 and x.dtype == torch.float32):
        return False
    H, W = x.shape[2], x.shape[3]
    return (H * W) % 4 == 0 and (not pool or (H % 2 == 0 and W % 2 == 0))


def batch_norm2d_hardtanh_pool(x, bn, hardtanh=True, pool=2):
    """Apply an ``nn.BatchNorm2d`` module (torch ``_BatchNorm.forward`` semantics), then Hardtanh
    and MaxPool2d(2, 2) (pool = 2) through libbnn."""
    rm, rv, bn_training, factor = _bn_module_args(bn)
    return BatchNorm2dHardtanhPoolFunction.apply(x, bn.weight, bn.bias, rm, rv, bn_training, factor, bn.eps,
                                                 hardtanh, pool)


class BNHardtanhBinaryLinearFunction(torch.autograd.Function):
    """fc(hardtanh(bn(z))) with fc a BinarizeLinear whose input is binarised (the hidden layers
    of the reference Net, mnist-dist2.py:66-71): BatchNorm statistics, then ONE pass writes the
    next GEMM's ternary operand (FP4 or int8 rows + int8 transpose) straight from z -- the fp32
    hardtanh output the reference materialises is never written.  Backward: dh = dY.W_b and
    dW = dY^T.sign(h) on the digit GEMM, then the fused BatchNorm+Hardtanh backward."""

    @staticmethod
    def forward(ctx, z, bn_w, bn_b, rm, rv, training, momentum, eps, weight, bias, backend, emit_z16=False,
                emit_stats=False):
        _check(z, bn_w, bn_b, rm, rv, weight, bias)
        ctx.q6 = _q6_wanted(z, z.shape[-1], training)
        ctx.i8c = (I8C_HANDOFF and bool(getattr(z, _I8C_WANT, False)) and training and not ctx.q6
                   and z.dim() == 2 and z.shape[-1] % 4 == 0)
        zz = _z16_of(z)                       # (int16, bias): z in its compact form
        zs = _s20_of(z)                       # (int16 low bits, nibbles, bias, scale): fc1's compact z1
        if zz is None and zs is None:
            z = _c2d(z)
        M, C = z.shape
        N = weight.shape[0]
        fp4 = backend == "fp4"
        ctx.fp6 = fp4 and DIGIT_GEMM == "fp6"
        if zz is not None and not (training and ctx.fp6 and ctx.q6 and C % 256 == 0):
            raise RuntimeError("a z16 pre-activation needs the training-mode FP4/FP6 consumer (z16_ok)")
        if zs is not None and not (training and ctx.fp6 and ctx.i8c and C % 256 == 0 and _fstats_of(z, M, C)):
            raise RuntimeError("an s20 pre-activation needs the training-mode FP4/FP6 consumer with the "
                               "int8 column-digit backward and the GEMM-epilogue statistics")
        gw = bn_w.detach() if bn_w is not None else None
        gb = bn_b.detach() if bn_b is not None else None
        if training:
            mean, invstd, mlo = _bn_stat_buffers(C, z.device)
            ws = _bn_ws(M, C, z.device)
            mom = float(momentum if momentum is not None else -1.0)
            with _timed("bn_fwd_stats", 0, (4 if zz is None else 2) * M * C):
                fs = _fstats_of(z, M, C)
                if fs is not None:
                    global PIX_STATS_USES, FP4_STATS_USES
                    if fs[5] == "pixels":
                        PIX_STATS_USES += 1
                    else:
                        FP4_STATS_USES += 1
                    L.call("bnn_bn_fwd_final_parts", L.ptr(fs[0]), fs[1], fs[2], M, C, L.ptr(rm), L.ptr(rv), mom,
                           float(eps), L.ptr(mean), L.ptr(invstd), L.ptr(mlo), L.stream())
                elif zz is None:
                    assert zs is None
                    L.call("bnn_bn_fwd_train", L.ptr(z), M, C, L.ptr(gw), L.ptr(gb), L.ptr(rm), L.ptr(rv), mom,
                           float(eps), L.ptr(mean), L.ptr(invstd), L.ptr(mlo), None, 1, L.ptr(ws), L.stream())
                else:
                    L.call("bnn_bn_fwd_train_i16", L.ptr(zz[0]), L.ptr(zz[1]), M, C, L.ptr(gw), L.ptr(gb), L.ptr(rm),
                           L.ptr(rv), mom, float(eps), L.ptr(mean), L.ptr(invstd), L.ptr(mlo), 0.0, 0, None,
                           L.ptr(ws), L.stream())
        else:
            mean, mlo = rm.contiguous(), None
            invstd = (rv + eps).rsqrt()
        need_dh = any(ctx.needs_input_grad[:3])
        need_dw = ctx.needs_input_grad[8] or zz is not None
        # FP6 backward: both GEMMs' B operands (this layer's X_b^T and W_b^T) are written straight in
        # the FP4 panel layout gemm_fp6 stages from (no panel pass)
        qf = "fp4p" if ctx.fp6 else "i8"
        q = torch.empty((M, round_up(C, 256) // 2) if fp4 else (M, round_up(C)),
                        dtype=torch.uint8 if fp4 else torch.int8, device=z.device)
        ctx.qt_panel = need_dw and qf == "fp4p"
        qt = _qt_buffer(C, M, qf, z.device) if need_dw else None
        nx = 2.5 if zs is not None else (4 if zz is None else 2)
        with _timed("bn_apply_pack", 0, nx * M * C + q.numel() + (qt.numel() if qt is not None else 0)):
            if zs is not None:
                L.call("bnn_bn_apply_pack_s20", L.ptr(zs[0]), L.ptr(zs[1]), L.ptr(zs[2]), zs[3], M, C, L.ptr(mean),
                       L.ptr(invstd), L.ptr(mlo), L.ptr(gw), L.ptr(gb), L.ptr(q), q.shape[1], L.ptr(qt), qt.shape[1],
                       1 if ctx.qt_panel else 0, L.stream())
            elif zz is None:
                L.call("bnn_bn_apply_pack", L.ptr(z), M, C, L.ptr(mean), L.ptr(invstd), L.ptr(mlo), L.ptr(gw),
                       L.ptr(gb), 1 if fp4 else 0, L.ptr(q), q.shape[1], L.ptr(qt), qt.shape[1] if qt is not None else 0,
                       _QT_CODE[qf], L.stream())
            else:
                L.call("bnn_bn_apply_pack_i16", L.ptr(zz[0]), L.ptr(zz[1]), M, C, L.ptr(mean), L.ptr(invstd),
                       L.ptr(mlo), L.ptr(gw), L.ptr(gb), L.ptr(q), q.shape[1], L.ptr(qt), qt.shape[1],
                       1 if ctx.qt_panel else 0, L.stream())
        b = bias.detach() if bias is not None else None
        wq, wqt = packed_weight(weight, "fp4" if fp4 else "i8", True, need_dh, cache=True, qt_fmt=qf)
        chunk = (int(L.lib().bnn_gemm_fp4_bnstats_chunk(M, N, q.shape[1]))
                 if emit_stats and FP4_STATS and fp4 and M > 0 and N % 4 == 0 else 0)
        drop = tuple(emit_stats) if isinstance(emit_stats, tuple) else (0.0, 0)   # (p, seed) of a fused dropout
        if emit_z16 and fp4 and training:
            # the next BatchNorm reads z = fl(I + bias) from int16 I and the bias (a detached view of
            # the Parameter: its consumer saves it for backward, so torch refuses a backward after an
            # in-place update of it)
            bs = b
            if chunk:
                y16, fst = _fp4_fwd_with_stats(q, wq, M, N, C, None, bs, chunk, True, drop)
                y = _z16_carrier(y16, bs)
                setattr(y, _FSTATS_ATTR, fst)
            else:
                y = _z16_carrier(gemm_fp4_i16(q, wq, M, N, k_true=C), bs)
        elif fp4 and chunk:
            y, fst = _fp4_fwd_with_stats(q, wq, M, N, C, b, b, chunk, False, drop)
            setattr(y, _FSTATS_ATTR, fst)
        elif fp4:
            y = gemm_fp4(q, wq, M, N, bias=b, k_true=C)
        else:
            y = gemm_i8(q, 1, wq, 1, M, N, bias=b, k_true=C)
        if zs is not None:
            ctx.save_for_backward(zs[0], gw, gb, mean, invstd, mlo, qt, wqt, zs[2])
            ctx.s20 = (zs[1], zs[3])          # the nibble plane and the scale
        elif zz is None:
            ctx.save_for_backward(z, gw, gb, mean, invstd, mlo, qt, wqt, None)
        else:
            ctx.save_for_backward(zz[0], gw, gb, mean, invstd, mlo, qt, wqt, zz[1])
        if zs is None:
            ctx.s20 = None
        ctx.z16 = zz is not None
        ctx.weight_ref = weight
        ctx.training = training
        ctx.dims = (M, C, N)
        ctx.has_bias = bias is not None
        if ctx.fp6:
            setattr(y, _Q6_WANT, True)
        return y

    @staticmethod
    def backward(ctx, dy):
        z, gw, gb, mean, invstd, mlo, qt, wqt, zb = ctx.saved_tensors
        M, C, N = ctx.dims
        pre = _q6_take_required(dy) if ctx.fp6 else None       # digits of dy from the BatchNorm backward
        if pre is None:
            dy = _c2d(dy)
        dz = dgw = dgb = dw = db = None
        need_db = ctx.has_bias and ctx.needs_input_grad[9]
        sink, ex = _grad_sink(ctx.weight_ref) if ctx.needs_input_grad[8] and ctx.fp6 else (None, None)
        if ctx.needs_input_grad[8] or need_db:
            if ctx.fp6:
                dt, cs = (pre[1], (pre[2] if need_db else None)) if pre is not None else \
                    quant6_cols_t(dy, want_colsum=need_db)
                if ctx.needs_input_grad[8]:
                    if ctx.qt_panel:
                        dw = gemm_fp6(dt, None, C, k_true=M, out=sink, panels=qt, panel_ks=qt.shape[1] // 32)
                    else:
                        dw = gemm_fp6(dt, qt, C, k_true=M, out=sink)           # dY^T . sign(h)
                    if sink is not None:        # written into the bucket view: nothing to accumulate
                        ex.grad_written(ctx.weight_ref)
                        dw = None
            else:
                dt, sc, cs = quant_cols_t(dy, want_colsum=need_db)
                if ctx.needs_input_grad[8]:
                    dw = gemm_i8(dt, 3, qt, 1, N, C, a_scale=sc, k_true=M)
            db = cs
        if any(ctx.needs_input_grad[:3]):
            st = None
            if ctx.fp6:
                A = pre[0] if pre is not None else quant6_rows(dy)
                if ctx.training and (ctx.q6 or ctx.i8c) and ctx.s20 is None and _bn_epi_ok(M, C, A.Kp):
                    # the BatchNorm backward's statistics come with dh from the GEMM's epilogue
                    dh, part, R = gemm_fp6_bnstats(A, wqt, wqt.shape[1] // 32, C, z, zb if ctx.z16 else None,
                                                   ctx.z16, mean, mlo, invstd, gw, gb, 1 if ctx.q6 else 2)
                    st = (part, R)
                else:
                    dh = gemm_fp6(A, None, C, k_true=N, panels=wqt, panel_ks=wqt.shape[1] // 32)   # dY . W_b
                del A
            else:
                d, s = quant_rows(dy)
                dh = gemm_i8(d, 3, wqt, 1, M, C, a_scale=s, k_true=N)
            del pre
            dgw = torch.empty((C,), dtype=torch.float32, device=z.device) if gw is not None else None
            dgb = torch.empty((C,), dtype=torch.float32, device=z.device) if gb is not None else None
            ws = _bn_ws(M, C, z.device)
            if ctx.q6:
                dz = _bn_bwd_q6(z, dh, M, C, gw, gb, mean, invstd, mlo, True, 0.0, 0, dgw, dgb, ws, "bn_bwd_q6",
                                z16=(z, zb) if ctx.z16 else None, pre=st)
            elif ctx.i8c:
                dz = _bn_bwd_i8c(z, dh, M, C, gw, gb, mean, invstd, mlo, dgw, dgb, pre=st,
                                 s20=(z, ctx.s20[0], zb, ctx.s20[1]) if ctx.s20 is not None else None)
            else:
                dz = torch.empty_like(z)
                with _timed("bn_bwd", 0, 16 * M * C):
                    _bn_bwd_call(ctx.training, z, dh, M, C, gw, gb, mean, invstd, mlo, True, dz, dgw, dgb, ws)
        return (dz, dgw if ctx.needs_input_grad[1] else None, dgb if ctx.needs_input_grad[2] else None,
                None, None, None, None, None, dw, db, None, None, None)


def bn_hardtanh_binary_linear(z, bn, fc, backend="fp4", emit_z16=False, emit_stats=False):
    """fc(hardtanh(bn(z))) through BNHardtanhBinaryLinearFunction (bn: nn.BatchNorm1d, fc: a
    BinarizeLinear holding its latent weight, i.e. ``org_protocol = False``).  emit_z16: return
    fc's output as a z16 placeholder (its consumer must be a z16-aware libbnn BatchNorm pass:
    bn_hardtanh_binary_linear or dropout_bn_hardtanh_linear in training mode; see z16_ok)."""
    rm, rv, bn_training, factor = _bn_module_args(bn)
    return BNHardtanhBinaryLinearFunction.apply(z, bn.weight, bn.bias, rm, rv, bn_training, factor, bn.eps,
                                                fc.weight, fc.bias, backend, bool(emit_z16),
                                                emit_stats if isinstance(emit_stats, tuple) else bool(emit_stats))

"""CPU-side checks of the C-ABI library: it loads, exports every symbol include/bnn.h declares,
and rejects bad arguments without launching anything (no GPU needed for these)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "bnn.h")


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|const char\*)\s+(bnn_\w+)\(", text, re.M)))


@pytest.fixture(scope="module")
def L():
    from bnn_amd import _lib
    return _lib.lib()


def test_header_declares_the_bound_signatures():
    from bnn_amd import _lib
    assert declared_symbols() == sorted(_lib.SIGNATURES)


def test_library_exports_every_declared_symbol(L):
    for name in declared_symbols():
        assert hasattr(L, name), name


def test_version_and_error_string(L):
    assert L.bnn_version() >= 1
    assert isinstance(L.bnn_last_error(), bytes)


def test_bad_arguments_are_rejected_without_a_gpu(L):
    from bnn_amd import _lib
    # K not a multiple of 64 -> BNN_EINVAL before any launch
    rc = L.bnn_gemm_i8(ctypes.c_void_p(16), 64, 0, 1, ctypes.c_void_p(16), 64, 0, 1, None, None, None,
                       ctypes.c_void_p(16), 8, 8, 8, 63, None)
    assert rc == -1
    assert b"bad arguments" in L.bnn_last_error()
    # unsupported digit combination (1,3)
    rc = L.bnn_gemm_i8(ctypes.c_void_p(16), 64, 0, 1, ctypes.c_void_p(16), 64, 64 * 8, 3, None, None, None,
                       ctypes.c_void_p(16), 8, 8, 8, 64, None)
    assert rc == -1
    rc = L.bnn_sign_pack_i8(ctypes.c_void_p(16), 4, 100, 100, ctypes.c_void_p(16), 100, None, 0, None)
    assert rc == -1  # ldq must be a multiple of 64
    with pytest.raises(_lib.BnnError):
        _lib.call("bnn_quant_rows", None, 1, 1, 1, None, 64, 64, None, None)


def test_workspace_queries(L):
    assert L.bnn_quant_cols_workspace(65536, 8192) > 0
    assert L.bnn_conv2d_bwd_filter_workspace(4096, 16, 32, 5, 5, 1) > 0


def test_ops_refuse_cpu_tensors():
    import torch
    from bnn_amd import functional as F
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        F.sign(torch.zeros(4))
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        F.binary_linear(torch.zeros(2, 8), torch.zeros(3, 8))


def test_conv_bf3_plans_are_bank_conflict_free(L):
    """The bf16x3 conv backward kernels' LDS layouts for the BinCNN's conv2 (host-only plan query):
    the data kernel's pixel / weight pitches are 16 (mod 32) bf16 with one image row per pixel
    tile, the filter kernel's dY pitch likewise, and its shifted input copies are padded so the
    modelled B-fragment ds_read_b128 is conflict-free (4 LDS cycles; the plain layout put all five
    kw copies of a combo row on the same banks)."""
    out = (ctypes.c_int64 * 9)()
    assert L.bnn_conv_bf3_plan(4096, 16, 14, 14, 32, 5, 5, 1, 2, 1, 1, out) == 0
    ps, ws, rowt, lds_d, kd, cs, xl, lds_f, cyc = list(out)
    assert ps % 32 == 16 and ws % 32 == 16 and rowt == 1 and lds_d <= 160 * 1024
    assert kd % 32 == 16 and cs % 8 == 0 and xl % 8 == 0 and lds_f <= 160 * 1024
    assert cyc == 400
    # shapes neither kernel takes report -1
    assert L.bnn_conv_bf3_plan(4, 8, 9, 9, 8, 3, 3, 2, 1, 1, 1, out) == 0 and out[0] == -1 and out[4] == -1


def test_bn_dropin_rejects_cpu_and_non_2d_inputs():
    """bnn_amd.nn.BatchNorm1d raises for what it does not run on the GPU (no silent torch fallback)."""
    import pytest
    import torch
    from bnn_amd.nn import BatchNorm1d
    bn = BatchNorm1d(8)
    assert isinstance(bn, torch.nn.BatchNorm1d) and set(bn.state_dict()) == set(torch.nn.BatchNorm1d(8).state_dict())
    with pytest.raises(TypeError, match="float32 CUDA"):
        bn(torch.randn(4, 8))

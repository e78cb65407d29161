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

"""Drop-in for the reference's ``models/binarized_modules.py`` on MI355X.

The reference scripts import exactly::

    from models.binarized_modules import BinarizeLinear, BinarizeConv2d   # mnist-dist2.py:15
    from models.binarized_modules import Binarize, HingeLoss              # mnist-dist2.py:16

Put ``distributed-mnist-bnns_amd/`` ahead of the reference checkout on ``sys.path`` (or copy
this ``models/`` package next to the scripts together with ``bnn_amd/`` and ``lib/``) and the
same lines bind to the libbnn-backed modules below, with the reference's ``weight.org``
protocol and input side effects preserved (bnn_amd/nn.py documents each one).
"""
import os
import sys

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _PKG_ROOT not in sys.path:
    sys.path.insert(0, _PKG_ROOT)

from bnn_amd.nn import (Binarize, BinarizeConv2d, BinarizeLinear, HingeLoss,  # noqa: E402,F401
                        Quantize, SqrtHingeLossFunction)

__all__ = ["Binarize", "HingeLoss", "SqrtHingeLossFunction", "Quantize", "BinarizeLinear",
           "BinarizeConv2d"]

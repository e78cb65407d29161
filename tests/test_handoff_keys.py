"""Host logic of the autograd hand-offs (functional._placeholder / _q6_key): every gradient
placeholder is a stride-0 view of one cached zero per device, so they all share data_ptr and the
version counter; each carries a unique token that the hand-offs' staleness key includes, so two
placeholders of the same shape never key alike."""
import torch

from bnn_amd import functional as F


def test_placeholders_key_apart():
    a = F._placeholder((4, 5), "cpu")
    b = F._placeholder((4, 5), "cpu")
    assert a.data_ptr() == b.data_ptr() and a.stride() == (0, 0)
    assert F._q6_key(a) != F._q6_key(b)
    assert F._q6_key(a) == F._q6_key(a)


def test_stale_handoff_refused():
    """A hand-off attached to one placeholder is not taken through another of the same shape."""
    a = F._placeholder((3, 64), "cpu")
    b = F._placeholder((3, 64), "cpu")
    setattr(b, F._Q6_ATTR, (F._q6_key(a), "rows", "cols", "cs"))      # a key that is not b's
    assert F._q6_take(b) is None
    setattr(a, F._Q6_ATTR, (F._q6_key(a), "rows", "cols", "cs"))
    assert F._q6_take(a) == ("rows", "cols", "cs")
    assert isinstance(torch.zeros(1), torch.Tensor)

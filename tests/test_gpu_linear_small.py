"""GPU parity of the narrow fp32 Linear (bnn_linear_nsmall_*): the BinCNN's classifier
nn.Linear(7*7*32, 10) (BASELINE config 4), forward and backward, against float64.

Bars: y, dx, dw, db within 1e-6 norm-wise of float64 (fp32 products and sums, another order than
torch's GEMM); deterministic (two runs bit-identical); an empty batch gives zero dw / db."""
import numpy as np
import pytest
import torch

from conftest import rel_err

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def F():
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    from bnn_amd import functional
    return functional


def host(t):
    torch.cuda.synchronize()
    return t.detach().cpu().numpy()


@pytest.mark.parametrize("M,K,N", [(4096, 1568, 10), (77, 36, 10), (1000, 1024, 16), (5, 8, 1), (300, 260, 4),
                                   (20000, 1568, 10)])
def test_linear_nsmall_vs_float64(F, M, K, N):
    g = torch.Generator(device="cuda").manual_seed(M + K + N)
    x = torch.randn(M, K, generator=g, device="cuda").requires_grad_(True)
    w = (torch.randn(N, K, generator=g, device="cuda") * 0.05).requires_grad_(True)
    b = torch.randn(N, generator=g, device="cuda").requires_grad_(True)
    dy = torch.randn(M, N, generator=g, device="cuda")
    y = F.linear_nsmall(x, w, b)
    y.backward(dy)
    xd, wd, bd, dyd = (host(t).astype(np.float64) for t in (x, w, b, dy))
    assert rel_err(host(y), xd @ wd.T + bd) <= 1e-6
    assert rel_err(host(x.grad), dyd @ wd) <= 1e-6
    assert rel_err(host(w.grad), dyd.T @ xd) <= 1e-6
    assert rel_err(host(b.grad), dyd.sum(0)) <= 1e-6
    # deterministic
    gx, gw, gb = x.grad.clone(), w.grad.clone(), b.grad.clone()
    x.grad = w.grad = b.grad = None
    y2 = F.linear_nsmall(x, w, b)
    y2.backward(dy)
    assert torch.equal(y, y2) and torch.equal(gx, x.grad) and torch.equal(gw, w.grad) and torch.equal(gb, b.grad)


def test_linear_nsmall_no_bias_and_empty_batch(F):
    w = torch.randn(10, 64, device="cuda", requires_grad=True)
    x = torch.randn(33, 64, device="cuda", requires_grad=True)
    y = F.linear_nsmall(x, w, None)
    assert rel_err(host(y), host(x).astype(np.float64) @ host(w).astype(np.float64).T) <= 1e-6
    b = torch.randn(10, device="cuda", requires_grad=True)
    e = torch.zeros((0, 64), device="cuda", requires_grad=True)
    F.linear_nsmall(e, w, b).sum().backward()
    assert w.grad is not None and not w.grad.any() and not b.grad.any()


def test_bincnn_uses_the_narrow_linear(F):
    from bnn_amd import nets
    m = nets.BinCNN(org_protocol=False, mutate_input=False, fused_bn=True).cuda()
    x = torch.randn(64, 1, 28, 28, device="cuda")
    timer = F.KernelTimer()
    with F.timing(timer):
        torch.nn.functional.nll_loss(m(x), torch.randint(0, 10, (64,), device="cuda")).backward()
    names = set(timer.summary())
    assert "linear_nsmall_fwd" in names and "linear_nsmall_bwd" in names

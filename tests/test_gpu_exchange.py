"""GPU checks of the gradient exchange's direct-write path (parallel.GradExchange, direct_write):
the fused layers write their FP6 weight gradients straight into the flat bucket views instead of
returning a tensor for AccumulateGrad to add.  A one-rank gloo group on the GPU process (the
collective itself is skipped at world size 1; tests/test_parallel_gloo.py covers the N = 2
exchange against torch DDP on CPU).

* gradients (every parameter) equal those of the plain step without an exchange, bit for bit;
* the weights written directly are views of the flat buffer, and every bucket was released;
* the direct-write path actually ran (the fused layers' sinks were armed and taken).
"""
import os

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def group():
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29561")
    if not dist.is_initialized():
        dist.init_process_group("gloo", rank=0, world_size=1)
    yield
    dist.destroy_process_group()


def _run(widths, M, mode):
    from bnn_amd import nets
    from bnn_amd.parallel import GradExchange
    torch.manual_seed(0)
    m = nets.MLP(*widths, org_protocol=False, mutate_input=False, fused_bn=True).cuda().train()
    g = torch.Generator(device="cuda").manual_seed(5)
    u = torch.randint(0, 256, (M, 1, 28, 28), generator=g, device="cuda").to(torch.uint8)
    y = torch.randint(0, 10, (M,), generator=g, device="cuda")
    ex = None
    if mode != "none":
        ex = GradExchange(m, bucket_mb=1, direct_write=(mode == "direct"))
        ex.zero_grad()
    torch.manual_seed(1)
    torch.nn.CrossEntropyLoss()(m(u), y).backward()
    written = None
    if ex is not None:
        written = ex.direct_writes
        ex.finish()
        assert all(b.pending <= 0 for b in ex.buckets)
        for flat, plist, _ in ex._flats:
            for p in plist:
                assert ex._is_view(p, flat)
    grads = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
    if ex is not None:
        ex.remove()
    return grads, written


def test_direct_write_equals_accumulate(group):
    widths, M = (1024, 1024, 512), 1024
    ref, _ = _run(widths, M, "none")
    acc, _ = _run(widths, M, "accumulate")
    dw, written = _run(widths, M, "direct")
    for k in ref:
        assert torch.equal(ref[k], acc[k]), k
        assert torch.equal(ref[k], dw[k]), k
    # fc2 and fc3 (the FP6 weight-gradient GEMMs) took the sink; nothing did without direct_write
    assert written == 2
    assert _run(widths, M, "accumulate")[1] == 0

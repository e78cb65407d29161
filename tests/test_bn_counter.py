"""functional.bn_counter_batch: the fused BatchNorm ops' num_batches_tracked += 1 (torch's
_BatchNorm.forward bookkeeping) deferred to one multi-tensor launch at the end of the nets' forward
(CPU: host-side logic only, no kernels)."""
import torch


def _bn(momentum=0.1):
    bn = torch.nn.BatchNorm1d(8, momentum=momentum)
    bn.train()
    return bn


def test_counters_deferred_inside_and_immediate_outside():
    from bnn_amd import functional as BF
    a, b = _bn(), _bn()
    BF._bn_module_args(a)
    assert int(a.num_batches_tracked) == 1            # no batch open: at once
    with BF.bn_counter_batch():
        BF._bn_module_args(a)
        BF._bn_module_args(b)
        assert int(a.num_batches_tracked) == 1 and int(b.num_batches_tracked) == 0
    assert int(a.num_batches_tracked) == 2 and int(b.num_batches_tracked) == 1


def test_cumulative_average_module_increments_at_once():
    from bnn_amd import functional as BF
    c = _bn(momentum=None)
    with BF.bn_counter_batch():
        _, _, _, factor = BF._bn_module_args(c)
        assert int(c.num_batches_tracked) == 1 and factor == 1.0
        _, _, _, factor = BF._bn_module_args(c)
        assert int(c.num_batches_tracked) == 2 and factor == 0.5


def test_nested_batches_and_eval_modules():
    from bnn_amd import functional as BF
    a, e = _bn(), _bn()
    e.eval()
    with BF.bn_counter_batch():
        with BF.bn_counter_batch():
            BF._bn_module_args(a)
        assert int(a.num_batches_tracked) == 1           # the inner batch flushed its own
        BF._bn_module_args(e)                              # eval: never counted
    assert int(e.num_batches_tracked) == 0

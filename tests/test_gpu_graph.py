"""HIP-graph training steps (bnn_amd.graph.GraphedStep + functional.DeviceStep).

* Adam with its bias corrections read from the device table (bnn_adam_*_sched) equals the
  per-launch form bit for bit (the table is the same host arithmetic);
* a captured step replayed n times equals n eager device-step steps bit for bit -- parameters,
  Adam moments, BatchNorm running statistics and the loss -- dropout included (the device counter
  gives every replay its own mask, the same one the eager step draws);
* distinct replays are distinct steps (the weights move, dropout masks differ).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def F():
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    from bnn_amd import functional
    return functional


def _model(seed, widths=(256, 128, 64), p_drop=0.3):
    from bnn_amd import nets
    torch.manual_seed(seed)
    return nets.MLP(*widths, p_drop=p_drop, org_protocol=False, mutate_input=False, fused_bn=True).cuda().train()


def _batch(M=256, seed=3):
    g = torch.Generator(device="cuda").manual_seed(seed)
    u = torch.randint(0, 256, (M, 1, 28, 28), generator=g, device="cuda").to(torch.uint8)
    y = torch.randint(0, 10, (M,), generator=g, device="cuda")
    return u, y


def _state(m, opt):
    out = {k: v.detach().cpu().numpy().copy() for k, v in m.state_dict().items()}
    for i, p in enumerate(m.parameters()):
        st = opt.state.get(p, {})
        for k in ("exp_avg", "exp_avg_sq"):
            if k in st:
                out[f"opt{i}.{k}"] = st[k].cpu().numpy().copy()
    return out


def _step_fn(m, opt, u, y):
    crit = torch.nn.CrossEntropyLoss()

    def step():
        for p in m.parameters():
            p.grad = None
        loss = crit(m(u), y)
        loss.backward()
        opt.step()
        return loss
    return step


def test_device_step_adam_equals_per_launch(F):
    from bnn_amd.nets import binary_params
    from bnn_amd.optim import LatentAdam
    u, y = _batch()
    states = []
    for dev_step in (False, True):
        m = _model(11, p_drop=0.0)
        ds = F.DeviceStep().activate() if dev_step else None
        try:
            opt = LatentAdam(m.parameters(), lr=0.01, clamp_params=binary_params(m), device_step=ds)
            step = _step_fn(m, opt, u, y)
            for _ in range(4):
                step()
            torch.cuda.synchronize()
            states.append(_state(m, opt))
        finally:
            if ds is not None:
                ds.deactivate()
    a, b = states
    for k in a:
        assert np.array_equal(a[k], b[k]), k


def test_device_step_eager_with_missing_gradients(F):
    """An eager device-step LatentAdam step where a parameter got no gradient (a frozen fc4 bias)
    takes the per-launch bias corrections for its group instead of raising (only a captured step
    needs one schedule per group): equal to LatentAdam without a device step, bit for bit."""
    from bnn_amd.nets import binary_params
    from bnn_amd.optim import LatentAdam
    u, y = _batch()
    states = []
    for dev_step in (False, True):
        m = _model(12, p_drop=0.0)
        m.fc4.bias.requires_grad_(False)
        ds = F.DeviceStep().activate() if dev_step else None
        try:
            opt = LatentAdam(m.parameters(), lr=0.01, clamp_params=binary_params(m), device_step=ds)
            step = _step_fn(m, opt, u, y)
            for _ in range(3):
                step()
            torch.cuda.synchronize()
            states.append(_state(m, opt))
        finally:
            if ds is not None:
                ds.deactivate()
    a, b = states
    for k in a:
        assert np.array_equal(a[k], b[k]), k


@pytest.mark.parametrize("widths,M", [((256, 128, 64), 256), ((192, 192, 192), 64)])
def test_graph_replays_equal_eager_device_steps(F, widths, M):
    from bnn_amd.graph import GraphedStep
    from bnn_amd.nets import binary_params
    from bnn_amd.optim import LatentAdam
    u, y = _batch(M)
    runs = []
    for graphed in (False, True):
        m = _model(5, widths)
        torch.manual_seed(99)                       # the DeviceStep's base dropout seed
        ds = F.DeviceStep().activate()
        try:
            opt = LatentAdam(m.parameters(), lr=0.01, clamp_params=binary_params(m), device_step=ds)
            step = _step_fn(m, opt, u, y)
            losses = []
            if graphed:
                g = GraphedStep(step, opt, ds, warmup=2)       # 2 eager steps + capture
                for _ in range(3):
                    losses.append(float(g().item()))
            else:
                for i in range(5):
                    loss = step()
                    if i >= 2:
                        losses.append(float(loss.item()))
            torch.cuda.synchronize()
            assert ds.steps == 5 and int(ds.ctr.item()) == 5
            runs.append((_state(m, opt), losses))
        finally:
            ds.deactivate()
    (a, la), (b, lb) = runs
    assert la == lb
    for k in a:
        assert np.array_equal(a[k], b[k]), k


def test_replays_are_distinct_steps(F):
    from bnn_amd.graph import GraphedStep
    from bnn_amd.nets import binary_params
    from bnn_amd.optim import LatentAdam
    u, y = _batch()
    m = _model(7)
    ds = F.DeviceStep().activate()
    try:
        opt = LatentAdam(m.parameters(), lr=0.01, clamp_params=binary_params(m), device_step=ds)
        g = GraphedStep(_step_fn(m, opt, u, y), opt, ds, warmup=1)
        w0 = m.fc2.weight.detach().clone()
        l1 = float(g().item())
        w1 = m.fc2.weight.detach().clone()
        l2 = float(g().item())
        assert not torch.equal(w0, w1) and not torch.equal(w1, m.fc2.weight)
        assert l1 != l2
        assert int(m.bn1.num_batches_tracked.item()) == 3       # warm-up + 2 replays
    finally:
        ds.deactivate()


def test_trainer_graph_mode(F):
    """bnn_amd.trainer --graph: full batches replay one captured step, the short last batch runs
    eagerly; every batch is one optimizer step and the device counter tracks them."""
    from bnn_amd import trainer
    args = trainer.parse(["--model", "small", "--epochs", "2", "--dataset-size", "600", "--batch-size", "128",
                          "--log-interval", "2", "--graph"])
    m = trainer.train(0, args)
    assert F._DEVICE_STEP is None                       # the trainer releases the seed counter
    nb = -(-600 // 128)
    for p in m.parameters():
        assert torch.isfinite(p).all()
    assert int(m.bn1.num_batches_tracked.item()) == 2 * nb


def test_trainer_graph_quirk_and_recapture(F):
    """An lr-quirk epoch (mnist-dist2.py:126-127: lr *= 0.1 on every batch) in --graph mode runs
    eagerly with per-launch Adam bias corrections (no device table rebuilt per batch), then the
    next epoch recaptures at the new lr.  The whole run equals its eager twin (--device-step: same
    device-counter dropout seeds, no graphs) bit for bit."""
    from bnn_amd import trainer
    base = ["--model", "small", "--epochs", "3", "--dataset-size", "640", "--batch-size", "128",
            "--log-interval", "100", "--lr-quirk-period", "2"]
    states = []
    for mode in ("--graph", "--device-step"):
        torch.manual_seed(0)
        m = trainer.train(0, trainer.parse(base + [mode]))
        torch.cuda.synchronize()
        states.append({k: v.detach().cpu().numpy().copy() for k, v in m.state_dict().items()})
    assert F._DEVICE_STEP is None
    a, b = states
    for k in a:
        assert np.array_equal(a[k], b[k]), k


def test_graph_replay_past_schedule_raises(F):
    """Replays that would index past the device Adam table raise instead of reading beyond it."""
    from bnn_amd.graph import GraphedStep
    from bnn_amd.nets import binary_params
    from bnn_amd.optim import LatentAdam
    u, y = _batch()
    m = _model(3, p_drop=0.0)
    ds = F.DeviceStep().activate()
    try:
        opt = LatentAdam(m.parameters(), lr=0.01, clamp_params=binary_params(m), device_step=ds)
        opt.SCHEDULE_STEPS = 4                  # a short table: built for counter values 0 .. 4
        g = GraphedStep(_step_fn(m, opt, u, y), opt, ds, warmup=1)
        g(3)
        with pytest.raises(RuntimeError, match="past the Adam schedule"):
            g(2)
    finally:
        ds.deactivate()


def test_graph_captures_totensor_recognition_with_guard(F):
    """fp32 ToTensor images (mnist-dist2.py:96-99, the GPU's fl(u * fl(1 / 255))) at fc1: the
    warm-up recognises them, the capture replays the recognition (nn.BinarizeLinear's guard), so
    the replays equal the eager device-step steps bit for bit -- the graph does not fall back to the
    fp32-digit GEMMs the eager steps skipped.  A replay over inputs that are not ToTensor images then
    makes the next call (and check()) raise."""
    from bnn_amd.graph import GraphedStep
    from bnn_amd.nets import binary_params
    from bnn_amd.optim import LatentAdam
    u, y = _batch(256)
    x = u.float() / 255.0
    runs = []
    for graphed in (False, True):
        m = _model(5)
        torch.manual_seed(99)
        ds = F.DeviceStep().activate()
        try:
            opt = LatentAdam(m.parameters(), lr=0.01, clamp_params=binary_params(m), device_step=ds)
            xs = x.clone()
            step = _step_fn(m, opt, xs, y)
            losses = []
            if graphed:
                n0 = F.UNIT_PIXELS
                g = GraphedStep(step, opt, ds, warmup=2)
                assert F.UNIT_PIXELS == n0 + 3 and len(g.guards) == 1      # 2 warm-up + the capture
                for _ in range(3):
                    losses.append(float(g().item()))
                g.check()
                runs.append((_state(m, opt), losses))
                xs.mul_(1.0001)                                           # no longer fl(u / 255)
                g()
                with pytest.raises(RuntimeError, match="not ToTensor images"):
                    g()
                with pytest.raises(RuntimeError, match="not ToTensor images"):
                    g.check()
            else:
                for i in range(5):
                    loss = step()
                    if i >= 2:
                        losses.append(float(loss.item()))
                runs.append((_state(m, opt), losses))
            torch.cuda.synchronize()
        finally:
            ds.deactivate()
    (a, la), (b, lb) = runs
    assert la == lb
    for k in a:
        assert np.array_equal(a[k], b[k]), k

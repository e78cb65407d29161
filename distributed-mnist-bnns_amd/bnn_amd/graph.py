"""One training step captured as a HIP graph (torch.cuda.CUDAGraph on ROCm) and replayed.

The reference's loop (mnist-dist2.py:118-137) launches every op of every step from Python; at
the published configuration (mnist-dist3.py: 784-192x3-10, batch 64) the GPU work per step is a
few hundred microseconds, so launch overhead is most of the step.  ``GraphedStep`` captures the
whole step -- forward, loss, backward, the fused latent update -- once and replays it:

* inputs are static tensors (copy the next batch into them before each replay);
* the quantities the host would pass per step by value -- Adam's bias corrections and the dropout
  seed -- come from a ``functional.DeviceStep`` counter that the captured optimizer advances on
  the device (bnn_adam_*_sched, bnn_set_seed_counter), so every replay is a distinct step and
  the sequence equals the same number of eager device-step steps bit for bit;
* data parallel: a step that runs a ``parallel.GradExchange`` is captured with its collectives --
  the per-forward buffer broadcast and every bucket all-reduce, issued from the backward hooks on
  RCCL's stream as in the eager step (torch joins that stream into the capture) -- so a replay
  issues the same collectives in the same order, overlapped with the backward kernels as before
  (tests/test_gpu_rccl.py::test_rccl_exchange_captured_in_graph: replays equal eager steps bit for
  bit on a one-rank RCCL group).  Every rank captures and replays the same step.
"""
import time

import torch
import torch.distributed as dist

from . import _lib as L
from . import functional as BF


class GraphedStep:
    def __init__(self, step_fn, optimizer, device_step, warmup=2):
        if device_step is None or not device_step.active:
            raise ValueError("GraphedStep: needs an active functional.DeviceStep")
        if getattr(optimizer, "device_step", None) is not device_step:
            raise ValueError("GraphedStep: the optimizer must run on the same DeviceStep")
        self.opt, self.ds = optimizer, device_step
        # eager warm-up on a side stream (torch's capture recipe): builds the packed-weight caches,
        # constant vectors and the Adam schedule outside the capture
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(max(1, warmup)):
                step_fn()
        torch.cuda.current_stream().wait_stream(side)
        # the captured Adam reads its bias corrections from device tables built for the current lr
        if hasattr(optimizer, "build_schedules"):
            optimizer.build_schedules()
        # let RCCL's watchdog retire the warm-up's collectives (it polls every 100 ms), and capture in
        # thread-local mode so that its event queries from another thread cannot invalidate the capture
        torch.cuda.synchronize()
        if dist.is_available() and dist.is_initialized() and dist.get_backend() == "nccl":
            time.sleep(0.25)
        self.graph = torch.cuda.CUDAGraph()
        BF.CAPTURE_GUARDS.clear()
        with torch.cuda.graph(self.graph, capture_error_mode="thread_local"):
            self.out = step_fn()
        # sticky mismatch flags of the fp32-image recognitions the step captured (nn.BinarizeLinear)
        self.guards = list(BF.CAPTURE_GUARDS)
        BF.CAPTURE_GUARDS.clear()
        # the capture ran the host side of one step without executing it on the device
        self._shadow(-1)

    def _shadow(self, n):
        self.ds.note_replays(n)
        for group in self.opt.param_groups:
            for p in group["params"]:
                st = self.opt.state.get(p)
                if st and "step" in st:
                    st["step"] += n

    def check(self):
        """Raise if a replay so far saw fp32 inputs that are not ToTensor images at a layer whose
        capture took the u8-pixel path (one host read per guard; __call__ runs it first)."""
        for g in self.guards:
            if int(g.item()) != 0:
                raise L.BnnError("GraphedStep: a replay fed fp32 inputs that are not ToTensor images "
                                  "(fl(u / 255)) to a BinarizeLinear captured on its u8-pixel path; that "
                                  "replay's step is wrong -- set detect_pixels = False on the layer (or "
                                  "feed uint8 pixels) and capture again")

    def __call__(self, n=1):
        """Replay the captured step n times; returns the step function's (static) output.  A step
        with captured pixel recognitions is checked before the replays (GraphedStep.check) --
        that waits for the previous replay; call check() after the last one."""
        if self.guards:
            self.check()
        limit = self.opt.schedule_limit() if hasattr(self.opt, "schedule_limit") else None
        if limit is not None and self.ds.steps + int(n) > limit:
            # the *_sched kernels index the table by the device counter without a bound
            raise RuntimeError(f"GraphedStep: {n} replays would run past the Adam schedule "
                               f"({self.ds.steps} of {limit} steps used); recapture to rebuild it")
        for _ in range(n):
            self.graph.replay()
        self._shadow(n)
        return self.out


__all__ = ["GraphedStep"]

"""Latent-weight update.

The reference's protocol around ``torch.optim.Adam`` (mnist-dist2.py:91, :131-137)::

    for p in model.parameters():            # restore the latent weight
        if hasattr(p, 'org'): p.data.copy_(p.org)
    optimizer.step()
    for p in model.parameters():            # clamp it and keep it as the new latent
        if hasattr(p, 'org'): p.org.copy_(p.data.clamp_(-1, 1))

``org_protocol_step`` is that loop, for models running with ``org_protocol = True``.
``LatentAdam`` is the fused form for models whose Parameters hold the latent weights directly
(``org_protocol = False``): one libbnn kernel per tensor does Adam (torch's formula) and the clamp
of the parameters the reference clamps, with an optional gradient scale (1/world_size when the
gradient exchange summed instead of averaged).  For a binarized layer's weight the same kernel
also rewrites the next forward's packed ternary operands (bnn_adam_clamp_pack), replacing the
per-forward sign-pack of the weight.

With ``device_step`` (a ``functional.DeviceStep``) the step is graph-capturable: the bias
corrections come from a device table indexed by the device step counter (bit-identical to the
per-launch values), and the counter is advanced on the device after the last update.
"""
import os

import torch

from . import functional as BF

# Side streams for the binarized weights' Adam + pack launches (bnn_adam_clamp_pack): the k-th such
# launch of a step runs on stream k mod (1 + ADAM_STREAMS), 0 = the caller's, each forked from the
# caller's stream just before its launch and joined back after the last.  Every launch touches only
# its own tensors, so the results are bit-identical.  Measured, off by default (0 = one stream): at
# 2 the captured graphs' parallel branches made config 3's step 0.76-0.81 ms against 0.69 and the
# 192-wide net's 0.42 against 0.25; the wide step did not move (profiles/r06_af_adam_streams_ab.txt).
ADAM_STREAMS = int(os.environ.get("BNN_ADAM_STREAMS", "0"))


def org_protocol_step(model, optimizer):
    """mnist-dist2.py:131-137 verbatim in behaviour."""
    params = list(model.parameters())
    for p in params:
        if hasattr(p, "org"):
            p.data.copy_(p.org)
    optimizer.step()
    for p in params:
        if hasattr(p, "org"):
            p.org.copy_(p.data.clamp_(-1, 1))


class LatentAdam(torch.optim.Optimizer):
    """Adam (torch defaults) fused with clamp(-1, 1) for the parameters in ``clamp_params``."""

    SCHEDULE_STEPS = 1 << 20      # device-step table length (8 MiB per parameter group)

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, clamp_params=(),
                 grad_scale=1.0, device_step=None):
        defaults = dict(lr=lr, betas=betas, eps=eps)
        super().__init__(params, defaults)
        self._clamp = {id(p) for p in clamp_params}
        self.grad_scale = grad_scale
        self.device_step = device_step
        self._sched = {}              # group index -> (device table, (lr, betas) it was built for)
        self._sides = {}              # device -> side streams (ADAM_STREAMS)

    def _side_streams(self, device):
        ss = self._sides.get(device)
        if ss is None:
            ss = [torch.cuda.Stream(device=device) for _ in range(ADAM_STREAMS)]
            self._sides[device] = ss
        return ss

    def _schedule(self, gi, group, step, device, build):
        """Device table for this group covering the device counter's steps: entry c holds the bias
        corrections of Adam step (step at table build) + c - (counter at build).  ``build``: make
        one if the cached table is missing or was built for another lr / betas; else None."""
        ds = self.device_step
        key = (group["lr"], tuple(group["betas"]))
        ent = self._sched.get(gi)
        if ent is None or ent[1] != key:
            if not build:
                return None
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("LatentAdam: build the device schedule (build_schedules) before capturing")
            first = step - ds.steps
            if first < 1:
                raise RuntimeError("LatentAdam: device step counter ahead of the optimizer's steps")
            tab = BF.adam_schedule(group["lr"], *group["betas"], first, ds.steps + self.SCHEDULE_STEPS, device)
            ent = (tab, key)
            self._sched[gi] = ent
        if ds.steps >= ent[0].shape[0]:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("LatentAdam: device-step schedule exhausted")
            return None             # eager: per-launch bias corrections
        return ent[0]

    def build_schedules(self):
        """(Re)build every group's device table for its current lr / betas, between steps -- before
        a HIP-graph capture (graph.GraphedStep calls it)."""
        ds = self.device_step
        if ds is None:
            return
        for gi, group in enumerate(self.param_groups):
            steps = {self.state[p]["step"] for p in group["params"] if self.state.get(p)}
            if not steps:
                continue
            if len(steps) != 1:
                raise RuntimeError("LatentAdam: device_step needs every parameter of a group stepped together")
            self._sched.pop(gi, None)
            self._schedule(gi, group, steps.pop() + 1, group["params"][0].device, build=True)

    def schedule_limit(self):
        """Device counter value at which the first device table runs out (None: no table)."""
        lens = [ent[0].shape[0] for ent in self._sched.values()]
        return min(lens) if lens else None

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        ds = self.device_step
        capturing = ds is not None and torch.cuda.is_current_stream_capturing()
        npack = 0
        joined = {}                   # id(side stream) -> stream to join back into the caller's
        for gi, group in enumerate(self.param_groups):
            b1, b2 = group["betas"]
            sched = None
            small = []                # plain Adam + clamp tensors: one multi-tensor launch per 16
            live = [p for p in group["params"] if p.grad is not None]
            steps = {self.state[p]["step"] if self.state.get(p) else 0 for p in live}
            uniform = len(steps) == 1 and len(live) == len(group["params"])
            if ds is not None and live and not uniform and capturing:
                # one table per group is indexed by the shared device counter
                raise RuntimeError("LatentAdam: a captured device step needs every parameter of a group to "
                                   "get a gradient on every step")
            if ds is not None and live and uniform:
                # the table of this lr: built on the group's first step (or by build_schedules before
                # a capture); an eager step at another lr (the trainer's lr-quirk epochs) -- or an
                # eager step where some parameter got no gradient -- uses the per-launch bias
                # corrections (bit-identical) instead of a table
                sched = self._schedule(gi, group, steps.pop() + 1, live[0].device,
                                       build=gi not in self._sched)
                if sched is None and capturing:
                    raise RuntimeError("LatentAdam: no device schedule for this lr (build_schedules before capturing)")
            for p in live:
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                st["step"] += 1
                g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
                args = (g, st["exp_avg"], st["exp_avg_sq"], st["step"], group["lr"], b1, b2, group["eps"],
                        self.grad_scale, id(p) in self._clamp)
                kw = dict(sched=sched, ctr=ds.ctr) if sched is not None else {}
                # a binarized layer's weight also gets its next-forward ternary operands rewritten in
                # the same pass (bnn_adam_clamp_pack); anything else: plain fused Adam + clamp
                side = None
                if ADAM_STREAMS > 0 and p.is_cuda and p.dim() == 2 and getattr(p, "_bnn_pack", None) is not None:
                    j = npack % (ADAM_STREAMS + 1)
                    npack += 1
                    if j > 0:
                        side = self._side_streams(p.device)[j - 1]
                if side is None:
                    done = BF.adam_clamp_pack_(p, *args, **kw)
                else:
                    main = torch.cuda.current_stream(p.device)
                    side.wait_stream(main)       # the gradient, the state and the counter are ready
                    with torch.cuda.stream(side):
                        done = BF.adam_clamp_pack_(p, *args, **kw)
                    if done:
                        joined[id(side)] = (side, main)
                        if g is not p.grad:
                            g.record_stream(side)
                if not done:
                    small.append((p, g, st["exp_avg"], st["exp_avg_sq"], st["step"], id(p) in self._clamp))
            if small:
                BF.adam_clamp_multi_(small, group["lr"], b1, b2, group["eps"], self.grad_scale,
                                     sched=sched, ctr=ds.ctr if sched is not None else None)
        for side, main in joined.values():
            main.wait_stream(side)
        if ds is not None:
            ds.advance()
        return loss

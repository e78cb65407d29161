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
"""
import torch

from . import functional as BF


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

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, clamp_params=(),
                 grad_scale=1.0):
        defaults = dict(lr=lr, betas=betas, eps=eps)
        super().__init__(params, defaults)
        self._clamp = {id(p) for p in clamp_params}
        self.grad_scale = grad_scale

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        for group in self.param_groups:
            b1, b2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                st["step"] += 1
                g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
                args = (g, st["exp_avg"], st["exp_avg_sq"], st["step"], group["lr"], b1, b2, group["eps"],
                        self.grad_scale, id(p) in self._clamp)
                # a binarized layer's weight also gets its next-forward ternary operands rewritten in
                # the same pass (bnn_adam_clamp_pack); anything else: plain fused Adam + clamp
                if not BF.adam_clamp_pack_(p, *args):
                    BF.adam_clamp_(p, *args)
        return loss

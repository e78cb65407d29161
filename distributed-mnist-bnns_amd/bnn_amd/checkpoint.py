"""Checkpoints that keep what binarized training needs to resume.

The reference saves ``ddp_model.state_dict()`` from rank 0, barriers, and loads it on every rank
with a ``map_location`` (mnist-distributed-BNNS2.py:152-191, ``demo_checkpoint``).  For a BNN
that state_dict is lossy: after a forward, ``weight.data`` holds ``sign(weight.org)`` and the
latent weight the optimizer updates lives only in the ``.org`` attribute, which ``state_dict``
never sees (binarized_modules.py:77-79).  A resumed run would restart from the binarised
weights.  This format stores:

* ``model``: the state_dict with every binarized layer's weight replaced by its latent
  ``.org`` when one exists (so ``weight`` is always the latent value, whichever protocol the
  layer runs), BatchNorm running stats and ``num_batches_tracked`` included;
* ``latent``: the names of the weights that came from ``.org``;
* ``optimizer``: the optimizer's state_dict (Adam moments and step counts);
* ``epoch`` and an optional ``extra`` dict.

Files are written with ``torch.save`` and read with ``torch.load(weights_only=True)``: tensors,
dicts, lists, numbers and strings only, nothing executable.
"""
import os

import torch
import torch.distributed as dist

from . import functional as BF
from .nn import BinarizeConv2d, BinarizeLinear

FORMAT = "bnn_amd.checkpoint/1"


def _binary_modules(model):
    for name, m in model.named_modules():
        if isinstance(m, (BinarizeLinear, BinarizeConv2d)):
            yield name, m


def state_with_latents(model):
    """``model.state_dict()`` with each binarized weight replaced by its latent ``.org``."""
    sd = {k: v.detach().clone() for k, v in model.state_dict().items()}
    latent = []
    for name, m in _binary_modules(model):
        org = getattr(m.weight, "org", None)
        if org is not None:
            key = f"{name}.weight" if name else "weight"
            sd[key] = org.detach().clone()
            latent.append(key)
    return sd, latent


def save_checkpoint(path, model, optimizer=None, epoch=0, extra=None):
    """Write a checkpoint from rank 0 (every rank holds the same replica after the gradient
    all-reduce), then barrier so no rank reads a half-written file -- the reference's
    ``demo_checkpoint`` order."""
    rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
    if rank == 0:
        sd, latent = state_with_latents(model)
        blob = {"format": FORMAT, "model": sd, "latent": latent, "epoch": int(epoch),
                "optimizer": optimizer.state_dict() if optimizer is not None else None,
                "extra": extra or {}}
        tmp = f"{path}.tmp"
        torch.save(blob, tmp)
        os.replace(tmp, path)      # atomic: a crash never leaves a truncated checkpoint
    if dist.is_available() and dist.is_initialized():
        dist.barrier()


def load_checkpoint(path, model, optimizer=None, map_location=None):
    """Restore a checkpoint written by ``save_checkpoint``.  Binarized layers running the
    reference's ``.org`` protocol get ``weight.org`` = the latent weight and ``weight.data`` =
    its sign (the state their next forward would produce); layers holding the latent weight
    in the Parameter get it directly.  Returns the stored epoch."""
    if map_location is None:
        p = next(model.parameters(), None)
        map_location = p.device if p is not None else "cpu"
    blob = torch.load(path, map_location=map_location, weights_only=True)
    if blob.get("format") != FORMAT:
        raise ValueError(f"{path}: not a {FORMAT} checkpoint (format={blob.get('format')!r})")
    model.load_state_dict(blob["model"])
    for prm in model.parameters():
        BF.invalidate_packed(prm)
    latent = set(blob["latent"])
    for name, m in _binary_modules(model):
        key = f"{name}.weight" if name else "weight"
        if m.org_protocol and key in latent:
            m.weight.org = m.weight.data.clone()
            m.weight.data = m.weight.org.sign()
    if optimizer is not None and blob.get("optimizer") is not None:
        optimizer.load_state_dict(blob["optimizer"])
    return blob["epoch"]

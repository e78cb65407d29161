"""Input side of the reference trainers, kept on the device.

* ``synthetic_mnist`` -- MNIST-shaped batches: 80.7 % exact-zero pixels (the t10k
  zero fraction), the rest u8/255, labels uniform 0-9; generated on the GPU from a seeded
  generator, so the timed step reads inputs already resident in HBM.
* ``shard_indices`` -- the ``DistributedSampler`` order the trainers rely on
  (mnist-dist2.py:100-102): randperm(seed + epoch), padded to a multiple of the world size by
  repeating its head, then ``indices[rank::world]``.  The reference never calls ``set_epoch`` so
  every epoch repeats epoch 0's order; ``epoch`` defaults to 0 accordingly.
* ``read_idx`` -- an idx-ubyte reader (the torchvision MNIST files' format) for real data when
  present; nothing is downloaded.
"""
import gzip
import struct

import numpy as np
import torch

ZERO_FRACTION = 0.807


def synthetic_mnist(n, seed=1234, device="cuda", normalize=None):
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    u = torch.rand((n, 1, 28, 28), generator=g, device=device)
    v = torch.randint(1, 256, (n, 1, 28, 28), generator=g, device=device).float()
    x = torch.where(u < ZERO_FRACTION, torch.zeros_like(v), v) / 255.0
    if normalize is not None:      # mnist-distributed-BNNS2.py:82 Normalize((0.1307,), (0.3081,))
        mean, std = normalize
        x = (x - mean) / std
    y = torch.randint(0, 10, (n,), generator=g, device=device)
    return x, y


def shard_indices(n, world, rank, seed=0, epoch=0, drop_last=False):
    g = torch.Generator()
    g.manual_seed(seed + epoch)
    idx = torch.randperm(n, generator=g).tolist()
    if drop_last:
        total = (n // world) * world
        idx = idx[:total]
    else:
        total = -(-n // world) * world
        pad = total - n
        while pad > 0:
            take = idx[:min(pad, len(idx))]
            idx = idx + take
            pad -= len(take)
    return idx[rank:total:world]


def read_idx(path):
    """Read an idx-ubyte file (optionally .gz) into a numpy array."""
    opener = gzip.open if path.endswith(".gz") else open
    with opener(path, "rb") as f:
        magic = f.read(4)
        ndim = magic[3]
        dims = struct.unpack(">" + "I" * ndim, f.read(4 * ndim))
        data = np.frombuffer(f.read(), dtype=np.uint8)
    return data.reshape(dims)

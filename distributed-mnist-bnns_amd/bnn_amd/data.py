"""Input side of the reference trainers, kept on the device.

* ``synthetic_mnist`` -- MNIST-shaped batches: 80.7 % exact-zero pixels (the t10k
  zero fraction), the rest u8/255, labels uniform 0-9; generated on the GPU from a seeded
  generator, so the timed step reads inputs already resident in HBM.  ``as_u8=True`` returns the
  bytes themselves (the same draw): the nets' fc1 consumes them directly (f3), so
  a resident dataset costs 784 B per image instead of 3136 and no fp32 image is ever built.
* ``load_idx_dataset`` -- idx files -> (u8 images [N,1,28,28], int64 labels), on the device.
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


def synthetic_mnist(n, seed=1234, device="cuda", normalize=None, as_u8=False):
    if as_u8 and normalize is not None:
        raise ValueError("synthetic_mnist: u8 pixels carry no Normalize; pass normalize=(mean, std) to the "
                         "model instead (nets.MLP(normalize=...) -> fc1.pixel_normalize)")
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    u = torch.rand((n, 1, 28, 28), generator=g, device=device)
    v = torch.randint(1, 256, (n, 1, 28, 28), generator=g, device=device)
    pix = torch.where(u < ZERO_FRACTION, torch.zeros_like(v), v)
    if as_u8:                      # normalize then belongs to the model (MLP(normalize=...))
        y = torch.randint(0, 10, (n,), generator=g, device=device)
        return pix.to(torch.uint8), y
    x = pix.float() / 255.0
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
        if len(magic) != 4 or magic[0] != 0 or magic[1] != 0 or magic[2] != 0x08:
            raise ValueError(f"read_idx: {path} is not an unsigned-byte idx file (magic {magic!r})")
        ndim = magic[3]
        dims = struct.unpack(">" + "I" * ndim, f.read(4 * ndim))
        data = np.frombuffer(f.read(), dtype=np.uint8)
    if data.size != int(np.prod(dims, dtype=np.int64)):
        raise ValueError(f"read_idx: {path} holds {data.size} bytes for dims {dims}")
    return data.reshape(dims)


def load_idx_dataset(images, labels, device="cuda"):
    """(u8 images [N, 1, 28, 28], int64 labels [N]) from idx(-ubyte)(.gz) files, on ``device``."""
    imgs = read_idx(images)
    lab = read_idx(labels)
    if imgs.ndim != 3 or lab.ndim != 1 or imgs.shape[0] != lab.shape[0]:
        raise ValueError(f"load_idx_dataset: images {imgs.shape} / labels {lab.shape} do not pair")
    x = torch.from_numpy(imgs.copy()).unsqueeze(1).to(device)
    y = torch.from_numpy(lab.astype(np.int64)).to(device)
    return x, y

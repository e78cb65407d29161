"""Input pipeline (f3): the idx reader against the MNIST files the reference ships
(data/MNIST/raw/, copied as fixtures: data, not source), the u8 synthetic set against its fp32
form, and the pixel affine map fc1 folds into its integer sums (bnn_pixels.hip)."""
import hashlib
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import bnn_np as O

LABELS = os.path.join(GOLDEN, "t10k-labels-idx1-ubyte.gz")
IMAGES = os.path.join(GOLDEN, "t10k-images-idx3-ubyte.gz")
# class counts of the MNIST test set (the published ones) and checksums of the decoded arrays
T10K_COUNTS = [980, 1135, 1032, 1010, 982, 892, 958, 1028, 974, 1009]
T10K_LABELS_SHA256 = "ddeff807876a9661a1110d45c266c86239a3a1b7d37da0c3716a7a683c852ff5"
T10K_IMAGES_SHA256 = "6d87418db22cc8025d05968bec9bd5c3932904b23485740db143a061a2c9d161"


def test_read_idx_labels():
    from bnn_amd.data import read_idx
    lab = read_idx(LABELS)
    assert lab.shape == (10000,) and lab.dtype == np.uint8
    assert np.bincount(lab).tolist() == T10K_COUNTS
    assert hashlib.sha256(lab.tobytes()).hexdigest() == T10K_LABELS_SHA256


def test_read_idx_images_and_zero_fraction():
    from bnn_amd.data import ZERO_FRACTION, read_idx
    img = read_idx(IMAGES)
    assert img.shape == (10000, 28, 28) and img.dtype == np.uint8
    assert hashlib.sha256(img.tobytes()).hexdigest() == T10K_IMAGES_SHA256
    assert abs((img == 0).mean() - ZERO_FRACTION) < 1e-3      # the synthetic set's zero fraction
    assert int((img.reshape(10000, -1).max(0) == 0).sum()) == 116   # pixels never lit in t10k


def test_read_idx_rejects_nothing_silently(tmp_path):
    from bnn_amd.data import read_idx
    p = tmp_path / "bad-idx1-ubyte"
    p.write_bytes(bytes([0, 0, 8, 1]) + (5).to_bytes(4, "big") + bytes(3))   # 5 announced, 3 present
    with pytest.raises(ValueError):
        read_idx(str(p))


def test_load_idx_dataset_cpu():
    from bnn_amd.data import load_idx_dataset
    x, y = load_idx_dataset(IMAGES, LABELS, device="cpu")
    assert x.shape == (10000, 1, 28, 28) and x.dtype == torch.uint8
    assert y.dtype == torch.int64 and np.bincount(y.numpy()).tolist() == T10K_COUNTS


def test_synthetic_u8_is_the_fp32_draw():
    from bnn_amd.data import synthetic_mnist
    xf, yf = synthetic_mnist(257, seed=7, device="cpu")
    xu, yu = synthetic_mnist(257, seed=7, device="cpu", as_u8=True)
    assert xu.dtype == torch.uint8 and torch.equal(yf, yu)
    assert np.array_equal(O.to_tensor(xu.numpy()), xf.numpy())       # ToTensor of the bytes, bitwise


@pytest.mark.parametrize("normalize", [None, (0.1307, 0.3081)])
def test_pixel_affine_is_the_transform(normalize):
    """x = a * (v + s0) with v = u - 128 reproduces ToTensor (+ Normalize) to float64 rounding;
    for ToTensor s0 = 128 exactly, so v + s0 is the byte itself."""
    from bnn_amd.functional import pixel_affine
    a, s0 = pixel_affine(normalize)
    u = np.arange(256, dtype=np.float64)
    x = a * ((u - 128.0) + s0)
    ref = u / 255.0 if normalize is None else (u / 255.0 - normalize[0]) / normalize[1]
    assert np.max(np.abs(x - ref)) < 1e-14
    if normalize is None:
        assert s0 == 128.0
    # and the fp32 transform the reference applies is within fp32 rounding of it
    assert np.max(np.abs(O.to_tensor(np.arange(256, dtype=np.uint8), normalize) - ref)) < 4e-7 * max(1, np.abs(ref).max())

"""Phase timing of the q6 BatchNorm-backward passes on the wide step, from a Q6_DIAG_STAMPS build
(bash tools/build_variant.sh stamps -DQ6_DIAG_STAMPS): wave 0 of each of the first 4096 workgroups
stamps s_memtime (shader clocks) at each sub-tile's start, after its dz phase + barrier, after the
previous sub-tile's record stores + barrier, and after its quantisation + barrier.

    BNN_LIB=ab/stamps/libbnn.so python tools/q6_stamps.py
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-mnist-bnns_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bnn_amd import _lib as L  # noqa: E402
from bnn_amd import nets  # noqa: E402
from bnn_amd.data import synthetic_mnist  # noqa: E402
from bnn_amd.nets import binary_params  # noqa: E402
from bnn_amd.optim import LatentAdam  # noqa: E402


def main():
    torch.manual_seed(0)
    m = nets.MODELS["wide"](org_protocol=False, mutate_input=False, fused_bn=True).cuda().train()
    opt = LatentAdam(m.parameters(), lr=0.01, clamp_params=binary_params(m))
    x, y = synthetic_mnist(65536, seed=1, device="cuda", as_u8=True)
    crit = torch.nn.CrossEntropyLoss()
    for _ in range(3):
        for p in m.parameters():
            p.grad = None
        loss = crit(m(x), y)
        loss.backward()
        opt.step()
    torch.cuda.synchronize()
    buf = np.zeros((2, 4096, 8, 4), dtype=np.uint64)
    lib = L.lib()
    lib.bnn_q6_stamps_copy.restype = ctypes.c_int
    lib.bnn_q6_stamps_copy.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    assert lib.bnn_q6_stamps_copy(buf.ctypes.data, buf.nbytes) == 0
    names = ["bn_bwd_apply_q6_k<0> (bn2)", "bn_bwd_apply_q6_k<10> (head)"]
    for k in range(2):
        st = buf[k].astype(np.int64)
        ok = (st > 0).all(axis=(1, 2))
        st = st[ok]
        if len(st) == 0:
            print(names[k], "no stamps")
            continue
        d01 = st[:, :, 1] - st[:, :, 0]
        d12 = st[:, :, 2] - st[:, :, 1]
        d23 = st[:, :, 3] - st[:, :, 2]
        d30 = st[:, 1:, 0] - st[:, :-1, 3]
        tot = st[:, -1, 3] - st[:, 0, 0]
        print(f"{names[k]}: {len(st)} workgroups, cycles per sub-tile (median / p90):")
        for lab, d in (("dz phase + barrier", d01), ("stores(prev) + barrier", d12),
                       ("loads(next) + quantise + barrier", d23), ("loop to next sub-tile", d30)):
            print(f"   {lab:34s} {np.median(d):9.0f} {np.percentile(d, 90):9.0f}")
        print(f"   {'8 sub-tiles, first to last stamp':34s} {np.median(tot):9.0f} {np.percentile(tot, 90):9.0f}")
        wg_start = st[:, 0, 0]
        print(f"   workgroup start spread (cycles): {np.percentile(wg_start - wg_start.min(), 50):.0f} median, "
              f"{wg_start.max() - wg_start.min():.0f} max")


if __name__ == "__main__":
    main()

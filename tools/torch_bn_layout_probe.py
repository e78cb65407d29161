"""How fast is torch's own BatchNorm1d (the drop-in path's largest cost: the reference's Net keeps
nn.BatchNorm1d around the binarized layers) on a [B, C] activation stored row-major (the layout a
Linear returns: torch picks its channels-last reduction kernels for stride(1) == 1) against the
same values stored column-major (a [C, B] buffer viewed as [B, C], strides (1, B))?

    python tools/torch_bn_layout_probe.py [B] [C]
"""
import sys

import torch


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    C = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
    dev = "cuda"
    torch.manual_seed(0)
    base = torch.randn(B, C, device=dev)
    g = torch.randn(B, C, device=dev)
    ref_out = ref_grad = None
    for layout in ("row-major [B][C]", "column-major [C][B] viewed as [B, C]"):
        if layout.startswith("row"):
            x0, gy = base.clone(), g.clone()
        else:
            x0, gy = base.t().contiguous().t(), g.t().contiguous().t()
        bn = torch.nn.BatchNorm1d(C).to(dev).train()
        x = x0.detach().requires_grad_(True)

        def fwd():
            return bn(x)

        def fwdbwd():
            y = bn(x)
            x.grad = None
            bn.weight.grad = bn.bias.grad = None
            y.backward(gy)

        y = fwd()
        fwdbwd()
        t_f, t_fb = timed(fwd), timed(fwdbwd)
        ht = torch.nn.Hardtanh()
        t_h = timed(lambda: ht(y))
        print(f"{layout:40s} out strides {tuple(y.stride())}: BN fwd {t_f:8.2f} ms, fwd+bwd {t_fb:8.2f} ms, "
              f"hardtanh {t_h:6.2f} ms", flush=True)
        if ref_out is None:
            ref_out, ref_grad = y.detach().clone(), x.grad.detach().clone()
        else:
            print(f"  same values as row-major: out max|d| {float((y.detach() - ref_out).abs().max()):.2e}, "
                  f"grad max|d| {float((x.grad - ref_grad).abs().max()):.2e}", flush=True)
        del x, y, x0, gy, bn
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

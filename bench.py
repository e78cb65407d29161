#!/usr/bin/env python3
"""Training-step benchmark of the binarized-network hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config wide|mlp|cnn|small] [--batch B]

N > 1 is launched by the driver as one process per GPU (torch.distributed.run, RCCL).
A "step" = one training step of the reference loop (mnist-dist2.py:118-137) on one batch of
synthetic MNIST-shaped input resident in HBM: forward through the libbnn layers (torch BatchNorm
/ Hardtanh / Dropout / LogSoftmax in between, as the reference's Net), CrossEntropy, backward
(libbnn STE GEMMs), bucketed RCCL gradient all-reduce overlapped with backward (N > 1), and the
fused latent Adam + clamp update.  Per-GPU batch is fixed (weak scaling).

Default workload = BASELINE config 5 (the one the metric's 1/2/4/8-GPU curve is quoted on):
wide binarized MLP 784-8192x3-10, batch 65536 per GPU.

Prints ONE JSON line (rank 0) with the contract fields plus ``roofline`` (dominant libbnn
kernel, HIP-event timed on its stream inside the timed region) and ``cpu_baseline`` (the
oracle's torch-CPU restatement of the reference path on this box's host cores, N=1 only).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "distributed-mnist-bnns_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

MI355X_INT8_DENSE_TOPS = 256 * 4 * 2048 * 2.4e9 / 1e12   # 32x32x32 i8 MFMA: 2048 ops/clk/SIMD
MI355X_HBM_GBS = 8000.0

CONFIGS = {
    # name: (model factory kwargs, default per-GPU batch, description)
    "wide": ("wide", 65536, "wide binarized MLP 784-8192x3-10 (BASELINE config 5)"),
    "mlp": ("mlp", 4096, "binarized MLP 784-3072-1536-768-10 (mnist-dist2 Net, BASELINE config 3)"),
    "small": ("small", 4096, "binarized MLP 784-192x3-10 (mnist-dist3 Net)"),
    "cnn": ("cnn", 4096, "binarized CNN conv5(1-16)-conv5(16-32)-fc (BASELINE config 4)"),
}
CPU_WIDTHS = {"wide": (8192, 8192, 8192), "mlp": (3072, 1536, 768), "small": (192, 192, 192), "cnn": "cnn"}
MI355X_F32_MFMA_TFLOPS = 256 * 4 * 64 * 2.4e9 / 1e12     # v_mfma_f32_16x16x4_f32: 64 FLOP/clk/SIMD
MI355X_DOT4_TOPS = 256 * 64 * 8 * 2.4e9 / 1e12           # v_dot4_i32_i8 on the VALU: 64 lanes x 8 ops /clk/CU


def op_peak(kernel):
    """(bound, peak TFLOP/s or TOPS, unit of the count) of an ops-counted kernel."""
    if kernel.startswith("conv2d_bwd"):
        return "mfma", MI355X_F32_MFMA_TFLOPS, "f32 MFMA flops (2*N*Co*OH*OW*C*KH*KW)"
    if kernel.startswith("conv2d_fwd"):   # C=1 layer on VALU dot4; C%16==0 layers on int8 MFMA (looser bound)
        return "valu", MI355X_DOT4_TOPS, "int8 dot4 / MFMA ops (2*N*Co*OH*OW*C*KH*KW)"
    return "mfma", MI355X_INT8_DENSE_TOPS, "int8 MFMA ops (2*M*N*K*digit_pairs)"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="wide", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=0, help="per-GPU batch (0 = config default)")
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--bucket-mb", type=float, default=64.0)
    ap.add_argument("--backend", default="fp4", choices=["fp4", "mfma", "xnor"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0, help="seconds of CPU baseline work")
    ap.add_argument("--no-kernel-timing", action="store_true")
    return ap.parse_args()


def build(cfg, backend):
    from bnn_amd import nets
    name = CONFIGS[cfg][0]
    if name == "cnn":
        model = nets.BinCNN(org_protocol=False, mutate_input=False, fused_bn=True)
    else:
        model = nets.MODELS[name](org_protocol=False, mutate_input=False, backend=backend, fused_bn=True)
    return model


def cpu_baseline(cfg, budget):
    sys.path.insert(0, ROOT)
    from oracle import bnn_torch
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    widths = CPU_WIDTHS.get(cfg)
    if widths is None:
        return None
    batch = 512 if cfg == "wide" else (256 if cfg == "cnn" else 1024)
    sps, steps, secs = bnn_torch.time_training(widths, batch, threads, budget_s=budget, max_steps=100000)
    return {"value": round(sps, 2), "unit": "samples/s", "cores": threads, "kind": "port",
            "sample": f"{steps} fp32 torch-CPU train steps (oracle/bnn_torch.py restatement of the "
                      f"reference path, .org protocol + Adam) of the same net at batch {batch}, "
                      f"{secs:.1f} s"}


def pmc_traffic(kernel):
    """HBM/fabric bytes per launch of ``kernel`` from the newest committed rocprofv3 PMC summary
    (profiles/*_pmc_traffic.json, written by tools/pmc_summary.py from separate FETCH_SIZE and
    WRITE_SIZE passes of this bench, gfx950-corrected).  None when no pass covers the kernel."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_traffic.json")))
    prefix = kernel.rstrip(">")
    for f in reversed(files):
        try:
            ks = json.load(open(f))["kernels"]
        except (OSError, ValueError, KeyError):
            continue
        for name, v in ks.items():
            if name == kernel or (name.startswith(prefix) and name[len(prefix):len(prefix) + 1] in (",", ">")):
                return v["traffic_bytes_per_launch"], os.path.relpath(f, ROOT)
    return None, None


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from bnn_amd import functional as BF
    from bnn_amd.data import synthetic_mnist
    from bnn_amd.nets import binary_params
    from bnn_amd.optim import LatentAdam
    from bnn_amd.parallel import GradExchange

    batch = args.batch or CONFIGS[args.config][1]
    torch.manual_seed(0)
    model = build(args.config, args.backend).to(dev).train()
    exchange = GradExchange(model, bucket_mb=args.bucket_mb) if world > 1 else None
    opt = LatentAdam(model.parameters(), lr=args.lr, clamp_params=binary_params(model))
    x, y = synthetic_mnist(batch, seed=1234 + rank, device=dev)
    crit = torch.nn.CrossEntropyLoss()

    def step():
        if exchange is not None:
            exchange.zero_grad()
        else:
            for p in model.parameters():
                p.grad = None
        loss = crit(model(x), y)
        loss.backward()
        if exchange is not None:
            exchange.finish()
        opt.step()
        return loss

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()

    timer = BF.KernelTimer()
    ctx = BF.timing(timer) if not args.no_kernel_timing else BF.timing(None)
    t0 = time.perf_counter()
    with ctx:
        for _ in range(args.steps):
            loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    final_loss = float(loss.item())

    ksum = timer.summary() if not args.no_kernel_timing else {}
    roofline = None
    if ksum:
        dom = max(ksum, key=lambda k: ksum[k]["ms"])
        d = ksum[dom]
        if d["avg_ops"] > 0:
            ach = d["avg_ops"] / (d["avg_ms"] * 1e-3) / 1e12
            bound, peak, ops_unit = op_peak(dom)
            roofline = {"bound": bound, "achieved": round(ach, 2), "peak": round(peak, 1),
                        "unit": "TFLOP/s", "frac": round(ach / peak, 4), "traffic": None,
                        "kernel": dom, "launches_per_step": d["launches"] / args.steps,
                        "avg_us": round(d["avg_ms"] * 1e3, 1), "ops_unit": ops_unit}
        else:
            ach = d["avg_bytes"] / (d["avg_ms"] * 1e-3) / 1e9
            roofline = {"bound": "hbm", "achieved": round(ach, 1), "peak": MI355X_HBM_GBS, "unit": "GB/s",
                        "frac": round(ach / MI355X_HBM_GBS, 4), "traffic": None, "kernel": dom,
                        "launches_per_step": d["launches"] / args.steps, "avg_us": round(d["avg_ms"] * 1e3, 1)}

    ms = elapsed / args.steps * 1e3
    samples = batch * world * args.steps
    result = {
        "metric": "train samples/sec (node) + binary GEMM TOPS",
        "value": round(samples / elapsed, 2),
        "unit": "samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp4/int8 MFMA (ternary operands as FP4 e2m1 / int8, fp32 digit planes as int8; exact integer sums; fp32 I/O)",
        "data": "synthetic MNIST-shaped (80.7% zero pixels, u8/255), random-init weights, resident in HBM",
        "config": {"workload": CONFIGS[args.config][2], "model": args.config, "global_batch": batch * world,
                   "per_gpu_batch": batch, "seq_len": 1, "parallelism": f"dp{world}",
                   "backend": args.backend, "loss_last_step": round(final_loss, 5)},
    }
    if ksum:
        # binary-GEMM TOPS: in-kernel rate of the ternary x ternary forward GEMMs (logical 2MNK)
        # ternary GEMM forms, and the binary convolutions' forward (im2col-free) for the CNN
        fwd = [v for k, v in ksum.items() if (k.startswith("gemm_i8") and "<1, 1," in k) or k == "conv2d_fwd"]
        if fwd:
            ops, ms_ = sum(v["ops"] for v in fwd), sum(v["ms"] for v in fwd)
            result["binary_gemm_tops"] = round(ops / (ms_ * 1e-3) / 1e12, 2)
        result["kernels"] = {k: {"launches": v["launches"], "avg_us": round(v["avg_ms"] * 1e3, 1),
                                 "share": round(v["ms"] / (elapsed * 1e3), 4)} for k, v in ksum.items()}
    if roofline is not None:
        traffic, src = pmc_traffic(roofline["kernel"])
        roofline["traffic"] = traffic
        roofline["traffic_source"] = src
        if traffic and d.get("avg_bytes"):
            roofline["algorithmic_bytes"] = int(d["avg_bytes"])
    result["roofline"] = roofline
    result["cpu_baseline"] = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args.config, args.cpu_budget)
        if result["cpu_baseline"]:
            result["speedup_vs_cpu"] = round(result["value"] / result["cpu_baseline"]["value"], 1)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

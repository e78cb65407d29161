#!/usr/bin/env python3
"""Training-step benchmark of the binarized-network hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config wide|mlp|cnn|small] [--batch B]
                    [--exchange]

N > 1 is launched by the driver as one process per GPU (torch.distributed.run, RCCL).
A "step" = one training step of the reference loop (mnist-dist2.py:118-137) on one batch of
synthetic MNIST-shaped input resident in HBM: forward through the libbnn layers (fused
BatchNorm+Hardtanh, BN -> sign-pack -> FP4 GEMM between the binarized layers), CrossEntropy,
backward (libbnn STE GEMMs), the bucketed RCCL gradient all-reduce overlapped with backward
(N > 1, or --exchange at N = 1), and the fused latent Adam + clamp + weight re-pack.  Per-GPU
batch is fixed (weak scaling).

Default workload = BASELINE config 5 (the one the metric's 1/2/4/8-GPU curve is quoted on):
wide binarized MLP 784-8192x3-10, batch 65536 per GPU.

Timing: W untimed warmup steps, then K steps between barrier + synchronize on both sides with
NO per-kernel instrumentation (``value``); the max over ranks.  Afterwards (outside the timed
region) a few instrumented steps time every libbnn launch with HIP events on its stream for the
``roofline`` object, whose ``achieved`` is ALGORITHMIC work (2*M*N*K ops per GEMM launch,
SURVEY §8(d); the digit passes that emulate fp32 operands on the int8 MFMA are not work) or
algorithmic bytes (HBM-bound kernels) per launch over the average launch time.

Prints ONE JSON line (rank 0) with the contract fields plus ``roofline``, ``cpu_baseline`` (the
oracle's torch-CPU restatement of the reference path on this box's host cores, N = 1 only:
the bench config itself, plus BASELINE configs 1 and 2) and ``gpu_torch_fp32`` (the same
restatement run on this GPU with torch's fp32 kernels: the naive-GPU comparator).
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "distributed-mnist-bnns_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

# Dense MFMA peaks of MI355X (MI355X_MICROARCH.md § Matrix cores; 256 CUs x 4 SIMDs x 2.4 GHz):
MI355X_INT8_DENSE_TOPS = 256 * 4 * 2048 * 2.4e9 / 1e12   # 32x32x32 i8 MFMA: 2048 ops/clk/SIMD
MI355X_FP4_DENSE_TOPS = 256 * 4 * 4096 * 2.4e9 / 1e12    # 32x32x64 f8f6f4 MFMA (FP4/FP6): 4096 ops/clk/SIMD
MI355X_F32_MFMA_TFLOPS = 256 * 4 * 64 * 2.4e9 / 1e12     # v_mfma_f32_16x16x4_f32: 64 FLOP/clk/SIMD
MI355X_BF16_DENSE_TFLOPS = 256 * 4 * 1024 * 2.4e9 / 1e12  # 16x16x32 / 32x32x16 bf16 MFMA: 1024 FLOP/clk/SIMD
MI355X_DOT4_TOPS = 256 * 64 * 8 * 2.4e9 / 1e12           # v_dot4_i32_i8 on the VALU: 64 lanes x 8 ops /clk/CU
# ternary XNOR-popcount on the VALU: 5 ops (and, xor, and, 2 x v_bcnt_u32 accumulate) per 32 MACs,
# 4 SIMDs x 16 lanes per CU per clock (tools/xnor_probe.py)
MI355X_XNOR_TOPS = 64 * 256 * 2.4e9 * (2 * 32 / 5) / 1e12
MI355X_HBM_GBS = 8000.0
PUBLISHED_SMALL_SPS = 60000 / 8.248   # MNIST_EPOCH_TIME(PersonalCom).csv:2-6 mean epoch, BASELINE.md §1

CONFIGS = {
    # name: (model key, default per-GPU batch, description)
    "wide": ("wide", 65536, "wide binarized MLP 784-8192x3-10 (BASELINE config 5)"),
    "mlp": ("mlp", 4096, "binarized MLP 784-3072-1536-768-10 (mnist-dist2 Net, BASELINE config 3)"),
    "small": ("small", 64, "binarized MLP 784-192x3-10 (mnist-dist3 Net: the published CSV config, batch 64)"),
    "cnn": ("cnn", 4096, "binarized CNN conv5(1-16)-conv5(16-32)-fc (BASELINE config 4)"),
}
CPU_WIDTHS = {"wide": (8192, 8192, 8192), "mlp": (3072, 1536, 768), "small": (192, 192, 192), "cnn": "cnn"}
CPU_BATCH = {"wide": 512, "mlp": 1024, "small": 64, "cnn": 256}


def digit_pairs(kernel):
    """MFMA passes per algorithmic MAC of a GEMM kernel instance: fp32 operands enter as digit
    planes -- 3 int8 planes on gemm_i8 ((3,1) = 3 passes, (3,3) = 6), 4 FP6 e2m3 planes against
    an FP4 ternary operand on gemm_fp6 (4 passes; 5 with a dX operand's residual FP4 plane)."""
    if kernel.startswith("gemm_fp6"):    # + the residual FP4 plane of a dX operand: a fifth pass
        return 5 if kernel.endswith("+res") else 4
    if kernel.startswith("conv2d_bwd"):   # dY as 3 exact bf16 terms (bf16x3) on the bf16 MFMA
        return 3
    for tag, n in (("<3, 3,", 6), ("<3, 1,", 3)):
        if tag in kernel:
            return n
    return 1


def op_peak(kernel):
    """(bound, dense peak TOPS, what is counted) of an ops-counted kernel."""
    if kernel.startswith("conv2d_bwd"):   # the default bf16x3 kernels (bnn_conv_set_mfma(1))
        return "mfma", MI355X_BF16_DENSE_TFLOPS, "algorithmic conv flops 2*N*Co*OH*OW*C*KH*KW on the bf16 MFMA (3 bf16 terms of dY)"
    if kernel.startswith("conv2d_fwd"):   # C=1 layer on VALU dot4; C%16==0 layers on int8 MFMA (looser bound)
        return "valu", MI355X_DOT4_TOPS, "int8 dot4 / MFMA ops (2*N*Co*OH*OW*C*KH*KW)"
    if kernel.startswith("gemm_fp4"):
        return "mfma", MI355X_FP4_DENSE_TOPS, "ternary GEMM ops 2*M*N*K on the FP4 MFMA"
    if kernel.startswith("gemm_fp6"):   # same f8f6f4 MFMA, FP6 x FP4 issues at the FP4 rate
        passes = ("4 FP6 digit planes + the FP4 residual plane: 5 MFMA passes" if kernel.endswith(" +res")
                  else "4 FP6 digit planes: 4 MFMA passes")
        return "mfma", MI355X_FP4_DENSE_TOPS, f"algorithmic GEMM ops 2*M*N*K on the FP6 x FP4 MFMA ({passes})"
    if kernel.startswith("gemm_xnor"):   # VALU popcount bound with the nonzero-mask plane
        return "valu", MI355X_XNOR_TOPS, "ternary popcount ops 2*M*N*K"
    return "mfma", MI355X_INT8_DENSE_TOPS, "algorithmic GEMM ops 2*M*N*K on the int8 MFMA"


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
    ap.add_argument("--exchange", action="store_true",
                    help="run the gradient-exchange path at N=1 too: flat buckets, hooks and the RCCL "
                         "bucket all-reduces / buffer broadcast on a one-rank group")
    ap.add_argument("--graph", action="store_true",
                    help="capture the training step as a HIP graph and time replays (bnn_amd.graph; with the "
                         "exchange, its collectives are captured too)")
    ap.add_argument("--dropin", action="store_true",
                    help="time the unchanged-script path instead: the reference Net through the drop-in "
                         "models.binarized_modules (.org protocol, torch BatchNorm / Hardtanh / CrossEntropyLoss, "
                         "torch.optim.Adam + the .org copy loop of mnist-dist2.py:131-137) on fp32 images")
    ap.add_argument("--dropin-bn", action="store_true",
                    help="with --dropin: bn1..bn3 as bnn_amd.nn.BatchNorm1d (torch's module on libbnn's passes)")
    ap.add_argument("--no-dropin", action="store_true", help="skip the drop-in path's secondary timing")
    ap.add_argument("--fp32-input", action="store_true",
                    help="feed fp32 images (u/255) instead of the u8 pixels the MLPs' fc1 consumes")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=10.0, help="seconds of CPU baseline work per config")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--no-gpu-torch", action="store_true", help="skip the torch-fp32-on-GPU comparator")
    ap.add_argument("--timing-steps", type=int, default=3, help="instrumented steps for the roofline")
    return ap.parse_args()


def build(cfg, backend):
    from bnn_amd import nets
    name = CONFIGS[cfg][0]
    if name == "cnn":
        model = nets.BinCNN(org_protocol=False, mutate_input=False, fused_bn=True)
    else:
        model = nets.MODELS[name](org_protocol=False, mutate_input=False, backend=backend, fused_bn=True)
    return model


def build_dropin(cfg, dropin_bn=False):
    """The reference's own call pattern on the drop-in module (mnist-dist2.py:46-76 Net built from
    models.binarized_modules' BinarizeLinear / BinarizeConv2d with torch's BatchNorm, Hardtanh,
    Dropout, LogSoftmax): ``org_protocol`` and ``mutate_input`` left at the reference's behaviour.
    dropin_bn: bn1..bn3 swapped for bnn_amd.nn.BatchNorm1d as well (MLPs)."""
    from bnn_amd import nets
    name = CONFIGS[cfg][0]
    if name == "cnn":
        return nets.BinCNN()
    return nets.MODELS[name](dropin_bn=True) if dropin_bn else nets.MODELS[name]()


def dropin_step_fn(model, x, y, lr):
    """mnist-dist2.py:118-137 unchanged: zero_grad, forward, nn.CrossEntropyLoss, backward, then the
    .org restore -> torch.optim.Adam.step -> clamp loop (optim.org_protocol_step)."""
    from bnn_amd.optim import org_protocol_step
    opt = torch.optim.Adam(model.parameters(), lr=lr)
    crit = torch.nn.CrossEntropyLoss()

    def step():
        opt.zero_grad()
        loss = crit(model(x), y)
        loss.backward()
        org_protocol_step(model, opt)
        return loss
    return step


def time_dropin(cfg, batch, dev, lr, steps, warmup, dropin_bn=False):
    """(ms per step, samples/s) of the drop-in path on this GPU: the same batch shape as fp32 images."""
    from bnn_amd.data import synthetic_mnist
    torch.manual_seed(0)
    model = build_dropin(cfg, dropin_bn).to(dev).train()
    x, y = synthetic_mnist(batch, seed=1234, device=dev, as_u8=False)
    step = dropin_step_fn(model, x, y, lr)
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    out = {"ms_per_step": round(dt * 1e3, 3), "value": round(batch / dt, 2), "unit": "samples/s", "steps": steps,
           "warmup": warmup, "loss_last_step": round(float(loss.item()), 5),
           "path": ("models.binarized_modules drop-in (.org protocol, "
                    + ("bnn_amd.nn.BatchNorm1d, torch " if dropin_bn else "torch BatchNorm/")
                    + "Hardtanh/CrossEntropyLoss, torch.optim.Adam + .org copy loop), fp32 images")}
    del model, x, y, step
    torch.cuda.empty_cache()
    return out


def _dropin_with_exchange(model, x, y, opt, exchange):
    from bnn_amd.optim import org_protocol_step
    loss = torch.nn.CrossEntropyLoss()(model(x), y)
    loss.backward()
    exchange.finish()
    org_protocol_step(model, opt)
    return loss


def host_threads():
    return int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))


def cpu_baselines(cfg, budget):
    """Reference semantics timed on this box's host cores (runs BEFORE this process touches the
    GPU).  Returns (entry for the bench config, list of entries for BASELINE configs 1 and 2)."""
    sys.path.insert(0, ROOT)
    from oracle import bnn_torch
    threads = host_threads()
    main = None
    widths = CPU_WIDTHS.get(cfg)
    batch = CPU_BATCH[cfg]
    sps, steps, secs = bnn_torch.time_training(widths, batch, threads, budget_s=budget, max_steps=100000)
    main = {"value": round(sps, 2), "unit": "samples/s", "cores": threads, "kind": "port",
            "sample": f"{steps} fp32 torch-CPU train steps (oracle/bnn_torch.py restatement of the reference "
                      f"path: .org protocol + Adam) of the same net at batch {batch}, {secs:.1f} s"}
    extra = []
    sps, steps, secs = bnn_torch.time_training((3072, 1536, 768), 100, threads, budget_s=budget, max_steps=100000)
    extra.append({"config": "BASELINE config 1: MLP 784-3072-1536-768-10, batch 100, 1 process, CPU",
                  "value": round(sps, 2), "unit": "samples/s", "cores": threads, "kind": "port",
                  "sample": f"{steps} steps, {secs:.1f} s"})
    per_rank = max(1, threads // 2)
    try:
        out = subprocess.run([sys.executable, "-m", "oracle.bnn_torch", "gloo", "3072", "1536", "768", "100", "2",
                              str(per_rank), str(budget)], cwd=ROOT, capture_output=True, text=True,
                             timeout=300, check=True)
        r = json.loads(out.stdout.strip().splitlines()[-1])
        extra.append({"config": "BASELINE config 2: same MLP, gloo DDP world_size 2 on CPU, batch 100 per rank",
                      "value": round(r["samples_per_s"], 2), "unit": "samples/s (both ranks)",
                      "cores": 2 * per_rank, "kind": "port",
                      "sample": f"{r['steps']} steps, {r['seconds']:.1f} s, {per_rank} threads per rank"})
    except (subprocess.SubprocessError, ValueError, IndexError, KeyError) as e:
        extra.append({"config": "BASELINE config 2", "error": repr(e)[:200]})
    return main, extra


def gpu_torch_baseline(cfg, batch, budget=4.0):
    """The reference semantics (oracle/bnn_torch.py: sign() + torch fp32 F.linear / F.conv2d,
    BatchNorm, Adam, .org protocol) run with GPU tensors: what the reference would do on this
    GPU without libbnn."""
    sys.path.insert(0, ROOT)
    from oracle import bnn_torch
    widths = CPU_WIDTHS.get(cfg)
    sps, steps, secs = bnn_torch.time_training(widths, batch, 1, budget_s=budget, max_steps=1000, device="cuda")
    torch.cuda.empty_cache()
    return {"value": round(sps, 2), "unit": "samples/s", "kind": "reference semantics, torch fp32 on this GPU",
            "sample": f"{steps} steps at batch {batch}, {secs:.1f} s"}


# Timers named after a C-ABI call rather than one kernel: the kernels one call launches (the
# first family counts the calls; the others -- the dW fold -- add their bytes to each call).
TIMER_KERNELS = {
    "conv2d_bwd_filter": ("conv_bwd_filter_bf3_k<", "conv_filter_tile_reduce1_k", "conv_filter_tile_reduce2_k"),
    "conv2d_bwd_data": ("conv_bwd_data_bf3_k<",),
    "conv2d_fwd": ("conv_fwd_",),
}


def pmc_traffic(kernel):
    """HBM/fabric bytes per launch of ``kernel`` from the newest committed rocprofv3 PMC summary
    (profiles/*_pmc_traffic.json, written by tools/pmc_summary.py from separate FETCH_SIZE and
    WRITE_SIZE passes of this bench, gfx950-corrected).  For a timer in TIMER_KERNELS: all bytes of
    the call's kernels over the number of calls.  None when no pass covers the kernel."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_traffic.json")))
    # a timer name "<kernel> +res" is the RES = 1 instance of the FP6 GEMM template (last parameter 1)
    res = kernel.endswith(" +res")
    if res:
        kernel = kernel[:-len(" +res")]
    prefix = kernel.rstrip(">")
    for f in reversed(files):
        try:
            ks = json.load(open(f))["kernels"]
        except (OSError, ValueError, KeyError):
            continue
        if kernel in TIMER_KERNELS:
            fams = TIMER_KERNELS[kernel]
            calls, total = 0, 0
            for name, v in ks.items():
                for i, fam in enumerate(fams):
                    if name.startswith(fam):
                        n = sum(gv["launches"] for gv in v["grids"].values())
                        total += v["traffic_bytes_per_launch"] * n
                        calls += n if i == 0 else 0
            if calls:
                return int(total / calls), os.path.relpath(f, ROOT)
            continue
        hits = [(name, v) for name, v in ks.items()
                if name == kernel or (name.startswith(prefix) and name[len(prefix):len(prefix) + 1] in (",", ">"))]
        if kernel.startswith("gemm_fp6_k") and len(hits) > 1:   # the instance with / without the residual plane
            hits = [(n, v) for n, v in hits if n.endswith(", 1>") == res] or hits
        if hits:
            return hits[0][1]["traffic_bytes_per_launch"], os.path.relpath(f, ROOT)
    return None, None


def roofline_of(ksum, steps):
    dom = max(ksum, key=lambda k: ksum[k]["ms"])
    d = ksum[dom]
    common = {"kernel": dom, "launches_per_step": d["launches"] / steps, "avg_us": round(d["avg_ms"] * 1e3, 1)}
    if d["avg_ops"] > 0:
        ach = d["avg_ops"] / (d["avg_ms"] * 1e-3) / 1e12
        bound, peak, ops_unit = op_peak(dom)
        r = {"bound": "mfma" if bound == "mfma" else bound, "achieved": round(ach, 2), "peak": round(peak, 1),
             "unit": "TFLOP/s", "frac": round(ach / peak, 4), "traffic": None, **common, "ops_unit": ops_unit}
        pairs = digit_pairs(dom)
        if pairs > 1:   # the MFMA passes the fp32-operand emulation issues (secondary, not the work)
            r["mfma_pass_rate_tops"] = round(ach * pairs, 2)
            r["mfma_pass_frac"] = round(ach * pairs / peak, 4)
    else:
        ach = d["avg_bytes"] / (d["avg_ms"] * 1e-3) / 1e9
        r = {"bound": "hbm", "achieved": round(ach, 1), "peak": MI355X_HBM_GBS, "unit": "GB/s",
             "frac": round(ach / MI355X_HBM_GBS, 4), "traffic": None, **common}
    traffic, src = pmc_traffic(dom)
    r["traffic"] = traffic
    r["traffic_source"] = src
    r["algorithmic_bytes_per_launch"] = int(d["avg_bytes"])
    return r


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("BNN_BENCH_ONE_DEVICE") == "1":   # rehearsal only: every rank on device 0
        local = 0
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    cpu_main, cpu_extra = None, []
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu_main, cpu_extra = cpu_baselines(args.config, args.cpu_budget)   # before any GPU work
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    use_exchange = world > 1 or args.exchange
    if use_exchange:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        backend = os.environ.get("BNN_BENCH_BACKEND", "nccl")   # rehearsal on one device: "gloo"
        if backend == "nccl":
            from bnn_amd.parallel import init_rccl
            init_rccl(dev, rank, world)
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)

    from bnn_amd import functional as BF
    from bnn_amd.data import synthetic_mnist
    from bnn_amd.nets import binary_params
    from bnn_amd.optim import LatentAdam
    from bnn_amd.parallel import GradExchange

    batch = args.batch or CONFIGS[args.config][1]
    torch.manual_seed(0)
    if args.dropin_bn and not args.dropin:
        raise SystemExit("--dropin-bn goes with --dropin")
    model = (build_dropin(args.config, args.dropin_bn) if args.dropin else build(args.config, args.backend)).to(dev).train()
    # --exchange at N = 1: a one-rank RCCL group issuing every collective of an N-GPU step
    exchange = (GradExchange(model, bucket_mb=args.bucket_mb, force_collectives=args.exchange)
                if use_exchange else None)
    if args.dropin and args.graph:
        raise SystemExit("--dropin times the reference's eager loop")
    dstep = BF.DeviceStep(dev).activate() if args.graph else None
    as_u8 = args.config != "cnn" and not args.fp32_input and not args.dropin
    x, y = synthetic_mnist(batch, seed=1234 + rank, device=dev, as_u8=as_u8)
    if args.dropin:
        # the unchanged reference loop on the drop-in module (its torch.optim.Adam + .org loop);
        # the exchange's hooks and finish() bracket it as DDP's would
        inner = dropin_step_fn(model, x, y, args.lr)

        def step():
            if exchange is not None:
                exchange.zero_grad()
            loss = inner() if exchange is None else _dropin_with_exchange(model, x, y, inner_opt, exchange)
            return loss
        inner_opt = torch.optim.Adam(model.parameters(), lr=args.lr) if exchange is not None else None
    else:
        opt = LatentAdam(model.parameters(), lr=args.lr, clamp_params=binary_params(model), device_step=dstep)
        from bnn_amd.nn import CrossEntropyLoss
        crit = CrossEntropyLoss()     # nn.CrossEntropyLoss() on libbnn (mnist-dist2.py's criterion)

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

    run = step
    coll_per_step = None
    if args.graph:
        from bnn_amd.graph import GraphedStep
        c0 = exchange.collectives if exchange is not None else 0
        run = GraphedStep(step, opt, dstep, warmup=max(1, args.warmup))   # eager warm-up + capture
        if exchange is not None:    # replays issue what the capture issued: count warm-up + capture
            coll_per_step = (exchange.collectives - c0) / (max(1, args.warmup) + 1)
    else:
        for _ in range(args.warmup):
            step()
    if use_exchange:
        dist.barrier()
    torch.cuda.synchronize()

    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = run()
    torch.cuda.synchronize()
    if use_exchange:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    dist_info = None
    if use_exchange:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        ranks = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(ranks, t)
        per_rank = [float(v.item()) for v in ranks]
        elapsed = max(per_rank)
        try:
            nccl_v = ".".join(str(v) for v in torch.cuda.nccl.version())
        except Exception:     # noqa: BLE001 -- informational only
            nccl_v = None
        dist_info = {"world_size": dist.get_world_size(), "backend": dist.get_backend(),
                     "rccl_version": nccl_v, "devices": world,
                     "rank_ms_per_step_min": round(min(per_rank) / args.steps * 1e3, 3),
                     "rank_ms_per_step_max": round(max(per_rank) / args.steps * 1e3, 3),
                     "collectives_per_step": (coll_per_step if coll_per_step is not None else
                                              exchange.collectives / max(1, args.warmup + args.steps)
                                              if exchange is not None else None)}
    final_loss = float(loss.item())

    # instrumented steps (outside the timed region): per-launch HIP events -> roofline
    ksum, tsteps = {}, 0
    if not args.no_kernel_timing and args.timing_steps > 0:
        timer = BF.KernelTimer()
        with BF.timing(timer):
            for _ in range(args.timing_steps):
                step()
        tsteps = args.timing_steps
        ksum = timer.summary()

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
        # the reference's only published figure is this config's CSV epoch time
        # (mnist-dist3.py, 784-192x3-10, batch 64, one GPU: 60000 / 8.248 s = 7,274 samples/s)
        "vs_baseline": (round(samples / elapsed / PUBLISHED_SMALL_SPS, 2)
                        if args.config == "small" and batch == 64 and world == 1 else None),
        "dtype": "fp4/fp6/int8 MFMA (ternary operands as FP4 e2m1, fp32 operands as 4 FP6 e2m3 digit planes "
                 "with E8M0 block scales + an FP4 residual plane on the dX operands (backward: within "
                 "2^-19 / 2^-22 of the block maximum) or 3 int8 digit planes (first layer); fp32 accumulate, "
                 "fp32 I/O)",
        "data": ("synthetic MNIST-shaped (80.7% zero pixels), resident in HBM as "
                 + ("u8 pixels (fc1 applies ToTensor on the bytes)" if as_u8 else "fp32 u8/255 images")
                 + ", random-init weights"),
        "config": {"workload": CONFIGS[args.config][2] + (" -- drop-in path (the unchanged reference loop)"
                                                           if args.dropin else ""),
                   "model": args.config + ("-dropin" + ("-bn" if args.dropin_bn else "") if args.dropin else ""), "global_batch": batch * world,
                   "per_gpu_batch": batch, "seq_len": 1, "parallelism": f"dp{world}",
                   "backend": args.backend, "exchange": bool(use_exchange), "hip_graph": bool(args.graph),
                   "loss_last_step": round(final_loss, 5)},
    }
    if ksum:
        # binary-GEMM TOPS: in-kernel rate of the ternary x ternary forward GEMMs (2*M*N*K) and the
        # binary convolutions' forward for the CNN; the first layer's u8-pixel x ternary GEMM (any
        # "[pixels" label: not a binary GEMM) is reported on its own as fc1_tops
        fwd = [v for k, v in ksum.items()
               if "[pixels" not in k and (k.startswith("gemm_fp4") or (k.startswith("gemm_i8") and "<1, 1," in k)
                                          or k == "conv2d_fwd" or k == "gemm_xnor_k")]
        if fwd:
            ops, ms_ = sum(v["ops"] for v in fwd), sum(v["ms"] for v in fwd)
            result["binary_gemm_tops"] = round(ops / (ms_ * 1e-3) / 1e12, 2)
        pix = [v for k, v in ksum.items() if "[pixels" in k and "<1, 1," in k and v["ops"] > 0]   # fc1's forward
        if pix:
            ops, ms_ = sum(v["ops"] for v in pix), sum(v["ms"] for v in pix)
            result["fc1_tops"] = round(ops / (ms_ * 1e-3) / 1e12, 2)
        step_ms = sum(v["ms"] for v in ksum.values()) / tsteps
        result["kernels"] = {k: {"launches_per_step": v["launches"] / tsteps, "avg_us": round(v["avg_ms"] * 1e3, 1),
                                 "share_of_step": round(v["ms"] / tsteps / ms, 4)}
                             for k, v in sorted(ksum.items(), key=lambda kv: -kv[1]["ms"])}
        result["libbnn_kernel_ms_per_step"] = round(step_ms, 3)
        result["roofline"] = roofline_of(ksum, tsteps)
    else:
        result["roofline"] = None
    if dist_info is not None:
        result["distributed"] = dist_info
    result["cpu_baseline"] = cpu_main
    if cpu_main:
        result["cpu_baselines_other"] = cpu_extra
        result["speedup_vs_cpu"] = round(result["value"] / cpu_main["value"], 1)
    if rank == 0 and world == 1 and not args.dropin and not args.no_dropin and not args.graph:
        # the unchanged-script path (models.binarized_modules drop-in + the reference's loop) on the
        # same GPU and batch, timed after the main measurement: what a user of mnist-dist2.py gets
        try:
            result["dropin"] = time_dropin(args.config, batch, dev, args.lr, steps=5, warmup=2)
        except RuntimeError as e:        # e.g. out of memory: report, never fail the bench line
            result["dropin"] = {"error": repr(e)[:200]}
        if CONFIGS[args.config][0] != "cnn":
            # the same with bn1..bn3 swapped for bnn_amd.nn.BatchNorm1d
            try:
                result["dropin_bn"] = time_dropin(args.config, batch, dev, args.lr, steps=5, warmup=2, dropin_bn=True)
            except RuntimeError as e:
                result["dropin_bn"] = {"error": repr(e)[:200]}
    if rank == 0 and world == 1 and not args.no_gpu_torch and args.config in CPU_WIDTHS:
        try:
            gb = min(batch, 16384) if args.config == "wide" else batch
            result["gpu_torch_fp32"] = gpu_torch_baseline(args.config, gb)
        except RuntimeError as e:        # e.g. out of memory: report, never fail the bench line
            result["gpu_torch_fp32"] = {"error": repr(e)[:200]}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if use_exchange:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

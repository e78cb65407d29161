"""The reference's data-parallel BNN training loop (mnist-dist2.py:22-155), on libbnn + RCCL.

    # one process per GPU (torchrun or the reference's mp.spawn style):
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        -m bnn_amd.trainer --model wide --batch-size 65536 --epochs 1
    python -m bnn_amd.trainer -g 2 --epochs 1          # spawns 2 local ranks itself

Flags keep the reference's names (-n/--nodes, -g/--gpus, -nr/--nr, --epochs, --seed, --lr,
--log-interval; mnist-dist2.py:23-37).  Semantics kept: batch 64 by default (:88), Adam(lr) on
the latent weights (:91), DistributedSampler order with seed 0 and no set_epoch (:100-108),
1-based epochs with the per-batch ``lr *= 0.1`` whenever ``epoch % 40 == 0`` (:126-127), the
.org restore -> step -> clamp protocol (:131-137, here fused into LatentAdam), AverageMeter batch
timing and the reference's log line (:139-146), optional CSVs in the reference's format
(mnist-dist3.py:132-135).  Differences: RCCL instead of gloo, inputs held in HBM
(synthetic MNIST-shaped data unless --idx-images/--idx-labels point at real idx files), fused
BatchNorm+Hardtanh, no fp32 copy of sign(input).
"""
import argparse
import os
import time
from datetime import datetime

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from . import functional as BF
from . import nets
from .checkpoint import load_checkpoint, save_checkpoint
from .graph import GraphedStep
from .data import load_idx_dataset, shard_indices, synthetic_mnist
from .optim import LatentAdam
from .parallel import GradExchange


class AverageMeter:
    """utils.py:86-102 semantics (val / sum / count / avg)."""

    def __init__(self):
        self.val = self.avg = self.sum = 0.0
        self.count = 0

    def update(self, val, n=1):
        self.val = val
        self.sum += val * n
        self.count += n
        self.avg = self.sum / self.count


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("-n", "--nodes", default=1, type=int)
    ap.add_argument("-g", "--gpus", default=1, type=int, help="processes (GPUs) per node")
    ap.add_argument("-nr", "--nr", default=0, type=int, help="rank of this node")
    ap.add_argument("--epochs", default=10, type=int)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--log-interval", type=int, default=10)
    ap.add_argument("--batch-size", type=int, default=64)
    ap.add_argument("--model", default="mlp", choices=sorted(nets.MODELS))
    ap.add_argument("--dataset-size", type=int, default=60000, help="synthetic training set size")
    ap.add_argument("--idx-images", default=None)
    ap.add_argument("--idx-labels", default=None)
    ap.add_argument("--graph", action="store_true", help="replay each full batch's step from a HIP graph "
                    "(one process; bnn_amd.graph)")
    ap.add_argument("--fp32-input", action="store_true", help="keep the dataset as fp32 images (u/255) "
                    "instead of u8 pixels")
    ap.add_argument("--max-steps", type=int, default=0, help="stop each epoch after this many steps")
    ap.add_argument("--no-lr-quirk", action="store_true", help="drop the per-batch lr*=0.1 at epoch%%40==0")
    ap.add_argument("--lr-quirk-period", type=int, default=40, help="the 40 of epoch%%40==0 (mnist-dist2.py:126)")
    ap.add_argument("--device-step", action="store_true", help="eager steps on the device step counter (dropout "
                    "seeds and Adam as --graph draws them: an eager twin of a --graph run)")
    ap.add_argument("--csv-prefix", default=None, help="write <prefix>_BATCH_TIME.csv / _EPOCH_TIME.csv")
    ap.add_argument("--checkpoint", default=None, help="write a latent-weight checkpoint here after every epoch")
    ap.add_argument("--resume", default=None, help="resume from a checkpoint written by --checkpoint")
    ap.add_argument("--backend", default="nccl")
    ap.add_argument("--master-addr", default=os.environ.get("MASTER_ADDR", "127.0.0.1"))
    ap.add_argument("--master-port", default=os.environ.get("MASTER_PORT", "23456"))
    return ap.parse_args(argv)


def load_dataset(args, device, rank, as_u8=True):
    """Resident training set: u8 pixels (fc1 applies ToTensor on the bytes) unless the model
    needs the fp32 images (the CNN) or --fp32-input asks for them."""
    if args.idx_images:
        imgs, labels = load_idx_dataset(args.idx_images, args.idx_labels, device)
        return (imgs if as_u8 else imgs.float().div_(255.0)), labels
    # identical synthetic set on every rank (seed 1234); the sampler shards it
    return synthetic_mnist(args.dataset_size, seed=1234, device=device, as_u8=as_u8)


def train(gpu, args):
    world = args.gpus * args.nodes
    rank = args.nr * args.gpus + gpu
    if "RANK" in os.environ and "WORLD_SIZE" in os.environ:      # launched by torch.distributed.run
        rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
        gpu = int(os.environ.get("LOCAL_RANK", gpu))
    torch.cuda.set_device(gpu)
    device = torch.device("cuda", gpu)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", args.master_addr)
        os.environ.setdefault("MASTER_PORT", str(args.master_port))
        if args.backend == "nccl":
            from .parallel import init_rccl
            init_rccl(device, rank, world, init_method="env://")
        else:
            dist.init_process_group(args.backend, init_method="env://", world_size=world, rank=rank)
    torch.cuda.manual_seed(args.seed)
    model = nets.MODELS[args.model](org_protocol=False, mutate_input=False,
                                    fused_bn=True).to(device)
    exchange = GradExchange(model) if world > 1 else None
    if args.graph and world > 1:
        raise SystemExit("--graph runs one process (the gradient exchange is not captured)")
    dstep = BF.DeviceStep(device).activate() if (args.graph or args.device_step) else None
    opt = LatentAdam(model.parameters(), lr=args.lr, clamp_params=nets.binary_params(model), device_step=dstep)
    crit = torch.nn.CrossEntropyLoss()
    first_epoch = 1
    if args.resume:
        first_epoch = load_checkpoint(args.resume, model, opt, map_location=device) + 1
    data, targets = load_dataset(args, device, rank, as_u8=args.model != "cnn" and not args.fp32_input)
    idx = torch.tensor(shard_indices(len(data), world, rank), device=device)
    nb = (len(idx) + args.batch_size - 1) // args.batch_size
    T, E = [], []
    graphed = static_x = static_y = None

    def _step(xb, yb):
        for p in model.parameters():
            p.grad = None
        lo = crit(model(xb), yb)
        lo.backward()
        opt.step()
        return lo

    starts = datetime.now()
    for epoch in range(first_epoch, args.epochs + 1):
        T.append(["epoch", epoch])
        start = datetime.now()
        meter = AverageMeter()
        end = time.time()
        model.train()
        for batch_idx in range(nb):
            if args.max_steps and batch_idx >= args.max_steps:
                break
            sel = idx[batch_idx * args.batch_size:(batch_idx + 1) * args.batch_size]
            x, y = data.index_select(0, sel), targets.index_select(0, sel)
            quirk = epoch % args.lr_quirk_period == 0 and not args.no_lr_quirk
            if args.graph and len(sel) == args.batch_size and not quirk:
                # full batches replay one captured step on static buffers (the last, short batch
                # and lr-quirk epochs run eagerly)
                if graphed is None:
                    static_x, static_y = x.clone(), y.clone()
                    loss = None             # drop the last eager step's autograd graph before capturing
                    graphed = GraphedStep(lambda: _step(static_x, static_y), opt, dstep, warmup=1)
                else:
                    static_x.copy_(x)
                    static_y.copy_(y)
                    graphed()
                loss = graphed.out
            else:
                if exchange is not None:
                    exchange.zero_grad()
                else:
                    opt.zero_grad(set_to_none=True)
                loss = crit(model(x), y)
                if quirk:
                    opt.param_groups[0]["lr"] *= 0.1
                    graphed = None          # the captured step holds the old lr's Adam schedule
                loss.backward()
                if exchange is not None:
                    exchange.finish()
                opt.step()
            meter.update(time.time() - end)     # host time per batch, as utils.AverageMeter use
            end = time.time()
            if batch_idx % args.log_interval == 0:
                lv = loss.item()                # syncs, like the reference's loss.item()
                if batch_idx * len(x) != 0:
                    T.append([batch_idx * len(x), meter.val])
                if rank == 0:
                    print("Train Epoch: {} [{}/{} ({:.0f}%)]\tLoss: {:.6f} \t Time: {:.3f}({:.3f})".format(
                        epoch, batch_idx * len(x), len(data), 100.0 * batch_idx / nb, lv, meter.val, meter.avg),
                        flush=True)
        torch.cuda.synchronize()
        if rank == 0:
            print("Training ", epoch, " : " + str(datetime.now() - start), flush=True)
        E.append([datetime.now() - start])
        if args.checkpoint:
            save_checkpoint(args.checkpoint, model, opt, epoch)
    if rank == 0:
        print("Training complete in: " + str(datetime.now() - starts), flush=True)
        if args.csv_prefix:
            import pandas as pd
            pd.DataFrame(T).to_csv(f"{args.csv_prefix}_BATCH_TIME.csv")
            pd.DataFrame(E).to_csv(f"{args.csv_prefix}_EPOCH_TIME.csv")
    if dstep is not None:
        dstep.deactivate()
    if world > 1:
        dist.destroy_process_group()
    return model


def main(argv=None):
    args = parse(argv)
    if "RANK" in os.environ and "WORLD_SIZE" in os.environ:
        train(int(os.environ.get("LOCAL_RANK", 0)), args)
    elif args.gpus > 1:
        os.environ.setdefault("MASTER_ADDR", args.master_addr)
        os.environ.setdefault("MASTER_PORT", str(args.master_port))
        mp.spawn(train, nprocs=args.gpus, args=(args,))
    else:
        train(0, args)


if __name__ == "__main__":
    main()

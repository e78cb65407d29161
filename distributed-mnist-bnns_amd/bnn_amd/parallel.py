"""Subsystem (4): data-parallel gradient exchange over RCCL (torch.distributed "nccl" on ROCm).

Replaces the reference's ``nn.parallel.DistributedDataParallel(model)`` over gloo
(mnist-dist2.py:83 + :93; the all-reduce fires inside ``loss.backward()`` at :130).  Same
contract as DDP there:

* at construction, parameters and buffers are broadcast from rank 0 (the reference seeds only
  the CUDA RNG, mnist-dist2.py:84, so CPU-initialised weights differ per rank until then);
* before every forward, buffers (BatchNorm running stats) are broadcast from rank 0
  (DDP ``broadcast_buffers=True``); batch statistics themselves stay per rank (no SyncBN);
* gradients are averaged across ranks, bucketed and overlapped with backward.

MI355X design:

* every gradient lives inside ONE flat buffer per (dtype, device) -- ``p.grad`` is a view, so
  there is no copy in or out and zeroing is one memset;
* buckets are contiguous slices of that buffer in reverse registration order (the order
  autograd produces gradients), at most ``bucket_mb`` each (64 MB default: xGMI rings are
  per-link bound, so fewer large collectives amortise launch cost while still overlapping);
  a gradient larger than the cap (the wide MLP's 268 MB fc2 / fc3 weights) is split into
  equal slices of at most the cap;
* a post-accumulate-grad hook launches each bucket's async all-reduce on the process group's
  own stream as soon as every gradient overlapping it has landed, strictly in bucket order on
  every rank; ``finish()`` joins them before the optimizer.  With RCCL the reduction is
  ``ReduceOp.AVG``; gloo (CPU tests) has no AVG, so it sums and divides;
* DDP's per-forward buffer broadcast is ONE collective per device over a flat byte staging
  buffer (not one per running_mean / running_var / num_batches_tracked);
* direct write (``direct_write=True``): a libbnn layer whose weight gradient is one GEMM writes it
  straight into the weight's bucket view (functional._grad_sink) and reports it
  (``grad_written``), instead of returning a fresh tensor that autograd's AccumulateGrad then adds
  into the zeroed view -- one read-modify-write pass over the 563 MB of wide-MLP gradients fewer
  per step.  Valid while each weight gets one gradient per backward (no accumulation across
  micro-batches); the sink is armed by ``zero_grad`` and disarmed once the weight is written.
* ``force_collectives=True`` issues every collective even on a one-rank group (the bucket
  all-reduces, the per-forward buffer broadcast): the RCCL path of a multi-GPU run, exercised and
  profiled on one GPU (an AVG over one rank leaves every gradient bit-identical).
"""
import math
import os

import torch
import torch.distributed as dist

from . import functional as BF

_ALIGN_BYTES = 256


def init_rccl(device, rank, world_size, init_method=None):
    """torch.distributed over RCCL ("nccl" on ROCm), one process per GPU, bound to ``device``, with
    RCCL's internal stream created at high priority.  HIP spreads normal-priority streams over a few
    hardware queues (GPU_MAX_HW_QUEUES = 4): in the r03 trace of bench.py --exchange the pool stream
    RCCL got shared hardware queue 4 with the compute stream, so every bucket reduction ran
    strictly between two backward kernels (profiles/r03_exchange_rccl_overlap_normalprio.txt: the
    last 24 collectives, 1,599.5 us, 0.00 % overlapped by compute kernels); a high-priority stream
    is given a queue of its own (profiles/r03_exchange_rccl_overlap_hiprio.txt: 5,886.1 us, 85.37 %
    overlapped -- one-rank collectives, so the durations are not xGMI traffic)."""
    # graph.GraphedStep captures collectives: keep RCCL work events out of torch's recycling cache,
    # so the watchdog thread never queries an event a capture has re-recorded
    os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")
    opts = dist.ProcessGroupNCCL.Options(is_high_priority_stream=True)
    kw = {"init_method": init_method} if init_method else {}
    dist.init_process_group("nccl", rank=rank, world_size=world_size, device_id=device, pg_options=opts, **kw)


class _Bucket:
    __slots__ = ("flat", "start", "end", "pending", "nparams", "work")

    def __init__(self, flat, start, end, nparams):
        self.flat = flat
        self.start = start
        self.end = end
        self.nparams = nparams
        self.pending = nparams
        self.work = None

    def view(self):
        return self.flat[self.start:self.end]


class GradExchange:
    def __init__(self, module, process_group=None, bucket_mb=64, broadcast_buffers=True,
                 init_broadcast=True, direct_write=True, force_collectives=False):
        if not dist.is_available() or not dist.is_initialized():
            raise RuntimeError("GradExchange needs an initialised torch.distributed process group")
        self.module = module
        self.pg = process_group
        self.world = dist.get_world_size(process_group)
        self.force = bool(force_collectives)
        self.collectives = 0       # collectives issued (all-reduces + buffer broadcasts)
        self.launch_log = []       # (bucket, start, end) of this step's all-reduces, in launch order
        # group rank 0 as a global rank: torch's src= arguments are global ranks
        self.src = dist.get_global_rank(process_group, 0) if process_group is not None else 0
        self.broadcast_buffers = broadcast_buffers
        self.use_avg = dist.get_backend(process_group) == "nccl"
        params = [p for p in module.parameters() if p.requires_grad]
        self._flat_buffers = self._coalesce_buffers(module)
        if init_broadcast:
            for p in params:
                dist.broadcast(p.data, src=self.src, group=self.pg)
                BF.invalidate_packed(p)     # written through .data: cached packed operands are stale
            self.sync_buffers()
        self.cap_bytes = max(1, int(bucket_mb * 2 ** 20))
        self.buckets, self._param_buckets, self._flats = self._build_buckets(list(reversed(params)))
        self._next = 0
        self._handles = []
        self._armed = set()        # weights whose zeroed bucket view a layer may overwrite
        self._counted = set()      # params already counted toward their buckets this step
        self.direct_write = direct_write
        self.direct_writes = 0     # gradients written straight into their views (tests, logs)
        for p in params:
            self._handles.append(p.register_post_accumulate_grad_hook(self._make_hook(self._param_buckets[p])))
            if direct_write:
                p._bnn_grad_sink = self
        if broadcast_buffers:
            self._handles.append(module.register_forward_pre_hook(lambda m, inp: self.sync_buffers()))

    # -------------------------------------------------------------- setup
    @staticmethod
    def _coalesce_buffers(module):
        """Staging for the per-forward buffer broadcast: one flat uint8 tensor per device with a
        typed view per registered buffer.  (The buffers themselves are NOT re-homed as views of
        it: views share a version counter, and torch's BatchNorm saves its running statistics
        for backward, so an in-place update of one would invalidate the others.)"""
        entries = [b for m in module.modules() for b in m._buffers.values() if b is not None]
        by_dev = {}
        for b in entries:
            by_dev.setdefault(b.device, []).append(b)
        groups = []
        for device, bufs in by_dev.items():
            offs, total = [], 0
            for b in bufs:
                offs.append(total)
                total += -(-max(b.numel() * b.element_size(), 1) // _ALIGN_BYTES) * _ALIGN_BYTES
            flat = torch.zeros(total, dtype=torch.uint8, device=device)
            by_dtype = {}
            for b, off in zip(bufs, offs):
                v = flat[off:off + b.numel() * b.element_size()].view(b.dtype).view(b.shape)
                src, dst = by_dtype.setdefault(b.dtype, ([], []))
                src.append(b)
                dst.append(v)
            groups.append((flat, list(by_dtype.values())))
        return groups

    def _build_buckets(self, params):
        """Flat gradient storage per (dtype, device) and the bucket slices over it."""
        groups = {}
        for p in params:
            groups.setdefault((p.dtype, p.device), []).append(p)
        buckets, param_buckets, flats = [], {}, []
        for (dtype, device), plist in groups.items():
            es = torch.empty((), dtype=dtype).element_size()
            # every gradient view starts on a 256-B boundary: the kernels that read or write them
            # (the fused latent update, the GEMMs writing into a view) take their vector paths
            # (a 10-float fc4 bias first misaligned every view after it); the gaps stay zero
            align = max(1, _ALIGN_BYTES // es)
            offsets, total = {}, 0
            for p in plist:
                offsets[p] = total
                total += -(-p.numel() // align) * align
            flat = torch.zeros(total, dtype=dtype, device=device)
            flats.append((flat, plist, offsets))
            cap = max(1, self.cap_bytes // es)
            cur, cur_start, cur_n = [], 0, 0      # cur_n: the bucket's span, gaps included
            for p in plist:
                n, off = p.numel(), offsets[p]
                if cur and (n > cap or off + n - cur_start > cap):
                    self._close(buckets, param_buckets, flat, cur, cur_start, cur_n)
                    cur, cur_n = [], 0
                if n > cap:                                 # split into equal slices <= cap
                    k = math.ceil(n / cap)
                    step = -(-n // k)
                    for i in range(k):
                        a, b = off + i * step, min(off + n, off + (i + 1) * step)
                        buckets.append(_Bucket(flat, a, b, 1))
                        param_buckets.setdefault(p, []).append(len(buckets) - 1)
                    continue
                if not cur:
                    cur_start = off
                cur.append(p)
                cur_n = off + n - cur_start
            if cur:
                self._close(buckets, param_buckets, flat, cur, cur_start, cur_n)
            self._bind(flat, plist, offsets)
        return buckets, param_buckets, flats

    @staticmethod
    def _close(buckets, param_buckets, flat, cur, start, n):
        buckets.append(_Bucket(flat, start, start + n, len(cur)))
        for q in cur:
            param_buckets.setdefault(q, []).append(len(buckets) - 1)

    @staticmethod
    def _bind(flat, plist, offsets):
        for p in plist:
            p.grad = flat[offsets[p]:offsets[p] + p.numel()].view_as(p)

    # -------------------------------------------------------------- per step
    def sync_buffers(self):
        """DDP broadcast_buffers: rank 0's buffers to every rank -- packed into the staging
        buffer (one multi-tensor copy per dtype), ONE collective per device, unpacked."""
        if self.world <= 1 and not self.force:
            return
        root = dist.get_rank() == self.src
        for flat, lists in self._flat_buffers:
            if root:
                for bufs, views in lists:
                    torch._foreach_copy_(views, bufs)
            dist.broadcast(flat, src=self.src, group=self.pg)
            self.collectives += 1
            if not root:
                for bufs, views in lists:
                    torch._foreach_copy_(bufs, views)

    def zero_grad(self):
        """Zero the flat gradient buffers (one memset each) and re-arm the hooks.  Gradients
        accumulate in place into the views, so they must start at zero, not None (an optimizer's
        ``zero_grad(set_to_none=True)`` detaches them; they are re-bound here)."""
        for flat, plist, offsets in self._flats:
            if not all(self._is_view(p, flat) for p in plist):
                self._bind(flat, plist, offsets)
            flat.zero_()
        for b in self.buckets:
            b.pending = b.nparams
            b.work = None
        self._next = 0
        self.launch_log = []
        self._counted = set()
        if self.direct_write:
            self._armed = {id(p) for _, plist, _ in self._flats for p in plist}

    def grad_sink(self, p):
        """The zeroed bucket view a layer's backward may write p's whole gradient into, or None
        (not armed: outside zero_grad .. backward, or already written this step)."""
        if id(p) not in self._armed:
            return None
        return p.grad

    def grad_written(self, p):
        """p's gradient was written into its view by the layer (what the accumulate hook reports)."""
        self._armed.discard(id(p))
        self.direct_writes += 1
        self._count(p)

    def _count(self, p):
        """p's gradient is complete in its view: count it toward its buckets ONCE per step.  A weight
        written by its layer gets no gradient from autograd, but torch still runs its post-accumulate
        hook (with nothing accumulated): counted twice, its bucket would be all-reduced before the
        parameters after it in backward order had their gradients (config 2's fc1.bias,
        tools/ddp_config2_diag.py, profiles/r05_ddp_config2_hook_order.log)."""
        if id(p) in self._counted:
            return
        self._counted.add(id(p))
        for bi in self._param_buckets[p]:
            self.buckets[bi].pending -= 1
        self._launch_ready()

    @staticmethod
    def _is_view(p, flat):
        g = p.grad
        if g is None:
            return False
        start = flat.data_ptr()
        end = start + flat.numel() * flat.element_size()
        return start <= g.data_ptr() < end

    def _make_hook(self, bucket_ids):
        def hook(p):
            self._armed.discard(id(p))
            self._count(p)
        return hook

    def _launch_ready(self):
        while self._next < len(self.buckets) and self.buckets[self._next].pending <= 0:
            b = self.buckets[self._next]
            if self.world > 1 or self.force:
                op = dist.ReduceOp.AVG if self.use_avg else dist.ReduceOp.SUM
                b.work = dist.all_reduce(b.view(), op=op, group=self.pg, async_op=True)
                self.collectives += 1
                self.launch_log.append((self._next, b.start, b.end))
            self._next += 1

    def finish(self):
        """Join all bucket reductions (launching any a hook did not reach, e.g. unused params)."""
        self._armed = set()
        for b in self.buckets:
            b.pending = 0
        self._launch_ready()
        for b in self.buckets:
            if b.work is not None:
                b.work.wait()
                if not self.use_avg and self.world > 1:
                    b.view().div_(self.world)
                b.work = None

    def remove(self):
        for h in self._handles:
            h.remove()
        self._handles = []
        self._armed = set()
        for _, plist, _ in self._flats:
            for p in plist:
                if getattr(p, "_bnn_grad_sink", None) is self:
                    del p._bnn_grad_sink

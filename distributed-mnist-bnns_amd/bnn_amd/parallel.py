"""Subsystem (4): data-parallel gradient exchange over RCCL (torch.distributed "nccl" on ROCm).

Replaces the reference's ``nn.parallel.DistributedDataParallel(model)`` over gloo
(mnist-dist2.py:83 + :93; the all-reduce fires inside ``loss.backward()`` at :130).  Same
contract as DDP there:

* at construction, parameters and buffers are broadcast from rank 0 (the reference seeds only
  the CUDA RNG, mnist-dist2.py:84, so CPU-initialised weights differ per rank until then);
* before every forward, buffers (BatchNorm running stats) are broadcast from rank 0
  (DDP ``broadcast_buffers=True``); batch statistics themselves stay per rank (no SyncBN);
* gradients are averaged across ranks, bucketed and overlapped with backward.

MI355X design: every gradient lives inside a flat per-bucket buffer (``p.grad`` is a view, so
there is no copy in or out); buckets follow reverse registration order (the order autograd
produces gradients) and are capped at ``bucket_mb`` (64 MB default: xGMI rings are per-link
bound, fewer larger collectives amortise launch cost while still overlapping); a
post-accumulate-grad hook launches the bucket's async all-reduce on the process group's own
stream as soon as its last gradient lands, strictly in bucket order on every rank.
``finish()`` joins them before the optimizer.  With RCCL the reduction is ``ReduceOp.AVG``;
gloo (CPU tests) has no AVG, so it sums and divides.
"""
import torch
import torch.distributed as dist


class _Bucket:
    __slots__ = ("params", "flat", "pending", "work")

    def __init__(self, params, flat):
        self.params = params
        self.flat = flat
        self.pending = len(params)
        self.work = None


class GradExchange:
    def __init__(self, module, process_group=None, bucket_mb=64, broadcast_buffers=True,
                 init_broadcast=True):
        if not dist.is_available() or not dist.is_initialized():
            raise RuntimeError("GradExchange needs an initialised torch.distributed process group")
        self.module = module
        self.pg = process_group
        self.world = dist.get_world_size(process_group)
        self.broadcast_buffers = broadcast_buffers
        self.use_avg = dist.get_backend(process_group) == "nccl"
        params = [p for p in module.parameters() if p.requires_grad]
        if init_broadcast:
            self._broadcast([p.data for p in params] + [b for b in module.buffers()])
        self.buckets = self._build_buckets(list(reversed(params)), int(bucket_mb * 2 ** 20))
        self._next = 0
        self._handles = []
        for bi, b in enumerate(self.buckets):
            for p in b.params:
                self._handles.append(p.register_post_accumulate_grad_hook(self._make_hook(bi)))
        if broadcast_buffers:
            self._handles.append(module.register_forward_pre_hook(lambda m, inp: self.sync_buffers()))

    # -------------------------------------------------------------- setup
    def _build_buckets(self, params, cap_bytes):
        buckets, cur, size = [], [], 0
        for p in params:
            nbytes = p.numel() * p.element_size()
            if cur and (size + nbytes > cap_bytes or p.dtype != cur[0].dtype or p.device != cur[0].device):
                buckets.append(cur)
                cur, size = [], 0
            cur.append(p)
            size += nbytes
        if cur:
            buckets.append(cur)
        out = []
        for plist in buckets:
            n = sum(p.numel() for p in plist)
            flat = torch.zeros(n, dtype=plist[0].dtype, device=plist[0].device)
            off = 0
            for p in plist:
                p.grad = flat[off:off + p.numel()].view_as(p)
                off += p.numel()
            out.append(_Bucket(plist, flat))
        return out

    def _broadcast(self, tensors):
        for t in tensors:
            dist.broadcast(t, src=0, group=self.pg)

    # -------------------------------------------------------------- per step
    def sync_buffers(self):
        if self.world > 1:
            self._broadcast(list(self.module.buffers()))

    def zero_grad(self):
        """Zero every bucket (one memset each) and re-arm the hooks.  Gradients accumulate in
        place into the bucket views, so they must start at zero, not None (an optimizer's
        ``zero_grad(set_to_none=True)`` detaches them; they are re-bound here)."""
        for b in self.buckets:
            if not all(self._is_view(p, b) for p in b.params):
                self._rebind(b)
            b.flat.zero_()
            b.pending = len(b.params)
            b.work = None
        self._next = 0

    @staticmethod
    def _is_view(p, b):
        g = p.grad
        if g is None:
            return False
        start = b.flat.data_ptr()
        end = start + b.flat.numel() * b.flat.element_size()
        return start <= g.data_ptr() < end

    @staticmethod
    def _rebind(b):
        off = 0
        for p in b.params:
            p.grad = b.flat[off:off + p.numel()].view_as(p)
            off += p.numel()

    def _make_hook(self, bi):
        def hook(p):
            b = self.buckets[bi]
            b.pending -= 1
            if b.pending == 0:
                self._launch_ready()
        return hook

    def _launch_ready(self):
        while self._next < len(self.buckets) and self.buckets[self._next].pending == 0:
            b = self.buckets[self._next]
            if self.world > 1:
                op = dist.ReduceOp.AVG if self.use_avg else dist.ReduceOp.SUM
                b.work = dist.all_reduce(b.flat, op=op, group=self.pg, async_op=True)
            self._next += 1

    def finish(self):
        """Join all bucket reductions (launching any a hook did not reach, e.g. unused params)."""
        for b in self.buckets:
            b.pending = 0
        self._launch_ready()
        for b in self.buckets:
            if b.work is not None:
                b.work.wait()
                if not self.use_avg:
                    b.flat.div_(self.world)
                b.work = None

    def remove(self):
        for h in self._handles:
            h.remove()
        self._handles = []

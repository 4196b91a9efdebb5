"""Data-parallel training step of the head (BASELINE.json configs[3]: CMTCoop
DDP training on 8 GPUs with RCCL gradient all-reduce over xGMI).

Reference: tools/dist_train.sh:10-20 (one process per GPU), tools/train.py:
197-204 (init_dist 'nccl'), mmcv MMDistributedDataParallel (bucketed gradient
all-reduce, sum then / world), mmcv OptimizerHook with grad_clip max_norm 35
(configs e.g. CMTCoop_TUMTraf/fusion/coop/...py:373-376), torch.optim.AdamW
(lr 1e-4, weight_decay 0.01, ...py:362-372).

MI355X design: every trainable parameter of the head is re-pointed into ONE
flat fp32 buffer and its .grad into ONE flat gradient buffer (autograd then
accumulates straight into it), so the gradient exchange is a few large
RCCL all-reduces over contiguous buckets (fewer, larger collectives: each
xGMI ring step moves bucket/world bytes per link) launched from
post-accumulate-grad hooks while backward is still running, the clip's global
norm is one native sum-of-squares pass and the AdamW update one native launch
over the whole buffer.  With world size 1 there is no collective at all.
"""
import gc

import torch
import torch.distributed as dist

from . import native_train as T
from .models.utils.train_ops import direct_param_grads
from .runtime import OPTIONS

__all__ = ["FlatParams", "Trainer", "PeerBackwardError", "allreduce_buckets"]


class FlatParams:
    """Trainable parameters of ``module`` as views of one flat buffer.

    With ``status_words`` > 0 the buffers start with that many words that are
    no parameter (kept 256-byte aligned for the parameters after them); the
    data-parallel exchange uses gradient word 0 as a per-step failure flag."""

    def __init__(self, module, status_words=0):
        self.params = [p for p in module.parameters() if p.requires_grad]
        if not self.params:
            raise ValueError("no trainable parameters")
        dev = self.params[0].device
        self.head = int(status_words)
        n = self.head + sum(p.numel() for p in self.params)
        self.flat = torch.zeros(n, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(n, dtype=torch.float32, device=dev)
        off = self.head
        self.slices = []
        for p in self.params:
            k = p.numel()
            self.flat[off:off + k].copy_(p.data.reshape(-1))
            p.data = self.flat[off:off + k].view_as(p)
            p.grad = self.grad[off:off + k].view_as(p)
            self.slices.append((off, k))
            off += k

    def zero_grad(self):
        self.grad.zero_()
        # autograd accumulates in place into existing .grad tensors (grad mode is off during backward);
        # re-attach in case a caller replaced one
        for p, (off, k) in zip(self.params, self.slices):
            if p.grad is None or p.grad.data_ptr() != self.grad[off:].data_ptr():
                p.grad = self.grad[off:off + k].view_as(p)


def allreduce_buckets(flat, bucket_bytes=25 << 20, group=None):
    """Mean over ranks of ``flat`` in place: contiguous buckets of at most
    ``bucket_bytes``, all launched asynchronously (RCCL over xGMI on the GPU
    box, gloo in the CPU tests), then one scale by 1/world."""
    if not (dist.is_available() and dist.is_initialized()):
        return 0
    world = dist.get_world_size(group)
    if world == 1:
        return 0
    per = max(1, bucket_bytes // flat.element_size())
    works = [dist.all_reduce(flat[i:i + per], group=group, async_op=True) for i in range(0, flat.numel(), per)]
    for w in works:
        w.wait()
    flat.mul_(1.0 / world)
    return len(works)


class PeerBackwardError(RuntimeError):
    """Another rank's backward raised in this step; no rank applies it."""


class _GradBuckets:
    """Gradient all-reduce overlapped with backward (mmcv
    MMDistributedDataParallel / torch DDP semantics, tools/train.py:282-289):
    the flat gradient buffer is cut at parameter boundaries into buckets of
    ~bucket_bytes in REVERSE parameter order (backward produces the last
    layers' gradients first); a post-accumulate-grad hook counts each bucket's
    parameters and, once a bucket is complete, launches the async all-reduces
    of every complete bucket in bucket order -- the same launch sequence on
    every rank whatever order autograd finishes them in, so the collectives
    pair up.  finish() flushes buckets whose parameters got no gradient, waits
    for all of them and scales by 1 / world.

    A backward that raises on SOME ranks only: the failing rank's abort()
    sets the step's failure flag (gradient word 0, in the last bucket) and
    launches every bucket it has not launched yet, so each rank still issues
    the same sequence of all-reduces and none is paired with a later step's;
    every rank's finish() then sees the summed flag, drops the step's
    gradients and raises PeerBackwardError.  (A backward that raises after
    its last bucket was launched -- all gradients already exchanged -- is not
    covered: the flag no longer travels; abort() then returns False and the
    Trainer refuses every later step, since this rank's weights can no longer
    follow the others'.)"""

    def __init__(self, fp, bucket_bytes, group):
        self.fp, self.group = fp, group
        self.world = dist.get_world_size(group)
        self.buckets = []                      # (lo, hi, n_params), in launch order
        self.of_param = [0] * len(fp.params)
        lo = hi = None
        members = 0
        for i in reversed(range(len(fp.params))):
            off, k = fp.slices[i]
            if hi is None:
                hi = off + k
            lo = off
            members += 1
            self.of_param[i] = len(self.buckets)
            if (hi - lo) * 4 >= bucket_bytes:
                self.buckets.append((lo, hi, members))
                lo = hi = None
                members = 0
        if hi is not None:
            self.buckets.append((lo, hi, members))
        lo, hi, members = self.buckets[-1]
        self.buckets[-1] = (0, hi, members)    # the last bucket also carries the status words
        self.handles = [p.register_post_accumulate_grad_hook(self._make_hook(i)) for i, p in enumerate(fp.params)]
        self.reset()

    def reset(self):
        self.pending = [n for _, _, n in self.buckets]
        self.next = 0
        self.works = []

    def _launch_ready(self, upto=None):
        end = len(self.buckets) if upto is None else upto
        while self.next < end and (upto is not None or self.pending[self.next] == 0):
            lo, hi, _ = self.buckets[self.next]
            self.works.append(dist.all_reduce(self.fp.grad[lo:hi], group=self.group, async_op=True))
            self.next += 1

    def _make_hook(self, i):
        def hook(_param):
            b = self.of_param[i]
            self.pending[b] -= 1
            if self.pending[b] == 0:
                self._launch_ready()
        return hook

    def drain(self):
        """Wait for the all-reduces launched so far and restart the bucket
        state: a backward() that step() never finished (called twice on every
        rank) must not leave ``next`` / ``pending`` behind, or the next step
        would exchange nothing and the ranks would drift apart."""
        for w in self.works:
            w.wait()
        self.reset()

    def abort(self):
        """This rank's backward raised: flag the step and complete its
        all-reduce sequence (see the class docstring).  Returns whether the
        flag travels (False: the last bucket was already launched)."""
        travels = self.next < len(self.buckets)
        if travels:
            self.fp.grad[0] = 1.0
        self._launch_ready(upto=len(self.buckets))
        for w in self.works:
            w.wait()
        self.reset()
        return travels

    def finish(self):
        self._launch_ready(upto=len(self.buckets))
        for w in self.works:
            w.wait()
        n = len(self.works)
        self.reset()
        failed = self.fp.grad[0].item() if self.fp.head else 0.0
        if failed > 0:
            self.fp.grad.zero_()
            raise PeerBackwardError(f"the backward of {int(failed)} rank(s) failed in this step: "
                                    "its gradients were dropped on every rank")
        self.fp.grad.mul_(1.0 / self.world)
        return n


class Trainer:
    """One optimisation step: backward of the summed loss dict with the
    bucketed gradient all-reduce overlapped (world > 1), clip_grad_norm_
    (max_norm), AdamW.  At construction, rank 0's parameters and buffers are
    broadcast to every rank (as MMDistributedDataParallel does), so ranks
    that started from different initialisations train the same model."""

    def __init__(self, module, lr=1e-4, weight_decay=0.01, betas=(0.9, 0.999), eps=1e-8, max_norm=35.0,
                 bucket_mb=25, group=None, freeze_gc=False):
        self.module = module
        # freeze_gc (opt-in, PROCESS-WIDE): after the first step gc.freeze() moves every object alive
        # in the process then -- the module, weight packs, optimizer state, but also the caller's
        # objects and iterators -- out of the cyclic collector's generations, so the one collection
        # a step triggers scans only that step's objects (33.1-33.8 -> 34.6-34.9 steps/s coop,
        # profiles/r5_experiments.txt r5aw).  Cycles among the frozen objects are not collected
        # until close() (or leaving the Trainer's `with` block) calls gc.unfreeze().
        self.freeze_gc = freeze_gc
        self._gc_frozen = False
        self._broken = None
        multi = dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1
        self.fp = FlatParams(module, status_words=64 if multi else 0)
        self.lr, self.wd, self.betas, self.eps, self.max_norm = lr, weight_decay, betas, eps, max_norm
        self.bucket_bytes = int(bucket_mb * (1 << 20))
        self.group = group
        self.exp_avg = torch.zeros_like(self.fp.flat)
        self.exp_avg_sq = torch.zeros_like(self.fp.flat)
        self.sumsq = torch.zeros(1, dtype=torch.float32, device=self.fp.flat.device)
        self.step_count = 0
        self.buckets = None
        if multi:
            src = dist.get_global_rank(group, 0) if group is not None else 0
            dist.broadcast(self.fp.flat, src, group=group)
            for b in module.buffers():
                if b.dtype.is_floating_point or b.dtype in (torch.int64, torch.int32):
                    dist.broadcast(b, src, group=group)
            self._bump_versions()
            self.buckets = _GradBuckets(self.fp, self.bucket_bytes, group)

    def set_hyperparams(self, lr=None, betas=None):
        """Per-step learning rate / momentum (the reference's cyclic lr and
        momentum schedules are applied by the caller through this)."""
        if lr is not None:
            self.lr = float(lr)
        if betas is not None:
            self.betas = tuple(betas)

    def _bump_versions(self):
        # the native AdamW (and the broadcast) write the parameters through their pointers: bump
        # Tensor._version so weight packs keyed on it (packing.PackCache) are rebuilt
        for p in self.fp.params:
            torch.autograd.graph.increment_version(p)

    def close(self):
        """Undo the process-wide gc.freeze() of ``freeze_gc`` and detach the
        gradient hooks; the Trainer takes no further step."""
        if self._gc_frozen:
            gc.unfreeze()
            self._gc_frozen = False
        if self.buckets is not None:
            for h in self.buckets.handles:
                h.remove()
            self.buckets = None
        self._broken = self._broken or "the Trainer was closed"

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

    def _check_usable(self):
        if self._broken:
            raise RuntimeError(f"Trainer unusable: {self._broken}")

    def backward(self, losses):
        """Backward of the summed losses into freshly zeroed flat gradients
        (no accumulation across calls: a second backward() before step()
        replaces the first one's gradients and exchange)."""
        self._check_usable()
        total = sum(losses.values()) if isinstance(losses, dict) else losses
        if self.buckets is not None:
            self.buckets.drain()   # outstanding all-reduces write fp.grad: finish them before zeroing it
        self.fp.zero_grad()
        # world size 1 (no accumulation hooks), no graph capture: the native backward adds each
        # Linear / LayerNorm weight gradient straight into the flat gradient buffer (train_ops)
        direct = self.buckets is None and not OPTIONS.train_graph
        try:
            with direct_param_grads(direct):
                total.backward()
        except BaseException:
            if self.buckets is not None and not self.buckets.abort():
                # every gradient was already exchanged: the other ranks apply this step and this
                # rank cannot, so its weights would drift from theirs -- refuse every later step
                self._broken = ("a backward raised after its last gradient bucket was exchanged; "
                                "the other ranks applied that step and this rank did not")
            raise
        return total

    def step(self, losses):
        self._check_usable()
        total = self.backward(losses)
        if self.buckets is not None:
            self.buckets.finish()
        self.step_count += 1
        self.sumsq.zero_()
        if self.max_norm and self.max_norm > 0:
            T.sumsq(self.fp.grad, self.sumsq)
        T.adamw_step(self.fp.flat, self.fp.grad, self.exp_avg, self.exp_avg_sq, step=self.step_count, lr=self.lr,
                     beta1=self.betas[0], beta2=self.betas[1], eps=self.eps, weight_decay=self.wd,
                     max_norm=self.max_norm or 0.0, sumsq_buf=self.sumsq)
        self._bump_versions()
        if self.freeze_gc and not self._gc_frozen:
            gc.collect()
            gc.freeze()
            self._gc_frozen = True
        return total.detach()

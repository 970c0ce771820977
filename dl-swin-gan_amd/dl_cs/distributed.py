"""Data-parallel gradient exchange for the unrolled network.

One cine slice per rank, parameters replicated; the only collective is the
gradient average (the reference's DDP all-reduce, train_swin.py:143 under
Lightning/DeepSpeed).  Gradients live in one flat fp32 bucket per distinct
regularizer network (param.grad are views into it); a bucket is all-reduced
asynchronously (RCCL over xGMI on GPU, gloo in the CPU tests) as soon as
backward has produced every gradient of that network, so the collective for
unroll i overlaps the backward of unrolls < i.

* SHARE_WEIGHTS (urs:61-63): one network used by every unroll gets one bucket,
  and its all-reduce starts after the LAST of its backward passes in the step
  (GRAD_READY callbacks are counted against the number of unrolls using it).
* Trainable parameters outside the regularizers (step_size when FIX_STEP_SIZE
  is False, urs:88-89; HQS lamda, urs:148) go into a final bucket that
  finish() reduces, so replicas never drift.
* Parameters the HIP path never touches (the unused SwinTransformer3D.norm,
  vst:633) get zero gradients outside the buckets.
* DLCS_FORCE_COLLECTIVES=1 (or collective=True) takes the multi-rank branches at
  world size 1 as well: with a one-rank RCCL communicator (a legal process group)
  the per-unroll async all-reduce, its wait and the exposed-wait events run on
  a single-GPU box exactly as they do in the driver's 8-rank run.
"""
import os
import time

import torch
import torch.distributed as dist


class GradBuckets:
    """direct=True (the fast path) makes the fused SwinNet backward write into
    the bucket views itself (swin3D.DIRECT_GRADS) and launch the bucket's
    all-reduce from swin3D.GRAD_READY; direct=False uses per-parameter
    post-accumulate-grad hooks (any autograd producer).

    Call zero() before every forward (it re-attaches the bucket views, so an
    optimizer.zero_grad(set_to_none=True) in between is harmless) and finish()
    after backward; close() unregisters the callback.

    Gradient accumulation: set `armed = False` for the micro-batches of a
    window that are not its last -- their backward accumulates into the
    buckets without starting an all-reduce (an all-reduce in flight while the
    next micro-batch accumulates into the same buffer would race, and the later
    micro-batches would never be reduced); the last micro-batch (armed = True,
    the default) starts them and finish() waits."""

    def __init__(self, model, world, direct=True, collective=None):
        from .models import swin3D
        self.world = world
        if collective is None:
            collective = world > 1 or os.environ.get("DLCS_FORCE_COLLECTIVES", "0") == "1"
        if collective and not dist.is_initialized():
            raise RuntimeError("dl_cs GradBuckets: collectives requested (world > 1 or DLCS_FORCE_COLLECTIVES=1) "
                               "without an initialised process group")
        self.collective = collective
        self.launched = 0                          # bucket all-reduces started (diagnostics / tests)
        self.direct = direct
        self.buckets, self.handles = [], []
        self.armed = True
        self.index, self.uses, self.seen, self.views = {}, {}, {}, {}
        nets = []
        regs = model.cnn_update if hasattr(model, "cnn_update") else model.nn_update      # Swin / ResNet, DiT
        for net in regs:
            if id(net) not in self.index:
                self.index[id(net)] = len(nets)
                self.uses[len(nets)] = 0
                nets.append(net)
            self.uses[self.index[id(net)]] += 1
        covered = set()
        self.unused = []
        for i, net in enumerate(nets):
            eps = net.engine_params() if hasattr(net, "engine_params") else dict(net.named_parameters())
            ps = list({id(p): p for p in eps.values() if p.requires_grad}.values())
            used = {id(p) for p in ps}
            for p in net.parameters():
                covered.add(id(p))
                if p.requires_grad and id(p) not in used:
                    self.unused.append(p)
            self.buckets.append(self._bucket(ps))
            if collective and not direct:
                for p in ps:
                    p.register_post_accumulate_grad_hook(self._hook(i, len(ps)))
        # everything else that trains (step size, HQS lamda): reduced in finish()
        extra = [p for p in model.parameters() if p.requires_grad and id(p) not in covered]
        self.extra = self._bucket(extra) if extra else None
        self._swin3D = swin3D
        if direct:
            swin3D.DIRECT_GRADS = True
            if collective:
                swin3D.GRAD_READY.append(self._ready)
        self.zero()

    @staticmethod
    def _bucket(ps):
        n = sum(p.numel() for p in ps)
        flat = torch.zeros(n, dtype=torch.float32, device=ps[0].device)
        return flat, ps

    def _attach(self, flat, ps):
        off = 0
        for p in ps:
            view = flat[off:off + p.numel()].view_as(p)
            self.views[id(p)] = view
            if p.grad is None or p.grad.data_ptr() != view.data_ptr():
                p.grad = view
            off += p.numel()

    def _home(self, p):
        """Put p.grad back into its bucket view if autograd replaced the tensor."""
        v = self.views[id(p)]
        if p.grad is not None and p.grad.data_ptr() != v.data_ptr():
            v.copy_(p.grad)
            p.grad = v

    def _launch(self, i):
        self.launched += 1
        self.handles.append(dist.all_reduce(self.buckets[i][0], op=dist.ReduceOp.SUM, async_op=True))

    def _ready(self, net):
        i = self.index.get(id(net))
        if i is None or not self.armed:
            return
        self.seen[i] = self.seen.get(i, 0) + 1
        if self.seen[i] == self.uses[i]:          # last backward pass of this network in the step
            self._launch(i)

    def _hook(self, i, n):
        # each parameter of the network fires once per backward (after all its uses)
        def fn(p):
            self._home(p)
            if not self.armed:
                return
            self.seen[i] = self.seen.get(i, 0) + 1
            if self.seen[i] == n:                  # autograd sums a shared leaf's uses before accumulating
                self._launch(i)
        return fn

    def _attached(self, ps):
        """True if the bucket's gradients are still its views: checked on the first and
        last parameter (an optimizer.zero_grad(set_to_none=True) or a replaced .grad
        detaches them all), so a steady step skips the per-parameter loop (~2 ms of
        host time at 10 unrolls)."""
        for p in (ps[0], ps[-1]):
            v = self.views.get(id(p))
            if v is None or p.grad is None or p.grad.data_ptr() != v.data_ptr():
                return False
        return True

    def zero(self):
        for flat, ps in self.buckets:
            flat.zero_()
            if not self._attached(ps):
                self._attach(flat, ps)
        if self.extra is not None:
            self.extra[0].zero_()
            self._attach(*self.extra)
        for p in self.unused:
            if p.grad is None:
                p.grad = torch.zeros_like(p)
        self.seen.clear()

    # Exposed-communication probe (bench.py): when a list, every finish() of a
    # multi-rank step appends (start_event, end_event, host_seconds) around its
    # waits -- the time the compute stream stood still for the all-reduces that
    # backward did not hide (events on the current stream; host time for gloo,
    # whose wait blocks the host).
    WAIT_PROFILE = None

    def finish(self):
        """Wait for the bucket all-reduces and turn sums into means."""
        if self.extra is not None:
            for p in self.extra[1]:
                self._home(p)
        for flat, ps in self.buckets:
            for p in (ps[0], ps[-1]):
                if p.grad is not None and p.grad.data_ptr() != self.views[id(p)].data_ptr():
                    raise RuntimeError("dl_cs GradBuckets: a gradient left its bucket between zero() and finish()")
        if not self.armed:
            raise RuntimeError("dl_cs GradBuckets: finish() on a disarmed micro-batch (set armed = True "
                               "for the last micro-batch of the accumulation window)")
        if self.collective:
            if len(self.handles) != len(self.buckets):
                raise RuntimeError(f"dl_cs GradBuckets: {len(self.handles)} of {len(self.buckets)} bucket "
                                   f"all-reduces were started by backward")
            prof = self.WAIT_PROFILE is not None
            if prof:
                cuda = self.buckets[0][0].is_cuda
                e0 = torch.cuda.Event(enable_timing=True) if cuda else None
                if cuda:
                    e0.record()
                t0 = time.perf_counter()
            for h in self.handles:
                h.wait()
            self.handles.clear()
            if self.extra is not None:
                dist.all_reduce(self.extra[0], op=dist.ReduceOp.SUM)
            if prof:
                e1 = torch.cuda.Event(enable_timing=True) if cuda else None
                if cuda:
                    e1.record()
                self.WAIT_PROFILE.append((e0, e1, time.perf_counter() - t0))
            if self.world > 1:
                for flat, _ in self.buckets + ([self.extra] if self.extra is not None else []):
                    flat.mul_(1.0 / self.world)

    def close(self):
        if self._ready in self._swin3D.GRAD_READY:
            self._swin3D.GRAD_READY.remove(self._ready)


def broadcast_parameters(model, src=0):
    """Identical replicas on every rank (rank src's initialisation)."""
    for p in model.parameters():
        dist.broadcast(p.data, src)

"""Data-parallel gradient exchange for the unrolled network.

One cine slice per rank, parameters replicated; the only collective is the
gradient average (the reference's DDP all-reduce, train_swin.py:143 under
Lightning/DeepSpeed).  Gradients live in one flat fp32 bucket per unroll
(param.grad are views into it); a bucket is all-reduced asynchronously (RCCL
over xGMI on GPU, gloo in the CPU tests) as soon as backward has produced every
gradient of that unroll, so the collective for unroll i overlaps the backward
of unrolls < i.  Parameters the HIP path never touches (the unused
SwinTransformer3D.norm, vst:633) get zero gradients outside the buckets.
"""
import torch
import torch.distributed as dist


class GradBuckets:
    """direct=True (the fast path) makes the fused SwinNet backward write into
    the bucket views itself (swin3D.DIRECT_GRADS) and launch the bucket's
    all-reduce from swin3D.GRAD_READY; direct=False uses per-parameter
    post-accumulate-grad hooks (any autograd producer)."""

    def __init__(self, model, world, direct=True):
        from .models import swin3D
        self.world = world
        self.direct = direct
        self.buckets, self.handles, self.pending = [], [], {}
        self.index = {}
        for i, net in enumerate(model.cnn_update):
            self.index[id(net)] = i
            ps = list({id(p): p for p in net.engine_params().values()}.values())
            used = {id(p) for p in ps}
            for p in net.parameters():
                if p.requires_grad and id(p) not in used:
                    p.grad = torch.zeros_like(p)
            n = sum(p.numel() for p in ps)
            flat = torch.zeros(n, dtype=torch.float32, device=ps[0].device)
            off = 0
            for p in ps:
                p.grad = flat[off:off + p.numel()].view_as(p)
                off += p.numel()
            self.buckets.append((flat, ps))
            if world > 1 and not direct:
                for p in ps:
                    p.register_post_accumulate_grad_hook(self._hook(i, len(ps)))
        if direct:
            swin3D.DIRECT_GRADS = True
            if world > 1:
                swin3D.GRAD_READY.append(self._ready)

    def _ready(self, net):
        i = self.index.get(id(net))
        if i is not None:
            self.handles.append(dist.all_reduce(self.buckets[i][0], op=dist.ReduceOp.SUM, async_op=True))

    def _hook(self, i, n):
        def fn(_):
            self.pending[i] = self.pending.get(i, 0) + 1
            if self.pending[i] == n:
                self.handles.append(dist.all_reduce(self.buckets[i][0], op=dist.ReduceOp.SUM, async_op=True))
        return fn

    def zero(self):
        for flat, _ in self.buckets:
            flat.zero_()
        self.pending.clear()

    def finish(self):
        """Wait for the bucket all-reduces and turn sums into means."""
        if self.world > 1:
            for h in self.handles:
                h.wait()
            self.handles.clear()
            for flat, _ in self.buckets:
                flat.mul_(1.0 / self.world)


def broadcast_parameters(model, src=0):
    """Identical replicas on every rank (rank src's initialisation)."""
    for p in model.parameters():
        dist.broadcast(p.data, src)

"""The training step's optimizer: torch.optim.Adam with the reference's arguments
(train_swin.py:155-166 passes only lr; betas / eps default), run as ONE fused
multi-tensor kernel per launch group when every parameter lives on the GPU.

The reference's torch.optim.Adam on CUDA takes the foreach path: per parameter group
a chain of multi_tensor_apply launches (98 launches per 10-unroll step here, for
~0.3 ms of HBM traffic).  fused=True is the same update rule (Adam, no AMSGrad, no
weight decay, bias-corrected moments) evaluated in one pass over p, grad, m, v.

The fused kernel does NOT bump the parameters' in-place version counters (the foreach
path does), and every packed-weight cache here is keyed by them (swin3D._net_weights,
engine._CONV_NORMS, dit_engine._packs, patchgan._patch_h3r): without the post-step
hook below the next forward would reuse the packing of the previous weights.  The
hook bumps every parameter's version after each step, so the caches rebuild exactly
as after a foreach step."""
import torch

from .. import diag as _diag


def adam(params, lr, fused=None, **kw):
    params = [p for p in params]
    if fused is None:
        fused = (bool(params) and all(p.is_cuda and p.dtype == torch.float32 for p in params)
                 and _diag.knob("DLCS_ADAM_FOREACH", "0") != "1")       # DIAG A/B: the foreach path
    if not fused:
        return torch.optim.Adam(params, lr=lr, foreach=True, **kw)
    opt = torch.optim.Adam(params, lr=lr, fused=True, **kw)
    opt.register_step_post_hook(lambda o, args, kwargs: torch.autograd.graph.increment_version(params))
    return opt

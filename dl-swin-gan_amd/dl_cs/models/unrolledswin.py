"""Unrolled reconstruction networks with the Swin regularizer, MI355X build.

Same classes, config keys and state_dict schema as the reference
(urs = dl_cs/models/unrolledswin.py).  ProximalGradientDescent runs each
data-consistency step as the fused SENSE normal operator + DC epilogue
(dlcs_sense_fwd / dlcs_sense_adj) when A is the HIP SenseModel, and each
regularizer as one fused kernel graph (SwinTransformer3DNet).
"""
import torch
from torch import nn
import torch.utils.checkpoint as cp

from .swin3D import SwinTransformer3DNet
from ..mri import transforms as T


class UnrolledSwinNet(nn.Module):
    """urs:15-75 -- abstract unrolled network."""

    def __init__(self, config):
        super().__init__()
        P = config.MODEL.PARAMETERS
        self.num_unrolls = P.NUM_UNROLLS
        self.num_swinblocks = P.NUM_SWINBLOCKS
        self.num_features = P.NUM_FEATURES
        self.kernel_size = P.CONV_BLOCK.KERNEL_SIZE[0]
        self.num_emaps = P.NUM_EMAPS
        self.share_weights = P.SHARE_WEIGHTS
        self.fix_step_size = P.FIX_STEP_SIZE
        self.use_complex_layers = P.CONV_BLOCK.COMPLEX
        self.circular_pad = P.CONV_BLOCK.CIRCULAR_PAD
        self.do_checkpoint = P.GRAD_CHECKPOINT
        self.window_size = P.WINDOW_SIZE          # read but unused, as in the reference (urs:33, s3d:315)
        self.num_heads = P.NUM_HEAD
        self.num_layers = P.NUM_LAYERS
        self.cnn_update = self.init_nets()

    def init_nets(self):
        """urs:40-68"""
        in_chans = self.num_emaps if self.use_complex_layers else 2 * self.num_emaps
        swin_params = dict(in_chans=in_chans, chans=self.num_features, num_swinblocks=self.num_swinblocks,
                           use_complex_layers=self.use_complex_layers, window_size=self.window_size,
                           kernel_size=self.kernel_size, circular_pad=self.circular_pad,
                           num_heads=self.num_heads, num_layers=self.num_layers)
        if self.share_weights:
            return nn.ModuleList([SwinTransformer3DNet(**swin_params)] * self.num_unrolls)
        return nn.ModuleList([SwinTransformer3DNet(**swin_params) for _ in range(self.num_unrolls)])

    def forward(self, y, A, x0=None):
        raise NotImplementedError


def _host_scalar(p):
    """float(p) of a fixed (no-grad) scalar parameter, read from the device once
    per (storage, in-place version) and cached ON the parameter: a per-unroll
    .item() would stall the host launch queue on every unroll.  (A cache keyed
    by address alone returned a freed parameter's value for a new one that the
    caching allocator placed at the same address.)"""
    key = (p.data_ptr(), p._version)
    c = getattr(p, "_dlcs_host_scalar", None)
    if c is None or c[0] != key:
        c = (key, float(p))
        p._dlcs_host_scalar = c
    return c[1]


def _dc_step(A, x, ATy, step_size):
    """urs:109 -- x + s * (A^H A x - A^H y)."""
    if isinstance(A, T.SenseModel) and not step_size.requires_grad:
        return A.normal_dc(x, ATy, _host_scalar(step_size))
    return x + step_size * (A(A(x), adjoint=True) - ATy)


class ProximalGradientDescent(UnrolledSwinNet):
    """urs:77-122 -- unrolled PGD: x <- R_i(x + s (A^H A x - A^H y)), s = -2 fixed."""

    def __init__(self, config):
        super().__init__(config)
        self.step_size = nn.Parameter(torch.tensor([-2.0], dtype=torch.float32),
                                      requires_grad=(not self.fix_step_size))

    def forward(self, y, A, x0=None):
        ATy = A(y, adjoint=True)
        xi = ATy if x0 is None else x0
        if self.training and self.do_checkpoint:
            xi.requires_grad_()

        def update(i):
            def update_fn(x):
                x = _dc_step(A, x, ATy, self.step_size)
                return self.cnn_update[i](x)
            return update_fn

        for i in range(self.num_unrolls):
            if self.do_checkpoint:
                xi = cp.checkpoint(update(i), xi, use_reentrant=False)
            else:
                xi = update(i)(xi)
        return xi


class HalfQuadraticSplitting(UnrolledSwinNet):
    """urs:125-172 -- HQS / MoDL with a conjugate-gradient data-consistency solve
    (the normal operator runs on the HIP SENSE kernels)."""

    def __init__(self, config):
        super().__init__(config)
        self.num_cg_iter = config.MODEL.PARAMETERS.MODL.NUM_CG_STEPS
        self.lamda = nn.Parameter(torch.tensor([0.1], dtype=torch.float32),
                                  requires_grad=(not self.fix_step_size))

    def _normal(self, A):
        """model_normal of urs:151.  HIP SenseModel: the fused normal operator
        (dlcs_sense_normal, lamda in its epilogue) when lamda is fixed; A^H A
        through the same call plus a differentiable lamda * m when it learns."""
        if isinstance(A, T.SenseModel) and A.maps.is_cuda:
            if not self.lamda.requires_grad:
                lam = _host_scalar(self.lamda)
                return lambda m: A.normal(m, lam)
            return lambda m: A.normal(m, 0.0) + self.lamda * m
        return lambda m: A(A(m), adjoint=True) + self.lamda * m

    def forward(self, y, A, x0=None):
        from ..mri.algorithms import ConjugateGradient
        ATy = A(y, adjoint=True)
        xi = ATy if x0 is None else x0
        if self.training and self.do_checkpoint:
            xi.requires_grad_()
        cg_solve = ConjugateGradient(self._normal(A), self.num_cg_iter)
        # no autograd needed: the whole CG solve stays on the device (dlcs_sense_cg)
        fused = (isinstance(A, T.SenseModel) and A.maps.is_cuda and not torch.is_grad_enabled())

        def update(i):
            def update_fn(x):
                z = self.cnn_update[i](x)
                b = ATy + self.lamda * z
                if fused:
                    return A.cg(x, b, _host_scalar(self.lamda), self.num_cg_iter)
                return cg_solve(x, b)
            return update_fn

        for i in range(self.num_unrolls):
            if self.do_checkpoint:
                xi = cp.checkpoint(update(i), xi, use_reentrant=False)
            else:
                xi = update(i)(xi)
        return xi

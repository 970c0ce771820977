"""Unrolled drivers with the DiT denoiser (BASELINE config 5), MI355X build.

Same classes, config keys, forward signatures and state_dict schema as the
reference (udit = dl_cs/models/unrolledDiT.py): the nn_update ModuleList of
DiTResNet networks (udit:41-92), DDPM (udit:102-135), DataConsistency
(udit:137-181, META_ARCHITECTURE "DDPM_X" of config_dit.yaml),
ProximalGradientDescent (udit:183-231) and HalfQuadraticSplitting
(udit:268-315).  Each DiTResNet call is one HIP autograd node
(dl_cs.models.dit_engine); the PGD data-consistency step is the fused SENSE
normal operator (dlcs_sense_normal) when A is the HIP SenseModel.
"""
import torch
from torch import nn
import torch.utils.checkpoint as cp

from .DiT import DiTResNet
from .unrolledswin import _dc_step, _host_scalar
from ..mri import transforms as T


class UnrolledDiTNet(nn.Module):
    """udit:16-98 (NET: the regularizer class -- DiTResNet here, LatteNet in
    unrolledLatte, whose drivers are otherwise identical)."""

    NET = DiTResNet

    def __init__(self, config):
        super().__init__()
        P = config.MODEL.PARAMETERS
        self.num_unrolls = P.NUM_UNROLLS
        self.num_blocks = P.NUM_RESBLOCKS
        self.num_features = P.NUM_FEATURES
        self.num_layers = P.NUM_LAYERS
        self.num_heads = P.NUM_HEADS
        self.kernel_size = P.CONV_BLOCK.KERNEL_SIZE[0]
        self.num_emaps = P.NUM_EMAPS
        self.share_weights = P.SHARE_WEIGHTS
        self.fix_step_size = P.FIX_STEP_SIZE
        self.use_complex_layers = P.CONV_BLOCK.COMPLEX
        self.circular_pad = P.CONV_BLOCK.CIRCULAR_PAD
        self.do_checkpoint = P.GRAD_CHECKPOINT
        self.learn_sigma = P.LEARN_SIGMA
        self.nn_update = self.init_nets()

    def init_nets(self):
        """udit:41-92 (LEARN_SIGMA True -- a final DiT predicting the variance for the
        VB loss -- is not built: config_dit.yaml sets it False)."""
        if self.learn_sigma:
            raise NotImplementedError("dl_cs DiT: LEARN_SIGMA False (config_dit.yaml)")
        in_chans = self.num_emaps if self.use_complex_layers else 2 * self.num_emaps
        params = dict(in_chans=in_chans, chans=self.num_features, num_blocks=self.num_blocks,
                      use_complex_layers=self.use_complex_layers, kernel_size=self.kernel_size,
                      circular_pad=self.circular_pad, num_heads=self.num_heads, num_layers=self.num_layers,
                      learn_sigma=False)
        if self.share_weights:
            return nn.ModuleList([self.NET(**params)] * self.num_unrolls)
        return nn.ModuleList([self.NET(**params) for _ in range(self.num_unrolls)])

    def _run(self, xi, update):
        if self.training and self.do_checkpoint:
            xi.requires_grad_()
        for i in range(self.num_unrolls):
            if self.do_checkpoint:
                xi = cp.checkpoint(update(i), xi, use_reentrant=False)
            else:
                xi = update(i)(xi)
        return xi

    def forward(self, y, A, t, c, x0=None):
        raise NotImplementedError


class DDPM(UnrolledDiTNet):
    """udit:102-135 -- the networks chained, no data consistency (DDPM_E)."""

    def forward(self, x0, t, A, A_1, A_F, fs, c):
        return self._run(x0, lambda i: (lambda x: self.nn_update[i](x, t, c)))


def _dc_project(x, x0, A, A_1, A_F):
    """udit:170 -- A_F^H (A_1 x + A x0) with A = S(maps, M), A_1 = S(maps, 1 - M),
    A_F = S(maps): the measured k-space of x0 replaces x's on the mask."""
    return A_F(A_1(x) + A(x0), adjoint=True)


class DataConsistency(UnrolledDiTNet):
    """udit:137-181 -- x <- A_F^H (A_1 R_i(x) + A x0) (META_ARCHITECTURE DDPM_X)."""

    def forward(self, x0, t, A, A_1, A_F, A_S, fs, c):
        def update(i):
            return lambda x: _dc_project(self.nn_update[i](x, t, c), x0, A, A_1, A_F)
        return self._run(x0, update)


class ProximalGradientDescent(UnrolledDiTNet):
    """udit:183-231 -- x <- R_i(x + s (A^H A x - x0)), ATy = x0 (the diffusion model
    feeds A^H y directly), s = -2 fixed."""

    def __init__(self, config):
        super().__init__(config)
        self.step_size = nn.Parameter(torch.tensor([-2.0], dtype=torch.float32),
                                      requires_grad=(not self.fix_step_size))

    def forward(self, x0, t, A, c):
        ATy = x0

        def update(i):
            return lambda x: self.nn_update[i](_dc_step(A, x, ATy, self.step_size), t, c)
        return self._run(x0, update)


class HalfQuadraticSplitting(UnrolledDiTNet):
    """udit:268-315 -- HQS / MoDL with the CG data-consistency solve on the HIP
    SENSE normal operator (as unrolledswin.HalfQuadraticSplitting)."""

    def __init__(self, config):
        super().__init__(config)
        self.num_cg_iter = config.MODEL.PARAMETERS.MODL.NUM_CG_STEPS
        self.lamda = nn.Parameter(torch.tensor([0.1], dtype=torch.float32),
                                  requires_grad=(not self.fix_step_size))

    def forward(self, y, t, A, c, x0=None):
        from ..mri.algorithms import ConjugateGradient
        from .unrolledswin import HalfQuadraticSplitting as _H
        ATy = A(y, adjoint=True)
        xi = ATy if x0 is None else x0
        cg_solve = ConjugateGradient(_H._normal(self, A), self.num_cg_iter)
        fused = isinstance(A, T.SenseModel) and A.maps.is_cuda and not torch.is_grad_enabled()

        def update(i):
            def fn(x):
                z = self.nn_update[i](x, t, c)
                b = ATy + self.lamda * z
                if fused:
                    return A.cg(x, b, _host_scalar(self.lamda), self.num_cg_iter)
                return cg_solve(x, b)
            return fn
        return self._run(xi, update)

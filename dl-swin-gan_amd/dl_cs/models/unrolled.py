"""Unrolled reconstruction networks with the 3D ResNet regularizer ("dlespirit",
BASELINE config 1, configs/example.yaml), MI355X build.

Same classes, config keys and state_dict schema as the reference
(ur = dl_cs/models/unrolled.py:15-172).  The data-consistency steps are the
Swin path's: the fused SENSE normal operator (PGD, ur:97-122) and the
device-resident conjugate gradient (HQS, ur:125-172); the regularizer is
resnet3d.ResNet on the HIP conv kernels.
"""
import torch
from torch import nn

from .resnet3d import ResNet
from . import unrolledswin as _us


class UnrolledNet(nn.Module):
    """ur:15-66 -- abstract unrolled network with ResNet regularizers."""

    def __init__(self, config):
        super().__init__()
        P = config.MODEL.PARAMETERS
        self.num_unrolls = P.NUM_UNROLLS
        self.num_resblocks = P.NUM_RESBLOCKS
        self.num_features = P.NUM_FEATURES
        self.kernel_size = P.CONV_BLOCK.KERNEL_SIZE[0]
        self.num_emaps = P.NUM_EMAPS
        self.share_weights = P.SHARE_WEIGHTS
        self.fix_step_size = P.FIX_STEP_SIZE
        self.use_complex_layers = P.CONV_BLOCK.COMPLEX
        self.circular_pad = P.CONV_BLOCK.CIRCULAR_PAD
        self.do_checkpoint = P.GRAD_CHECKPOINT
        self.cnn_update = self.init_nets()

    def init_nets(self):
        """ur:37-66"""
        in_chans = self.num_emaps if self.use_complex_layers else 2 * self.num_emaps
        params = dict(in_chans=in_chans, chans=self.num_features, num_resblocks=self.num_resblocks,
                      use_complex_layers=self.use_complex_layers, kernel_size=self.kernel_size,
                      circular_pad=self.circular_pad)
        if self.share_weights:
            return nn.ModuleList([ResNet(**params)] * self.num_unrolls)
        return nn.ModuleList([ResNet(**params) for _ in range(self.num_unrolls)])

    def forward(self, y, A, x0=None):
        raise NotImplementedError


class ProximalGradientDescent(UnrolledNet):
    """ur:69-122 -- x <- R_i(x + s (A^H A x - A^H y)), s = -2 (learnable unless FIX_STEP_SIZE)."""

    def __init__(self, config):
        super().__init__(config)
        self.step_size = nn.Parameter(torch.tensor([-2.0], dtype=torch.float32),
                                      requires_grad=(not self.fix_step_size))

    forward = _us.ProximalGradientDescent.forward


class HalfQuadraticSplitting(UnrolledNet):
    """ur:125-172 -- z = R_i(x); x <- CG(A^H A + lamda I, A^H y + lamda z)."""

    def __init__(self, config):
        super().__init__(config)
        self.num_cg_iter = config.MODEL.PARAMETERS.MODL.NUM_CG_STEPS
        self.lamda = nn.Parameter(torch.tensor([0.1], dtype=torch.float32),
                                  requires_grad=(not self.fix_step_size))

    _normal = _us.HalfQuadraticSplitting._normal
    forward = _us.HalfQuadraticSplitting.forward

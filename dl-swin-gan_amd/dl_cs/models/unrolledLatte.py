"""Unrolled drivers with the Latte denoiser (BASELINE config 5: config_latte.yaml),
MI355X build.

The reference's dl_cs/models/unrolledLatte.py is unrolledDiT.py with LatteNet in
place of DiTResNet (ulat:16-98 vs udit:16-98; the DDPM, DataConsistency,
ProximalGradientDescent and HalfQuadraticSplitting forwards are identical), so
these classes are the unrolledDiT drivers with NET = LatteNet: same names,
config keys, forward signatures and state_dict schema (nn_update.{i}.Latte...).
"""
from . import unrolledDiT as _udit
from .Latte import LatteNet


class UnrolledLatteNet(_udit.UnrolledDiTNet):
    """ulat:15-98"""
    NET = LatteNet


class DDPM(_udit.DDPM):
    """ulat:101-134"""
    NET = LatteNet


class DataConsistency(_udit.DataConsistency):
    """ulat:136-180 (META_ARCHITECTURE DDPM_X of config_latte.yaml)"""
    NET = LatteNet


class ProximalGradientDescent(_udit.ProximalGradientDescent):
    """ulat:182-265"""
    NET = LatteNet


class HalfQuadraticSplitting(_udit.HalfQuadraticSplitting):
    """ulat:267-315"""
    NET = LatteNet

"""Loss / metrics (met = dl_cs/utils/metrics.py:20-39, :121-125), LOSS_WEIGHT
support included.  Reductions run as device tensor ops (tiny, once per step)."""
import torch


def calc_weight(ref):
    """met:11-17 -- through-time std weighting.  The reference repeats |std_t|
    ([B, C, Y, X]) nt times along its Y axis and reinterprets that buffer as
    [B, C, nt, Y, X]; expanding a new axis after Y gives the same memory order."""
    B, C, nt, Y, X = ref.shape
    w = torch.abs(torch.std(ref, dim=2))
    return w.unsqueeze(3).expand(B, C, Y, nt, X).reshape(ref.shape)


def _w(ref, weight):
    return calc_weight(ref) if weight is True else None


def l2(ref, pred, weight=False):
    W = _w(ref, weight)
    d = ref - pred if W is None else W * (ref - pred)
    return torch.sqrt(torch.mean(torch.abs(d) ** 2))


def l1(ref, pred, weight=False):
    W = _w(ref, weight)
    d = ref - pred if W is None else W * (ref - pred)
    return torch.mean(torch.abs(d))


def psnr(ref, pred, weight=False):
    scale = torch.abs(ref).max()
    return 20 * torch.log10(scale / l2(ref, pred, weight))


def perp_loss(ref, pred, weight=False):
    """met:128-153"""
    W = calc_weight(ref) if weight is True else torch.ones(ref.shape, device=ref.device)
    assert ref.is_complex() and pred.is_complex()
    P = torch.abs(W * pred.real * ref.imag - W * pred.imag * ref.real) / torch.abs(W * ref)
    M = torch.abs(torch.abs(W * ref) - torch.abs(W * pred))
    return torch.mean(P + M)


def vggloss(ref, pred):
    raise NotImplementedError("VGG loss needs torchvision vgg16(pretrained=True) weights (out of scope)")

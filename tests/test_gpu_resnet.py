"""HIP "dlespirit" unrolled ResNet (BASELINE config 1, configs/example.yaml;
ur = dl_cs/models/unrolled.py, r3d = dl_cs/models/resnet3d.py) vs the
reference's own outputs: prediction, loss and every parameter gradient of a
2-unroll training step, and the state_dict schema.  Tolerances as the Swin PGD
test (test_gpu_swin.py): outputs NRMSE <= 1e-5, parameter gradients held to the
float64 floor with the HIP forward's ReLU decisions (goldutil.assert_masked_f64)."""
import pytest
import torch

from goldutil import HipMasks, assert_masked_f64, golden_err, grad_keys
from oracle import recipe

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _model(n, seed, hqs=False):
    from dl_cs.config import get_cfg
    from dl_cs.models import unrolled
    cfg = get_cfg()
    P = cfg.MODEL.PARAMETERS
    P.NUM_UNROLLS, P.NUM_RESBLOCKS, P.NUM_FEATURES, P.NUM_EMAPS = n, 2, 64, 1
    P.CONV_BLOCK.COMPLEX, P.FIX_STEP_SIZE = False, True
    m = (unrolled.HalfQuadraticSplitting if hqs else unrolled.ProximalGradientDescent)(cfg)
    m.eval()
    recipe.fill_module(m, seed)
    return m.to(DEV)


def test_resnet_pgd2_training_step(golden):
    from dl_cs.models import swin3D
    from dl_cs.mri import transforms as T
    swin3D.set_compute_dtype(torch.float32)
    g = golden("resnet")
    B, E, C, Tt, Y, X = 1, 1, 8, 20, 32, 32
    model = _model(2, 81)
    named = dict(model.named_parameters())
    assert set(grad_keys(g, "res2_")) <= set(named), "state_dict schema differs from the reference"
    maps = recipe.sense_maps(82, B, E, C, Y, X).to(DEV)
    mask = recipe.binary_mask(83, (B, 1, Tt, Y, X))
    y = (recipe.crandn(84, (B, C, Tt, Y, X)) * mask).to(DEV)
    target = recipe.crandn(85, (B, E, Tt, Y, X)).to(DEV)
    from dl_cs.models import engine
    engine.CAPTURE = []
    try:
        pred = model(y=y, A=T.SenseModel(maps, weights=mask.to(DEV)), x0=None)
    finally:
        caps, engine.CAPTURE = engine.CAPTURE, None
    loss = torch.mean(torch.abs(target - pred))
    loss.backward()
    assert golden_err(g, "res2_pred", pred) < 1e-5
    assert abs(float(loss) - float(g["res2_loss"])) < 1e-5 * float(g["res2_loss"])
    from oracle import dlcs_oracle as O
    mc, yc, tc = maps.cpu(), y.cpu(), target.cpu()

    def lf(P, c, mk):
        reg = lambda Pu, xu: O.resnet(Pu, xu, relu=mk.relu())                 # noqa: E731
        pred_o = O.pgd(O.split_unrolls(P, 2), c(yc), c(mc), c(mask), reg=reg)
        return torch.mean(torch.abs(c(tc) - pred_o))
    assert_masked_f64({n: p.grad for n, p in named.items() if p.grad is not None}, lf, model.state_dict(),
                      lambda k: "step_size" not in k, HipMasks(caps), "resnet pgd2")


def test_resnet_hqs_runs_and_matches_oracle():
    """HQS with the ResNet regularizer (ur:125-172) through the device CG vs the
    oracle's restatement (no reference golden for this combination)."""
    from oracle import dlcs_oracle as O
    from dl_cs.mri import transforms as T
    B, E, C, Tt, Y, X = 1, 1, 8, 20, 32, 32
    model = _model(2, 91, hqs=True)
    maps = recipe.sense_maps(92, B, E, C, Y, X)
    mask = recipe.binary_mask(93, (B, 1, Tt, Y, X))
    y = recipe.crandn(94, (B, C, Tt, Y, X)) * mask
    with torch.no_grad():
        pred = model(y=y.to(DEV), A=T.SenseModel(maps.to(DEV), weights=mask.to(DEV)), x0=None).cpu()
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    Ps = O.split_unrolls(sd, 2)
    ATy = O.sense_adjoint(y, maps, mask)
    x = ATy
    normal = lambda m: O.sense_adjoint(O.sense_forward(m, maps, mask), maps, mask) + 0.1 * m
    for P in Ps:
        x = O.conjugate_gradient(normal, x, ATy + 0.1 * O.resnet(P, x), 10)
    assert O.nrmse(x, pred) < 1e-5

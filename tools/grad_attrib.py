"""Per-tensor gradient error of the fp32 Swin regularizer vs a float64 oracle
evaluation with the HIP forward's ReLU decisions (the masked-f64 check of
tests/goldutil.py), printed for every parameter -- run once per kernel
configuration (env knobs are read once per process) to attribute the error:

    python tools/grad_attrib.py [X] [seed]
"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "dl-swin-gan_amd"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)
from goldutil import HipMasks, nrmse, oracle_grads  # noqa: E402
from oracle import dlcs_oracle as O  # noqa: E402
from oracle import recipe  # noqa: E402


def main():
    X = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 71
    nb = int(os.environ.get("NB", "1"))
    torch.set_num_threads(16)
    from dl_cs.models import engine, swin3D
    swin3D.set_compute_dtype(torch.float32)
    if os.environ.get("INPUT") == "aty":
        # bench.py's probe: the config_swin regularizer (default init) on the BASELINE
        # slice's A^H y
        import bench
        sys.argv = [sys.argv[0], "--nx", str(X)]
        args = bench.parse()
        model, _ = bench.build_model(args, torch.device("cuda", 0))
        net = model.cnn_update[0]
        net.eval()
        x = bench.make_slice(args, 0, torch.device("cuda", 0))["x0"].detach().cpu()
        nb = net.num_swinblocks if hasattr(net, "num_swinblocks") else nb
    else:
        net = swin3D.SwinTransformer3DNet(num_swinblocks=nb, in_chans=4, chans=160, kernel_size=3,
                                          window_size=(4, 4))
        net.eval()
        recipe.fill_module(net, seed)
        net = net.cuda()
        x = recipe.crandn(seed + 1, (1, 2, 20, 192, X))
    engine.CAPTURE = []
    try:
        y = net(x.cuda())
    finally:
        caps, engine.CAPTURE = engine.CAPTURE, None
    g = recipe.crandn(seed + 2, y.shape)
    (y.real * g.real.cuda() + y.imag * g.imag.cuda()).sum().backward()
    hip = {n: p.grad.detach().cpu().double().numpy() for n, p in net.named_parameters() if p.grad is not None}
    masks = HipMasks(caps)

    def lf(P, c, mk):
        yo, gc = O.swinnet(P, c(x), num_swinblocks=nb, relu=mk.relu()), c(g)
        return (yo.real * gc.real + yo.imag * gc.imag).sum()
    tr = lambda k: "relative_position_index" not in k           # noqa: E731
    masks.reset()
    o32 = oracle_grads(lambda P, c: lf(P, c, masks), net.state_dict(), torch.float32, tr)
    masks.relus = []
    masks.reset()
    o64 = oracle_grads(lambda P, c: lf(P, c, masks), net.state_dict(), torch.float64, tr)
    rows = []
    for n in sorted(set(hip) & set(o64)):
        fl = nrmse(o64[n], o32[n])
        er = nrmse(o64[n], hip[n])
        rows.append((er / max(1e-5, 4 * fl), er, fl, n))
    rows.sort(reverse=True)
    knobs = {k: v for k, v in os.environ.items() if k.startswith("DLCS_")}
    print(f"config {knobs or 'default'}  X={X} nb={nb}: {len(rows)} grads; "
          f"{sum(r[0] > 1 for r in rows)} over max(1e-5, 4 floor)")
    for r in rows[:24]:
        print(f"  ratio {r[0]:7.3f}  err {r[1]:.3e}  floor {r[2]:.3e}  {r[3]}")
    print("  outside the Swin blocks:")
    for r in rows:
        if ".blocks." not in r[3]:
            print(f"  ratio {r[0]:7.3f}  err {r[1]:.3e}  floor {r[2]:.3e}  {r[3]}")
    print(f"  median err {np.median([r[1] for r in rows]):.3e}  median floor {np.median([r[2] for r in rows]):.3e}")


if __name__ == "__main__":
    main()

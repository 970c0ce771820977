"""bench.py's grad_nrmse_vs_f64 probe after the bench's own training history:
n_fp32 fp32 train steps (the headline phase), n_bf16 bf16 steps (the secondary
phase), n_full more fp32 steps (the all-branches phase), then the probe -- run once
per kernel configuration (env knobs are read once per process).

    python tools/grad_trained_diag.py [n_fp32 n_bf16 n_full]
"""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def main():
    n32, n16, nfull = (int(a) for a in (sys.argv[1:4] if len(sys.argv) > 3 else (13, 11, 11)))
    sys.argv = sys.argv[:1]
    args = bench.parse()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from dl_cs.distributed import GradBuckets
    from dl_cs.models import swin3D
    from dl_cs.mri import transforms as T
    model, cfg = bench.build_model(args, dev)
    model.train()
    data = bench.make_slice(args, 0, dev)
    A = T.SenseModel(data["maps"], weights=data["mask"])
    opt = torch.optim.Adam([p for p in model.parameters() if p.requires_grad], lr=cfg.OPTIMIZER.ADAM.LR, foreach=True)
    buckets = GradBuckets(model, 1)

    def step():
        buckets.zero()
        pred = model(y=data["y"], A=A, x0=data["x0"])
        loss = torch.mean(torch.abs(data["target"] - pred))
        loss.backward()
        buckets.finish()
        opt.step()

    for dt, n in ((torch.float32, n32), (torch.bfloat16, n16), (torch.float32, nfull)):
        swin3D.set_compute_dtype(dt)
        for _ in range(n):
            step()
    torch.cuda.synchronize()
    r = bench.grad_accuracy(model, data, 16)
    knobs = {k: v for k, v in os.environ.items() if k.startswith("DLCS_")}
    print(json.dumps({"knobs": knobs, "steps": [n32, n16, nfull], "max": r["max_nrmse"], "median": r["median_nrmse"],
                      "over_bar": r["over_bar"], "worst": r["worst"]}))


if __name__ == "__main__":
    main()

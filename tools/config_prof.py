"""One BASELINE config phase of bench.py on its own, for rocprofv3 kernel traces:
    python tools/config_prof.py {gan|dit|latte|config2} [steps]
Prints the phase's bench entry (JSON) on one line."""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def main():
    which = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    sys.argv = [sys.argv[0]]
    args = bench.parse()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    data = bench.make_slice(args, 0, dev)
    if which == "dit":
        res = bench.dit_phase(args, dev, data, steps)
    elif which == "latte":
        res = bench.dit_phase(args, dev, data, steps, "config_latte.yaml")
    elif which == "config2":
        res = bench.config2_phase(args, dev, data, steps)
    elif which == "gan":
        from dl_cs.distributed import GradBuckets
        from dl_cs.mri import transforms as T
        model, cfg = bench.build_model(args, dev)
        model.train()
        A = T.SenseModel(data["maps"], weights=data["mask"])
        opt = torch.optim.Adam([p for p in model.parameters() if p.requires_grad], lr=cfg.OPTIMIZER.ADAM.LR,
                               foreach=True)
        buckets = GradBuckets(model, 1)
        res = bench.gan_phase(args, model, data, A, buckets, opt, steps)
    else:
        raise SystemExit(f"unknown phase {which}")
    print(json.dumps({which: res}))


if __name__ == "__main__":
    main()

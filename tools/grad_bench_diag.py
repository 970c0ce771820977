"""bench.py's grad_nrmse_vs_f64 probe in isolation: fresh model from config_swin
(no training steps, no gradient buckets), the BASELINE slice's A^H y input; then
the same with recipe-random weights, and with a recipe-random input.
    python tools/grad_bench_diag.py [X]"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import bench  # noqa: E402
from oracle import recipe  # noqa: E402


def main():
    X = int(sys.argv[1]) if len(sys.argv) > 1 else 160
    sys.argv = [sys.argv[0], "--nx", str(X)]
    args = bench.parse()
    dev = torch.device("cuda", 0)
    model, cfg = bench.build_model(args, dev)
    data = bench.make_slice(args, 0, dev)
    r = bench.grad_accuracy(model, data, 16)
    print("config model, A^H y input:", {k: r[k] for k in ("max_nrmse", "median_nrmse", "over_bar")}, r["worst"])
    net = model.cnn_update[0]
    recipe.fill_module(net, 71)
    r = bench.grad_accuracy(model, data, 16)
    print("recipe weights, A^H y input:", {k: r[k] for k in ("max_nrmse", "median_nrmse", "over_bar")}, r["worst"])
    data = dict(data, x0=recipe.crandn(72, tuple(data["x0"].shape)).to(dev))
    r = bench.grad_accuracy(model, data, 16)
    print("recipe weights, recipe input:", {k: r[k] for k in ("max_nrmse", "median_nrmse", "over_bar")}, r["worst"])


if __name__ == "__main__":
    main()

"""Per-shape GEMM time of one training step (--dtype bf16|fp32) (10-unroll PGD, BASELINE slice)."""
import collections
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "dl-swin-gan_amd"))
import torch  # noqa: E402
import bench  # noqa: E402
from dl_cs.models import _ops, swin3D  # noqa: E402

args = bench.parse()
swin3D.set_compute_dtype(torch.bfloat16 if args.dtype == "bf16" else torch.float32)
dev = torch.device("cuda", 0)
model, cfg = bench.build_model(args, dev)
model.train()
data = bench.make_slice(args, 0, dev)
from dl_cs.mri import transforms as T  # noqa: E402
A = T.SenseModel(data["maps"], weights=data["mask"])


def step():
    model.zero_grad(set_to_none=False)
    pred = model(y=data["y"], A=A, x0=data["x0"])
    torch.mean(torch.abs(data["target"] - pred)).backward()


step()
torch.cuda.synchronize()
_ops.GEMM_TRACE = []
step()
torch.cuda.synchronize()
agg = collections.defaultdict(lambda: [0, 0.0])
for key, e0, e1 in _ops.GEMM_TRACE:
    agg[key][0] += 1
    agg[key][1] += e0.elapsed_time(e1)
tot = sum(v[1] for v in agg.values())
print(f"GEMM total {tot:.2f} ms over {len(_ops.GEMM_TRACE)} calls")
print("   ms  calls   us/call  TF/s   (M, N, K, a_t, b_t, act, splitk, acc, C, rowmap)")
for key, (n, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    M, N, K = key[:3]
    print(f"{ms:7.2f} {n:5d} {1000 * ms / n:9.1f} {2.0 * M * N * K * n / (ms * 1e-3) / 1e12:6.1f}   {key}")

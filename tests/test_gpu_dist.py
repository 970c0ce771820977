"""The data-parallel step with REAL gradients: two ranks on the one
GPU (gloo over GPU tensors -- RCCL refuses two ranks per device), each running
the HIP fused forward + backward of a 2-unroll PGD on its own slice, gradients
written straight into the bucket views and all-reduced per network from the
backward (GradBuckets direct mode).  Rank 0 then recomputes each slice's
gradients single-process and checks that the bucket average equals their mean
(fp32, NRMSE <= max(1e-5, 4x the run-to-run floor of the same slice's
gradients: the step's reductions are fixed-order -- the weight gradients'
per-range slabs and the split-K partials are summed by separate kernels in a
fixed order -- so the floor is normally 0; the max() keeps the bar meaningful
should a reduction ever become order-dependent))."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _setup(rank):
    import sys
    for p in (REPO, os.path.join(REPO, "dl-swin-gan_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    from oracle import recipe
    from dl_cs.config import get_cfg
    from dl_cs.models import swin3D, unrolledswin
    swin3D.set_compute_dtype(torch.float32)
    cfg = get_cfg()
    cfg.merge_from_file(os.path.join(REPO, "configs", "config_swin.yaml"))
    P = cfg.MODEL.PARAMETERS
    P.NUM_UNROLLS = 2
    model = unrolledswin.ProximalGradientDescent(cfg)
    model.eval()                                     # DropPath off: deterministic gradients
    recipe.fill_module(model, 21)
    return model.cuda(), recipe


def _slice(recipe, r):
    B, E, C, T, Y, X = 1, 2, 8, 4, 32, 32
    maps = recipe.sense_maps(100 + r, B, E, C, Y, X).cuda()
    mask = recipe.binary_mask(200 + r, (B, 1, T, Y, X)).cuda()
    target = recipe.crandn(300 + r, (B, E, T, Y, X)).cuda()
    return maps, mask, target


def _loss(model, maps, mask, target):
    from dl_cs.mri import transforms as T
    A = T.SenseModel(maps, weights=mask)
    y = A(target)
    return torch.mean(torch.abs(target - model(y=y, A=A)))


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    model, recipe = _setup(rank)
    from dl_cs.distributed import GradBuckets
    from dl_cs.models import swin3D
    buckets = GradBuckets(model, world)
    buckets.zero()
    _loss(model, *_slice(recipe, rank)).backward()
    buckets.finish()
    buckets.close()
    avg = {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}
    ok = True
    if rank == 0:
        swin3D.DIRECT_GRADS = False                  # plain autograd gradients for the reference
        single = []
        for r in list(range(world)) + [0]:           # slice 0 twice: the run-to-run floor
            model.zero_grad(set_to_none=True)
            _loss(model, *_slice(recipe, r)).backward()
            single.append({n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None})

        def err(a, b):
            den = float(torch.linalg.vector_norm(b.double()))
            return float(torch.linalg.vector_norm(a.double() - b.double())) / den if den > 0 else 0.0

        errs, floor = {}, {}
        for n, g in avg.items():
            if n not in single[0]:
                continue
            errs[n] = err(g, (single[0][n].double() + single[1][n].double()) / world)
            floor[n] = err(single[2][n], single[0][n])
        worst = max(errs.values())
        top = sorted(errs, key=lambda n: -errs[n])[:4]
        ok = all(errs[n] <= max(1e-5, 4 * floor[n]) for n in errs)
        with open(os.path.join(out_dir, "worst.txt"), "w") as f:
            f.write(f"{worst:.3e} " + " ".join(f"{n}={errs[n]:.2e}/floor {floor[n]:.2e}" for n in top))
    with open(os.path.join(out_dir, f"rank{rank}.txt"), "w") as f:
        f.write("ok" if ok else "fail")
    dist.barrier()
    dist.destroy_process_group()


def test_dp_step_real_gradients_two_ranks(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    worst = (tmp_path / "worst.txt").read_text()
    for r in range(world):
        assert (tmp_path / f"rank{r}.txt").read_text() == "ok", worst

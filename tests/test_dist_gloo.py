"""Multi-rank path on CPU (gloo, world size 2): replica broadcast and the
per-unroll bucketed gradient average of dl_cs.distributed (the only collective
of the data-parallel step); the GPU run uses the same code over
RCCL."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _model(seed):
    from dl_cs.config import get_cfg
    from dl_cs.models import unrolledswin
    cfg = get_cfg()
    cfg.merge_from_file(os.path.join(REPO, "configs", "config_swin.yaml"))
    cfg.MODEL.PARAMETERS.NUM_UNROLLS = 2
    torch.manual_seed(seed)
    return unrolledswin.ProximalGradientDescent(cfg)


def _worker(rank, world, port, out_dir, direct):
    import sys
    sys.path.insert(0, os.path.join(REPO, "dl-swin-gan_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    from dl_cs.distributed import GradBuckets, broadcast_parameters
    model = _model(1000 + rank)                  # different init per rank ...
    broadcast_parameters(model, 0)               # ... made identical by the broadcast
    from dl_cs.models import swin3D
    buckets = GradBuckets(model, world, direct=direct)
    ok = []
    for step in range(2):                        # the buckets are reused across steps
        buckets.zero()
        if direct:
            # what the fused SwinNet backward does: accumulate into p.grad in
            # place, then announce the finished unroll (last unroll first)
            for i, net in reversed(list(enumerate(model.cnn_update))):
                for k, (name, p) in enumerate(sorted(net.engine_params().items())):
                    p.grad.add_((rank + 1) * (step + 1) * (k + 1) * (i + 1))
                for cb in swin3D.GRAD_READY:
                    cb(net)
        else:
            loss = 0.0
            for i, net in enumerate(model.cnn_update):
                for k, (name, p) in enumerate(sorted(net.engine_params().items())):
                    loss = loss + (rank + 1) * (step + 1) * (k + 1) * (i + 1) * p.sum()
            loss.backward()
        buckets.finish()
        mean_scale = sum(r + 1 for r in range(world)) / world
        for i, net in enumerate(model.cnn_update):
            flat = buckets.buckets[i][0]
            lo, hi = flat.data_ptr(), flat.data_ptr() + flat.numel() * 4
            for k, (name, p) in enumerate(sorted(net.engine_params().items())):
                want = mean_scale * (step + 1) * (k + 1) * (i + 1)
                ok.append(bool(torch.all(p.grad == want)))
                ok.append(lo <= p.grad.data_ptr() < hi)          # still a view into the bucket
            used = {id(p) for p in net.engine_params().values()}
            for p in net.parameters():
                if id(p) not in used and p.requires_grad:
                    ok.append(bool(torch.all(p.grad == 0)))
    first = next(iter(model.parameters())).detach().clone()
    others = [torch.zeros_like(first) for _ in range(world)]
    dist.all_gather(others, first)
    ok.append(all(torch.equal(o, first) for o in others))
    with open(os.path.join(out_dir, f"rank{rank}.txt"), "w") as f:
        f.write("ok" if all(ok) else f"fail {ok.count(False)} of {len(ok)}")
    dist.destroy_process_group()


@pytest.mark.parametrize("direct", [False, True])
def test_bucketed_grad_allreduce_gloo(tmp_path, direct):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), direct), nprocs=world, join=True)
    for r in range(world):
        assert (tmp_path / f"rank{r}.txt").read_text() == "ok"

"""The RCCL branch of the data-parallel step on a single-GPU box (SURVEY 8(e);
reference entry: `Trainer(gpus=devices)`, scripts/train_swin.py:253-261).

The driver's 1->8 GPU run goes through code that gloo never touches: the nccl
process group (`bench.py`, `init_process_group("nccl", device_id=...)`), the
async per-unroll bucket all-reduce launched from inside the fused backward
(`GradBuckets._ready` via `swin3D.GRAD_READY`), `Work.wait()` on the compute
stream and the exposed-wait events.  A one-rank RCCL communicator is legal, and
`GradBuckets(collective=True)` / `DLCS_FORCE_COLLECTIVES=1` take every
multi-rank branch at world size 1, so this file runs that path here:

* in a fresh spawned process, a 2-unroll PGD training step with the nccl
  process group: every bucket is snapshotted the moment backward hands it to
  RCCL; after `finish()` each bucket must be BITWISE its snapshot (an all-reduce
  SUM over one rank is the identity; the 1/world scale is skipped at world 1),
  the number of all-reduces must equal the number of buckets, and the gradients
  must match a run without any process group within the run-to-run floor;
* `bench.py --gpus 1` under DLCS_FORCE_COLLECTIVES=1 prints backend "nccl" with
  the `allreduce` block filled from RCCL events.
"""
import json
import os
import socket
import subprocess
import sys

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


def _worker(rank, port, out_dir):
    for p in (REPO, os.path.join(REPO, "dl-swin-gan_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    from oracle import recipe
    from dl_cs.config import get_cfg
    from dl_cs.distributed import GradBuckets
    from dl_cs.models import swin3D, unrolledswin
    from dl_cs.mri import transforms as T
    msg = "ok"
    try:
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        swin3D.set_compute_dtype(torch.float32)
        cfg = get_cfg()
        cfg.merge_from_file(os.path.join(REPO, "configs", "config_swin.yaml"))
        cfg.MODEL.PARAMETERS.NUM_UNROLLS = 2
        model = unrolledswin.ProximalGradientDescent(cfg)
        model.eval()                                  # DropPath off: the same computation every run
        recipe.fill_module(model, 21)
        model = model.to(dev)
        B, E, C, Tt, Y, X = 1, 2, 8, 4, 32, 32
        maps = recipe.sense_maps(100, B, E, C, Y, X).to(dev)
        mask = recipe.binary_mask(200, (B, 1, Tt, Y, X)).to(dev)
        target = recipe.crandn(300, (B, E, Tt, Y, X)).to(dev)
        A = T.SenseModel(maps, weights=mask)
        y = A(target)

        def step(buckets):
            buckets.zero()
            torch.mean(torch.abs(target - model(y=y, A=A))).backward()
            buckets.finish()
            return {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}

        # no process group: the single-process gradients, twice (run-to-run floor)
        b0 = GradBuckets(model, 1, collective=False)
        g_ref, g_ref2 = step(b0), step(b0)
        b0.close()

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        assert dist.get_backend() == "nccl", dist.get_backend()
        bk = GradBuckets(model, 1, collective=True)
        snaps = {}

        def snap(net):                                # runs before GradBuckets._ready enqueues the all-reduce
            i = bk.index[id(net)]
            snaps[i] = bk.buckets[i][0].clone()
        swin3D.GRAD_READY.insert(0, snap)
        try:
            g_nccl = step(bk)
        finally:
            swin3D.GRAD_READY.remove(snap)
        launched = bk.launched
        bk.close()
        torch.cuda.synchronize()
        if launched != len(bk.buckets):
            msg = f"{launched} all-reduces for {len(bk.buckets)} buckets"
        elif sorted(snaps) != list(range(len(bk.buckets))):
            msg = f"snapshots of buckets {sorted(snaps)}"
        else:
            for i, (flat, _) in enumerate(bk.buckets):
                if not torch.equal(flat, snaps[i]):
                    d = (flat - snaps[i]).abs().max().item()
                    msg = f"bucket {i}: RCCL all-reduce over one rank changed the data (max |diff| {d:.3e})"
                    break
        if msg == "ok":
            def err(a, b):
                den = float(torch.linalg.vector_norm(b.double()))
                return float(torch.linalg.vector_norm(a.double() - b.double())) / den if den > 0 else 0.0
            for n in g_ref:
                e, fl = err(g_nccl[n], g_ref[n]), err(g_ref2[n], g_ref[n])
                if e > max(1e-6, 4 * fl):
                    msg = f"{n}: nccl-path gradient NRMSE {e:.3e} vs the no-process-group run (floor {fl:.3e})"
                    break
        dist.barrier()
        dist.destroy_process_group()
    except Exception as ex:                           # noqa: BLE001 -- reported through the file
        msg = f"exception: {type(ex).__name__}: {ex}"
    with open(os.path.join(out_dir, "rccl.txt"), "w") as f:
        f.write(msg)


def test_gradbuckets_rccl_world1_bitwise(tmp_path):
    mp.spawn(_worker, args=(_free_port(), str(tmp_path)), nprocs=1, join=True)
    assert (tmp_path / "rccl.txt").read_text() == "ok"


def test_bench_forced_collectives_nccl():
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env["DLCS_FORCE_COLLECTIVES"] = "1"
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "1", "--steps", "2", "--warmup", "1",
                        "--unrolls", "2", "--frames", "4", "--ny", "32", "--nx", "32", "--no-secondary", "--no-configs",
                        "--no-cpu-baseline", "--no-all-branches"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=REPO)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 1 and line["world_size"] == 1 and line["backend"] == "nccl"
    ar = line["allreduce"]
    assert ar is not None and ar["backend"] == "nccl" and ar["world_size"] == 1
    assert ar["allreduces_per_step"] == 2                      # one bucket per unroll (no shared weights)
    assert len(ar["exposed_allreduce_ms_per_step"]) == 1 and ar["exposed_allreduce_ms_per_step"][0] >= 0.0
    assert line["value"] > 0 and line["loss"] == line["loss"]

"""Headline benchmark: cine slices/s of the Swin-unrolled PGD training step.

BASELINE.json metric: "cine slices/sec (fwd+bwd) at 10-iter unroll, 1/2/4/8 GPU;
PSNR vs ref".  One step = one training iteration on one synthetic cine slice
per rank (8 coils x 20 frames x 192 x 160, 2 ESPIRiT maps, VDkt mask, seed
1000): forward through 10 unrolls (SENSE normal op + Swin regularizer), complex
L1 loss, backward, RCCL gradient all-reduce (N > 1), Adam step.  Inputs are
resident in HBM before timing.  Weak scaling: one slice per rank.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    (N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N)

Prints ONE JSON line on rank 0 (see the harness contract in DESIGN.md).
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "dl-swin-gan_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

MI355X_BF16_DENSE_TFLOPS = 2500.0      # MI355X_MICROARCH.md chip table (dense, no sparsity)
MI355X_FP32_TFLOPS = 157.3
MI355X_HBM_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--unrolls", type=int, default=10)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--coils", type=int, default=8)
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--ny", type=int, default=192)
    ap.add_argument("--nx", type=int, default=160)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0)
    return ap.parse_args()


def vdkt_mask(T, Y, X):
    """VDktMaskFunc((10,15), partial_kx=.25, partial_ky=.25), seed 1000, produced by
    the reference (tests/golden/misc.npz, data only); recipe mask for other sizes."""
    if (T, Y, X) == (20, 192, 160):
        g = np.load(os.path.join(REPO, "tests", "golden", "misc.npz"))
        bits = np.unpackbits(g["vdkt_seed1000_bits"])[: 20 * 192 * 160]
        return torch.from_numpy(bits.reshape(1, 1, T, Y, X).astype(np.float32))
    gen = torch.Generator().manual_seed(1000)
    return (torch.rand((1, 1, T, Y, X), generator=gen) < 0.08).float()


def make_slice(args, rank, dev):
    from dl_cs.mri import transforms as T
    gen = torch.Generator().manual_seed(1000 + rank)
    E, C, Tt, Y, X = 2, args.coils, args.frames, args.ny, args.nx
    x_true = torch.complex(torch.randn((1, E, Tt, Y, X), generator=gen), torch.randn((1, E, Tt, Y, X), generator=gen))
    maps = torch.complex(torch.randn((1, E, C, 1, Y, X), generator=gen), torch.randn((1, E, C, 1, Y, X), generator=gen))
    maps = maps / torch.sqrt((maps.abs() ** 2).sum(dim=(1, 2), keepdim=True))      # sum_{e,c} |S|^2 = 1
    mask = vdkt_mask(Tt, Y, X)
    x_true, maps, mask = x_true.to(dev), maps.to(dev), mask.to(dev)
    A = T.SenseModel(maps, weights=mask)
    with torch.no_grad():
        y = A(x_true)
        x0 = A(y, adjoint=True)
    return dict(y=y, maps=maps, mask=mask, x0=x0, target=x_true)


def build_model(args, dev):
    from dl_cs.config import get_cfg
    from dl_cs.models import unrolledswin
    cfg = get_cfg()
    cfg.merge_from_file(os.path.join(REPO, "configs", "config_swin.yaml"))
    cfg.MODEL.PARAMETERS.NUM_UNROLLS = args.unrolls
    torch.manual_seed(cfg.SEED)
    return unrolledswin.ProximalGradientDescent(cfg).to(dev), cfg


def pmc_traffic(dtype):
    """HBM bytes per launch of the roofline kernel from the newest committed PMC
    pass (profiles/*_traffic_conv3d_k3_v5.json, tools/profile_round.sh); the
    bf16 kernel only."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "*_traffic_conv3d_k3_v5.json")))
    if dtype != "bf16" or not files:
        return None
    with open(files[-1]) as f:
        return json.load(f)["hbm_bytes_per_launch"]


def secondary(prof, bound, peak, unit, scale, what):
    """Roofline entry of a secondary kernel from (start, end, algorithmic work) events."""
    if not prof:
        return None
    ms = [e0.elapsed_time(e1) for e0, e1, _ in prof]
    work = float(np.mean([w for _, _, w in prof]))
    achieved = work / (float(np.mean(ms)) * 1e-3) / scale
    return {"bound": bound, "kernel": what, "achieved": achieved, "peak": peak, "unit": unit,
            "frac": achieved / peak, "launches": len(ms), "avg_us": 1e3 * float(np.mean(ms)),
            "work_per_launch": work}


def cpu_baseline(model, data, args, threads):
    """The oracle (fp32 PyTorch-CPU restatement, pinned to the reference's goldens)
    timed on one of the `unrolls` unrolls at full size, fwd+bwd, scaled to a slice."""
    sys.path.insert(0, REPO)
    from oracle import dlcs_oracle as O
    torch.set_num_threads(threads)
    net0 = model.cnn_update[0]
    P = {k: v.detach().float().cpu().clone().requires_grad_(torch.is_floating_point(v) and
                                                              "relative_position_index" not in k)
         for k, v in net0.state_dict().items()}
    maps, mask = data["maps"].cpu(), data["mask"].cpu()
    y, x0, target = data["y"].cpu(), data["x0"].cpu(), data["target"].cpu()
    t0 = time.perf_counter()
    aty = O.sense_adjoint(y, maps, mask)
    x = x0.clone().requires_grad_()
    xx = x + (-2.0) * (O.sense_adjoint(O.sense_forward(x, maps, mask), maps, mask) - aty)
    out = O.swinnet(P, xx)
    loss = O.l1(target, out)
    loss.backward()
    dt = time.perf_counter() - t0
    slices_per_s = 1.0 / (dt * args.unrolls)
    # parity: the same unroll on the GPU path (eval semantics, compute dtype) vs the fp32 oracle
    with torch.no_grad():
        model.eval()
        from dl_cs.mri import transforms as T
        A = T.SenseModel(data["maps"], weights=data["mask"])
        aty_g = A(data["y"], adjoint=True)
        xg = A.normal_dc(data["x0"], aty_g, -2.0)
        out_g = net0(xg).cpu()
        model.train()
    ref = out.detach().to(torch.complex128)
    rmse = torch.sqrt(torch.mean(torch.abs(out_g.to(torch.complex128) - ref) ** 2))
    psnr = float(20 * torch.log10(ref.abs().max() / rmse))
    nrmse = float(torch.linalg.vector_norm(out_g.to(torch.complex128) - ref) / torch.linalg.vector_norm(ref))
    return dict(value=slices_per_s, unit="slices/s", cores=threads, kind="port",
                sample=f"1 of {args.unrolls} unrolls (SENSE normal op + SwinTransformer3DNet) fwd+bwd at "
                       f"{tuple(data['y'].shape)} k-space, fp32, {dt:.2f} s, scaled x{args.unrolls}"), \
        dict(psnr_db=psnr, nrmse=nrmse, what="1 unroll, GPU path vs fp32 CPU oracle, same weights/input")


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    from dl_cs.models import engine, swin3D
    from dl_cs.distributed import GradBuckets, broadcast_parameters
    swin3D.set_compute_dtype(torch.bfloat16 if args.dtype == "bf16" else torch.float32)
    model, cfg = build_model(args, dev)
    model.train()
    if world > 1:
        broadcast_parameters(model, 0)
    data = make_slice(args, rank, dev)
    from dl_cs.mri import transforms as T
    A = T.SenseModel(data["maps"], weights=data["mask"])
    opt = torch.optim.Adam([p for p in model.parameters() if p.requires_grad], lr=cfg.OPTIMIZER.ADAM.LR,
                           foreach=True)
    buckets = GradBuckets(model, world)

    def step():
        buckets.zero()
        pred = model(y=data["y"], A=A, x0=data["x0"])
        loss = torch.mean(torch.abs(data["target"] - pred))          # Train/complex_l1 (train_swin.py:134)
        loss.backward()
        buckets.finish()
        opt.step()
        return loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    engine.PROFILE, engine.ATTN_PROFILE, T.PROFILE = [], [], []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    prof, engine.PROFILE = engine.PROFILE, None
    aprof, engine.ATTN_PROFILE = engine.ATTN_PROFILE, None
    sprof, T.PROFILE = T.PROFILE, None
    t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t)
    conv_ms = [e0.elapsed_time(e1) for e0, e1, _ in prof]
    conv_flops = prof[0][2] if prof else 0.0
    if rank == 0:
        avg_ms = float(np.mean(conv_ms)) if conv_ms else float("nan")
        achieved = conv_flops / (avg_ms * 1e-3) / 1e12 if conv_ms else 0.0
        peak = MI355X_BF16_DENSE_TFLOPS if args.dtype == "bf16" else MI355X_FP32_TFLOPS
        line = {
            "metric": "cine slices/sec (fwd+bwd) at 10-iter unroll, 1/2/4/8 GPU; PSNR vs ref",
            "value": world * args.steps / elapsed,
            "unit": "slices/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1000.0 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic (random x_true, normalised random maps, reference VDkt mask seed 1000; random-init weights)",
            "config": {"workload": f"configs/config_swin.yaml, PGD {args.unrolls}-iter unroll, Swin regularizer, "
                                   f"1 cine slice per rank: {args.coils} coils x {args.frames} frames x "
                                   f"{args.ny} x {args.nx}, 2 ESPIRiT maps, train step (fwd+bwd+Adam)",
                       "global_batch": world, "unrolls": args.unrolls,
                       "parallelism": f"dp{world} (one slice per rank, RCCL grad all-reduce)"},
            "roofline": {"bound": "mfma",
                         "kernel": ("conv3d_k3_v5_kernel" if args.dtype == "bf16" else "conv3d_k3_kernel<float,5>")
                         + " (Conv3d 160->160 k3 fwd, ResSwin/DFE tails)",
                         "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                         "frac": achieved / peak, "traffic": pmc_traffic(args.dtype),
                         "launches": len(conv_ms), "avg_ms": avg_ms,
                         "flops_per_launch": conv_flops},
            # the north star's two named secondary kernels, timed the same way
            "roofline_sense": secondary(sprof, "hbm", MI355X_HBM_GBS, "GB/s", 1e9,
                                        "SenseModel forward / adjoint (+ fused PGD DC update): dlcs_sense_fwd/adj, "
                                        "2 launches per op; algorithmic bytes = x, maps, mask, k-space (and DC "
                                        "operands) each read or written once"),
            "roofline_attention": secondary(aprof, "mfma", MI355X_BF16_DENSE_TFLOPS if args.dtype == "bf16"
                                            else MI355X_FP32_TFLOPS, "TFLOP/s", 1e12,
                                            "attn_fwd_v2_kernel (fused window attention forward: Q K^T + bias + "
                                            "mask + softmax + P V, 30 windows x 8 heads x 448^2, head dim 20)"),
            "loss": float(loss.detach()),
        }
        if world == 1 and not args.no_cpu_baseline:
            threads = args.cpu_threads or min(16, os.cpu_count() or 1)
            cb, parity = cpu_baseline(model, data, args, threads)
            line["cpu_baseline"] = cb
            line["psnr_vs_ref"] = parity
        else:
            line["cpu_baseline"] = None
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

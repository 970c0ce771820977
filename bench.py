"""Headline benchmark: cine slices/s of the Swin-unrolled PGD training step.

BASELINE.json metric: "cine slices/sec (fwd+bwd) at 10-iter unroll, 1/2/4/8 GPU;
PSNR vs ref".  One step = one training iteration on one synthetic cine slice
per rank (8 coils x 20 frames x 192 x 160, 2 ESPIRiT maps, VDkt mask, seed
1000): forward through 10 unrolls (SENSE normal op + Swin regularizer), complex
L1 loss, backward, RCCL gradient all-reduce (N > 1), Adam step.  Inputs are
resident in HBM before timing.  Weak scaling: one slice per rank.

    python bench.py [--gpus N] [--steps K] [--warmup W]

N > 1: under torchrun (`python -m torch.distributed.run --nproc-per-node N ...
bench.py --gpus N`, RANK / WORLD_SIZE in the environment) each process is one
rank; a plain `python bench.py --gpus N` starts the N ranks itself as fresh child
processes (before anything touches the GPU) with a 127.0.0.1 rendezvous, the way
the reference's `Trainer(gpus=devices)` does (train_swin.py:253-261).  Either way
the world size must equal --gpus, or the run exits non-zero.

The headline runs in fp32 (the reference's own arithmetic); a second
phase in bf16 (BASELINE config 2's dtype) follows in the same process and is
reported under the "bf16" key.  Prints ONE JSON line on rank 0 (see the harness
contract in DESIGN.md).
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

# the reference's own PyTorch-CPU Swin PGD train step, 10 unrolls,
# measured in the survey container (8-core Xeon, fp32): ~148 s / slice.  Not a published
# number (BASELINE.md section 1 has none); quoted for context only -- vs_baseline divides by
# the cpu_baseline measured in the same run on the same box.
REFERENCE_CPU_SLICES_PER_S = 0.0068
MI355X_BF16_DENSE_TFLOPS = 2500.0      # MI355X_MICROARCH.md chip table (dense, no sparsity)
MI355X_FP32_TFLOPS = 157.3
MI355X_HBM_GBS = 8000.0


def log(msg):
    """Progress on stderr (the JSON line stays the only stdout line): long CPU legs
    (oracle reconstruction, float64 gradient probe, the measured CPU baseline) run
    for minutes, and a silent process looks hung to a watchdog."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--unrolls", type=int, default=10)
    ap.add_argument("--dtype", default="fp32", choices=["bf16", "fp32"],
                    help="headline compute dtype (fp32 = the reference's own precision)")
    ap.add_argument("--no-secondary", dest="secondary", action="store_false",
                    help="skip the second phase in the other dtype (reported under its dtype key)")
    ap.add_argument("--coils", type=int, default=8)
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--ny", type=int, default=192)
    ap.add_argument("--nx", type=int, default=160)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-configs", dest="configs", action="store_false",
                    help="skip the BASELINE config 2 / 3 / 5 keys (5-unroll bf16, Swin-GAN, DiT DDPM_X)")
    ap.add_argument("--config-steps", type=int, default=5)
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-all-branches", dest="all_branches", action="store_false",
                    help="skip the DropPath all-branches phase (profiling runs: exactly warmup + steps train steps)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher / rendezvous / timing plumbing only, on the CPU with gloo: each step all-reduces a "
                         "gradient-sized flat bucket (no HIP path; tests/test_bench_launch.py)")
    ap.add_argument("--dry-run-numel", type=int, default=1 << 20)
    return ap.parse_args()


def launch_ranks(args):
    """`bench.py --gpus N` (N > 1) outside torchrun: start N fresh interpreters, one
    per rank (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / a free
    MASTER_PORT), before this process touches the GPU; rank 0 prints the line.
    Returns the first nonzero exit status (the other ranks are then terminated)."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:
                    q.terminate()
        time.sleep(0.2)
    for p in procs:
        p.wait()
    return rc


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


CONV_KERNELS = {   # (dtype, role) -> kernel the 160->160 conv launches (conv3d.hip dispatch)
    ("bf16", "conv_fwd"): "conv3d_k3_v5_kernel", ("bf16", "conv_dgrad"): "conv3d_k3_v5_kernel<4, 0>",
    ("bf16", "conv_wgrad"): "conv3d_wgrad_c160_kernel",
    ("fp32", "conv_fwd"): "conv3d_k3_f32_kernel", ("fp32", "conv_dgrad"): "conv3d_k3_f32_kernel",
    ("fp32", "conv_wgrad"): "conv3d_wgrad_f32_kernel",
    ("x6", "conv_fwd"): "conv3d_k3_x6_kernel", ("x6", "conv_dgrad"): "conv3d_k3_x6_kernel<4>",
    ("x6", "conv_wgrad"): "conv3d_wgrad_x6_kernel",
    ("f16x3", "conv_fwd"): "conv3d_k3_f16x3_kernel", ("f16x3", "conv_dgrad"): "conv3d_k3_f16x3_kernel<4>",
    ("f16x3", "conv_wgrad"): "conv3d_wgrad_f16x3_kernel",
}
SPLIT_PRODUCTS = {"x6": (6, "six bf16 plane products"), "f16x3": (3, "three fp16 plane products")}


def pmc_traffic(dtype, role):
    """HBM bytes per launch of a conv kernel from the newest committed PMC pass
    (profiles/*_traffic_<dtype>_<role>.json, tools/profile_round.sh): FETCH_SIZE
    (x2, gfx950 correction) + WRITE_SIZE, separate --pmc runs; None if absent."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", f"*_traffic_{dtype}_{role}.json")))
    if not files and (dtype, role) == ("bf16", "conv_fwd"):
        files = sorted(glob.glob(os.path.join(REPO, "profiles", "*_traffic_conv3d_k3_v5.json")))
    if not files:
        return None
    with open(files[-1]) as f:
        return json.load(f)["hbm_bytes_per_launch"]


def secondary(prof, bound, peak, unit, scale, what):
    """Roofline entry of a kernel from (start, end, algorithmic work) events."""
    if not prof:
        return None
    ms = [ev[0].elapsed_time(ev[1]) for ev in prof]
    work = float(np.mean([ev[2] for ev in prof]))
    achieved = work / (float(np.mean(ms)) * 1e-3) / scale
    return {"bound": bound, "kernel": what, "achieved": achieved, "peak": peak, "unit": unit,
            "frac": achieved / peak, "launches": len(ms), "avg_us": 1e3 * float(np.mean(ms)),
            "total_ms": float(np.sum(ms)), "work_per_launch": work}


def sense_entry(prof, what):
    """roofline_sense(_adj): `achieved` counts the bytes the entry point needs
    (row-sparse operators: only the mask's sampled k-space lines); `survey`
    re-prices the same measured time with SURVEY.md §8(d)'s per-call accounting
    of the reference's dense SenseModel calls (A and A^H at 55.54 MB each at the
    headline geometry, transforms._call_bytes) -- the same work, priced as the
    reference's operator moves it."""
    e = secondary(prof, "hbm", MI355X_HBM_GBS, "GB/s", 1e9, what)
    if e is not None:
        ms = float(np.mean([ev[0].elapsed_time(ev[1]) for ev in prof]))
        work = float(np.mean([ev[4] for ev in prof]))
        a = work / (ms * 1e-3) / 1e9
        e["survey"] = {"achieved": a, "frac": a / MI355X_HBM_GBS, "bytes_per_launch": work,
                       "note": "SURVEY.md §8(d): each SenseModel call reads/writes its operands once "
                               "(A = A^H = 55.54 MB at [1, 8, 20, 192, 160]); the normal operator = A + A^H"}
    return e


# fp32 window attention on fp16 matrix cores (csrc/attention_h3.inc, default; DLCS_ATTN_H3=0
# with DLCS_DIAG=1 restores the f32-MFMA kernels): v_mfma_f32_32x32x16_f16 instructions executed per 32 x 32
# (query, key) tile -- forward 12 (QK^T and P V, 3 plane products x 2 k-steps), backward
# 24 (dK / dV kernel: S, dP, dV, dK) + 18 (dQ kernel: S, dP, dQ) -- against the algorithmic
# fp32 flops per tile (forward 4 * 32 * 32 * 20, backward twice that)
_DIAG = os.environ.get("DLCS_DIAG", "0") == "1"
ATTN_H3 = not (_DIAG and os.environ.get("DLCS_ATTN_H3", "1") == "0")
ATTN_H3_BWD = ATTN_H3 and not (_DIAG and os.environ.get("DLCS_ATTN_H3_BWD", "1") == "0")
ATTN_TILE_FLOPS = 4.0 * 32 * 32 * 20
ATTN_H3_MFMA = {"fwd": 12, "bwd": 42}


def h3_attention_entry(prof, executed_per_tile, algo_per_tile, what):
    """MFMA roofline of an fp32 attention kernel that runs every product as three fp16
    plane products on v_mfma_f32_32x32x16_f16: `achieved` / `frac` = EXECUTED
    matrix-core flops (head dim padded to 32, 3 plane products) against the dense fp16
    peak -- the kernel's own matrix-core roofline, never above 1; `fp32_equiv` = the
    algorithmic fp32 flops per second (the reference's arithmetic), for comparison with
    the 157 TFLOP/s f32 MFMA the kernel replaces."""
    if not prof:
        return None
    ratio = executed_per_tile * 32768.0 / algo_per_tile
    e = secondary([(e0, e1, w * ratio) for e0, e1, w in prof], "mfma", MI355X_BF16_DENSE_TFLOPS, "TFLOP/s", 1e12,
                  what + " -- fp32 as three fp16 plane products on v_mfma_f32_32x32x16_f16; achieved = executed "
                         "matrix-core flops (incl. head-dim padding to 32) against the dense fp16 peak")
    alg = e["achieved"] / ratio
    e["fp32_equiv"] = {"achieved": alg, "unit": "TFLOP/s", "algorithmic_work_per_launch": e["work_per_launch"] / ratio,
                       "ratio_to_f32_mfma_peak": alg / MI355X_FP32_TFLOPS,
                       "note": "algorithmic fp32 flops (Q K^T + P V) per second; the f32 MFMA peak is not this "
                               "kernel's roofline (it runs on fp16 matrix cores), so this is a ratio, not a frac"}
    e["executed_per_tile"] = executed_per_tile
    return e


def attention_entry(prof, dtype, which, what):
    """roofline_attention(_bwd) of the Swin window attention: bf16 kernels against the
    dense bf16 peak; the fp32 kernels (fp16 split, attention_h3.inc) by executed
    matrix-core flops against the dense fp16 peak (h3_attention_entry)."""
    h3 = dtype == "fp32" and (ATTN_H3 if which == "fwd" else ATTN_H3_BWD)
    if h3:
        return h3_attention_entry(prof, ATTN_H3_MFMA[which], ATTN_TILE_FLOPS * (1 if which == "fwd" else 2),
                                  what + " (csrc/attention_h3.inc)")
    peak = MI355X_BF16_DENSE_TFLOPS if dtype == "bf16" else MI355X_FP32_TFLOPS
    return secondary(prof, "mfma", peak, "TFLOP/s", 1e12, what)


def conv_rooflines(prof, dtype, steps):
    """MFMA roofline of the three 160->160 conv kernels (fwd, dgrad, wgrad: 1.189
    TFLOP each per launch at BASELINE size) from HIP events around every launch;
    the dominant one (most total time) is the line's `roofline`."""
    from dl_cs.models import engine
    out = {}
    for role in ("conv_fwd", "conv_dgrad", "conv_wgrad"):
        split = engine.FP32_CONV if (dtype == "fp32" and engine.X6) else None
        peak = MI355X_BF16_DENSE_TFLOPS if (dtype == "bf16" or split) else MI355X_FP32_TFLOPS
        ev = prof.get(role)
        nprod, what = SPLIT_PRODUCTS.get(split, (1, ""))
        if split and ev:
            # fp32 on bf16 / fp16 matrix cores: the kernel executes nprod 16-bit plane
            # products per fp32 product -- its matrix-core roofline is the dense
            # bf16 / fp16 one (same peak) on nprod x the work
            ev = [(e0, e1, nprod * w) for e0, e1, w in ev]
        e = secondary(ev, "mfma", peak, "TFLOP/s", 1e12,
                      f"{CONV_KERNELS[(split or dtype, role)]} (Conv3d 160->160 k3 {role[5:]}, ResSwin/DFE tails"
                      + (f", fp32 as {what}" if split else "") + ")")
        if e is not None:
            if split:
                e["fp32_equiv_tflops"] = e["achieved"] / nprod
                e["work_note"] = (f"work_per_launch = {nprod} x the fp32 conv's 1.189 TFLOP "
                                  f"(16-bit MFMA flops executed)")
            e["traffic"] = pmc_traffic(split or dtype, role)
            e["ms_per_step"] = e["total_ms"] / steps
            out[role] = e
    dom = max(out, key=lambda r: out[r]["total_ms"]) if out else None
    return dom, out


def cpu_threads():
    """CPU cores this process may use (its affinity set, capped by OMP_NUM_THREADS
    when set -- the GPU box exports its CPU share there)."""
    n = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    return min(n, int(omp)) if omp and omp.isdigit() and int(omp) > 0 else n


def cpu_baseline(model, data, args, threads, timed=2):
    """The oracle (fp32 PyTorch-CPU restatement pinned to the reference's goldens)
    timed on the whole workload of one step, as BASELINE.md section 3 asks: the
    reference's training iteration at `unrolls` unrolls (A^H y, then per unroll the
    SENSE normal op + SwinTransformer3DNet, complex L1, backward through all of it,
    Adam over every unroll's parameters) at the BASELINE slice, after one warmup
    (one unroll fwd + bwd: the allocator and the thread pool warm, no cost model
    taken from it), `timed` timed iterations; value = 1 / their mean.  Nothing is
    extrapolated."""
    sys.path.insert(0, REPO)
    from oracle import dlcs_oracle as O
    torch.set_num_threads(threads)
    sd = {k: v.detach().float().cpu() for k, v in model.state_dict().items()}
    Ps = [{k: v.clone().requires_grad_(torch.is_floating_point(v) and "relative_position_index" not in k)
           for k, v in P.items()} for P in O.split_unrolls(sd, args.unrolls)]
    params = [v for P in Ps for v in P.values() if v.requires_grad]
    opt = torch.optim.Adam(params, lr=1e-4)
    maps, mask = data["maps"].cpu(), data["mask"].cpu()
    y, x0, target = data["y"].cpu(), data["x0"].cpu(), data["target"].cpu()
    t0 = time.perf_counter()                       # warmup: one unroll fwd + bwd
    O.l1(target, O.pgd(Ps[:1], y, maps, mask, x0=x0)).backward()
    warm = time.perf_counter() - t0
    log(f"cpu_baseline: warmup (1 unroll fwd+bwd) {warm:.1f} s on {threads} threads")
    times = []
    for it in range(timed):
        opt.zero_grad(set_to_none=True)
        t0 = time.perf_counter()
        loss = O.l1(target, O.pgd(Ps, y, maps, mask, x0=x0))     # Train/complex_l1 (train_swin.py:134)
        loss.backward()
        opt.step()
        times.append(time.perf_counter() - t0)
        log(f"cpu_baseline: timed iteration {it + 1}/{timed}: {times[-1]:.1f} s")
    dt = float(np.mean(times))
    return dict(value=1.0 / dt, unit="slices/s", cores=threads, kind="port", extrapolated=False,
                measured_unrolls=args.unrolls, iterations_s=times, warmup_s=warm,
                sample=f"the full step: {args.unrolls}-unroll PGD training iteration (A^H y, SENSE normal op + "
                       f"SwinTransformer3DNet per unroll, complex L1, backward, Adam) at {tuple(data['y'].shape)} "
                       f"k-space, fp32 PyTorch-CPU oracle, {threads} threads; 1 warmup (one unroll fwd+bwd) + "
                       f"{timed} timed iterations, mean {dt:.1f} s")


def psnr_vs_oracle(model, data, args, threads, dtypes):
    """Reconstruction parity: the full `unrolls`-unroll PGD forward (eval mode, same
    weights and slice) through the GPU path in each compute dtype vs the fp32
    PyTorch-CPU oracle (oracle.pgd).  Bar: fp32 NRMSE <= 1e-5
    (>= 100 dB), bf16 NRMSE <= 1e-2."""
    sys.path.insert(0, REPO)
    from oracle import dlcs_oracle as O
    from dl_cs.models import swin3D
    from dl_cs.mri import transforms as T
    torch.set_num_threads(threads)
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    Ps = O.split_unrolls(sd, args.unrolls)
    t0 = time.perf_counter()
    with torch.no_grad():
        ref = O.pgd(Ps, data["y"].cpu(), data["maps"].cpu(), data["mask"].cpu(), x0=data["x0"].cpu())
    t_oracle = time.perf_counter() - t0
    ref = ref.to(torch.complex128)
    out = {"what": f"{args.unrolls}-unroll PGD reconstruction (eval), GPU path vs fp32 CPU oracle, same weights "
                   f"and slice; oracle forward {t_oracle:.1f} s on {threads} threads"}
    old = swin3D.get_compute_dtype()
    model.eval()
    try:
        for name in dtypes:
            swin3D.set_compute_dtype(torch.bfloat16 if name == "bf16" else torch.float32)
            with torch.no_grad():
                A = T.SenseModel(data["maps"], weights=data["mask"])
                rec = model(y=data["y"], A=A, x0=data["x0"]).cpu().to(torch.complex128)
            rmse = torch.sqrt(torch.mean(torch.abs(rec - ref) ** 2))
            out[name] = {"psnr_db": float(20 * torch.log10(ref.abs().max() / rmse)),
                         "nrmse": float(torch.linalg.vector_norm(rec - ref) / torch.linalg.vector_norm(ref))}
    finally:
        model.train()
        swin3D.set_compute_dtype(old)
    return out


def grad_accuracy(model, data, threads):
    """Gradient accuracy of the fp32 path at the BASELINE slice: one unroll's
    regularizer (model.cnn_update[0], SwinTransformer3DNet) fwd + bwd through the
    HIP path on the slice's A^H y with a fixed random cotangent, against a float64
    evaluation of the CPU oracle with the HIP forward's ReLU decisions (the masked
    float64 check of tests/goldutil.py), next to the fp32 oracle's own distance from
    it (the floor).  Per parameter tensor NRMSE; the line reports the largest and
    the median, and the largest ratio to the bar max(1e-5, 4 x floor)."""
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from goldutil import HipMasks, nrmse, oracle_grads
    from oracle import dlcs_oracle as O
    from dl_cs.models import engine, swin3D
    torch.set_num_threads(threads)
    old = swin3D.get_compute_dtype()
    swin3D.set_compute_dtype(torch.float32)
    net = model.cnn_update[0]
    was = net.training
    net.eval()
    t0 = time.perf_counter()
    try:
        x = data["x0"].detach()
        gen = torch.Generator(device="cpu").manual_seed(7)
        g = torch.complex(torch.randn(x.shape, generator=gen), torch.randn(x.shape, generator=gen))
        for p in net.parameters():
            p.grad = None
        engine.CAPTURE = []
        try:
            y = net(x)
        finally:
            caps, engine.CAPTURE = engine.CAPTURE, None
        gd = g.to(x.device)
        (y.real * gd.real + y.imag * gd.imag).sum().backward()
        hip = {n: p.grad.detach().double().cpu().numpy() for n, p in net.named_parameters() if p.grad is not None}
        masks = HipMasks(caps)
        xc = x.cpu()

        def lf(P, c, mk):
            yo, gc = O.swinnet(P, c(xc), relu=mk.relu()), c(g)
            return (yo.real * gc.real + yo.imag * gc.imag).sum()
        tr = lambda k: "relative_position_index" not in k          # noqa: E731
        sd = {k: v.detach().cpu() for k, v in net.state_dict().items()}
        masks.reset()
        o32 = oracle_grads(lambda P, c: lf(P, c, masks), sd, torch.float32, tr)
        masks.relus = []
        masks.reset()
        o64 = oracle_grads(lambda P, c: lf(P, c, masks), sd, torch.float64, tr)
    finally:
        for p in net.parameters():
            p.grad = None
        net.train(was)
        swin3D.set_compute_dtype(old)
    rows = []
    for n in sorted(set(hip) & set(o64)):
        fl, er = nrmse(o64[n], o32[n]), nrmse(o64[n], hip[n])
        rows.append((er / max(1e-5, 4 * fl), er, fl, n))
    rows.sort(reverse=True)
    errs = [r[1] for r in rows]
    return {"what": "one unroll's SwinTransformer3DNet fwd+bwd at the BASELINE slice (fp32 path, input A^H y, fixed "
                    "random cotangent): per parameter tensor NRMSE of the HIP gradient vs a float64 oracle evaluation "
                    "with the HIP ReLU decisions; floor = the fp32 oracle's own NRMSE vs float64; bar max(1e-5, 4 x floor)",
            "tensors": len(rows), "max_nrmse": max(errs), "median_nrmse": float(np.median(errs)),
            "median_floor": float(np.median([r[2] for r in rows])), "worst": {"tensor": rows[0][3], "nrmse": rows[0][1],
                                                                             "floor": rows[0][2], "ratio_to_bar": rows[0][0]},
            "over_bar": sum(r[0] > 1.0 for r in rows), "seconds": time.perf_counter() - t0}


def _timed(step, steps, warmup):
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        out = step()
    torch.cuda.synchronize()
    return time.perf_counter() - t0, out


def config2_phase(args, dev, data, steps):
    """BASELINE config 2 (configs/config_swin.yaml: 5-iter unroll, bf16): the Swin PGD
    train step with 5 unrolls in bf16 (fp32 complex boundary and SENSE)."""
    from dl_cs.config import get_cfg
    from dl_cs.distributed import GradBuckets
    from dl_cs.utils import optim
    from dl_cs.models import swin3D, unrolledswin
    from dl_cs.mri import transforms as T
    cfg = get_cfg()
    cfg.merge_from_file(os.path.join(REPO, "configs", "config_swin.yaml"))
    cfg.MODEL.PARAMETERS.NUM_UNROLLS = 5
    torch.manual_seed(cfg.SEED)
    model = unrolledswin.ProximalGradientDescent(cfg).to(dev)
    model.train()
    A = T.SenseModel(data["maps"], weights=data["mask"])
    opt = optim.adam([p for p in model.parameters() if p.requires_grad], lr=1e-4)
    buckets = GradBuckets(model, 1)
    old = swin3D.get_compute_dtype()
    swin3D.set_compute_dtype(torch.bfloat16)

    def step():
        buckets.zero()
        pred = model(y=data["y"], A=A, x0=data["x0"])
        loss = torch.mean(torch.abs(data["target"] - pred))
        loss.backward()
        buckets.finish()
        opt.step()
        return loss
    try:
        el, loss = _timed(step, steps, 2)
    finally:
        swin3D.set_compute_dtype(old)
        buckets.close()
    return {"value": steps / el, "unit": "slices/s", "ms_per_step": 1000 * el / steps, "steps": steps,
            "dtype": "bf16", "loss": float(loss.detach()),
            "workload": "configs/config_swin.yaml PGD 5-iter unroll (BASELINE config 2), Swin regularizer, bf16 "
                        "activations / GEMM operands with fp32 accumulation and fp32 complex SENSE boundary, train "
                        "step (fwd+bwd+Adam), BASELINE slice"}


def gan_phase(args, model, data, A, buckets, opt, steps, adv_weight=0.01):
    """BASELINE config 3 (Swin-GAN; build-defined, the reference ships no
    discriminator): one generator step (complex L1 + adv_weight x BCE(D(G(y)), 1)
    through the config_swin PGD generator) and one PatchGAN discriminator step
    (BCE real / fake) per iteration at the BASELINE slice, fp32."""
    from dl_cs.models import patchgan, swin3D
    from dl_cs.utils import optim
    torch.manual_seed(1001)
    D = patchgan.PatchGANDiscriminator3D(4, 160).to(data["maps"].device)
    optD = optim.adam(D.parameters(), lr=1e-4)
    swin3D.set_compute_dtype(torch.float32)

    def step():
        buckets.zero()
        pred = model(y=data["y"], A=A, x0=data["x0"])
        g_loss = torch.mean(torch.abs(data["target"] - pred)) + adv_weight * patchgan.g_adv_loss(D(pred))
        g_loss.backward()
        buckets.finish()
        opt.step()
        optD.zero_grad(set_to_none=True)
        d_loss = patchgan.d_loss(D(data["target"]), D(pred.detach()))
        d_loss.backward()
        optD.step()
        return g_loss, d_loss
    el, (gl, dl) = _timed(step, steps, 2)
    return {"value": steps / el, "unit": "slices/s", "ms_per_step": 1000 * el / steps, "steps": steps,
            "dtype": "fp32", "g_loss": float(gl.detach()), "d_loss": float(dl.detach()),
            "workload": f"Swin-GAN (BASELINE config 3, build-defined spec, parity unpinned vs the reference): "
                        f"config_swin PGD {args.unrolls}-iter generator + 3-D PatchGAN (160 features) discriminator, "
                        f"G step (L1 + {adv_weight} adversarial) + D step per iteration, BASELINE slice, fp32"}


def dit_phase(args, dev, data, steps, cfg_name="config_dit.yaml"):
    """BASELINE config 5 (configs/config_dit.yaml, META_ARCHITECTURE DDPM_X): the
    reference's DiT training step (train_DiT.py:232-288 + optimizer_step's EMA,
    :424-427): x_t = q_sample(target, t), 4 DataConsistency unrolls of DiTResNet
    (6 DiT blocks, 384 features, 16 heads), k-space L1 vs the fully-sampled target,
    backward, Adam, EMA(0.9999); fp32; the sub-mask split of train_DiT.submask is
    drawn once outside the timed region (data preparation)."""
    import copy
    sys.path.insert(0, os.path.join(REPO, "scripts"))
    from dl_cs.config import load_cfg
    from dl_cs.diffusion import create_diffusion
    from dl_cs.models import dit_engine, swin3D, unrolledDiT
    from dl_cs.utils import optim
    from dl_cs.mri import transforms as T
    from train_DiT import submask
    from dl_cs.models import unrolledLatte
    cfg = load_cfg(os.path.join(REPO, "configs", cfg_name))
    torch.manual_seed(cfg.SEED)
    swin3D.set_compute_dtype(torch.float32)
    latte = cfg.MODEL.MODEL_TYPE == "Latte"
    model = (unrolledLatte if latte else unrolledDiT).DataConsistency(cfg).to(dev)
    model.train()
    ema = copy.deepcopy(model)
    for p in ema.parameters():
        p.requires_grad_(False)
    diff = create_diffusion(timestep_respacing="", noise_schedule=cfg.MODEL.PARAMETERS.NOISE_SCHED,
                            diffusion_steps=1000, learn_sigma=False, predict_xstart=True)
    maps, mask, target = data["maps"], data["mask"], data["target"]
    gen = torch.Generator(device="cpu").manual_seed(1000)
    mask_r, mask_p = submask(mask, 0.9, gen)
    kw = dict(A=T.SenseModel(maps, weights=mask_p), A_1=T.SenseModel(maps, weights=1 - mask_p),
              A_F=T.SenseModel(maps), A_S=T.SenseModel(maps, weights=mask_r), fs=target,
              c=torch.tensor([1], device=dev))
    params = [p for p in model.parameters() if p.requires_grad]
    opt = optim.adam(params, lr=cfg.OPTIMIZER.ADAM.LR)
    ep, mp = list(ema.parameters()), list(model.parameters())

    def step():
        opt.zero_grad(set_to_none=True)
        t = torch.randint(0, diff.num_timesteps, (1,), device=dev)
        terms, _, _ = diff.training_kspace_loss(model, target, t, kw)
        terms["loss"].backward()
        opt.step()
        with torch.no_grad():
            torch._foreach_lerp_(ep, mp, 1.0 - 0.9999)                  # update_ema (train_DiT.py:58-72)
        return terms["loss"]
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    dit_engine.PROFILE = []
    el, loss = _timed(step, steps, 0)
    prof, dit_engine.PROFILE = dit_engine.PROFILE, None
    # inference: one denoiser evaluation (the EMA model's 4 DataConsistency unrolls at
    # a fixed t, eval, no grad -- one step of the reverse diffusion) in fp32 and on
    # the fp8 token-Linear path; NRMSE of the fp8 output vs the fp32 one
    ema.eval()
    # every Linear of the evaluated copy drawn N(0, 0.02): under the reference's
    # adaLN-Zero init (gates and final layer zero) each block is an identity and the
    # fp8 GEMMs would not reach the output
    gen = torch.Generator(device=dev).manual_seed(7)
    with torch.no_grad():
        for p_ in ema.parameters():
            if p_.dim() == 2 and p_.requires_grad is False and p_.shape[0] > 1:
                p_.normal_(0.0, 0.02, generator=gen)
    from dl_cs.diffusion.gaussian_diffusion import tensor2complex, tensor2realimag
    tt = torch.tensor([500], device=dev)
    xt = tensor2complex(diff.q_sample(tensor2realimag(target), tt))

    def infer():
        with torch.no_grad():
            return ema(xt, tt, **kw)
    infer()
    el32, y32 = _timed(infer, steps, 0)
    dit_engine.set_fp8(True)
    try:
        infer()
        el8, y8 = _timed(infer, steps, 0)
    finally:
        dit_engine.set_fp8(False)
    fp8_err = float(((y8 - y32).abs().pow(2).sum() / y32.abs().pow(2).sum()).sqrt())
    inference = {"fp32": {"denoiser_evals_per_s": steps / el32, "ms": 1000 * el32 / steps},
                 "fp8": {"denoiser_evals_per_s": steps / el8, "ms": 1000 * el8 / steps,
                         "nrmse_vs_fp32": fp8_err},
                 "what": "one reverse-diffusion denoiser evaluation (EMA DataConsistency, t = 500, eval; its Linear "
                         "weights redrawn N(0, 0.02) so the adaLN-Zero gates are nonzero); "
                         "fp8 = the DiT blocks' token Linears (adaLN, qkv, proj, fc1, fc2) as OCP e4m3 row-scaled "
                         "GEMMs on v_mfma_f32_16x16x32_fp8_fp8 (dlcs_gemm_f8r), the rest fp32"}
    long = [(e0, e1, f) for e0, e1, f, n in prof if n > 64]
    if latte:
        P_ = cfg.MODEL.PARAMETERS
        what = (f"dlcs_mhsa_fwd -> mhsa_fwd_h3_kernel (flash attention, csrc/mhsa_h3.inc), Latte spatial blocks: the 1,920 "
                f"patches of each of the 24 padded frames, {P_.NUM_HEADS} heads, head dim "
                f"{P_.NUM_FEATURES // P_.NUM_HEADS}; flops = Q K^T + P V")
        workload = ("configs/config_latte.yaml (BASELINE config 5, MODEL_TYPE Latte): DDPM_X training step, "
                    f"{P_.NUM_UNROLLS} DataConsistency unroll(s) of LatteNet ({P_.NUM_LAYERS} Latte blocks = spatial / "
                    f"temporal pairs, hidden {P_.NUM_FEATURES}, {P_.NUM_HEADS} heads, 2-D patch (4,4)), diffusion "
                    f"k-space L1, Adam + EMA, BASELINE slice {tuple(data['y'].shape)} k-space, fp32; the fp8 MFMA path "
                    "under 'inference'")
    else:
        what = ("dlcs_mhsa_fwd -> mhsa_fwd_h3_kernel (flash attention, csrc/mhsa_h3.inc) over the 1,920 tokens of each "
                "frame: 12 frames x 16 heads, head dim 24; flops = Q K^T + P V")
        workload = ("configs/config_dit.yaml (BASELINE config 5): DDPM_X training step, 4 DataConsistency "
                    "unrolls of DiTResNet (SFE conv 4->384, DiT 6 x DiTBlockFactor, hidden 384, 16 heads, patch "
                    "(2,4,4), final conv 384->4), diffusion k-space L1, Adam + EMA, BASELINE slice "
                    f"{tuple(data['y'].shape)} k-space, fp32; the fp8 MFMA path under 'inference'")
    hd = cfg.MODEL.PARAMETERS.NUM_FEATURES // cfg.MODEL.PARAMETERS.NUM_HEADS
    # mhsa_fwd_h3_kernel per 32 x 32 (query, key) tile: Q K^T 2 k-steps + P V 2 k-steps, 3 plane
    # products each = 12 v_mfma_f32_32x32x16_f16, against 4 x 32 x 32 x hd algorithmic flops
    att = h3_attention_entry([(e0, e1, f) for e0, e1, f in long], 12, 4.0 * 32 * 32 * hd, what)
    return {"value": steps / el, "unit": "slices/s", "ms_per_step": 1000 * el / steps, "steps": steps,
            "dtype": "fp32", "loss": float(loss.detach()), "roofline_attention": att, "inference": inference,
            "workload": workload}


def world_timing(elapsed, steps, world, dev):
    """Max-over-ranks wall time plus every rank's ms/step (all_gather)."""
    t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
    if world == 1:
        return elapsed, [1000.0 * elapsed / steps]
    allt = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(allt, t)
    per = [float(x) for x in allt]
    return max(per), [1000.0 * x / steps for x in per]


def dry_run(args, world, rank, backend):
    """--dry-run: the multi-rank plumbing of main() without the HIP path (CPU, gloo):
    W + K steps, each all-reducing a flat fp32 bucket, barrier-bracketed timing, max
    over ranks, ONE line from rank 0."""
    if world > 1:
        dist.init_process_group(backend)
    bucket = torch.ones(args.dry_run_numel)
    for _ in range(args.warmup):
        dist.all_reduce(bucket) if world > 1 else None
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        if world > 1:
            dist.all_reduce(bucket)
    if world > 1:
        dist.barrier()
    elapsed, per_rank = world_timing(time.perf_counter() - t0, args.steps, world, "cpu")
    if rank == 0:
        print(json.dumps({"metric": "dry-run (launcher plumbing, no HIP path)", "value": world * args.steps / elapsed,
                          "unit": "steps/s", "n_gpus": world, "world_size": dist.get_world_size() if world > 1 else 1,
                          "backend": backend if world > 1 else None, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": 1000.0 * elapsed / args.steps, "per_rank_ms_per_step": per_rank,
                          "dry_run": True}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        rc = launch_ranks(args)
        sys.exit(rc if rc >= 0 else 128 - rc)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: world size {world} (WORLD_SIZE) != --gpus {args.gpus}", file=sys.stderr)
        sys.exit(3)
    # one rank per GPU (the driver's N-GPU launch); DLCS_DIST_BACKEND=gloo with more
    # ranks than GPUs rehearses the multi-rank path on one device (ranks share it)
    backend = os.environ.get("DLCS_DIST_BACKEND", "nccl")
    if args.dry_run:
        return dry_run(args, world, rank, "gloo")
    ndev = torch.cuda.device_count()
    if backend == "nccl" and world > ndev:
        raise SystemExit(f"bench.py: {world} ranks need {world} GPUs (found {ndev}); "
                         "DLCS_DIST_BACKEND=gloo shares one")
    local = local % ndev
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # DLCS_FORCE_COLLECTIVES=1 at --gpus 1: a one-rank process group (RCCL under the
    # default backend) and GradBuckets' multi-rank branches -- the per-unroll async
    # all-reduce from backward, its wait, the exposed-wait events -- so a single-GPU
    # box executes the code path of the driver's N-GPU run (dl_cs/distributed.py)
    use_pg = world > 1 or os.environ.get("DLCS_FORCE_COLLECTIVES", "0") == "1"
    if use_pg:
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if "MASTER_PORT" not in os.environ:
                import socket
                with socket.socket() as s_:
                    s_.bind(("127.0.0.1", 0))
                    os.environ["MASTER_PORT"] = str(s_.getsockname()[1])
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    from dl_cs.models import engine, swin3D
    from dl_cs.distributed import GradBuckets, broadcast_parameters
    from dl_cs.utils import optim
    model, cfg = build_model(args, dev)
    model.train()
    if use_pg:
        broadcast_parameters(model, 0)
    data = make_slice(args, rank, dev)
    from dl_cs.mri import transforms as T
    A = T.SenseModel(data["maps"], weights=data["mask"])
    buckets = GradBuckets(model, world, collective=use_pg)
    opt = optim.adam([p for p in model.parameters() if p.requires_grad], lr=cfg.OPTIMIZER.ADAM.LR)

    def step():
        buckets.zero()
        pred = model(y=data["y"], A=A, x0=data["x0"])
        loss = torch.mean(torch.abs(data["target"] - pred))          # Train/complex_l1 (train_swin.py:134)
        loss.backward()
        buckets.finish()
        opt.step()
        return loss

    def phase(dtype, steps, warmup):
        """W untimed + K timed training steps in one compute dtype; max over ranks."""
        swin3D.set_compute_dtype(torch.bfloat16 if dtype == "bf16" else torch.float32)
        for _ in range(warmup):
            step()
        torch.cuda.synchronize()
        if use_pg:
            dist.barrier()
        engine.PROFILE, engine.ATTN_PROFILE, engine.ATTN_BWD_PROFILE, T.PROFILE = {}, [], [], []
        buckets.WAIT_PROFILE = []
        buckets.launched = 0
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            loss = step()
        torch.cuda.synchronize()
        if use_pg:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        prof, engine.PROFILE = engine.PROFILE, None
        aprof, engine.ATTN_PROFILE = engine.ATTN_PROFILE, None
        abprof, engine.ATTN_BWD_PROFILE = engine.ATTN_BWD_PROFILE, None
        sprof, T.PROFILE = T.PROFILE, None
        wprof, buckets.WAIT_PROFILE = buckets.WAIT_PROFILE, None
        elapsed, per_rank = world_timing(elapsed, steps, world, dev)
        comm = None
        if use_pg:
            # the compute stream's stall in GradBuckets.finish() (events; host time under gloo)
            ev = [e0.elapsed_time(e1) if e0 is not None else 1000.0 * h for e0, e1, h in wprof]
            w = torch.tensor([float(np.mean(ev)) if ev else 0.0], device=dev, dtype=torch.float64)
            allw = [torch.zeros_like(w) for _ in range(world)]
            dist.all_gather(allw, w)
            comm = {"backend": dist.get_backend(), "world_size": dist.get_world_size(),
                    "allreduces_per_step": buckets.launched / steps,
                    "exposed_allreduce_ms_per_step": [float(x) for x in allw],
                    "bucket_mb": [round(4e-6 * f.numel(), 2) for f, _ in buckets.buckets],
                    "note": "per rank: time the compute stream waited in GradBuckets.finish() for the per-unroll "
                            "bucket all-reduces (launched asynchronously from backward) -- the communication "
                            "backward did not hide"}
        peak = MI355X_BF16_DENSE_TFLOPS if dtype == "bf16" else MI355X_FP32_TFLOPS
        dom, convs = conv_rooflines(prof, dtype, steps)
        res = {
            "value": world * steps / elapsed,
            "ms_per_step": 1000.0 * elapsed / steps,
            "per_rank_ms_per_step": per_rank,
            "allreduce": comm,
            "roofline": dict(convs[dom], dominant=dom) if dom else None,
            "roofline_conv": convs,
            # the north star's two named secondary kernels, timed the same way
            "roofline_sense": sense_entry([ev for ev in sprof if ev[3].startswith("dlcs_sense_normal")],
                                        "the PGD data-consistency step x + s (A^H W^2 A x - A^H y) of every unroll "
                                        "(forward and backward): dlcs_sense_normal_rows, the row-sparse normal "
                                        "operator for the VDkt k-t mask (3 launches: FFT_Y + sampled-line gather, "
                                        "FFT_X . W^2 . IFFT_X on the sampled lines, zero-filled IFFT_Y + conj-map "
                                        "coil sum + DC epilogue); algorithmic bytes = x, A^H y (forward only), maps "
                                        "and the output once, plus the sampled weight lines"),
            "roofline_sense_adj": sense_entry([ev for ev in sprof if ev[3].startswith("dlcs_sense_adj")],
                                            "the A^H y adjoint (dlcs_sense_adj_rows, 2 launches: IFFT_X of the "
                                            "sampled k-space lines with their weights, zero-filled IFFT_Y + "
                                            "conj-map coil sum); algorithmic bytes = the sampled lines of k-space "
                                            "and weights, maps and x once"),
            "roofline_attention": attention_entry(aprof, dtype, "fwd",
                                                  "fused window attention forward (Q K^T + bias + mask + softmax + "
                                                  "P V, 30 windows x 8 heads x 448^2, head dim 20)"),
            "roofline_attention_bwd": attention_entry(abprof, dtype, "bwd",
                                                      "window attention backward (dK / dV / bias-table kernel + dQ "
                                                      "kernel; algorithmic flops = dV, dP, dQ, dK = 2 x the "
                                                      "forward's -- the kernels' recomputation of P is not counted)"),
            "loss": float(loss.detach()),
        }
        return res

    head = phase(args.dtype, args.steps, args.warmup)
    log(f"{args.dtype} phase: {head['value']:.3f} slices/s")
    other = "bf16" if args.dtype == "fp32" else "fp32"
    sec = phase(other, args.steps, max(1, args.warmup)) if args.secondary else None
    if sec is not None:
        log(f"{other} phase: {sec['value']:.3f} slices/s")
    # DropPath: the timed train step draws stochastic depth (p = 0 .. 0.2, vst:603) and a
    # dropped branch skips its forward GEMMs and its whole backward (its gradient is zero);
    # the reference's autograd still computes it.  Same step with every branch computed:
    full = None
    if args.all_branches:
        dps = [m for m in model.modules() if type(m).__name__ == "DropPath"]
        saved = [m.drop_prob for m in dps]
        for m in dps:
            m.drop_prob = 0.0
        full = phase(args.dtype, args.steps, 1)
        for m, pr in zip(dps, saved):
            m.drop_prob = pr
    extra = {}
    if args.configs and world == 1:
        extra["config2_bf16_5unroll"] = config2_phase(args, dev, data, args.config_steps)
        log("config 2 done")
        extra["config3_swin_gan"] = gan_phase(args, model, data, A, buckets, opt, args.config_steps)
        log("config 3 done")
        extra["config5_dit_ddpm_x"] = dit_phase(args, dev, data, args.config_steps)
        log("config 5 (DiT) done")
        extra["config5_latte_ddpm_x"] = dit_phase(args, dev, data, args.config_steps, "config_latte.yaml")
        log("config 5 (Latte) done")
    if rank == 0:
        line = {
            "metric": "cine slices/sec (fwd+bwd) at 10-iter unroll, 1/2/4/8 GPU; PSNR vs ref",
            "value": head["value"],
            "unit": "slices/s",
            "n_gpus": world,
            "world_size": dist.get_world_size() if use_pg else 1,
            "backend": dist.get_backend() if use_pg else None,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": head["ms_per_step"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,            # value / cpu_baseline.value of this same run (set below)
            "vs_baseline_ref": "value / cpu_baseline.value measured in this run on this box's host cores "
                               "(no published number exists, BASELINE.md; null when the CPU leg is skipped). "
                               f"The survey's 8-core container figure was {REFERENCE_CPU_SLICES_PER_S} slices/s",
            "dtype": args.dtype,
            "data": "synthetic (random x_true, normalised random maps, reference VDkt mask seed 1000; random-init weights)",
            "config": {"workload": f"configs/config_swin.yaml, PGD {args.unrolls}-iter unroll, Swin regularizer, "
                                   f"1 cine slice per rank: {args.coils} coils x {args.frames} frames x "
                                   f"{args.ny} x {args.nx}, 2 ESPIRiT maps, train step (fwd+bwd+Adam)",
                       "global_batch": world, "unrolls": args.unrolls,
                       "parallelism": f"dp{world} (one slice per rank, RCCL grad all-reduce)"},
        }
        line.update({k: head[k] for k in ("per_rank_ms_per_step", "allreduce", "roofline", "roofline_conv",
                                          "roofline_sense", "roofline_sense_adj",
                                          "roofline_attention", "roofline_attention_bwd",
                                          "loss")})
        if sec is not None:
            line[other] = sec
        if full is not None:
            line["droppath"] = {
                "note": "headline = train mode with the reference's stochastic depth (DropPath p = linspace(0, 0.2, 6) "
                        "per Swin block, vst:603); a dropped branch skips its forward GEMMs and its backward here, "
                        "the reference's autograd computes them (x 0).  all_branches = the same step with "
                        "drop_prob 0 (every branch computed)",
                "all_branches": {"value": full["value"], "ms_per_step": full["ms_per_step"]},
                "attention_fwd_launches_per_step_headline":
                    (head["roofline_attention"] or {}).get("launches", 0) / args.steps,
            }
        line.update(extra)
        if world == 1 and not args.no_cpu_baseline:
            threads = args.cpu_threads or cpu_threads()
            line["psnr_vs_ref"] = psnr_vs_oracle(model, data, args, threads, [args.dtype] + ([other] if sec else []))
            log("psnr_vs_ref done")
            line["grad_nrmse_vs_f64"] = grad_accuracy(model, data, threads)
            log("grad_nrmse_vs_f64 done")
            line["cpu_baseline"] = cpu_baseline(model, data, args, threads)
            cb = (line["cpu_baseline"] or {}).get("value")
            line["vs_baseline"] = head["value"] / cb if cb else None
        else:
            line["cpu_baseline"] = None
        print(json.dumps(line), flush=True)
    if use_pg:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

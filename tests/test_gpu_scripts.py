"""The entry points on the GPU: scripts/train_swin.py trains a 2-unroll Swin PGD
on synthetic slices (GPU preprocessing, Adam + StepLR, validation, best /
last checkpoints, metrics log), resumes from its checkpoint, and
scripts/reconstruct.py reconstructs CFL k-space with that checkpoint."""
import importlib.util
import json
import math
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CFG = """MODEL:
  MODEL_TYPE: "SWIN"
  META_ARCHITECTURE: "dlespirit"
  PARAMETERS:
    NUM_UNROLLS: 2
    NUM_SWINBLOCKS: 1
    NUM_FEATURES: 160
    NUM_EMAPS: 2
    FIX_STEP_SIZE: True
    SLWIN_INIT: True
    CONV_BLOCK:
      COMPLEX: False
  RECON_LOSS:
    NAME: "complex_l1"
    RENORMALIZE_DATA: False
AUG_TRAIN:
  CROP_READOUT: 16
  UNDERSAMPLE:
    ACCELERATIONS: (4, 6)
    PARTIAL_KX: 0.25
    PARTIAL_KY: 0.25
OPTIMIZER:
  MAX_EPOCHS: 2
EVAL:
  RUN_EVERY_N_EPOCHS: 1
LOGGER:
  LOG_METRICS_EVERY_N_STEPS: 1
SEED: 1000
OUTPUT_DIR: "{out}"
"""


def _script(name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(REPO, "scripts", name + ".py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_train_resume_reconstruct(tmp_path):
    out = tmp_path / "out"
    cfg = tmp_path / "swin.yaml"
    cfg.write_text(CFG.format(out=str(out)))
    tr = _script("train_swin")
    common = ["--config-file", str(cfg), "--data", "synthetic", "--synthetic-slices", "2",
              "--synthetic-shape", "4", "2", "8", "32", "32"]
    tr.main(common)
    ckpts = sorted(p.name for p in out.glob("epoch=*.ckpt"))
    assert (out / "last.ckpt").exists() and len(ckpts) == 1, ckpts
    recs = [json.loads(line) for line in (out / "exp" / "metrics.jsonl").read_text().splitlines()]
    train = [r for r in recs if "Train/complex_l1" in r]
    val = [r for r in recs if "Validate/complex_l1" in r]
    assert len(train) == 4 and len(val) == 2                     # 2 epochs x 2 slices, 2 validations
    assert all(math.isfinite(r["Train/complex_l1"]) for r in train)
    ck = torch.load(out / "last.ckpt", weights_only=True)
    assert ck["epoch"] == 1 and ck["global_step"] == 4 and ck["lr_schedulers"][0]["last_epoch"] == 2
    # resume for one more epoch
    tr.main(common + ["--resume", "--ckpt", str(out / "last.ckpt"), "--max-epochs", "3"])
    ck = torch.load(out / "last.ckpt", weights_only=True)
    assert ck["epoch"] == 2 and ck["global_step"] == 6
    # the restored ModelCheckpoint state keeps one best file (save_top_k = 1) across the resume
    ckpts = sorted(p.name for p in out.glob("epoch=*.ckpt"))
    assert len(ckpts) == 1, ckpts

    # reconstruct CFL k-space (2 slices, 8 coils -> 4 coils to match the maps) with the best checkpoint
    from dl_cs.data.dataset import SyntheticCineDataset
    from dl_cs.fileio import cfl
    ds = SyntheticCineDataset(2, lambda k, m, t, f: (k, m), coils=4, emaps=2, frames=8, ny=32, nx=32, seed=5)
    ks = np.stack([ds[i][0] for i in range(2)])                  # [sl, C, T, Y, X]
    maps = np.stack([ds[i][1] for i in range(2)])                # [sl, E, C, 1, Y, X]
    ks[:, :, :, ::3] = 0                                         # undersample ky
    X, Y, S, C, T = 32, 32, 2, 4, 8
    cfl.write(str(tmp_path / "ks"), ks.transpose(4, 3, 0, 1, 2).reshape(X, Y, S, C, 1, 1, 1, T), order='F')
    cfl.write(str(tmp_path / "maps"), maps[:, :, :, 0].transpose(4, 3, 0, 2, 1), order='F')
    rc = _script("reconstruct")
    args = rc.create_arg_parser().parse_args(["--directory", str(tmp_path), "--ckpt", str(out / ckpts[0]),
                                              "--config-file", str(cfg), "--device", "0"])
    rc.main(args)
    im = cfl.read(str(tmp_path / "im.dl"), order='F')
    assert im.shape == (X, Y, S, 1, 2, 1, 1, T)
    assert np.isfinite(im).all() and np.abs(im).max() > 0


def _trainer(tmp_path, cfg_text, script="train_swin", cls="Trainer"):
    from dl_cs.config import load_cfg
    out = tmp_path / "out"
    cfg = tmp_path / "c.yaml"
    cfg.write_text(cfg_text.format(out=str(out)))
    mod = _script(script)
    args = mod.create_arg_parser().parse_args(["--config-file", str(cfg), "--data", "synthetic",
                                               "--synthetic-slices", "2", "--synthetic-shape", "4", "2", "8", "32",
                                               "32"])
    return getattr(mod, cls)(load_cfg(str(cfg)), args, 0, 1, torch.device("cuda", 0)), args


def test_train_swin_first_loss_vs_oracle(tmp_path):
    """The training script's forward + loss on its own first (GPU-preprocessed) batch
    vs the fp32 oracle on the same batch and weights (NRMSE of the prediction
    <= 1e-5, loss to 1e-5 relative)."""
    from oracle import dlcs_oracle as O
    tr, _ = _trainer(tmp_path, CFG)
    tr.model.eval()
    mod = _script("train_swin")
    batch = next(mod.batches(tr.train_ds, 1, 0, 1, True, tr.cfg.SEED))
    with torch.no_grad():
        pred, target = tr._forward(batch)
        loss = mod.compute_metrics(tr.cfg, pred, target)["Train/complex_l1"]
        kspace, mask, maps, init, scale, tgt = (t.cpu() for t in batch)
        sd = {k: v.detach().cpu() for k, v in tr.model.state_dict().items()}
        ref = O.pgd(O.split_unrolls(sd, 2), kspace, maps, mask, x0=init)
    assert O.nrmse(ref, pred.cpu()) < 1e-5
    lo = float(O.l1(tgt, ref))
    assert abs(float(loss) - lo) < 1e-5 * lo
    tr.buckets.close()


GAN_CFG = CFG + """GAN:
  ADV_WEIGHT: 0.01
  D_FEATURES: 32
  D_LR: 0.0001
  D_STEPS: 1
"""


def test_train_swin_gan_script(tmp_path):
    """scripts/train_swin_gan.py (BASELINE config 3, build-defined): alternating D / G
    steps train, checkpoint with the discriminator state, and resume."""
    out = tmp_path / "out"
    cfg = tmp_path / "gan.yaml"
    cfg.write_text(GAN_CFG.format(out=str(out)))
    gan = _script("train_swin_gan")
    common = ["--config-file", str(cfg), "--data", "synthetic", "--synthetic-slices", "2",
              "--synthetic-shape", "4", "2", "8", "32", "32", "--max-epochs", "1"]
    gan.main(common)
    ck = torch.load(out / "last.ckpt", weights_only=True)
    assert "discriminator_state_dict" in ck and ck["global_step"] == 2
    recs = [json.loads(line) for line in (out / "exp" / "metrics.jsonl").read_text().splitlines()]
    tr = [r for r in recs if "d_loss" in r]
    assert len(tr) == 2 and all(math.isfinite(r["d_loss"]) and math.isfinite(r["g_adv"]) for r in tr)
    gan.main(common[:-1] + ["2", "--resume", "--ckpt", str(out / "last.ckpt")])
    assert torch.load(out / "last.ckpt", weights_only=True)["global_step"] == 4


DIT_CFG = """MODEL:
  MODEL_TYPE: "DiT"
  META_ARCHITECTURE: "DDPM_X"
  PARAMETERS:
    NUM_UNROLLS: 2
    NUM_RESBLOCKS: 0
    NUM_LAYERS: 2
    NUM_HEADS: 16
    NUM_FEATURES: 384
    NUM_EMAPS: 2
    FIX_STEP_SIZE: True
    LEARN_SIGMA: False
    NOISE_SCHED: "linear"
    CONV_BLOCK:
      COMPLEX: False
  RECON_LOSS:
    NAME: "complex_l1"
    RENORMALIZE_DATA: False
AUG_TRAIN:
  CROP_READOUT: 16
  UNDERSAMPLE:
    ACCELERATIONS: (4, 6)
    PARTIAL_KX: 0.25
    PARTIAL_KY: 0.25
OPTIMIZER:
  MAX_EPOCHS: 1
EVAL:
  RUN_EVERY_N_EPOCHS: 1
LOGGER:
  LOG_METRICS_EVERY_N_STEPS: 1
SEED: 1000
OUTPUT_DIR: "{out}"
"""


def test_train_dit_script_and_loss_vs_oracle(tmp_path):
    """scripts/train_DiT.py (BASELINE config 5, DDPM_X): the k-space diffusion loss of
    a fixed batch / t / noise / sub-mask vs the oracle (fp32, 1e-5 relative), then a
    one-epoch run with EMA and checkpoints."""
    from oracle import dit_oracle as DO
    from oracle import dlcs_oracle as O
    from dl_cs.mri import transforms as T
    tr, args = _trainer(tmp_path, DIT_CFG, "train_DiT", "DiTTrainer")
    mod = _script("train_swin")
    _, mask, maps, init, scale, target = next(mod.batches(tr.train_ds, 1, 0, 1, True, tr.cfg.SEED))
    dit = _script("train_DiT")
    mask_r, mask_p = dit.submask(mask, 0.9, torch.Generator().manual_seed(3))
    # the split: per frame, the sampled ky lines partitioned 10 % / 90 %
    assert torch.equal((mask_r + mask_p), mask) and float((mask_r * mask_p).abs().sum()) == 0.0
    t = torch.tensor([321], device=mask.device)
    noise = torch.randn((1, 4) + tuple(target.shape[2:]), generator=torch.Generator().manual_seed(4)).to(mask.device)
    kw = dict(A=T.SenseModel(maps, weights=mask_p), A_1=T.SenseModel(maps, weights=1 - mask_p), A_F=T.SenseModel(maps),
              A_S=T.SenseModel(maps, weights=mask_r), fs=target, c=torch.tensor([1], device=mask.device))
    tr.model.eval()
    with torch.no_grad():
        terms, out, _ = tr.diffusion.training_kspace_loss(tr.model, target, t, kw, noise=noise)
        sd = {k: v.detach().cpu() for k, v in tr.model.state_dict().items()}
        Ps = DO.split_unrolls(sd, 2)
        mc, mpc = maps.cpu(), mask_p.cpu()
        model = lambda xt: DO.data_consistency(Ps, xt, t.cpu(), torch.tensor([1]), mc, mpc, 2, 16,  # noqa: E731
                                               pos_table=sd["nn_update.0.DiT.pos_embedder.pos_embed_table"][0])
        lo, ref, _ = DO.training_kspace_loss(model, target.cpu(), t.cpu(), mc, target.cpu(), noise.cpu())
    assert O.nrmse(ref, out.cpu()) < 1e-5
    assert abs(float(terms["loss"]) - float(lo)) < 1e-5 * float(lo)
    tr.fit()
    ck = torch.load(tmp_path / "out" / "last.ckpt", weights_only=True)
    # the EMA copy is a child of the reference's LightningModule: 'ema.<name>' entries
    ema_keys = {k[4:] for k in ck["state_dict"] if k.startswith("ema.")}
    assert ck["global_step"] == 2 and ema_keys == set(tr.ema.state_dict())
    # resume (train_DiT.py:537/563): model, optimizer, counters and the EMA weights come back
    tr2, _ = _trainer(tmp_path, DIT_CFG, "train_DiT", "DiTTrainer")
    tr2.resume(str(tmp_path / "out" / "last.ckpt"))
    assert tr2.global_step == 2 and tr2.epoch == ck["epoch"] + 1
    for k, v in tr2.ema.state_dict().items():
        assert torch.equal(v.cpu(), ck["state_dict"]["ema." + k]), k
    for k, v in tr2.model.state_dict().items():
        assert torch.equal(v.cpu(), ck["state_dict"]["model." + k]), k
    assert len(tr2.opt.state_dict()["state"]) == len(ck["optimizer_states"][0]["state"])


def test_reconstruct_h5(tmp_path):
    """scripts/reconstruct_h5.py (rh5:370-485) on a 2-slice file (.npz with the H5
    keys): --acceleration 4 undersamples with the seed-1000 VDkt mask and runs the
    model (vs calling the model on the same DataTransform outputs); --acceleration
    1 writes the scaled A^H y guess with no network call; CFL layout [x, y, sl,
    emap, phase, 1, 1, 1]."""
    from dl_cs import checkpoint
    from dl_cs.config import load_cfg
    from dl_cs.data.dataset import SyntheticCineDataset
    from dl_cs.data.preprocess import DataTransform
    from dl_cs.fileio import cfl
    from dl_cs.mri import subsample as ss
    from dl_cs.mri import transforms as T
    from oracle import recipe
    rc = _script("reconstruct_h5")
    cfgp = tmp_path / "swin.yaml"
    cfgp.write_text(CFG.format(out=str(tmp_path / "o")))
    config = load_cfg(str(cfgp))
    model = _script("reconstruct").build_model(config)
    recipe.fill_module(model, 77)
    ck = tmp_path / "m.ckpt"
    torch.save({"state_dict": {"model." + k: v for k, v in model.state_dict().items()}}, ck)
    ds = SyntheticCineDataset(2, lambda k, m, t, f: (k, m), coils=4, emaps=2, frames=8, ny=32, nx=32, seed=9)
    ks = np.stack([ds[i][0] for i in range(2)]).astype(np.complex64)          # [sl, C, T, Y, X]
    maps = np.stack([ds[i][1] for i in range(2)]).astype(np.complex64)        # [sl, E, C, 1, Y, X]
    f = tmp_path / "slices.npz"
    np.savez(f, kspace=ks, maps=maps, target=np.zeros((2, 2, 8, 32, 32), np.complex64))
    for accel in (4, 1):
        args = rc.create_arg_parser().parse_args(["--file", str(f), "--model", "SWIN", "--acceleration", str(accel),
                                                  "--out-directory", str(tmp_path), "--ckpt", str(ck),
                                                  "--config-file", str(cfgp), "--device", "0"])
        rc.main(args)
        im = cfl.read(str(tmp_path / f"slices_{accel}accel.im"), order='F')
        assert im.shape == (32, 32, 2, 2, 8, 1, 1, 1)
        got = np.transpose(im[..., 0, 0, 0], (2, 3, 4, 1, 0))                 # [sl, E, T, Y, X]
        tf = DataTransform(config, device="cuda", fftmod=False, acceleration=accel)
        m = model.to("cuda").eval()
        for sl in range(2):
            k_, mp_, mask_, init_, scale_ = tf(ks[sl], maps[sl])
            if accel > 1:
                ref_mask = ss.VDktMaskFunc((4, 4), sim_partial_kx=0.25, sim_partial_ky=0.25)((1, 1, 8, 32, 32), 1000)
                assert torch.equal(mask_.cpu().float(), ref_mask[0].float())
                with torch.no_grad():
                    x = m(y=k_[None], A=T.SenseModel(mp_[None], weights=mask_[None]), x0=init_[None])[0]
            else:
                x = init_
            want = (scale_ * x).cpu().numpy()
            err = np.linalg.norm(got[sl] - want) / np.linalg.norm(want)
            assert err < 1e-5, (accel, sl, err)

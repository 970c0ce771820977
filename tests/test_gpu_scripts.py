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

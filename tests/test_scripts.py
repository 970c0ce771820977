"""Entry points (scripts/train_swin.py, scripts/reconstruct.py) on CPU: the
reference's command lines parse unchanged, the checkpoint round-trips in the
Lightning layout with the reference's state_dict schema, and CFL data is
transposed the way reconstruct.py:59-107 does.  The GPU runs of both scripts
are tests/test_gpu_scripts.py."""
import importlib.util
import os

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _script(name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(REPO, "scripts", name + ".py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_train_cli_matches_reference():
    m = _script("train_swin")
    a = m.create_arg_parser().parse_args(["--config-file", "c.yaml", "--resume", "--ckpt", "x.ckpt",
                                          "--devices", "0", "1", "2", "--verbose"])
    assert a.config_file == "c.yaml" and a.resume and a.ckpt == "x.ckpt" and a.devices == [0, 1, 2] and a.verbose


def test_reconstruct_cli_matches_reference():
    m = _script("reconstruct")
    a = m.create_arg_parser().parse_args(["--directory", "d", "--ckpt", "c", "--config-file", "f"])
    assert (a.kspace, a.maps, a.out, a.batch_size, a.device, a.multi_gpu) == ("ks", "maps", "im.dl", 1, -1, False)


def test_checkpoint_roundtrip_reference_schema(tmp_path):
    from dl_cs import checkpoint
    from dl_cs.config import get_cfg
    from dl_cs.models import unrolledswin
    from oracle import shapes
    cfg = get_cfg()
    cfg.merge_from_file(os.path.join(REPO, "configs", "config_swin.yaml"))
    cfg.MODEL.PARAMETERS.NUM_UNROLLS = 2
    model = unrolledswin.ProximalGradientDescent(cfg)
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    sched = torch.optim.lr_scheduler.StepLR(opt, 1000, 0.5)
    path = checkpoint.save(str(tmp_path / "epoch=0-step=1.ckpt"), model, opt, sched, 0, 1)
    ck = checkpoint.load(path)
    assert all(k.startswith("model.") for k in ck["state_dict"])
    # the reference's parameter schema (oracle/shapes.py, with the DFE alias keys)
    want = set(shapes.swinnet_param_shapes(with_aliases=True))
    got = {k[len("model.cnn_update.0."):] for k in ck["state_dict"] if k.startswith("model.cnn_update.0.")}
    assert want <= got, sorted(want - got)[:5]
    model2 = unrolledswin.ProximalGradientDescent(cfg)
    checkpoint.load_model(model2, path)
    for (k, a), (_, b) in zip(model.state_dict().items(), model2.state_dict().items()):
        assert torch.equal(a, b), k


def test_cfl_dataset_layout(tmp_path):
    from dl_cs.fileio import cfl
    m = _script("reconstruct")
    X, Y, S, C, Ec, Ph, Em = 6, 5, 3, 4, 1, 7, 2
    rng = np.random.default_rng(0)
    ks = (rng.standard_normal((X, Y, S, C, 1, Ec, 1, Ph)) + 1j * rng.standard_normal((X, Y, S, C, 1, Ec, 1, Ph)))
    mp = (rng.standard_normal((X, Y, S, C, Em)) + 1j * rng.standard_normal((X, Y, S, C, Em)))   # BART ecalib layout
    cfl.write(str(tmp_path / "ks"), ks, order='F')
    cfl.write(str(tmp_path / "maps"), mp, order='F')
    ds = m.CflDataset(str(tmp_path / "ks"), str(tmp_path / "maps"))
    assert len(ds) == S * Ec
    k1, m1 = ds[1]
    assert k1.shape == (C, Ph, Y, X) and m1.shape == (Em, C, 1, Y, X)
    assert np.allclose(k1[2, 3, 4, 5], ks[5, 4, 1, 2, 0, 0, 0, 3])
    assert np.allclose(m1[1, 3, 0, 2, 1], mp[1, 2, 1, 3, 1])
    imgs = rng.standard_normal((S * Ec, Em, Ph, Y, X)).astype(np.complex64)
    ds.write(str(tmp_path / "im"), imgs)
    back = cfl.read(str(tmp_path / "im"), order='F')
    assert back.shape == (X, Y, S, 1, Em, Ec, 1, Ph)
    assert np.allclose(back[4, 2, 1, 0, 1, 0, 0, 5], imgs[1, 1, 5, 2, 4])


def test_shard_indices_pad_like_distributed_sampler():
    """Every rank gets the same number of items (hence batches and bucket
    all-reduces) whatever the dataset size; the union covers the dataset."""
    m = _script("train_swin")
    for n in range(1, 12):
        for world in (1, 2, 3, 4):
            shards = [m.shard_indices(n, r, world, True, 7) for r in range(world)]
            assert len({len(s) for s in shards}) == 1, (n, world)
            assert len(shards[0]) == -(-n // world)
            assert set().union(*map(set, shards)) == set(range(n))
            for bs in (1, 2, 3):
                counts = {len(range(0, len(s), bs)) for s in shards}
                assert len(counts) == 1


def test_resume_restores_model_checkpoint_state(tmp_path):
    """last.ckpt carries the ModelCheckpoint state (best score and file); after a
    resume a worse validation is not a new best, and a better one replaces the
    old best file (save_top_k=1)."""
    from dl_cs.config import get_cfg
    from dl_cs.models import unrolledswin
    m = _script("train_swin")
    cfg = get_cfg()
    cfg.merge_from_file(os.path.join(REPO, "configs", "config_swin.yaml"))
    cfg.MODEL.PARAMETERS.NUM_UNROLLS = 1

    def trainer():
        t = m.Trainer.__new__(m.Trainer)
        t.cfg, t.rank, t.out_dir = cfg, 0, str(tmp_path)
        t.model = unrolledswin.ProximalGradientDescent(cfg)
        t.opt = torch.optim.Adam(t.model.parameters(), lr=1e-4)
        t.sched = torch.optim.lr_scheduler.StepLR(t.opt, 1000, 0.5)
        t.epoch, t.global_step, t.best, t.best_path = 0, 3, float('inf'), None
        return t

    key = f'Validate/{cfg.MODEL.RECON_LOSS.NAME}'
    t1 = trainer()
    t1.checkpoint({key: 0.5})
    first = t1.best_path
    assert os.path.exists(first)
    t2 = trainer()
    t2.resume(str(tmp_path / "last.ckpt"))
    assert t2.best == 0.5 and t2.best_path == first and t2.epoch == 1
    t2.checkpoint({key: 0.7})                          # worse: not a new best
    assert t2.best == 0.5 and t2.best_path == first and os.path.exists(first)
    t2.global_step = 9
    t2.checkpoint({key: 0.3})                          # better: replaces the best file
    assert t2.best == 0.3 and t2.best_path != first and not os.path.exists(first)
    assert os.path.exists(t2.best_path)


def test_model_checkpoint_state_lightning_key():
    """Lightning (>= 1.5) keys the ModelCheckpoint callback state by its state_key, e.g.
    "ModelCheckpoint{'monitor': 'Validate MSE', 'mode': 'min', ...}" (reference
    train_DiT.py:360-375); a checkpoint written by the reference with that key resumes its
    best score / file, and the checkpoints written here carry both key forms."""
    import sys
    sys.path.insert(0, os.path.join(REPO, "dl-swin-gan_amd"))
    from dl_cs import checkpoint
    lk = "ModelCheckpoint{'monitor': 'Validate MSE', 'mode': 'min', 'every_n_train_steps': 0}"
    ck = {"callbacks": {lk: {"best_model_score": torch.tensor(0.25), "best_model_path": "/x/best.ckpt"}}}
    st = checkpoint.model_checkpoint_state(ck)
    assert float(st["best_model_score"]) == 0.25 and st["best_model_path"] == "/x/best.ckpt"
    assert checkpoint.model_checkpoint_state({}) == {}
    out = checkpoint.callback_state("Validate MSE", 0.5, "/y.ckpt")["callbacks"]
    assert out["ModelCheckpoint"]["best_model_score"] == 0.5
    lkeys = [k for k in out if k.startswith("ModelCheckpoint{")]
    assert len(lkeys) == 1 and "'monitor': 'Validate MSE'" in lkeys[0]
    assert checkpoint.model_checkpoint_state({"callbacks": {lkeys[0]: out[lkeys[0]]}})["best_model_path"] == "/y.ckpt"

"""Training entry point of the Swin-unrolled cine reconstruction on MI355X.

Same command line and training semantics as the reference's
scripts/train_swin.py (CLI :269-290, LitUnrolled :33-219, main :222-266), with
the Lightning/DeepSpeed trainer replaced by a plain loop over this package:

  * model: META_ARCHITECTURE 'dlespirit' -> ProximalGradientDescent, 'modl' ->
    HalfQuadraticSplitting (:46-51), forward y=kspace, A=SenseModel(maps,
    weights=mask), x0=initial guess (:116);
  * loss: metrics['Train/<RECON_LOSS.NAME>'] of the complex / magnitude l1, l2,
    psnr set (:53-78, :134), optional RENORMALIZE_DATA rescale (:119-123);
  * Adam(lr=OPTIMIZER.ADAM.LR) + StepLR(LR_SCHEDULER.STEP_SIZE, GAMMA) stepped
    per epoch (:155-166), GRAD_ACCUM_ITERS gradient accumulation;
  * validation every EVAL.RUN_EVERY_N_EPOCHS, best 'Validate/<loss>' checkpoint
    kept as OUTPUT_DIR/epoch=E-step=S.ckpt (save_top_k=1, :182-188) plus
    last.ckpt; --resume --ckpt continues from one (:273-274, :288);
  * data: per-slice files (H5 as the reference, or NPZ with the same keys) or
    synthetic slices, preprocessed ON THE GPU by dl_cs.data.preprocess
    (the reference runs it in CPU DataLoader workers);
  * --devices with several GPUs: one process per GPU, each on its own slices,
    gradients averaged by RCCL all-reduce per unroll (dl_cs.distributed) --
    the reference's Lightning DDP.  Also runs under torchrun.

Metrics are appended to OUTPUT_DIR/exp/metrics.jsonl (TensorBoard is not in
this image); rank 0 prints a progress line per LOG_METRICS_EVERY_N_STEPS.
"""
import argparse
import json
import logging
import os
import random
import socket
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dl-swin-gan_amd"))

from dl_cs import checkpoint  # noqa: E402
from dl_cs.config import load_cfg  # noqa: E402
from dl_cs.utils import metrics as metric  # noqa: E402
from dl_cs.utils import optim  # noqa: E402

logging.basicConfig(level=logging.INFO)
logger = logging.getLogger("train_swin")


def build_model(config):
    """train_swin.py:46-51 (MODEL_TYPE 'SWIN'); MODEL_TYPE 'RES' builds the reference's
    scripts/train.py model -- dl_cs.models.unrolled with the 3-D ResNet of
    configs/example.yaml (BASELINE config 1)."""
    from dl_cs.models import unrolled, unrolledswin
    mod = unrolledswin if config.MODEL.MODEL_TYPE.upper() == 'SWIN' else unrolled
    arch = config.MODEL.META_ARCHITECTURE
    if arch == 'dlespirit':
        return mod.ProximalGradientDescent(config)
    if arch == 'modl':
        return mod.HalfQuadraticSplitting(config)
    raise ValueError('Meta architecture in config file not recognized!')


def compute_metrics(config, prediction, target, is_training=True):
    """train_swin.py:53-78 (VGG losses need a network download: not built)."""
    tag = 'Train' if is_training else 'Validate'
    w = config.MODEL.RECON_LOSS.LOSS_WEIGHT
    m = {f'{tag}/complex_l1': metric.l1(target, prediction, w),
         f'{tag}/complex_l2': metric.l2(target, prediction, w),
         f'{tag}/complex_psnr': metric.psnr(target, prediction, w)}
    mp, mt = prediction.abs(), target.abs()
    m.update({f'{tag}/mag_l1': metric.l1(mt, mp, w), f'{tag}/mag_l2': metric.l2(mt, mp, w),
              f'{tag}/mag_psnr': metric.psnr(mt, mp, w)})
    return m


def make_dataset(config, kind, split, preprocess, n_synthetic, synth_shape):
    from dl_cs.data import dataset as D
    if kind == 'synthetic':
        C, E, T, Y, X = synth_shape
        return D.SyntheticCineDataset(n_synthetic, preprocess, coils=C, emaps=E, frames=T, ny=Y, nx=X,
                                      seed=config.SEED + (0 if split == 'train' else 10 ** 6))
    roots = config.DATASET.TRAIN if split == 'train' else config.DATASET.VAL
    if not roots:
        raise ValueError(f"config DATASET.{split.upper()} is empty (or pass --data synthetic)")
    cls = D.Hdf5Dataset if kind == 'h5' else D.NpzDataset
    return cls(root_directory=roots[0], transform=preprocess, sample_rate=config.DATALOADER.SUBSAMPLE)


def shard_indices(n, rank, world, shuffle, epoch_seed):
    """Per-rank indices of a DistributedSampler: the (shuffled) index list is
    padded by repeating from its start to a multiple of `world`, so every rank
    gets the same number of items -- and hence of batches and of bucket
    all-reduces (a rank with an extra batch would start collectives the others
    never join)."""
    idx = list(range(n))
    if shuffle:
        random.Random(epoch_seed).shuffle(idx)
    if n and n % world:
        pad = world - n % world
        idx += (idx * (pad // n + 1))[:pad]
    return idx[rank::world]


def batches(ds, batch_size, rank, world, shuffle, epoch_seed):
    """Per-rank shard of the dataset (shard_indices), stacked on device."""
    idx = shard_indices(len(ds), rank, world, shuffle, epoch_seed)
    for i in range(0, len(idx), batch_size):
        items = [ds[j] for j in idx[i:i + batch_size]]
        yield tuple(torch.stack([torch.as_tensor(it[k]) for it in items]) for k in range(len(items[0])))


class Trainer:
    def __init__(self, config, args, rank, world, device):
        from dl_cs.data.preprocess import CinePreprocess
        from dl_cs.distributed import GradBuckets, broadcast_parameters
        from dl_cs.models import swin3D
        self.cfg, self.args, self.rank, self.world, self.device = config, args, rank, world, device
        swin3D.set_compute_dtype(torch.bfloat16 if args.dtype == 'bf16' else torch.float32)
        torch.manual_seed(config.SEED)
        self.model = build_model(config).to(device)
        if world > 1:
            broadcast_parameters(self.model, 0)
        self.opt = optim.adam([p for p in self.model.parameters() if p.requires_grad], lr=config.OPTIMIZER.ADAM.LR)
        self.sched = torch.optim.lr_scheduler.StepLR(self.opt, step_size=config.LR_SCHEDULER.STEP_SIZE,
                                                     gamma=config.LR_SCHEDULER.GAMMA)
        # the fused Swin backward writes straight into the buckets; other networks use hooks
        self.buckets = GradBuckets(self.model, world, direct=config.MODEL.MODEL_TYPE.upper() == 'SWIN')
        synth = tuple(args.synthetic_shape)
        self.train_ds = make_dataset(config, args.data, 'train', CinePreprocess(config, use_seed=False, device=device),
                                     args.synthetic_slices, synth)
        self.val_ds = make_dataset(config, args.data, 'val', CinePreprocess(config, use_seed=True, device=device),
                                   max(1, args.synthetic_slices // 4), synth)
        self.epoch, self.global_step = 0, 0
        self.best, self.best_path = float('inf'), None
        self.out_dir = config.OUTPUT_DIR
        self.log_path = os.path.join(self.out_dir, 'exp', 'metrics.jsonl')
        if rank == 0:
            os.makedirs(os.path.dirname(self.log_path), exist_ok=True)

    # ---------------------------------------------------------------- state
    def resume(self, path):
        ck = checkpoint.load_model(self.model, path)
        if ck.get('optimizer_states'):
            self.opt.load_state_dict(ck['optimizer_states'][0])
        if ck.get('lr_schedulers'):
            self.sched.load_state_dict(ck['lr_schedulers'][0])
        self.epoch = int(ck.get('epoch', -1)) + 1
        self.global_step = int(ck.get('global_step', 0))
        mc = checkpoint.model_checkpoint_state(ck)     # Lightning's callback state (plain or state_key)
        if mc.get('best_model_score') is not None:
            self.best = float(mc['best_model_score'])
            self.best_path = mc.get('best_model_path')
        logger.info(f"resumed from {path}: epoch {self.epoch}, step {self.global_step}")

    def _log(self, rec):
        if self.rank == 0:
            with open(self.log_path, 'a') as f:
                f.write(json.dumps(rec) + '\n')

    # ---------------------------------------------------------------- steps
    def _forward(self, batch):
        from dl_cs.mri import transforms as T
        kspace, mask, maps, init, scale, target = batch                   # preprocess.py:180
        pred = self.model(y=kspace, A=T.SenseModel(maps, weights=mask), x0=init)
        if self.cfg.MODEL.RECON_LOSS.RENORMALIZE_DATA:                     # train_swin.py:119-123
            s = scale.view(-1, 1, 1, 1, 1)
            pred, target = pred * s, target * s
        return pred, target

    def train_epoch(self):
        cfg, accum = self.cfg, max(1, self.cfg.OPTIMIZER.GRAD_ACCUM_ITERS)
        self.model.train()
        t0 = time.time()
        for i, batch in enumerate(batches(self.train_ds, cfg.DATALOADER.TRAIN_BATCH_SIZE, self.rank, self.world,
                                          True, cfg.SEED + self.epoch)):
            if i % accum == 0:
                self.buckets.zero()
            # only the last micro-batch of an accumulation window starts the
            # bucket all-reduces: earlier ones accumulate locally
            self.buckets.armed = (i + 1) % accum == 0
            pred, target = self._forward(batch)
            m = compute_metrics(cfg, pred, target, is_training=True)
            loss = m[f'Train/{cfg.MODEL.RECON_LOSS.NAME}']
            (loss / accum).backward()
            if (i + 1) % accum == 0:
                self.buckets.finish()
                self.opt.step()
                self.global_step += 1
                if self.global_step % cfg.LOGGER.LOG_METRICS_EVERY_N_STEPS == 0 or self.args.verbose:
                    rec = {k: float(v) for k, v in m.items()}
                    rec.update(epoch=self.epoch, step=self.global_step, lr=self.sched.get_last_lr()[0],
                               slices_per_s=(i + 1) * self.world / (time.time() - t0))
                    self._log(rec)
                    if self.rank == 0:
                        logger.info(f"epoch {self.epoch} step {self.global_step} loss {float(loss):.5f}")
            if self.args.max_steps and self.global_step >= self.args.max_steps:
                break
        self.sched.step()                                                   # StepLR per epoch

    @torch.no_grad()
    def validate(self):
        cfg = self.cfg
        self.model.eval()
        sums, n = {}, 0
        for batch in batches(self.val_ds, cfg.DATALOADER.VAL_BATCH_SIZE, self.rank, self.world, False, 0):
            pred, target = self._forward(batch)
            for k, v in compute_metrics(cfg, pred, target, is_training=False).items():
                sums[k] = sums.get(k, 0.0) + float(v) * pred.shape[0]
            n += pred.shape[0]
        keys = sorted(sums) if sums else sorted(compute_metrics(cfg, torch.zeros(1, 1, 1, 1, 1, dtype=torch.complex64),
                                                                torch.ones(1, 1, 1, 1, 1, dtype=torch.complex64),
                                                                False))
        vec = torch.tensor([sums.get(k, 0.0) for k in keys] + [float(n)], dtype=torch.float64, device=self.device)
        if self.world > 1:
            dist.all_reduce(vec)                                             # sync_dist
        total = max(1.0, float(vec[-1]))
        res = {k: float(vec[i]) / total for i, k in enumerate(keys)}
        res.update(epoch=self.epoch, step=self.global_step)
        self._log(res)
        return res

    def checkpoint(self, val):
        if self.rank != 0:
            return
        key = f'Validate/{self.cfg.MODEL.RECON_LOSS.NAME}'
        if val is not None and val.get(key, float('inf')) < self.best:       # save_top_k=1, mode='min'
            self.best = val[key]
            path = os.path.join(self.out_dir, f'epoch={self.epoch}-step={self.global_step}.ckpt')
            checkpoint.save(path, self.model, self.opt, self.sched, self.epoch, self.global_step,
                            extra=self._callback_state(key, path))
            if self.best_path and self.best_path != path and os.path.exists(self.best_path):
                os.remove(self.best_path)
            self.best_path = path
            logger.info(f"new best {key} = {self.best:.6f}: {path}")
        # last.ckpt carries the ModelCheckpoint state too, so a resume keeps the best score / file
        checkpoint.save(os.path.join(self.out_dir, 'last.ckpt'), self.model, self.opt, self.sched,
                        self.epoch, self.global_step, extra=self._callback_state(key, self.best_path))

    def _callback_state(self, key, path):
        best = self.best if self.best != float('inf') else None
        return checkpoint.callback_state(key, best, path)

    def fit(self):
        cfg = self.cfg
        max_epochs = self.args.max_epochs or cfg.OPTIMIZER.MAX_EPOCHS
        while self.epoch < max_epochs:
            self.train_epoch()
            val = None
            if (self.epoch + 1) % cfg.EVAL.RUN_EVERY_N_EPOCHS == 0:
                val = self.validate()
            self.checkpoint(val)
            self.epoch += 1
            if self.args.max_steps and self.global_step >= self.args.max_steps:
                break
        self.buckets.close()


def run(rank, world, args, devices, port=None):
    if port is not None:
        os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK=str(rank))
    local = int(os.environ.get('LOCAL_RANK', rank))
    dev_index = devices[local] if devices else local
    torch.cuda.set_device(dev_index)
    device = torch.device('cuda', dev_index)
    if world > 1:
        dist.init_process_group('nccl', device_id=device)
    config = load_cfg(args.config_file)
    random.seed(config.SEED)                                                 # train_swin.py:283-285
    np.random.seed(config.SEED)
    torch.manual_seed(config.SEED)
    if rank == 0:
        os.makedirs(config.OUTPUT_DIR, exist_ok=True)
    cls = Trainer
    if getattr(args, 'trainer', None) == 'gan':            # scripts/train_swin_gan.py
        from train_swin_gan import GanTrainer as cls
    tr = cls(config, args, rank, world, device)
    if args.resume:
        if not args.ckpt:
            raise ValueError('--resume needs --ckpt')
        tr.resume(args.ckpt)
    tr.fit()
    if world > 1:
        dist.destroy_process_group()


def _spawn_entry(rank, world, args, devices, port):
    run(rank, world, args, devices, port)


def create_arg_parser():
    p = argparse.ArgumentParser(description="Training script for unrolled MRI recon.")
    p.add_argument('--config-file', type=str, required=True, help='Training config file (yaml)')
    p.add_argument('--resume', action='store_true', help='Resume training from checkpoint')
    p.add_argument('--ckpt', type=str, help='Checkpoint file to resume training from')
    p.add_argument('--devices', type=int, nargs='+', help='GPU devices')
    p.add_argument('--verbose', action='store_true', help='Turn on debug statements')
    # additions of this build
    p.add_argument('--data', choices=['h5', 'npz', 'synthetic'], default='h5',
                   help='slice files under DATASET.TRAIN / VAL (h5 as the reference, or npz), or synthetic slices')
    p.add_argument('--synthetic-slices', type=int, default=8, help='training slices with --data synthetic')
    p.add_argument('--synthetic-shape', type=int, nargs=5, default=[8, 2, 20, 192, 160], metavar=('C', 'E', 'T', 'Y', 'X'))
    p.add_argument('--dtype', choices=['fp32', 'bf16'], default='fp32', help='compute dtype of the regularizer')
    p.add_argument('--max-epochs', type=int, default=0, help='override OPTIMIZER.MAX_EPOCHS')
    p.add_argument('--max-steps', type=int, default=0, help='stop after this many optimizer steps')
    return p


def main(argv=None):
    main_args(create_arg_parser().parse_args(argv))


def main_args(args):
    devices = args.devices or []
    if 'RANK' in os.environ and 'WORLD_SIZE' in os.environ:                 # torchrun
        run(int(os.environ['RANK']), int(os.environ['WORLD_SIZE']), args, devices)
    elif len(devices) > 1:
        with socket.socket() as s:
            s.bind(('127.0.0.1', 0))
            port = s.getsockname()[1]
        torch.multiprocessing.spawn(_spawn_entry, args=(len(devices), args, devices, port), nprocs=len(devices),
                                    join=True)
    else:
        run(0, 1, args, devices)


if __name__ == '__main__':
    main()

"""Training entry point of the DiT- and Latte-unrolled cine reconstruction on MI355X
(BASELINE config 5: configs/config_dit.yaml, configs/config_latte.yaml -- MODEL_TYPE
'Latte' is the reference's scripts/train_Latte.py, the same loop on unrolledLatte).

Same command line and training semantics as the reference's scripts/train_DiT.py
(LitUnrolled :87-432, CLI at the end of the file), with the Lightning / DeepSpeed
trainer replaced by the plain loop of scripts/train_swin.py:

  * model: META_ARCHITECTURE 'DDPM_X' -> unrolledDiT.DataConsistency, 'DDPM_E' ->
    DDPM, 'dlespirit' -> ProximalGradientDescent, 'modl' -> HalfQuadraticSplitting
    (:101-113);
  * diffusion: create_diffusion('', NOISE_SCHED, 1000 steps, LEARN_SIGMA,
    predict_xstart) (:115-129);
  * training_step (:232-288): t ~ U{0..999}; DDPM_X: (mask_r, mask_p) =
    submask(mask, 0.9), A = S(maps, mask_p), A_1 = S(maps, 1 - mask_p),
    A_F = S(maps), A_S = S(maps, mask_r); loss = training_kspace_loss on the
    fully-sampled target; DDPM_E: training_losses (MSE);
  * Adam(lr) + StepLR (:386-395), EMA of the weights after every optimizer step
    (update_ema, decay 0.9999, :58-72, :429-432), best 'Validate MSE' checkpoint.
Data, multi-GPU (one process per GPU, RCCL gradient all-reduce) and checkpoint
layout as scripts/train_swin.py.
"""
import argparse
import copy
import logging
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dl-swin-gan_amd"))
sys.path.insert(0, os.path.join(REPO, "scripts"))

from dl_cs.utils import optim  # noqa: E402

logging.basicConfig(level=logging.INFO)
logger = logging.getLogger("train_DiT")


def submask(mask, factor, generator=None):
    """train_DiT.py:153-176 -- per frame, a random `factor` fraction of the sampled ky
    lines goes to mask_r (the rest zeroed there) and the complement to mask_p.
    mask [B, 1, T, Y, X]; returns (mask_r, mask_p).  The random permutation is drawn
    on the host (torch.randperm, like the reference)."""
    T = mask.shape[2]
    mask_r, mask_p = mask.detach().clone(), mask.detach().clone()
    rows = (mask.detach().sum(dim=(0, 1, 4)) != 0)                   # [T, Y]: sampled ky lines per frame
    for f in range(T):
        idx = torch.nonzero(rows[f], as_tuple=False).reshape(-1).cpu()
        n = idx.numel()
        perm = torch.randperm(n, generator=generator)
        k = int(n * factor)
        drop, keep = idx[perm[:k]].to(mask.device), idx[perm[k:]].to(mask.device)
        mask_r[:, :, f, drop, :] = 0
        mask_p[:, :, f, keep, :] = 0
    return mask_r, mask_p


def build_model(config):
    """MODEL_TYPE 'Latte' takes the unrolledLatte drivers (the reference's
    scripts/train_Latte.py, ulat:101-113 -- same training step), else unrolledDiT."""
    from dl_cs.models import unrolledDiT, unrolledLatte
    arch = config.MODEL.META_ARCHITECTURE
    mod = unrolledLatte if getattr(config.MODEL, "MODEL_TYPE", "DiT") == "Latte" else unrolledDiT
    table = {'dlespirit': mod.ProximalGradientDescent, 'modl': mod.HalfQuadraticSplitting,
             'DDPM_X': mod.DataConsistency, 'DDPM_E': mod.DDPM}
    if arch not in table:
        raise ValueError('Meta architecture in config file not recognized!')
    return table[arch](config)


@torch.no_grad()
def update_ema(ema_model, model, decay=0.9999):
    """train_DiT.py:58-72"""
    ep, mp = list(ema_model.parameters()), list(model.parameters())
    torch._foreach_lerp_(ep, mp, 1.0 - decay)


class DiTTrainer:
    def __init__(self, config, args, rank, world, device):
        from train_swin import make_dataset
        from dl_cs.data.preprocess import CinePreprocess
        from dl_cs.diffusion import create_diffusion
        from dl_cs.distributed import GradBuckets, broadcast_parameters
        self.cfg, self.args, self.rank, self.world, self.device = config, args, rank, world, device
        torch.manual_seed(config.SEED)
        self.model = build_model(config).to(device)
        if world > 1:
            broadcast_parameters(self.model, 0)
        self.ema = copy.deepcopy(self.model)
        for p in self.ema.parameters():
            p.requires_grad_(False)
        P = config.MODEL.PARAMETERS
        self.predict_xstart = config.MODEL.META_ARCHITECTURE != 'DDPM_E'
        self.diffusion = create_diffusion(timestep_respacing="", noise_schedule=P.NOISE_SCHED, diffusion_steps=1000,
                                          learn_sigma=P.LEARN_SIGMA, predict_xstart=self.predict_xstart)
        self.opt = optim.adam([p for p in self.model.parameters() if p.requires_grad], lr=config.OPTIMIZER.ADAM.LR)
        self.sched = torch.optim.lr_scheduler.StepLR(self.opt, step_size=config.LR_SCHEDULER.STEP_SIZE,
                                                     gamma=config.LR_SCHEDULER.GAMMA)
        self.buckets = GradBuckets(self.model, world, direct=False)
        synth = tuple(args.synthetic_shape)
        self.train_ds = make_dataset(config, args.data, 'train', CinePreprocess(config, use_seed=False, device=device),
                                     args.synthetic_slices, synth)
        self.val_ds = make_dataset(config, args.data, 'val', CinePreprocess(config, use_seed=True, device=device),
                                   max(1, args.synthetic_slices // 4), synth)
        self.epoch, self.global_step = 0, 0
        self.best, self.best_path = float('inf'), None
        self.gen = torch.Generator(device="cpu").manual_seed(config.SEED + rank)

    def loss(self, batch, initial=False):
        """train_DiT.py:232-265 (training) / :290-327 (validation: on the initial guess)."""
        from dl_cs.mri import transforms as T
        _, mask, maps, init, scale, target = batch
        t = torch.randint(0, self.diffusion.num_timesteps, (init.shape[0],), device=self.device)
        c = torch.tensor([1], device=self.device)
        if self.cfg.MODEL.RECON_LOSS.RENORMALIZE_DATA:
            s = scale.view(-1, 1, 1, 1, 1)
            init, target = init * s, target * s
        x_start = init if initial else target
        if self.cfg.MODEL.META_ARCHITECTURE == 'DDPM_E':
            kw = dict(A=T.SenseModel(maps, weights=mask), A_1=T.SenseModel(maps, weights=1 - mask),
                      A_F=T.SenseModel(maps), fs=target, c=c)
            terms, _, _ = self.diffusion.training_losses(self.model, x_start, t, kw)
            return terms["loss"].mean()
        mask_r, mask_p = submask(mask, 0.9, self.gen)
        kw = dict(A=T.SenseModel(maps, weights=mask_p), A_1=T.SenseModel(maps, weights=1 - mask_p),
                  A_F=T.SenseModel(maps), A_S=T.SenseModel(maps, weights=mask_r), fs=target, c=c)
        terms, _, _ = self.diffusion.training_kspace_loss(self.model, x_start, t, kw)
        return terms["loss"]

    def train_epoch(self):
        from train_swin import batches
        self.model.train()
        for batch in batches(self.train_ds, self.cfg.DATALOADER.TRAIN_BATCH_SIZE, self.rank, self.world, True,
                             self.cfg.SEED + self.epoch):
            self.buckets.zero()
            loss = self.loss(batch)
            loss.backward()
            self.buckets.finish()
            self.opt.step()
            update_ema(self.ema, self.model)
            self.global_step += 1
            if self.rank == 0 and (self.global_step % self.cfg.LOGGER.LOG_METRICS_EVERY_N_STEPS == 0 or
                                   self.args.verbose):
                logger.info(f"epoch {self.epoch} step {self.global_step} Train MSE {float(loss):.5f}")
            if self.args.max_steps and self.global_step >= self.args.max_steps:
                break
        self.sched.step()

    @torch.no_grad()
    def validate(self):
        from train_swin import batches
        self.model.eval()
        tot, n = 0.0, 0
        for batch in batches(self.val_ds, self.cfg.DATALOADER.VAL_BATCH_SIZE, self.rank, self.world, False, 0):
            tot += float(self.loss(batch, initial=True))
            n += 1
        v = torch.tensor([tot, n], dtype=torch.float64, device=self.device)
        if self.world > 1:
            torch.distributed.all_reduce(v)
        return float(v[0]) / max(1.0, float(v[1]))

    def checkpoint(self, val):
        from dl_cs import checkpoint
        if self.rank != 0:
            return
        os.makedirs(self.cfg.OUTPUT_DIR, exist_ok=True)
        # the EMA copy is a child of the reference's LightningModule (self.ema,
        # train_DiT.py:133): its weights go into the same state_dict as 'ema.<name>'
        sub = {'ema': self.ema}
        if val < self.best:
            self.best = val
            path = os.path.join(self.cfg.OUTPUT_DIR, f'epoch={self.epoch}-step={self.global_step}.ckpt')
            checkpoint.save(path, self.model, self.opt, self.sched, self.epoch, self.global_step,
                            extra=self._callback_state(path), submodules=sub)
            if self.best_path and os.path.exists(self.best_path) and self.best_path != path:
                os.remove(self.best_path)
            self.best_path = path
        checkpoint.save(os.path.join(self.cfg.OUTPUT_DIR, 'last.ckpt'), self.model, self.opt, self.sched,
                        self.epoch, self.global_step, extra=self._callback_state(self.best_path), submodules=sub)

    def _callback_state(self, path):
        from dl_cs import checkpoint
        best = self.best if self.best != float('inf') else None
        return checkpoint.callback_state('Validate MSE', best, path)

    def resume(self, path):
        """trainer.fit(ckpt_path=args.ckpt) (train_DiT.py:537/563): model, optimizer,
        scheduler, epoch / step counters, the best-checkpoint state and the EMA
        weights ('ema.<name>' entries; a checkpoint without them starts the EMA
        from the loaded model, as on_train_start's update_ema(decay=0), :424-427)."""
        from dl_cs import checkpoint
        ck = checkpoint.load_model(self.model, path)
        ema = checkpoint.submodule_state_dict(ck, 'ema') or ck.get('ema_state_dict')
        if ema:
            self.ema.load_state_dict(ema)
        else:
            update_ema(self.ema, self.model, decay=0.0)
        if ck.get('optimizer_states'):
            self.opt.load_state_dict(ck['optimizer_states'][0])
        if ck.get('lr_schedulers'):
            self.sched.load_state_dict(ck['lr_schedulers'][0])
        self.epoch = int(ck.get('epoch', -1)) + 1
        self.global_step = int(ck.get('global_step', 0))
        mc = checkpoint.model_checkpoint_state(ck)     # plain or Lightning state_key
        if mc.get('best_model_score') is not None:
            self.best = float(mc['best_model_score'])
            self.best_path = mc.get('best_model_path')
        logger.info(f"resumed from {path}: epoch {self.epoch}, step {self.global_step}")

    def fit(self):
        max_epochs = self.args.max_epochs or self.cfg.OPTIMIZER.MAX_EPOCHS
        while self.epoch < max_epochs:
            self.train_epoch()
            val = self.validate() if (self.epoch + 1) % self.cfg.EVAL.RUN_EVERY_N_EPOCHS == 0 else float('inf')
            if self.rank == 0:
                logger.info(f"epoch {self.epoch} Validate MSE {val:.5f}")
            self.checkpoint(val)
            self.epoch += 1
            if self.args.max_steps and self.global_step >= self.args.max_steps:
                break
        self.buckets.close()


def run(rank, world, args, devices, port=None):
    import random
    from dl_cs.config import load_cfg
    if port is not None:
        os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK=str(rank))
    local = int(os.environ.get('LOCAL_RANK', rank))
    dev_index = devices[local] if devices else local
    torch.cuda.set_device(dev_index)
    device = torch.device('cuda', dev_index)
    if world > 1:
        torch.distributed.init_process_group('nccl', device_id=device)
    config = load_cfg(args.config_file)
    random.seed(config.SEED)
    np.random.seed(config.SEED)
    torch.manual_seed(config.SEED)
    tr = DiTTrainer(config, args, rank, world, device)
    if args.resume:
        if not args.ckpt:
            raise ValueError('--resume needs --ckpt')
        tr.resume(args.ckpt)
    tr.fit()
    if world > 1:
        torch.distributed.destroy_process_group()


def create_arg_parser():
    from train_swin import create_arg_parser as base
    p = base()
    p.description = "Training script for DiT-unrolled MRI recon."
    return p


def main(argv=None):
    import socket
    args = create_arg_parser().parse_args(argv)
    if args.dtype != 'fp32':
        raise SystemExit('train_DiT: the DiT / Latte path trains in fp32 (--dtype bf16 is a Swin-path option)')
    devices = args.devices or []
    if 'RANK' in os.environ and 'WORLD_SIZE' in os.environ:
        run(int(os.environ['RANK']), int(os.environ['WORLD_SIZE']), args, devices)
    elif len(devices) > 1:
        with socket.socket() as s:
            s.bind(('127.0.0.1', 0))
            port = s.getsockname()[1]
        torch.multiprocessing.spawn(run, args=(len(devices), args, devices, port), nprocs=len(devices), join=True)
    else:
        run(0, 1, args, devices)


if __name__ == '__main__':
    main()

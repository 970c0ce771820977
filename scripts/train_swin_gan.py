"""Swin-GAN training (BASELINE config 3: configs/config_swingan.yaml) on MI355X.

The reference names this run (run_script.sh:29, :45-47, :144-155:
scripts/train_swin_gan.py with configs/config_swingan.yaml) but ships neither
the script nor a discriminator, so the adversarial part is this build's spec
(parity unpinned against the reference):

  * generator = the Swin-unrolled PGD of scripts/train_swin.py (same config keys);
  * discriminator = dl_cs.models.patchgan.PatchGANDiscriminator3D(2E, GAN.D_FEATURES);
  * per batch: GAN.D_STEPS discriminator steps on BCE(D(target), 1) + BCE(D(G(y)), 0)
    (G's output detached), then one generator step on
    Train/<RECON_LOSS.NAME> + GAN.ADV_WEIGHT * BCE(D(G(y)), 1);
  * Adam for both (OPTIMIZER.ADAM.LR for G, GAN.D_LR for D), StepLR for G.
Everything else (data, validation, checkpoints -- the discriminator's state is
stored under 'discriminator_state_dict' -- and multi-GPU) is scripts/train_swin.py.
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dl-swin-gan_amd"))
sys.path.insert(0, os.path.join(REPO, "scripts"))

import train_swin  # noqa: E402
from dl_cs.utils import optim  # noqa: E402


class GanTrainer(train_swin.Trainer):
    def __init__(self, config, args, rank, world, device):
        super().__init__(config, args, rank, world, device)
        from dl_cs.distributed import broadcast_parameters
        from dl_cs.models import patchgan
        E = config.MODEL.PARAMETERS.NUM_EMAPS
        torch.manual_seed(config.SEED + 1)
        self.D = patchgan.PatchGANDiscriminator3D(2 * E, config.GAN.D_FEATURES).to(device)
        if world > 1:
            broadcast_parameters(self.D, 0)
        self.optD = optim.adam(self.D.parameters(), lr=config.GAN.D_LR)

    def _d_allreduce(self):
        if self.world > 1:
            for p in self.D.parameters():
                torch.distributed.all_reduce(p.grad)
                p.grad.mul_(1.0 / self.world)

    def train_epoch(self):
        from dl_cs.models import patchgan
        cfg = self.cfg
        self.model.train()
        self.D.train()
        for i, batch in enumerate(train_swin.batches(self.train_ds, cfg.DATALOADER.TRAIN_BATCH_SIZE, self.rank,
                                                     self.world, True, cfg.SEED + self.epoch)):
            self.buckets.zero()
            pred, target = self._forward(batch)
            # discriminator steps (G's output detached)
            for _ in range(cfg.GAN.D_STEPS):
                self.optD.zero_grad(set_to_none=True)
                d_loss = patchgan.d_loss(self.D(target), self.D(pred.detach()))
                d_loss.backward()
                self._d_allreduce()
                self.optD.step()
            # generator step: reconstruction loss + adversarial term through D
            m = train_swin.compute_metrics(cfg, pred, target, is_training=True)
            g_adv = patchgan.g_adv_loss(self.D(pred))
            loss = m[f'Train/{cfg.MODEL.RECON_LOSS.NAME}'] + cfg.GAN.ADV_WEIGHT * g_adv
            self.optD.zero_grad(set_to_none=True)        # D's grads from the G step are not applied
            loss.backward()
            self.buckets.finish()
            self.opt.step()
            self.global_step += 1
            if self.global_step % cfg.LOGGER.LOG_METRICS_EVERY_N_STEPS == 0 or self.args.verbose:
                rec = {k: float(v) for k, v in m.items()}
                rec.update(epoch=self.epoch, step=self.global_step, d_loss=float(d_loss), g_adv=float(g_adv))
                self._log(rec)
                if self.rank == 0:
                    train_swin.logger.info(f"epoch {self.epoch} step {self.global_step} loss {float(loss):.5f} "
                                           f"d_loss {float(d_loss):.4f}")
            if self.args.max_steps and self.global_step >= self.args.max_steps:
                break
        self.sched.step()

    def _callback_state(self, key, path):
        st = super()._callback_state(key, path)
        st['discriminator_state_dict'] = {k: v.detach().cpu() for k, v in self.D.state_dict().items()}
        st['discriminator_optimizer'] = self.optD.state_dict()
        return st

    def resume(self, path):
        super().resume(path)
        from dl_cs import checkpoint
        ck = checkpoint.load(path)
        if 'discriminator_state_dict' in ck:
            self.D.load_state_dict(ck['discriminator_state_dict'])
        if 'discriminator_optimizer' in ck:
            self.optD.load_state_dict(ck['discriminator_optimizer'])


def main(argv=None):
    args = train_swin.create_arg_parser().parse_args(argv)
    args.trainer = 'gan'
    train_swin.main_args(args)


if __name__ == '__main__':
    main()

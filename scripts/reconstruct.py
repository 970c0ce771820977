"""Inference entry point: reconstruct BART CFL k-space with a trained Swin-unrolled
model on MI355X.

Same command line and file handling as the reference's scripts/reconstruct.py
(CLI :250-262, CflDataset :59-111, DataTransform :114-152, main :155-247), with
the model dispatch of reconstruct_h5.py (:98-122, :398-406): MODEL.MODEL_TYPE
'SWIN' (configs/config_swin.yaml) builds dl_cs.models.unrolledswin, and the
checkpoint's Lightning 'model.' prefix is stripped (dl_cs.checkpoint; loaded with
torch.load(weights_only=True)).  The inference preprocessing (data mask, fftmod,
95th-percentile scale, sliding-window initial guess) runs on the GPU
(dl_cs.data.preprocess.DataTransform); images are rescaled by that scale
(:233) and written as CFL [x, y, sl, 1, emap, echo, 1, phase] (:98-107).
--multi-gpu spreads the slices over every visible GPU (the reference's
nn.DataParallel): each GPU runs whole slices, launches interleave across devices.
"""
import argparse
import logging
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dl-swin-gan_amd"))

from dl_cs import checkpoint  # noqa: E402
from dl_cs.config import load_cfg  # noqa: E402
from dl_cs.fileio import cfl  # noqa: E402

logging.basicConfig(level=logging.INFO)
logger = logging.getLogger("reconstruct")


class CflDataset:
    """reconstruct.py:59-111 -- one example per (echo, slice) of BART-ordered
    k-space [x, y, sl, coil, 1, echo, 1, phase] and maps [x, y, sl, coil, emap]."""

    def __init__(self, file_ks, file_maps):
        ks = cfl.read(file_ks, order='F')
        maps = cfl.read(file_maps, order='F')
        X, Y, S, C = ks.shape[0], ks.shape[1], ks.shape[2], ks.shape[3]
        Ec = ks.shape[5] if ks.ndim > 5 else 1
        Ph = ks.shape[7] if ks.ndim > 7 else 1
        Em = maps.shape[4] if maps.ndim > 4 else 1
        ks = np.reshape(ks, (X, Y, S, C, Ec, Ph), order='F')
        maps = np.reshape(maps, (X, Y, S, 1, C, Em), order='F')
        self.kspace = np.transpose(ks, (2, 4, 3, 5, 1, 0))        # [sl, ec, coil, ph, y, x]
        self.maps = np.transpose(maps, (2, 5, 4, 3, 1, 0))        # [sl, em, coil, 1, y, x]
        self.image_dims = (S, Ec, Em, Ph, Y, X)
        self.examples = [(sl, ec) for ec in range(Ec) for sl in range(S)]

    def __len__(self):
        return len(self.examples)

    def __getitem__(self, i):
        sl, ec = self.examples[i]
        return np.ascontiguousarray(self.kspace[sl, ec]), np.ascontiguousarray(self.maps[sl])

    def write(self, file_im, images):
        """images: [n_examples, emap, phase, y, x] in example order.  Reshaped
        straight to [sl, ec, em, ph, y, x] exactly as reconstruct.py:98-107 does
        (with several echoes that reading differs from the echo-major example
        order; kept for output parity), then written [x, y, sl, 1, em, ec, 1, ph]."""
        im = np.reshape(np.asarray(images), self.image_dims)
        im = np.transpose(im, (5, 4, 0, 2, 1, 3))[:, :, :, None, :, :, None, :]
        cfl.write(file_im, im, order='F')


def build_model(config):
    """reconstruct_h5.py:398-406 -- MODEL_TYPE 'SWIN' (LitUnrolledSWIN, :97-122) or
    'RES' (LitUnrolledResNet: dl_cs.models.unrolled, the ResNet of configs/example.yaml)."""
    from dl_cs.models import unrolled, unrolledswin
    mods = {'SWIN': unrolledswin, 'RES': unrolled}
    if config.MODEL.MODEL_TYPE not in mods:
        raise NotImplementedError(f"MODEL_TYPE {config.MODEL.MODEL_TYPE}: SWIN and RES are built for MI355X")
    mod = mods[config.MODEL.MODEL_TYPE]
    if config.MODEL.META_ARCHITECTURE == 'dlespirit':
        return mod.ProximalGradientDescent(config)
    if config.MODEL.META_ARCHITECTURE == 'modl':
        return mod.HalfQuadraticSplitting(config)
    raise ValueError('Meta architecture in config file not recognized!')


def reconstruct(model_by_dev, transform_by_dev, dataset, batch_size):
    """Run every example through the model; batches go round-robin over devices."""
    from dl_cs.mri import transforms as T
    devs = list(model_by_dev)
    out = [None] * len(dataset)
    pending = []
    for b0 in range(0, len(dataset), batch_size):
        dev = devs[(b0 // batch_size) % len(devs)]
        with torch.cuda.device(dev):
            items = [transform_by_dev[dev](*dataset[i]) for i in range(b0, min(len(dataset), b0 + batch_size))]
            kspace, maps, mask, init, scale = (torch.stack([it[k] for it in items]) for k in range(5))
            with torch.no_grad():
                images = model_by_dev[dev](y=kspace, A=T.SenseModel(maps, weights=mask), x0=init)
            pending.append((b0, scale.view(-1, 1, 1, 1, 1) * images))          # reconstruct.py:233
    for b0, im in pending:
        im = im.cpu().numpy()
        for j in range(im.shape[0]):
            out[b0 + j] = im[j]
    return np.stack(out)


def main(args):
    from dl_cs.data.preprocess import DataTransform
    from dl_cs.models import swin3D
    swin3D.set_compute_dtype(torch.bfloat16 if args.dtype == 'bf16' else torch.float32)
    file_kspace = os.path.join(args.directory, args.kspace)
    file_maps = os.path.join(args.directory, args.maps)
    file_images = os.path.join(args.directory, args.out)
    if args.multi_gpu:
        devices = [torch.device('cuda', i) for i in range(torch.cuda.device_count())]
        logger.info(f'Running on {len(devices)} GPU devices...')
    else:
        if args.device < 0:
            raise RuntimeError("the Swin-unrolled model runs on the GPU (HIP kernels): pass --device N")
        devices = [torch.device('cuda', args.device)]
        logger.info(f'Running on GPU device #{args.device}...')
    logger.info(f'Loading model {args.ckpt}...')
    config = load_cfg(args.config_file)
    model_by_dev, tf_by_dev = {}, {}
    for d in devices:
        m = build_model(config)
        checkpoint.load_model(m, args.ckpt)
        m.eval()
        for p in m.parameters():                                            # freeze()
            p.requires_grad_(False)
        model_by_dev[d] = m.to(d)
        tf_by_dev[d] = DataTransform(config, device=d)
    logger.info('Loading CFL data...')
    data = CflDataset(file_kspace, file_maps)
    logger.info('Running inference...')
    start = time.time()
    images = reconstruct(model_by_dev, tf_by_dev, data, args.batch_size * len(devices))
    logger.info(f'Elapsed time (reconstruction): {time.time() - start} s')
    logger.info('Writing images...')
    data.write(file_images, images)


def create_arg_parser():
    parser = argparse.ArgumentParser(description="Inference script for unrolled MRI recon.")
    parser.add_argument('--directory', type=str, required=True, help='Directory with raw data files')
    parser.add_argument('--kspace', type=str, default='ks', help='k-Space file (CFL)')
    parser.add_argument('--maps', type=str, default='maps', help='Sensitivity maps file (CFL)')
    parser.add_argument('--out', type=str, default='im.dl', help='Output - images file (CFL)')
    parser.add_argument('--ckpt', type=str, required=True, help='Model checkpoint file')
    parser.add_argument('--batch-size', type=int, default=1, help='Slices per batch (per device)')
    parser.add_argument('--config-file', type=str, required=True, help='Training config file (yaml)')
    parser.add_argument('--device', type=int, default=-1, help='GPU device')
    parser.add_argument('--multi-gpu', action='store_true', help='Uses multiple GPUs for inference (overrides device flag)')
    parser.add_argument('--verbose', action='store_true', help='Turn on debug statements')
    parser.add_argument('--dtype', choices=['fp32', 'bf16'], default='fp32', help='compute dtype of the regularizer')
    return parser


if __name__ == '__main__':
    a = create_arg_parser().parse_args(sys.argv[1:])
    t0 = time.time()
    main(a)
    logger.info('Script complete.')
    logger.info(f'Elapsed time (total): {time.time() - t0} s')

"""Checkpoints in the reference's Lightning layout (train_swin.py:182-188,
reconstruct_h5.py:405-406): a dict with ``state_dict`` keyed ``model.<name>``
(the LightningModule wraps the unrolled net as ``self.model``), ``epoch``,
``global_step``, ``optimizer_states`` and ``lr_schedulers``.  Written with
torch.save and read back with ``torch.load(weights_only=True)``, so a
checkpoint can never execute code when loaded; the parameter names are the
reference's (including the DFE.layers / DFE.resswin_blocks aliases), so a
reference-trained state_dict loads into this package unchanged."""
import os

import torch

PREFIX = "model."


def model_state_dict(ckpt):
    """The unrolled network's state_dict from a checkpoint dict or a plain state_dict."""
    sd = ckpt.get("state_dict", ckpt)
    if any(k.startswith(PREFIX) for k in sd):
        return {k[len(PREFIX):]: v for k, v in sd.items() if k.startswith(PREFIX)}
    return dict(sd)


def submodule_state_dict(ckpt, prefix):
    """Entries ``<prefix>.<name>`` of a checkpoint's state_dict (e.g. the EMA copy a
    LightningModule holds as ``self.ema``, train_DiT.py:133), prefix stripped;
    empty when the checkpoint has none."""
    sd = ckpt.get("state_dict", {})
    p = prefix + "."
    return {k[len(p):]: v for k, v in sd.items() if k.startswith(p)}


def model_checkpoint_state(ckpt):
    """The ModelCheckpoint callback state of a checkpoint: Lightning keys it by the
    callback's ``state_key`` -- ``"ModelCheckpoint{'monitor': ..., 'mode': ...}"`` since
    PL 1.5 (e.g. reference train_DiT.py:360-375 checkpoints), plain
    ``"ModelCheckpoint"`` before; either form is accepted ({} if absent)."""
    cbs = ckpt.get("callbacks") or {}
    if "ModelCheckpoint" in cbs:
        return cbs["ModelCheckpoint"] or {}
    for k, v in cbs.items():
        if isinstance(k, str) and k.startswith("ModelCheckpoint"):
            return v or {}
    return {}


def callback_state(monitor, best_score, best_path, mode="min"):
    """``callbacks`` entry written with a checkpoint: the best score / file under both the
    plain key and the Lightning state_key (PL >= 1.5), so either reader resumes them."""
    st = {"monitor": monitor, "best_model_score": best_score, "best_model_path": best_path}
    lkey = "ModelCheckpoint" + repr({"monitor": monitor, "mode": mode, "every_n_train_steps": 0,
                                     "every_n_epochs": 1, "train_time_interval": None,
                                     "save_on_train_epoch_end": True})
    return {"callbacks": {"ModelCheckpoint": dict(st), lkey: dict(st)}}


def load(path, map_location="cpu"):
    return torch.load(path, map_location=map_location, weights_only=True)


def load_model(model, path, strict=True):
    """Load a .ckpt (or a bare state_dict file) into `model`; returns the checkpoint dict."""
    ckpt = load(path)
    model.load_state_dict(model_state_dict(ckpt), strict=strict)
    return ckpt


def save(path, model, optimizer=None, scheduler=None, epoch=0, global_step=0, extra=None, submodules=None):
    """submodules: {prefix: module} written into the same state_dict as
    ``<prefix>.<name>`` (the LightningModule's other children, e.g. ``ema``)."""
    sd = {PREFIX + k: v.detach().cpu() for k, v in model.state_dict().items()}
    for pre, mod in (submodules or {}).items():
        sd.update({f"{pre}.{k}": v.detach().cpu() for k, v in mod.state_dict().items()})
    ck = {"epoch": int(epoch), "global_step": int(global_step), "state_dict": sd,
          "optimizer_states": [optimizer.state_dict()] if optimizer is not None else [],
          "lr_schedulers": [scheduler.state_dict()] if scheduler is not None else [],
          "pytorch-lightning_version": "1.6.0"}
    if extra:
        ck.update(extra)
    tmp = path + ".tmp"
    torch.save(ck, tmp)
    os.replace(tmp, path)
    return path

"""Timestep respacing (respace = dl_cs/diffusion/respace.py of the reference)."""
import torch

from .gaussian_diffusion import GaussianDiffusion


def space_timesteps(num_timesteps, section_counts):
    """respace:12-62 -- the steps kept from each equal section of the process
    ("ddimN" = the fixed DDIM stride)."""
    if isinstance(section_counts, str):
        if section_counts.startswith("ddim"):
            want = int(section_counts[len("ddim"):])
            for stride in range(1, num_timesteps):
                if len(range(0, num_timesteps, stride)) == want:
                    return set(range(0, num_timesteps, stride))
            raise ValueError(f"cannot create exactly {num_timesteps} steps with an integer stride")
        section_counts = [int(x) for x in section_counts.split(",")]
    size_per, extra = divmod(num_timesteps, len(section_counts))
    start, steps = 0, []
    for i, count in enumerate(section_counts):
        size = size_per + (1 if i < extra else 0)
        if size < count:
            raise ValueError(f"cannot divide section of {size} steps into {count}")
        stride = 1 if count <= 1 else (size - 1) / (count - 1)
        steps += [start + round(k * stride) for k in range(count)]
        start += size
    return set(steps)


class _WrappedModel:
    """respace:117-129 -- maps the respaced step index to the original one."""

    def __init__(self, model, timestep_map, original_num_steps):
        self.model, self.timestep_map, self.original_num_steps = model, timestep_map, original_num_steps

    def __call__(self, x, ts, **kwargs):
        m = torch.tensor(self.timestep_map, device=ts.device, dtype=ts.dtype)
        return self.model(x, m[ts], **kwargs)


class SpacedDiffusion(GaussianDiffusion):
    """respace:65-114 -- a diffusion over a subset of the base process's steps
    (betas re-derived from the kept cumulative products)."""

    def __init__(self, use_timesteps, **kwargs):
        self.use_timesteps = set(use_timesteps)
        self.timestep_map = []
        self.original_num_steps = len(kwargs["betas"])
        base = GaussianDiffusion(**kwargs)
        last, new_betas = 1.0, []
        for i, ab in enumerate(base.alphas_cumprod):
            if i in self.use_timesteps:
                new_betas.append(1 - ab / last)
                last = ab
                self.timestep_map.append(i)
        kwargs["betas"] = new_betas
        super().__init__(**kwargs)

    def _wrap_model(self, model):
        if isinstance(model, _WrappedModel):
            return model
        return _WrappedModel(model, self.timestep_map, self.original_num_steps)

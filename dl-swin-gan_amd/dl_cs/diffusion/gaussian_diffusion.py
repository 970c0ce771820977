"""Gaussian diffusion of the DiT denoiser training (BASELINE config 5),
MI355X build: the schedule constants, the forward process q(x_t | x_0), the
posterior, the sampler, and the two training losses train_DiT.py uses
(gd = dl_cs/diffusion/gaussian_diffusion.py of the reference, itself from
OpenAI's improved / guided diffusion).  The constants are float64 numpy tables
indexed per sample and cast to fp32 (gd:1039-1051); everything per voxel is a
device-tensor expression around the HIP DiT networks.  Not built: the
variational-bound losses (KL / learned variances) and DDIM sampling, which
config_dit.yaml does not use (LEARN_SIGMA False, training_kspace_loss).
"""
import enum
import math

import numpy as np
import torch


def tensor2realimag(x):
    """gd:15-17 -- complex [B, E, ...] -> real [B, 2E, ...] (re | im)."""
    return torch.cat((x.real, x.imag), dim=1)


def tensor2complex(x):
    """gd:19-22"""
    c = x.shape[1] // 2
    return torch.complex(x[:, :c], x[:, c:])


def mean_flat(tensor):
    """gd:24-28"""
    return tensor.mean(dim=list(range(1, tensor.ndim)))


class ModelMeanType(enum.Enum):
    """gd:31-38"""
    PREVIOUS_X = enum.auto()
    START_X = enum.auto()
    EPSILON = enum.auto()


class ModelVarType(enum.Enum):
    """gd:41-51"""
    LEARNED = enum.auto()
    FIXED_SMALL = enum.auto()
    FIXED_LARGE = enum.auto()
    LEARNED_RANGE = enum.auto()


class LossType(enum.Enum):
    """gd:54-63"""
    MSE = enum.auto()
    RESCALED_MSE = enum.auto()
    KL = enum.auto()
    RESCALED_KL = enum.auto()

    def is_vb(self):
        return self in (LossType.KL, LossType.RESCALED_KL)


def get_beta_schedule(beta_schedule, *, beta_start, beta_end, num_diffusion_timesteps):
    """gd:73-103 (linear / quad / const / jsd / warmup)."""
    n = num_diffusion_timesteps
    if beta_schedule == "linear":
        return np.linspace(beta_start, beta_end, n, dtype=np.float64)
    if beta_schedule == "quad":
        return np.linspace(beta_start ** 0.5, beta_end ** 0.5, n, dtype=np.float64) ** 2
    if beta_schedule == "const":
        return beta_end * np.ones(n, dtype=np.float64)
    if beta_schedule == "jsd":
        return 1.0 / np.linspace(n, 1, n, dtype=np.float64)
    if beta_schedule in ("warmup10", "warmup50"):
        frac = 0.1 if beta_schedule == "warmup10" else 0.5
        b = beta_end * np.ones(n, dtype=np.float64)
        w = int(n * frac)
        b[:w] = np.linspace(beta_start, beta_end, w, dtype=np.float64)
        return b
    raise NotImplementedError(beta_schedule)


def betas_for_alpha_bar(num_diffusion_timesteps, alpha_bar, max_beta=0.999):
    """gd:135-152"""
    n = num_diffusion_timesteps
    return np.array([min(1 - alpha_bar((i + 1) / n) / alpha_bar(i / n), max_beta) for i in range(n)])


def get_named_beta_schedule(schedule_name, num_diffusion_timesteps):
    """gd:106-133 -- note the reference's 'linear' ends at 1000/T * 0.0008 (gd:117)."""
    if schedule_name == "linear":
        scale = 1000 / num_diffusion_timesteps
        return get_beta_schedule("linear", beta_start=scale * 0.0001, beta_end=scale * 0.0008,
                                 num_diffusion_timesteps=num_diffusion_timesteps)
    if schedule_name == "squaredcos_cap_v2":
        return betas_for_alpha_bar(num_diffusion_timesteps,
                                   lambda t: math.cos((t + 0.008) / 1.008 * math.pi / 2) ** 2)
    raise NotImplementedError(f"unknown beta schedule: {schedule_name}")


def _extract_into_tensor(arr, timesteps, broadcast_shape):
    """gd:1039-1051 -- float64 table rows at `timesteps`, as fp32 broadcast to the shape."""
    res = torch.from_numpy(arr).to(device=timesteps.device)[timesteps].float()
    while res.ndim < len(broadcast_shape):
        res = res[..., None]
    return res.expand(broadcast_shape)


class GaussianDiffusion:
    """gd:155-1036 (the parts on the config_dit path)."""

    def __init__(self, *, betas, model_mean_type, model_var_type, loss_type):
        self.model_mean_type = model_mean_type
        self.model_var_type = model_var_type
        self.loss_type = loss_type
        betas = np.array(betas, dtype=np.float64)
        assert betas.ndim == 1 and (betas > 0).all() and (betas <= 1).all()
        self.betas = betas
        self.num_timesteps = int(betas.shape[0])
        alphas = 1.0 - betas
        self.alphas_cumprod = np.cumprod(alphas, axis=0)
        self.alphas_cumprod_prev = np.append(1.0, self.alphas_cumprod[:-1])
        self.alphas_cumprod_next = np.append(self.alphas_cumprod[1:], 0.0)
        self.sqrt_alphas_cumprod = np.sqrt(self.alphas_cumprod)
        self.sqrt_one_minus_alphas_cumprod = np.sqrt(1.0 - self.alphas_cumprod)
        self.log_one_minus_alphas_cumprod = np.log(1.0 - self.alphas_cumprod)
        self.sqrt_recip_alphas_cumprod = np.sqrt(1.0 / self.alphas_cumprod)
        self.sqrt_recipm1_alphas_cumprod = np.sqrt(1.0 / self.alphas_cumprod - 1)
        self.posterior_variance = betas * (1.0 - self.alphas_cumprod_prev) / (1.0 - self.alphas_cumprod)
        self.posterior_log_variance_clipped = (
            np.log(np.append(self.posterior_variance[1], self.posterior_variance[1:]))
            if len(self.posterior_variance) > 1 else np.array([]))
        self.posterior_mean_coef1 = betas * np.sqrt(self.alphas_cumprod_prev) / (1.0 - self.alphas_cumprod)
        self.posterior_mean_coef2 = (1.0 - self.alphas_cumprod_prev) * np.sqrt(alphas) / (1.0 - self.alphas_cumprod)

    # ---------------------------------------------------------------- forward process
    def q_mean_variance(self, x_start, t):
        """gd:214-224"""
        mean = _extract_into_tensor(self.sqrt_alphas_cumprod, t, x_start.shape) * x_start
        var = _extract_into_tensor(1.0 - self.alphas_cumprod, t, x_start.shape)
        logv = _extract_into_tensor(self.log_one_minus_alphas_cumprod, t, x_start.shape)
        return mean, var, logv

    def q_sample(self, x_start, t, noise=None):
        """gd:226-241"""
        if noise is None:
            noise = torch.randn_like(x_start)
        assert noise.shape == x_start.shape
        return (_extract_into_tensor(self.sqrt_alphas_cumprod, t, x_start.shape) * x_start +
                _extract_into_tensor(self.sqrt_one_minus_alphas_cumprod, t, x_start.shape) * noise)

    def q_posterior_mean_variance(self, x_start, x_t, t):
        """gd:243-263"""
        assert x_start.shape == x_t.shape
        mean = (_extract_into_tensor(self.posterior_mean_coef1, t, x_t.shape) * x_start +
                _extract_into_tensor(self.posterior_mean_coef2, t, x_t.shape) * x_t)
        var = _extract_into_tensor(self.posterior_variance, t, x_t.shape)
        logv = _extract_into_tensor(self.posterior_log_variance_clipped, t, x_t.shape)
        return mean, var, logv

    # ---------------------------------------------------------------- reverse process
    def _predict_xstart_from_eps(self, x_t, t, eps):
        """gd:345-350"""
        return (_extract_into_tensor(self.sqrt_recip_alphas_cumprod, t, x_t.shape) * x_t -
                _extract_into_tensor(self.sqrt_recipm1_alphas_cumprod, t, x_t.shape) * eps)

    def _predict_eps_from_xstart(self, x_t, t, pred_xstart):
        """gd:352-355"""
        return ((_extract_into_tensor(self.sqrt_recip_alphas_cumprod, t, x_t.shape) * x_t - pred_xstart) /
                _extract_into_tensor(self.sqrt_recipm1_alphas_cumprod, t, x_t.shape))

    def _wrap_model(self, model):
        return model

    def p_mean_variance(self, model, x, t, clip_denoised=True, denoised_fn=None, model_kwargs=None):
        """gd:265-343 (fixed variances)."""
        model = self._wrap_model(model)
        model_kwargs = model_kwargs or {}
        assert t.shape == (x.shape[0],)
        out = model(x, t, **model_kwargs)
        extra = None
        if isinstance(out, tuple):
            out, extra = out
        if self.model_var_type in (ModelVarType.LEARNED, ModelVarType.LEARNED_RANGE):
            raise NotImplementedError("dl_cs diffusion: learned variances (LEARN_SIGMA False in config_dit)")
        if self.model_var_type == ModelVarType.FIXED_LARGE:
            var = np.append(self.posterior_variance[1], self.betas[1:])
            logv = np.log(var)
        else:
            var, logv = self.posterior_variance, self.posterior_log_variance_clipped
        var = _extract_into_tensor(var, t, x.shape)
        logv = _extract_into_tensor(logv, t, x.shape)

        def process(v):
            if denoised_fn is not None:
                v = denoised_fn(v)
            return v.clamp(-1, 1) if clip_denoised else v

        if self.model_mean_type == ModelMeanType.START_X:
            pred_xstart = process(out)
        else:
            pred_xstart = process(self._predict_xstart_from_eps(x_t=x, t=t, eps=out))
        mean, _, _ = self.q_posterior_mean_variance(x_start=pred_xstart, x_t=x, t=t)
        return {"mean": mean, "variance": var, "log_variance": logv, "pred_xstart": pred_xstart, "extra": extra}

    def p_sample(self, model, x, t, clip_denoised=True, denoised_fn=None, cond_fn=None, model_kwargs=None):
        """gd:387-428"""
        out = self.p_mean_variance(model, x, t, clip_denoised=clip_denoised, denoised_fn=denoised_fn,
                                   model_kwargs=model_kwargs)
        noise = torch.randn_like(x)
        nonzero = (t != 0).float().view(-1, *([1] * (x.ndim - 1)))
        if cond_fn is not None:
            g = cond_fn(x, t, **(model_kwargs or {}))
            out["mean"] = out["mean"].float() + out["variance"] * g.float()
        return {"sample": out["mean"] + nonzero * torch.exp(0.5 * out["log_variance"]) * noise,
                "pred_xstart": out["pred_xstart"]}

    def _loop(self, model, shape, noise, device, progress, step):
        if device is None:
            device = next(model.parameters()).device
        assert isinstance(shape, (tuple, list))
        img = noise if noise is not None else torch.randn(*shape, device=device)
        indices = list(range(self.num_timesteps))[::-1]
        if progress:
            from tqdm.auto import tqdm
            indices = tqdm(indices)
        init_img = img
        for i in indices:
            t = torch.tensor([i] * shape[0], device=device)
            with torch.no_grad():
                out = step(img, t, i, init_img)
                yield out
                img = out["sample"]

    def p_sample_loop_progressive(self, model, shape, noise=None, clip_denoised=True, denoised_fn=None,
                                  cond_fn=None, model_kwargs=None, device=None, progress=False):
        """gd:475-522"""
        def step(img, t, i, init_img):
            return self.p_sample(model, img, t, clip_denoised, denoised_fn, cond_fn, model_kwargs)
        return self._loop(model, shape, noise, device, progress, step)

    def p_sample_loop(self, model, shape, **kw):
        """gd:430-473"""
        final = None
        for final in self.p_sample_loop_progressive(model, shape, **kw):
            pass
        return final["sample"]

    def p_sample_loop_conditional_progressive(self, model, shape, noise=None, clip_denoised=True,
                                              denoised_fn=None, cond_fn=None, model_kwargs=None, device=None,
                                              progress=False):
        """gd:569-633 -- after every step but the last the sample's measured k-space is
        replaced by the initial image's: A_F^H (A_1 x + A x_init)."""
        A_F, A_1, A = model_kwargs["A_F"], model_kwargs["A_1"], model_kwargs["A"]

        def step(img, t, i, init_img):
            out = self.p_sample(model, img, t, clip_denoised, denoised_fn, cond_fn, model_kwargs)
            if i != 0:
                out["sample"] = A_F(A_1(out["sample"]) + A(init_img), adjoint=True)
            return out
        return self._loop(model, shape, noise, device, progress, step)

    def p_sample_loop_conditional(self, model, shape, **kw):
        """gd:524-567"""
        final = None
        for final in self.p_sample_loop_conditional_progressive(model, shape, **kw):
            pass
        return final["sample"]

    # ---------------------------------------------------------------- training losses
    def training_kspace_loss(self, model, x_start, t, model_kwargs=None, noise=None):
        """gd:837-873 -- mean |A_F out - A_F target| of the model run on x_t (the
        k-space L1 of META_ARCHITECTURE DDPM_X, train_DiT.py:249-256).  Returns
        (terms, model output, x_t)."""
        model_kwargs = model_kwargs or {}
        x_ri = tensor2realimag(x_start)
        if noise is None:
            noise = torch.randn_like(x_ri)
        x_t = tensor2complex(self.q_sample(x_ri, t, noise=noise))
        out = model(x_t, t, **model_kwargs)
        A_F, target = model_kwargs["A_F"], model_kwargs["fs"]
        l1 = torch.mean(torch.abs(A_F(out) - A_F(target)))
        return {"l1": l1, "MSE": l1, "loss": l1}, out, x_t

    def training_losses(self, model, x_start, t, model_kwargs=None, noise=None):
        """gd:876-965 -- the MSE losses (DDPM_E); the VB terms are not built."""
        if self.loss_type.is_vb() or self.model_var_type in (ModelVarType.LEARNED, ModelVarType.LEARNED_RANGE):
            raise NotImplementedError("dl_cs diffusion: variational-bound terms (config_dit: MSE, fixed variance)")
        model = self._wrap_model(model)
        model_kwargs = model_kwargs or {}
        x_ri = tensor2realimag(x_start)
        if noise is None:
            noise = torch.randn_like(x_ri)
        x_t = tensor2complex(self.q_sample(x_ri, t, noise=noise))
        out = tensor2realimag(model(x_t, t, **model_kwargs))
        x_t_ri = tensor2realimag(x_t)
        target = {ModelMeanType.PREVIOUS_X: lambda: self.q_posterior_mean_variance(x_ri, x_t_ri, t)[0],
                  ModelMeanType.START_X: lambda: x_ri,
                  ModelMeanType.EPSILON: lambda: noise}[self.model_mean_type]()
        assert out.shape == target.shape == x_ri.shape
        terms = {"mse": mean_flat((target - out) ** 2)}
        terms["loss"] = terms["mse"]
        return terms, tensor2complex(out), x_t

"""Drop-in for the reference's ``diffusion_model/sample_ddpm.py`` (unguided DDPM sampling).

Same public functions — ``load_config``, ``sample``, ``load_model``, ``load_scheduler``, ``infer`` —
with the reference's argument meaning.  Differences, all opt-in or fail-loud:
  * ``sample`` returns the final x0 tensor in addition to writing the PNG grid (``save_path=None``
    skips the file), and takes build-only keywords: ``noise`` ('torch_cpu' = reference RNG stream,
    'philox' = on-device counter-based noise), ``seed``, ``x_T``, ``graph``.
  * ``infer`` does not swallow exceptions (reference ``:84-87`` prints and continues).
Hot loop (reference ``:35-44``) per step: one UNet forward on the HIP engine + one fused scheduler
kernel.  ``graph=True`` captures the UNet forward + step into a HIP graph once and replays it.
"""
import math
import os
from datetime import datetime
from typing import Optional

import torch

from .config import Config, DiffusionConfig, ModelConfig, TrainingConfig, load_config  # noqa: F401
from .models.unet_base import Unet
from .scheduler.linear_noise_scheduler import LinearNoiseScheduler


def _device() -> torch.device:
    return torch.device('cuda' if torch.cuda.is_available() else 'cpu')


# ----------------------------------------------------------------------------------- image output
def make_grid(ims: torch.Tensor, nrow: int = 8, padding: int = 2, pad_value: float = 0.0) -> torch.Tensor:
    """torchvision.utils.make_grid (torchvision==0.18.0, reference requirements.txt:6; not a dependency
    here) for a (B, C, H, W) batch with its defaults normalize=False, scale_each=False: one image is
    returned as is, a 1-channel batch is repeated to 3 channels, images are laid out row-major
    ``min(nrow, B)`` per row with ``padding`` pixels of ``pad_value`` around each."""
    if ims.dim() == 3:
        ims = ims.unsqueeze(0)
    if ims.shape[1] == 1:
        ims = torch.cat((ims, ims, ims), 1)
    B, C, H, W = ims.shape
    if B == 1:
        return ims[0]
    xmaps = min(nrow, B)
    ymaps = int(math.ceil(B / xmaps))
    h, w = H + padding, W + padding
    grid = torch.full((C, ymaps * h + padding, xmaps * w + padding), pad_value, dtype=ims.dtype)
    k = 0
    for y in range(ymaps):
        for x in range(xmaps):
            if k >= B:
                break
            grid[:, y * h + padding:y * h + padding + H, x * w + padding:x * w + padding + W] = ims[k]
            k += 1
    return grid


def save_png(grid: torch.Tensor, path: str):
    """torchvision.transforms.ToPILImage()(grid).save(path) for a CHW tensor: a float tensor becomes
    ``mul(255).byte()`` (truncation, wrapping above 255 as the reference's does), a uint8 tensor is
    taken as is; 1 channel -> mode 'L', 3 -> 'RGB'."""
    from PIL import Image
    g = grid.detach().cpu()
    if g.is_floating_point():
        g = g.mul(255).byte()
    arr = g.permute(1, 2, 0).numpy()
    Image.fromarray(arr.squeeze(-1) if arr.shape[-1] == 1 else arr).save(path)


# ----------------------------------------------------------------------------------- sampling core
class _GraphStep:
    """One reverse step (UNet + fused scheduler update) captured into a HIP graph per timestep class.

    The UNet's shapes are static across steps; only the timestep value and the step scalars change.
    The graph reads the timestep from a device tensor and the scalars are baked per captured step, so
    we capture one graph per distinct step index lazily... which would be T graphs.  Instead we capture
    the UNet forward only (timestep read from device memory) and run the scheduler kernel eagerly.
    """

    def __init__(self, model: Unet, x: torch.Tensor, split: Optional[int] = None):
        self.model = model
        self.x_in = x.clone()
        self.t_in = torch.zeros(1, dtype=torch.long, device=x.device)
        # split > 1: the batch runs as `split` independent image groups on their own streams inside
        # the one graph (every UNet op is per image: bit-identical result, tests/test_gpu_unet.py);
        # concurrent groups fill each other's launch tails and hide the small launches (GroupNorm
        # finalize, scheduler) under the other group's convs.  Same-box A/B at 256 px B=16, 60-step
        # bench, two rounds (profiles/r06_graph_split_ab.txt): 23.74 / 23.73 (1), 23.34 / 23.39 (2),
        # 24.09 / 24.14 (4) ms/step -- two groups by default where each keeps >= 8 images (rounds 1-5
        # measured 1 vs 2 within box spread on slower kernels).  WC_GRAPH_SPLIT overrides.
        B = x.shape[0]
        if split is None:
            split = int(os.environ.get('WC_GRAPH_SPLIT', '2' if B >= 16 and B % 2 == 0 else '1'))
        self.split = split if split > 1 and B % split == 0 else 1
        self.streams = [torch.cuda.Stream(device=x.device) for _ in range(self.split - 1)]
        # concurrent groups: the pre-split convs with N % 256 == 0 on 8-wave workgroups, the form that
        # measured faster beside the other group's launches (slower alone: kernels.wino_vp_wide)
        from ..kernels import wino_vp_wide
        with wino_vp_wide(self.split > 1):
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(2):  # warm the allocator / engine pack outside capture
                    self.eps = self._forward()
            torch.cuda.current_stream().wait_stream(s)
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):
                self.eps = self._forward()

    def _forward(self) -> torch.Tensor:
        if self.split == 1:
            return self.model(self.x_in, self.t_in)
        g = self.x_in.shape[0] // self.split
        main = torch.cuda.current_stream()
        outs = [None] * self.split
        for i, st in enumerate(self.streams, 1):
            st.wait_stream(main)
            with torch.cuda.stream(st):
                outs[i] = self.model(self.x_in[i * g:(i + 1) * g], self.t_in)
        outs[0] = self.model(self.x_in[:g], self.t_in)
        for st in self.streams:
            main.wait_stream(st)
        return torch.cat(outs)

    def __call__(self, x: torch.Tensor, t_dev: torch.Tensor) -> torch.Tensor:
        self.x_in.copy_(x)
        self.t_in.copy_(t_dev)
        self.graph.replay()
        return self.eps


@torch.no_grad()
def sample_tensor(model: Unet, scheduler: LinearNoiseScheduler, batch: int, im_channels: int, im_size: int, *,
                  noise: str = 'torch_cpu', seed: Optional[int] = None, sample0: int = 0,
                  x_T: Optional[torch.Tensor] = None, graph: bool = False, total_batch: Optional[int] = None,
                  progress=None, progress_x=None) -> torch.Tensor:
    """The reverse loop of reference ``sample_ddpm.py:35-44``; returns x0 (not clamped).

    noise='torch_cpu': x_T and every z come from the CPU generator in the reference's order
    (``torch.randn`` of the full batch).  With ``total_batch`` > batch (sharded sampling) every
    rank draws the full-batch tensor and keeps rows [sample0, sample0+batch) — identical to one rank.
    noise='philox': x_T and z from Philox(seed, global sample, step) on the device.
    """
    dev = scheduler.device
    T = scheduler.num_timesteps
    shape = (batch, im_channels, im_size, im_size)
    full = total_batch or batch
    full_shape = (full, im_channels, im_size, im_size)
    if noise not in ('torch_cpu', 'philox'):
        raise ValueError(f"noise must be 'torch_cpu' or 'philox', got {noise!r}")
    if seed is not None and noise == 'torch_cpu':
        torch.manual_seed(seed)
    seed = 0 if seed is None else seed

    def cpu_noise():
        z = torch.randn(full_shape)
        return z[sample0:sample0 + batch].contiguous().to(dev)

    if x_T is not None:
        xt = x_T.to(dev, torch.float32).contiguous()
    elif noise == 'torch_cpu':
        xt = cpu_noise()
    else:
        from ..kernels import philox_normal
        xt = philox_normal(shape, dev, seed, sample0=sample0, step=T)  # step index T keys x_T
    ts = torch.arange(T, device=dev, dtype=torch.long)
    runner = _GraphStep(model, xt) if graph else None
    nxt = torch.empty_like(xt)
    # reference-RNG mode: the per-step z draws (the full-batch CPU tensor, in the reference's order)
    # run one step ahead on a worker thread while the GPU computes the UNet.  They come from a private
    # generator that continues the global CPU generator's state, and the global state is set to the
    # private one's at the end: the stream is exactly the reference's sequential one, and a callback
    # (progress / progress_x) drawing from the global generator meanwhile cannot interleave with it.
    pool = fut = gen = None
    if noise == 'torch_cpu' and T > 1:
        from concurrent.futures import ThreadPoolExecutor
        pool = ThreadPoolExecutor(1)
        gen = torch.Generator()
        gen.set_state(torch.get_rng_state())

        def cpu_draw():
            return torch.randn(full_shape, generator=gen)[sample0:sample0 + batch].contiguous()

        fut = pool.submit(cpu_draw)
    try:
        for i in reversed(range(T)):
            t_dev = ts[i:i + 1]
            eps = runner(xt, t_dev) if runner is not None else model(xt, t_dev)
            if i == 0:
                scheduler.step(xt, eps, 0, out=nxt)
            elif noise == 'torch_cpu':
                z = fut.result()
                fut = pool.submit(cpu_draw) if i > 1 else None
                scheduler.step(xt, eps, i, out=nxt, z=z.to(dev))
            else:
                scheduler.step(xt, eps, i, out=nxt, noise='philox', seed=seed, sample0=sample0)
            xt, nxt = nxt, xt
            if progress is not None:
                progress(i)
            if progress_x is not None:  # (t, x_{t-1}) after each step (tests / diagnostics)
                progress_x(i, xt)
    finally:
        if pool is not None:
            pool.shutdown(wait=True)
        if gen is not None:
            torch.set_rng_state(gen.get_state())
    return xt


def sample(model, scheduler: LinearNoiseScheduler, train_config: TrainingConfig, model_config: ModelConfig,
           diffusion_config: DiffusionConfig, save_path: Optional[str] = 'diffusion_model_v2/outputs/samples', *,
           noise: str = 'torch_cpu', seed: Optional[int] = None, x_T: Optional[torch.Tensor] = None,
           graph: bool = False) -> torch.Tensor:
    """Reference ``sample`` (:23-53): T-step reverse loop, clamp, [0,1], PNG grid.  Returns x0."""
    if diffusion_config.num_timesteps != scheduler.num_timesteps:
        raise RuntimeError('scheduler / diffusion_config timestep mismatch')
    xt = sample_tensor(model, scheduler, train_config.sample_size, model_config.im_channels, model_config.im_size,
                       noise=noise, seed=seed, x_T=x_T, graph=graph)
    if save_path is not None:
        ims = (torch.clamp(xt, -1., 1.).detach().cpu() + 1) / 2
        grid = make_grid(ims, nrow=train_config.num_grid_rows)
        now = datetime.now()
        os.makedirs(save_path, exist_ok=True)
        save_png(grid, os.path.join(save_path, f'x_410{now.hour}{now.minute}{now.second}.png'))
    return xt


def load_model(model_path: str, model_config: ModelConfig) -> torch.nn.Module:
    """Reference :56-61 — Unet + ``torch.load(...)['model_state_dict']`` (weights_only load)."""
    dev = _device()
    model = Unet(model_config).to(dev)
    checkpoint = torch.load(model_path, map_location=dev, weights_only=True)
    model.load_state_dict(checkpoint['model_state_dict'])
    model.eval()
    return model


def load_scheduler(diffusion_config: DiffusionConfig) -> LinearNoiseScheduler:
    """Reference :64-70."""
    return LinearNoiseScheduler(num_timesteps=diffusion_config.num_timesteps, beta_start=diffusion_config.beta_start,
                                beta_end=diffusion_config.beta_end)


def infer(config: Config, epoch: int = 410):
    """Reference :73-87 (checkpoint ``{checkpoints}/{epoch}-checkpoint.ckpt``); errors propagate."""
    checkpoint_path = os.path.join(config.folders.checkpoints, f'{epoch}-checkpoint.ckpt')
    model = load_model(checkpoint_path, config.model)
    scheduler = load_scheduler(config.diffusion)
    with torch.no_grad():
        return sample(model, scheduler, config.training, config.model, config.diffusion, config.folders.samples)


if __name__ == '__main__':
    infer(load_config())

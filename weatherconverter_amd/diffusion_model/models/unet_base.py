"""Drop-in ``Unet`` for the reference's ``diffusion_model/models/unet_base.py``.

Parameter tree: key-for-key and shape-for-shape identical to the reference (``unet_base.py:64-449``:
358 / 382 / 406 keys at im_size 256 / 128 / 64 with the default channels), so reference checkpoints
(``{'model_state_dict': ...}``) load with ``load_state_dict`` unchanged.

Forward: NOT PyTorch eager.  ``Unet.forward`` hands the parameters to
:class:`weatherconverter_amd.diffusion_model.models.engine.UnetEngine`, which repacks them once into
GEMM layouts on the GPU and runs the whole network as hand-written gfx950 HIP kernels (NHWC,
fp32 MFMA implicit-GEMM convolutions with fused GroupNorm+SiLU prologues, flash attention, fused
time-embedding).  There is no CPU fallback: on a machine without the HIP library or GPU the forward
raises.  The CPU reference restatement used to check it lives in ``oracle/`` (test-only).
"""
from typing import Optional, List

import torch
import torch.nn as nn

from ..config.models import ModelConfig


def get_time_embedding(time_steps: torch.Tensor, temb_dim: int) -> torch.Tensor:
    """Sinusoidal embedding with the reference's exact fp32 recipe (``unet_base.py:7-30``).

    Kept for API completeness (host-side helper); the UNet forward computes the embedding on the GPU
    inside ``wc_temb``.
    """
    assert temb_dim % 2 == 0, "time embedding dimension must be divisible by 2"
    half = temb_dim // 2
    k = torch.arange(half, dtype=torch.float32, device=time_steps.device)
    freq = 10000**(k / half)
    arg = time_steps.reshape(-1)[:, None].repeat(1, half) / freq
    return torch.cat([torch.sin(arg), torch.cos(arg)], dim=-1)


def _gn_silu_conv(c_in: int, c_out: int) -> nn.Sequential:
    # keys: .0 = GroupNorm(8), .1 = SiLU (no params), .2 = Conv2d 3x3
    return nn.Sequential(nn.GroupNorm(8, c_in), nn.SiLU(), nn.Conv2d(c_in, c_out, 3, 1, 1))


def _temb_proj(t_emb_dim: int, c_out: int) -> nn.Sequential:
    # keys: .1 = Linear (index 0 is the parameter-free SiLU)
    return nn.Sequential(nn.SiLU(), nn.Linear(t_emb_dim, c_out))


class _ResAttnStage(nn.Module):
    """Holds ``n_res`` ResBlocks and ``n_attn`` attention layers under the reference's attribute
    names (``resnet_conv_first``, ``t_emb_layers``, ``resnet_conv_second``, ``attention_norms``,
    ``attentions``, ``residual_input_conv``).  Registration order matches the reference so that
    ``state_dict()`` iterates keys in the same order."""

    def _build(self, c_in: int, c_out: int, t_emb_dim: int, n_res: int, n_attn: int, num_heads: int,
               use_attn: bool):
        ins = [c_in] + [c_out] * (n_res - 1)
        self.resnet_conv_first = nn.ModuleList([_gn_silu_conv(ci, c_out) for ci in ins])
        self.t_emb_layers = nn.ModuleList([_temb_proj(t_emb_dim, c_out) for _ in ins])
        self.resnet_conv_second = nn.ModuleList([_gn_silu_conv(c_out, c_out) for _ in ins])
        if use_attn:
            self.attention_norms = nn.ModuleList([nn.GroupNorm(8, c_out) for _ in range(n_attn)])
            self.attentions = nn.ModuleList(
                [nn.MultiheadAttention(c_out, num_heads, batch_first=True) for _ in range(n_attn)]
            )
        else:
            self.attention_norms = nn.ModuleList([nn.Identity() for _ in range(n_attn)])
            self.attentions = nn.ModuleList([nn.Identity() for _ in range(n_attn)])
        self.residual_input_conv = nn.ModuleList([nn.Conv2d(ci, c_out, 1) for ci in ins])

    def forward(self, *args, **kwargs):  # pragma: no cover - the engine executes the network
        raise RuntimeError('stages are executed by UnetEngine through Unet.forward')


class DownBlock(_ResAttnStage):
    """reference ``unet_base.py:64-164``: [ResBlock, Attn?] x num_layers, then 4x4/s2 conv."""

    def __init__(self, in_channels, out_channels, t_emb_dim, down_sample=True, num_heads=4, num_layers=1,
                 use_attn=True):
        super().__init__()
        self.num_layers = num_layers
        self.use_attn = use_attn
        self.down_sample = down_sample
        self._build(in_channels, out_channels, t_emb_dim, num_layers, num_layers, num_heads, use_attn)
        self.down_sample_conv = nn.Conv2d(out_channels, out_channels, 4, 2, 1) if down_sample else nn.Identity()


class MidBlock(_ResAttnStage):
    """reference ``unet_base.py:167-268``: ResBlock, [Attn, ResBlock] x num_layers."""

    def __init__(self, in_channels, out_channels, t_emb_dim, num_heads=4, num_layers=1, use_attn=False):
        super().__init__()
        self.num_layers = num_layers
        self.use_attn = use_attn
        self._build(in_channels, out_channels, t_emb_dim, num_layers + 1, num_layers, num_heads, use_attn)


class UpBlock(_ResAttnStage):
    """reference ``unet_base.py:271-369``: ConvT 4x4/s2, concat skip, [ResBlock, Attn?] x num_layers."""

    def __init__(self, in_channels, out_channels, t_emb_dim, up_sample=True, num_heads=4, num_layers=1,
                 use_attn=False):
        super().__init__()
        self.num_layers = num_layers
        self.up_sample = up_sample
        self.use_attn = use_attn
        self._build(in_channels, out_channels, t_emb_dim, num_layers, num_layers, num_heads, use_attn)
        half = in_channels // 2
        self.up_sample_conv = nn.ConvTranspose2d(half, half, 4, 2, 1) if up_sample else nn.Identity()


class Unet(nn.Module):
    """DDPM UNet (reference ``unet_base.py:372-488``) executed by hand-written gfx950 HIP kernels."""

    def __init__(self, model_config: ModelConfig):
        super().__init__()
        mc = model_config
        self.model_config = mc
        self.down_channels: List[int] = list(mc.down_channels)
        self.mid_channels: List[int] = list(mc.mid_channels)
        self.t_emb_dim = mc.time_emb_dim
        self.down_sample: List[bool] = list(mc.down_sample)
        self.num_down_layers = mc.num_down_layers
        self.num_mid_layers = mc.num_mid_layers
        self.num_up_layers = mc.num_up_layers
        self.attn_resolutions = list(mc.attn_resolutions)
        assert self.mid_channels[0] == self.down_channels[-1]
        assert self.mid_channels[-1] == self.down_channels[-2]
        assert len(self.down_sample) == len(self.down_channels) - 1

        d = self.t_emb_dim
        self.t_proj = nn.Sequential(nn.Linear(d, d), nn.SiLU(), nn.Linear(d, d))
        self.up_sample = list(reversed(self.down_sample))
        self.conv_in = nn.Conv2d(mc.im_channels, self.down_channels[0], kernel_size=3, padding=(1, 1))

        n_levels = len(self.down_channels) - 1
        self.downs = nn.ModuleList([
            DownBlock(self.down_channels[i], self.down_channels[i + 1], d, down_sample=self.down_sample[i],
                      num_layers=self.num_down_layers, num_heads=mc.num_heads,
                      use_attn=self.level_has_attn(i)) for i in range(n_levels)
        ])
        self.mids = nn.ModuleList([
            MidBlock(self.mid_channels[i], self.mid_channels[i + 1], d, num_layers=self.num_mid_layers,
                     use_attn=True, num_heads=mc.num_heads) for i in range(len(self.mid_channels) - 1)
        ])
        self.ups = nn.ModuleList([
            UpBlock(self.down_channels[i] * 2, self.down_channels[i - 1] if i != 0 else self.down_channels[0], d,
                    up_sample=self.down_sample[i], num_layers=self.num_up_layers, num_heads=mc.num_heads,
                    use_attn=self.level_has_attn(i)) for i in reversed(range(n_levels))
        ])
        self.norm_out = nn.GroupNorm(8, self.down_channels[0])
        self.conv_out = nn.Conv2d(self.down_channels[0], mc.im_channels, kernel_size=3, padding=1)
        self._engine = None
        self.conv_precision = None  # None = kernels.default_conv_precision()
        self.train_precision = None  # None = conv_precision (training only: also 'f16')

    def level_has_attn(self, i: int) -> bool:
        """Attention placement rule of ``unet_base.py:404-405,434-435``."""
        return (self.model_config.im_size // (2**i)) in self.attn_resolutions

    # -------------------------------------------------------------------------------- forward
    def engine(self):
        from .engine import UnetEngine
        if self._engine is None:
            self._engine = UnetEngine(self)
        return self._engine

    def set_conv_precision(self, precision: str) -> 'Unet':
        """Conv / attention arithmetic: 'f16x3' (the default: 2-piece fp16 split under power-of-two
        range bounds, bf16x6 where no bound exists), 'bf16x6' (exact 3-piece bf16 split everywhere) or
        'fp32' (fp32 MFMA).  The default comes from kernels.default_conv_precision(), which the
        WC_CONV_PRECISION environment variable overrides; see DESIGN.md §3.1."""
        from ... import kernels
        if precision not in kernels.CONV_PRECISIONS:
            raise ValueError(f'conv precision must be one of {kernels.CONV_PRECISIONS}')
        self.conv_precision = precision
        self._engine = None
        self._train_engine = None
        return self

    def set_train_precision(self, precision: Optional[str]) -> 'Unet':
        """Training arithmetic: None (= the conv precision: fp32-class), or a 16-bit line: 'bf16' (BASELINE
        config 3 trains in bf16) — the f16x3 kernels with one bf16 piece per operand on the bf16 MFMA
        (libwc_kernels_bf16.so), fp32 accumulation; or 'f16' — one fp16 piece per operand
        (libwc_kernels_single16.so, 3 more significand bits, the same range scaling).  Gradients about
        1e-3 (f16) / 1e-2 (bf16) relative to float64 instead of 1e-6."""
        from ... import kernels
        if precision is not None and precision not in kernels.CONV_PRECISIONS + ('f16', 'bf16'):
            raise ValueError(f"train precision must be None, 'f16', 'bf16' or one of {kernels.CONV_PRECISIONS}")
        self.train_precision = precision
        self._train_engine = None
        return self

    def train_engine(self):
        from .train_engine import TrainEngine
        if getattr(self, '_train_engine', None) is None:
            self._train_engine = TrainEngine(self)
        return self._train_engine

    def forward(self, x: torch.Tensor, t) -> torch.Tensor:
        if self.training and torch.is_grad_enabled():
            # training (train_ddpm.py:106-110): the HIP forward records its tape and loss.backward()
            # runs the HIP backward (models/train_engine.py), one gradient per parameter
            from .train_engine import UnetTrainFunction
            return UnetTrainFunction.apply(self.train_engine(), x, t, *self.parameters())
        return self.engine().forward(x, t)

    def _apply(self, fn, *args, **kwargs):
        # device / dtype moves invalidate the packed GPU weights
        self._engine = None
        self._train_engine = None
        return super()._apply(fn, *args, **kwargs)

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        self._engine = None
        return super().load_state_dict(state_dict, strict=strict, assign=assign)

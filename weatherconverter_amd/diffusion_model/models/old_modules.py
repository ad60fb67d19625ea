"""Drop-in for the reference's older UNet (``diffusion_model/models/old_modules.py:126-360``), the model
``sample_integrated.py`` samples with.

Parameter tree key-for-key identical to the reference (270 keys, 7.37 M params at the defaults) so
its checkpoints load.  The forward runs on HIP kernels through :class:`OldUnetEngine`:

* ResidualBlock (:126-160) = BN(eval)->conv3x3 ; SiLU->conv3x3 (+ 1x1 ``res`` conv or identity).
  BatchNorm is a per-channel affine applied in the first conv's PROLOGUE, i.e. before zero padding,
  exactly where the reference applies it (it cannot be folded into the weights at the borders);
  the SiLU is the second conv's prologue; the 1x1 ``res`` conv is extra K columns, the identity
  residual an epilogue add.
* Down/Up blocks: ``wc_avgpool2x2`` / ``wc_upsample2x_bilinear``; every skip is written by its
  producer straight into the channel slice of the up-path concat buffer that consumes it.
* SelfAttention (:73-94) = LayerNorm -> MHA (+x) -> LayerNorm -> Linear -> GELU -> Linear (+x):
  ``wc_layernorm_channels``, implicit-GEMM projections (GELU and residuals in the epilogues) and the
  flash attention kernel.
* The noise-level sinusoid (:283-317) is broadcast straight into its 32 concat channels.
Works at ``image_size=128`` only, like the reference (its attention sizes are hard-coded).
"""
import math

import torch
import torch.nn as nn

from ... import kernels as K
from ..._native import ACT_GELU
from ...kernels import Seg, View


class DiffusionUNet(nn.Module):
    requires_alpha_hat_timestep = False


class SelfAttention(nn.Module):

    def __init__(self, channels, size):
        super().__init__()
        self.channels = channels
        self.size = size
        self.mha = nn.MultiheadAttention(channels, 4, batch_first=True)
        self.ln = nn.LayerNorm([channels])
        self.ff_self = nn.Sequential(nn.LayerNorm([channels]), nn.Linear(channels, channels), nn.GELU(),
                                     nn.Linear(channels, channels))


class ResidualBlock(nn.Module):

    def __init__(self, in_channels, out_channels, mid_channels=None, residual=False):
        super().__init__()
        self.residual = residual
        mid = mid_channels or out_channels
        self.res = nn.Conv2d(in_channels, out_channels, kernel_size=1, bias=False)
        self.double_conv = nn.Sequential(nn.BatchNorm2d(in_channels),
                                         nn.Conv2d(in_channels, mid, kernel_size=3, padding=1, bias=False), nn.SiLU(),
                                         nn.Conv2d(mid, out_channels, kernel_size=3, padding=1, bias=False))


class DownBlock(nn.Module):

    def __init__(self, in_channels, out_channels, block_depth, emb_dim=256):
        super().__init__()
        self.residual_blocks = nn.ModuleList([
            ResidualBlock(in_channels if i == 0 else out_channels, out_channels, residual=(i == 0))
            for i in range(block_depth)
        ])
        self.downsample = nn.AvgPool2d(kernel_size=2)


class UpBlock(nn.Module):

    def __init__(self, in_channels, out_channels, skip_channels, block_depth, emb_dim=256):
        super().__init__()
        self.residual_blocks = nn.ModuleList([
            ResidualBlock((in_channels if i == 0 else out_channels) + skip_channels, out_channels, residual=True)
            for i in range(block_depth)
        ])
        self.upsample = nn.Upsample(scale_factor=2, mode='bilinear')


class UNet(DiffusionUNet):
    """reference old_modules.py:230-360 (defaults: 3->3 channels, 128 px, depth 3)."""

    def __init__(self, c_in=3, c_out=3, image_size=128, conv_dim=64, block_depth=3, time_emb_dim=256):
        super().__init__()
        self.requires_alpha_hat_timestep = True
        self.image_size = image_size
        self.pre_conv = nn.Conv2d(c_in, 32, kernel_size=3, padding=1, bias=False)
        self.embedding_upsample = nn.Upsample(size=(image_size, image_size), mode='nearest')
        self.down1 = DownBlock(64, 32, block_depth)
        self.down2 = DownBlock(32, 64, block_depth)
        self.attn_down3 = SelfAttention(64, 32)
        self.down3 = DownBlock(64, 96, block_depth)
        self.attn_down4 = SelfAttention(96, 16)
        self.down4 = DownBlock(96, 128, block_depth)
        self.bottleneck1 = ResidualBlock(128, 256, residual=True)
        self.attn_bottleneck = SelfAttention(256, 8)
        self.bottleneck2 = ResidualBlock(256, 256, residual=True)
        self.up1 = UpBlock(256, 128, 128, block_depth)
        self.attn_up1 = SelfAttention(128, 16)
        self.up2 = UpBlock(128, 96, 96, block_depth)
        self.attn_up2 = SelfAttention(96, 32)
        self.up3 = UpBlock(96, 64, 64, block_depth)
        self.up4 = UpBlock(64, 32, 32, block_depth)
        self.output = nn.Conv2d(32, c_out, kernel_size=3, padding=1, bias=False)
        self._engine = None

    def forward(self, x: torch.Tensor, t: torch.Tensor) -> torch.Tensor:
        if self.training and torch.is_grad_enabled():
            raise RuntimeError('old UNet: inference path only (no backward kernels)')
        if self._engine is None:
            self._engine = OldUnetEngine(self)
        return self._engine.forward(x, t)

    def _apply(self, fn, *args, **kwargs):
        self._engine = None
        return super()._apply(fn, *args, **kwargs)

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        self._engine = None
        return super().load_state_dict(state_dict, strict=strict, assign=assign)


TAPS3 = [(ky - 1, kx - 1) for ky in range(3) for kx in range(3)]


def _pack3(w):
    return w.detach().permute(0, 2, 3, 1).reshape(w.shape[0], -1).contiguous().float()


class OldUnetEngine:

    def __init__(self, m: UNet):
        p = next(m.parameters())
        if not p.is_cuda:
            raise RuntimeError('old UNet runs on the GPU only (HIP kernels, no CPU fallback)')
        if m.image_size != 128:
            raise RuntimeError('the reference old UNet only supports image_size=128 (hard-coded attention sizes)')
        K._native.load()
        self.m, self.dev = m, p.device
        self._sig = None
        self._pack()

    def _signature(self):
        return tuple((q.data_ptr(), q._version) for q in self.m.parameters())

    def _pack(self):
        m, dev = self.m, self.dev
        self._sig = self._signature()
        with torch.no_grad():
            self.pre_w = m.pre_conv.weight.detach().float().contiguous()
            self.pre_b = torch.zeros(32, device=dev)
            self.out_w = _pack3(m.output.weight)
            # noise-level sinusoid frequencies, computed with the reference's fp32 torch ops (:293-303)
            freq = torch.exp(torch.linspace(math.log(1.0), math.log(1000.0), 16))
            self.ang = (2.0 * math.pi * freq).float().contiguous().to(dev)
        self.rb = {}
        for name, mod in m.named_modules():
            if isinstance(mod, ResidualBlock):
                bn, c1, c2 = mod.double_conv[0], mod.double_conv[1], mod.double_conv[3]
                with torch.no_grad():
                    inv = 1.0 / torch.sqrt(bn.running_var.float() + bn.eps)
                    alpha = bn.weight.float() * inv
                    beta = bn.bias.float() - bn.running_mean.float() * alpha
                    w2 = _pack3(c2.weight)
                    if mod.residual:
                        w2 = torch.cat([w2, mod.res.weight.detach().reshape(w2.shape[0], -1).float()], 1).contiguous()
                self.rb[name] = dict(alpha=alpha, beta=beta, w1=_pack3(c1.weight), w2=w2, mid=c1.out_channels,
                                     cout=c2.out_channels, residual=mod.residual)
            elif isinstance(mod, SelfAttention):
                mha, ff = mod.mha, mod.ff_self
                with torch.no_grad():
                    self.rb[name] = dict(
                        ln_g=mod.ln.weight.float().contiguous(), ln_b=mod.ln.bias.float().contiguous(),
                        w_in=mha.in_proj_weight.float().contiguous(), b_in=mha.in_proj_bias.float().contiguous(),
                        w_out=mha.out_proj.weight.float().contiguous(), b_out=mha.out_proj.bias.float().contiguous(),
                        ln2_g=ff[0].weight.float().contiguous(), ln2_b=ff[0].bias.float().contiguous(),
                        w1=ff[1].weight.float().contiguous(), b1=ff[1].bias.float().contiguous(),
                        w2=ff[3].weight.float().contiguous(), b2=ff[3].bias.float().contiguous(), heads=mha.num_heads)

    def _new(self, B, H, W, C):
        return torch.empty((B, H, W, C), dtype=torch.float32, device=self.dev)

    def resblock(self, name: str, X: View, Y: View):
        p = self.rb[name]
        B, H, W = X.B, X.H, X.W
        sc = p['alpha'].expand(B, -1).contiguous()
        sh = p['beta'].expand(B, -1).contiguous()
        h = View.full(self._new(B, H, W, p['mid']))
        K.conv_igemm([Seg(X, TAPS3, scale=sc, shift=sh, silu=False)], p['w1'], None, h, Hm=H, Wm=W)
        one = torch.ones((B, p['mid']), device=self.dev)
        zero = torch.zeros((B, p['mid']), device=self.dev)
        segs = [Seg(h, TAPS3, scale=one, shift=zero, silu=True)]
        if p['residual']:
            segs.append(Seg(X, [(0, 0)], kbase=9 * p['mid']))
            K.conv_igemm(segs, p['w2'], None, Y, Hm=H, Wm=W)
        else:
            K.conv_igemm(segs, p['w2'], None, Y, Hm=H, Wm=W, res=X)

    def attention(self, name: str, X: View) -> View:
        p = self.rb[name]
        B, H, W, C = X.B, X.H, X.W, X.C
        N = H * W
        ln = View.full(self._new(B, H, W, C))
        K.layernorm_channels(X, p['ln_g'], p['ln_b'], ln)
        qkv = self._new(B, H, W, 3 * C)
        K.conv_igemm([Seg(ln, [(0, 0)])], p['w_in'], p['b_in'], View.full(qkv), Hm=H, Wm=W)
        o = self._new(B, H, W, C)
        K.attention(qkv.view(B * N, 3 * C), o.view(B * N, C), B, N, C, p['heads'])
        av = View.full(self._new(B, H, W, C))
        K.conv_igemm([Seg(View.full(o), [(0, 0)])], p['w_out'], p['b_out'], av, Hm=H, Wm=W, res=X)
        ln2 = View.full(self._new(B, H, W, C))
        K.layernorm_channels(av, p['ln2_g'], p['ln2_b'], ln2)
        hid = View.full(self._new(B, H, W, C))
        K.conv_igemm([Seg(ln2, [(0, 0)])], p['w1'], p['b1'], hid, Hm=H, Wm=W, act=ACT_GELU)
        out = View.full(self._new(B, H, W, C))
        K.conv_igemm([Seg(hid, [(0, 0)])], p['w2'], p['b2'], out, Hm=H, Wm=W, res=av)
        return out

    def forward(self, x: torch.Tensor, t: torch.Tensor) -> torch.Tensor:
        if self._signature() != self._sig:
            self._pack()
        x = x.to(self.dev, torch.float32).contiguous()
        B, _, S, _ = x.shape
        if S != 128:
            raise RuntimeError('old UNet expects 128x128 inputs')
        noise = torch.as_tensor(t, dtype=torch.float32, device=self.dev).reshape(-1).contiguous()
        if noise.numel() == 1 and B > 1:
            noise = noise.expand(B).contiguous()
        # concat buffers of the up path: [x | skip] per (level, up-block u); the down-path block j
        # writes its skip into slot u = 2 - j (UpBlock pops skips last-first)
        levels = [(128, 'down1', 'up4', 64, 32), (64, 'down2', 'up3', 96, 64), (32, 'down3', 'up2', 128, 96),
                  (16, 'down4', 'up1', 256, 128)]  # (res, down, up, up_in, cout)
        cat = {}
        for res, _, up, up_in, cout in levels:
            cat[up] = [self._new(B, res, res, (up_in if u == 0 else cout) + cout) for u in range(3)]

        def skip_view(up, j, cout):
            buf = cat[up][2 - j]
            return View(buf, buf.shape[-1] - cout, cout)

        d1in = self._new(B, S, S, 64)
        K.conv_in(x, self.pre_w, self.pre_b, View(d1in, 0, 32))
        K.noise_embed(noise, self.ang, View(d1in, 32, 32))
        cur = View.full(d1in)
        attn_before = {'down3': 'attn_down3', 'down4': 'attn_down4'}
        for res, down, up, up_in, cout in levels:
            if down in attn_before:
                cur = self.attention(attn_before[down], cur)
            for j in range(3):
                y = skip_view(up, j, cout)
                self.resblock(f'{down}.residual_blocks.{j}', cur, y)
                cur = y
            pooled = View.full(self._new(B, res // 2, res // 2, cout))
            K.avgpool2x2(cur, pooled)
            cur = pooled
        b1 = View.full(self._new(B, 8, 8, 256))
        self.resblock('bottleneck1', cur, b1)
        a = self.attention('attn_bottleneck', b1)
        b2 = View.full(self._new(B, 8, 8, 256))
        self.resblock('bottleneck2', a, b2)
        cur = b2
        attn_after = {'up1': 'attn_up1', 'up2': 'attn_up2'}
        for res, down, up, up_in, cout in reversed(levels):
            K.upsample2x_bilinear(cur, View(cat[up][0], 0, up_in))
            for u in range(3):
                src = View.full(cat[up][u])
                dst = View(cat[up][u + 1], 0, cout) if u < 2 else View.full(self._new(B, res, res, cout))
                self.resblock(f'{up}.residual_blocks.{u}', src, dst)
                cur = dst
            if up in attn_after:
                cur = self.attention(attn_after[up], cur)
        out = torch.empty((B, 3, S, S), dtype=torch.float32, device=self.dev)
        K.conv_igemm([Seg(cur, TAPS3)], self.out_w, None, None, Hm=S, Wm=S, out_nchw=out)
        return out

"""Swift-SRGAN x4 generator with the reference's parameter tree (``srgan_model/models.py:1-92``).

It runs every guided step (``translation.py:81``) between the diffusion space and the segmenter.
On a ROCm device the forward runs on HIP kernels (``SrganEngine``): per SeperableConv2d one
``wc_dwconv`` (LDS-tiled depthwise KxK) and one ``wc_conv_igemm`` (fp32-MFMA pointwise GEMM) whose
epilogue applies the folded eval-mode BatchNorm, PReLU, the residual add, PixelShuffle (four output
maps, one per sub-pixel) and the ``(tanh + 1) / 2`` head with an NCHW store.  On the CPU the module
runs its own PyTorch layers (the reference's eval semantics).  state_dict keys match the reference
so its ``{'model': ...}`` checkpoints load.
"""
import torch
from torch import nn


class SeperableConv2d(nn.Module):  # (sic) reference spelling, keeps the key names

    def __init__(self, cin, cout, kernel_size, stride=1, padding=1, bias=True):
        super().__init__()
        self.depthwise = nn.Conv2d(cin, cin, kernel_size, stride=stride, padding=padding, groups=cin, bias=bias)
        self.pointwise = nn.Conv2d(cin, cout, 1, bias=bias)

    def forward(self, x):
        return self.pointwise(self.depthwise(x))


class ConvBlock(nn.Module):

    def __init__(self, cin, cout, use_act=True, use_bn=True, discriminator=False, **kw):
        super().__init__()
        self.use_act = use_act
        self.cnn = SeperableConv2d(cin, cout, **kw, bias=not use_bn)
        self.bn = nn.BatchNorm2d(cout) if use_bn else nn.Identity()
        self.act = nn.LeakyReLU(0.2, inplace=True) if discriminator else nn.PReLU(num_parameters=cout)

    def forward(self, x):
        y = self.bn(self.cnn(x))
        return self.act(y) if self.use_act else y


class UpsampleBlock(nn.Module):

    def __init__(self, cin, scale_factor):
        super().__init__()
        self.conv = SeperableConv2d(cin, cin * scale_factor**2, kernel_size=3, stride=1, padding=1)
        self.ps = nn.PixelShuffle(scale_factor)
        self.act = nn.PReLU(num_parameters=cin)

    def forward(self, x):
        return self.act(self.ps(self.conv(x)))


class ResidualBlock(nn.Module):

    def __init__(self, c):
        super().__init__()
        self.block1 = ConvBlock(c, c, kernel_size=3, stride=1, padding=1)
        self.block2 = ConvBlock(c, c, kernel_size=3, stride=1, padding=1, use_act=False)

    def forward(self, x):
        return self.block2(self.block1(x)) + x


class Generator(nn.Module):
    """(tanh(final) + 1) / 2 output in [0, 1]; x4 by two PixelShuffle(2) stages."""

    def __init__(self, in_channels: int = 3, num_channels: int = 64, num_blocks: int = 16, upscale_factor: int = 4):
        super().__init__()
        self.initial = ConvBlock(in_channels, num_channels, kernel_size=9, stride=1, padding=4, use_bn=False)
        self.residual = nn.Sequential(*[ResidualBlock(num_channels) for _ in range(num_blocks)])
        self.convblock = ConvBlock(num_channels, num_channels, kernel_size=3, stride=1, padding=1, use_act=False)
        self.upsampler = nn.Sequential(*[UpsampleBlock(num_channels, 2) for _ in range(upscale_factor // 2)])
        self.final_conv = SeperableConv2d(num_channels, in_channels, kernel_size=9, stride=1, padding=4)
        self._engine = None

    def forward(self, x):
        if x.is_cuda or next(self.parameters()).is_cuda:
            if self.training:
                raise RuntimeError('weatherconverter_amd SRGAN: the HIP engine implements eval-mode inference')
            if self._engine is None or self._engine.stale():
                self._engine = SrganEngine(self)
            return self._engine.forward(x)
        initial = self.initial(x)
        x = self.convblock(self.residual(initial)) + initial
        return (torch.tanh(self.final_conv(self.upsampler(x))) + 1) / 2

    def _apply(self, fn, *args, **kwargs):
        self._engine = None  # device moves invalidate the packed weights
        return super()._apply(fn, *args, **kwargs)


class SrganEngine:
    """Packed HIP execution of an eval-mode ``Generator`` (NHWC fp32 activations)."""

    def __init__(self, gen: Generator):
        from .. import kernels as K
        self.K = K
        self.gen = gen
        self.dev = next(gen.parameters()).device
        self._sig = self._signature()
        with torch.no_grad():
            self.initial = self._pack_block(gen.initial, pad_in=32)  # wc_conv_igemm: C % 32
            self.blocks = [(self._pack_block(rb.block1), self._pack_block(rb.block2)) for rb in gen.residual]
            self.convblock = self._pack_block(gen.convblock)
            self.ups = [self._pack_up(u) for u in gen.upsampler]
            self.final = self._pack_sep(gen.final_conv.depthwise, gen.final_conv.pointwise, None)

    def _signature(self):
        return tuple((p.data_ptr(), p._version) for p in self.gen.parameters()) + tuple(
            (b.data_ptr(), b._version) for b in self.gen.buffers())

    def stale(self) -> bool:
        return self._signature() != self._sig

    def _pack_sep(self, dw: nn.Conv2d, pw: nn.Conv2d, bn, pad_in: int = 0):
        """(dw weight (Cp, K*K), dw bias, pw weight (N, Cin_p), pw bias); eval BN folded into the pw."""
        C, K = dw.in_channels, dw.kernel_size[0]
        Cp = (C + 3) // 4 * 4
        wd = torch.zeros((Cp, K * K), device=self.dev)
        wd[:C] = dw.weight.detach().float().reshape(C, K * K)
        bd = None
        if dw.bias is not None:
            bd = torch.zeros(Cp, device=self.dev)
            bd[:C] = dw.bias.detach().float()
        N = pw.out_channels
        w = pw.weight.detach().double().reshape(N, C)
        b = pw.bias.detach().double() if pw.bias is not None else torch.zeros(N, dtype=torch.float64, device=self.dev)
        if bn is not None and isinstance(bn, nn.BatchNorm2d):
            inv = bn.weight.detach().double() / torch.sqrt(bn.running_var.detach().double() + bn.eps)
            w = w * inv[:, None]
            b = (b - bn.running_mean.detach().double()) * inv + bn.bias.detach().double()
        cin = max(Cp, pad_in)
        wp = torch.zeros((N, cin), dtype=torch.float32, device=self.dev)
        wp[:, :C] = w.float()
        return wd, bd, wp.contiguous(), b.float().contiguous(), K, Cp

    def _pack_block(self, cb, pad_in: int = 0):
        sep = self._pack_sep(cb.cnn.depthwise, cb.cnn.pointwise, cb.bn, pad_in)
        slope = cb.act.weight.detach().float().contiguous() if (cb.use_act and isinstance(cb.act, nn.PReLU)) else None
        if cb.use_act and slope is None:
            raise RuntimeError('SrganEngine: only the generator (PReLU) blocks are supported')
        return sep, slope

    def _pack_up(self, ub):
        wd, bd, wp, b, K, Cp = self._pack_sep(ub.conv.depthwise, ub.conv.pointwise, None)
        r = ub.ps.upscale_factor
        C = wp.shape[0] // (r * r)
        # PixelShuffle: out[c, r*y + i, r*x + j] = in[c*r*r + i*r + j, y, x] -> one GEMM per sub-pixel (i, j)
        parts = []
        for i in range(r):
            for j in range(r):
                rows = torch.arange(C, device=self.dev) * r * r + i * r + j
                parts.append(((i, j), wp[rows].contiguous(), b[rows].contiguous()))
        return wd, bd, parts, K, Cp, r, ub.act.weight.detach().float().contiguous()

    # ------------------------------------------------------------------ execution
    def _new(self, B, H, W, C, zero: bool = False):
        f = torch.zeros if zero else torch.empty
        return f((B, H, W, C), dtype=torch.float32, device=self.dev)

    def _sep(self, x, pack, slope, out, res=None, out_nchw=None, act=None, tmp=None):
        K, V, Seg = self.K, self.K.View, self.K.Seg
        (wd, bd, wp, b, k, Cp), (B, H, W) = pack, (x.B, x.H, x.W)
        t = tmp if tmp is not None else V.full(self._new(B, H, W, wp.shape[1]))
        K.dwconv(x, wd, bd, V(t.t, 0, Cp), k)
        a = (K._native.ACT_PRELU if slope is not None else K._native.ACT_NONE) if act is None else act
        K.conv_igemm([Seg(V.full(t.t), [(0, 0)])], wp, b, out, Hm=H, Wm=W, res=res, out_nchw=out_nchw, act=a,
                     act_param=slope)

    @torch.no_grad()
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        K, V = self.K, self.K.View
        if x.dim() != 4 or x.shape[1] != self.gen.initial.cnn.depthwise.in_channels:
            raise RuntimeError(f'SRGAN expects (B, 3, H, W), got {tuple(x.shape)}')
        x = x.to(self.dev, torch.float32)
        B, Cin, H, W = x.shape
        xin = self._new(B, H, W, 4, zero=True)  # NHWC, channels padded to a float4
        xin[..., :Cin] = x.permute(0, 2, 3, 1)
        (sep0, slope0) = self.initial
        t32 = V.full(self._new(B, H, W, 32, zero=True))  # zero channels beyond Cin for the pointwise K
        C = sep0[2].shape[0]
        initial = V.full(self._new(B, H, W, C))
        self._sep(V(xin, 0, 4), sep0, slope0, initial, tmp=t32)
        tmp = V.full(self._new(B, H, W, C))
        cur = initial
        for (p1, s1), (p2, s2) in self.blocks:
            h = V.full(self._new(B, H, W, C))
            self._sep(cur, p1, s1, h, tmp=tmp)
            y = V.full(self._new(B, H, W, C))
            self._sep(h, p2, s2, y, res=cur, tmp=tmp)
            cur = y
        y = V.full(self._new(B, H, W, C))
        self._sep(cur, self.convblock[0], self.convblock[1], y, res=initial, tmp=tmp)
        cur = y
        for wd, bd, parts, k, Cp, r, slope in self.ups:
            Hc, Wc = cur.H, cur.W
            t = self._new(B, Hc, Wc, Cp)
            K.dwconv(cur, wd, bd, V.full(t), k)
            out = V.full(self._new(B, Hc * r, Wc * r, parts[0][1].shape[0]))
            for (i, j), wp, b in parts:
                K.conv_igemm([K.Seg(V.full(t), [(0, 0)])], wp, b, out, Hm=Hc, Wm=Wc, out_map=(r, r, i, j),
                             act=K._native.ACT_PRELU, act_param=slope)
            cur = out
        wd, bd, wp, b, k, Cp = self.final
        res = torch.empty((B, wp.shape[0], cur.H, cur.W), dtype=torch.float32, device=self.dev)
        self._sep(cur, self.final, None, None, out_nchw=res, act=K._native.ACT_TANH01)
        return res


def load_model(model_path: str, device=None) -> nn.Module:
    """reference srgan_model/inference.py:9-16 (weights_only checkpoint load)."""
    device = device or torch.device('cuda' if torch.cuda.is_available() else 'cpu')
    net = Generator(upscale_factor=4).to(device)
    net.load_state_dict(torch.load(model_path, map_location=device, weights_only=True)['model'])
    return net.eval()


@torch.no_grad()
def inference(netG: nn.Module, lr_image: torch.Tensor) -> torch.Tensor:
    """reference srgan_model/inference.py:35-39."""
    return netG(lr_image)

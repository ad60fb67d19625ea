"""UnetEngine: runs the reference ``Unet`` forward (``unet_base.py:451-488``) as gfx950 HIP kernels.

Data layout in HBM
------------------
* Activations are NHWC fp32.  The only NCHW tensors are the UNet's input (read by ``wc_conv_in``,
  which fuses the transpose) and its output (written by the last implicit-GEMM conv).
* Skip concatenation is free: for every level ``i`` the engine allocates one buffer
  ``U[i] = (B, S_i, S_i, 2*C_i)``.  The down path writes the level's input ``X_i`` (= the skip
  ``down_outs[i]``) straight into channels ``[C_i, 2C_i)``; the up path's ConvTranspose (or the
  stage below when it does not upsample) writes channels ``[0, C_i)``.  The up ResBlock then reads
  ``U[i]`` as one contiguous tensor, which is exactly ``torch.cat([x, out_down], dim=1)`` of
  ``unet_base.py:349``.
* Weights are repacked once per ``load_state_dict``: the ResBlock 3x3 convs into the Winograd
  F(2,3)-along-x operand layout (``U = (g0, (g0+g1+g2)/2, (g0-g1+g2)/2, g2)`` per kernel row, split
  into two fp16 pieces under a per-channel power-of-two scale), conv2 carrying the 1x1
  ``residual_input_conv`` as a 13th K-step per chunk (its bias folded into conv2's); the
  projections, down convs and ConvT into the pre-split ``[N][K]`` fp16-piece layouts.

Default (f16x3, fp32-class) launches per ResBlock (``unet_base.py:146-150``)::

    sc1, sh1, |X| = GN-finalize(partials of X)             wc_gn_finalize_part (partials came from
                                                            X's producer epilogue: no stats pass)
    h  = conv3x3(SiLU(X*sc1 + sh1)) + b1 + temb            wc_conv3x3_wino_f16x3 (GN+SiLU prologue,
                                                            transform, split per chunk in the conv;
                                                            epilogue writes h's GN partials)
    sc2, sh2 = GN-finalize(partials of h)                  wc_gn_finalize_part
    Y  = conv3x3(SiLU(h*sc2 + sh2)) + conv1x1(X) + b2      wc_conv3x3_wino_f16x3, residual in the
                                                            transform domain under |X|

For convs with >= 4 output-channel tiles of 128 the GN+SiLU + transform + split of segment 0 runs
once per input (``wc_wino_vsplit_f16x3``) and the conv copies its halo planes by LDS-DMA
(``wc_conv3x3_wino_f16x3_vp``); the 64-channel conv2 + residual stays on the direct halo kernel
(``wc_conv3x3_f16x3``, measured faster there).

Per attention layer (``unet_base.py:153-161``), in place on Y::

    sc, sh = GN-finalize(partials of Y)
    a3 = split(GN(Y))                                     wc_split_f16x3_tiled (once per element)
    Q, K, V = a3 W_in^T + b_in, written pre-split           wc_proj_f16x3_qkv (fp16 pieces, V in the
                                                            PV MFMA's key order)
    O = flash-attention(Q, K, V), written pre-split        wc_attention_fwd_f16x3_presplit_a3
    Y = Y + O W_out^T + b_out                              wc_proj_f16x3 (residual in place, Y's GN
                                                            partials from the epilogue)

Modes ``bf16x6`` / ``fp32`` (``set_conv_precision``) run the same structure on the direct halo
kernels (``wc_conv3x3_x6``) and implicit-GEMM convs (``wc_conv_igemm``).
"""
import os
from dataclasses import dataclass
from typing import List, Optional, Tuple

import torch

from ... import kernels as K
from ...kernels import Seg, View

TAPS3 = [(ky - 1, kx - 1) for ky in range(3) for kx in range(3)]
TAPS1 = [(0, 0)]
TAPS4S2 = [(ky - 1, kx - 1) for ky in range(4) for kx in range(4)]
# ConvTranspose2d(4, stride 2, pad 1): output row 2m+p gathers input rows m+dy with kernel row ky.
_CT_TAPS = {0: [(0, 1), (-1, 3)], 1: [(1, 0), (0, 2)]}


def pack_conv(w: torch.Tensor) -> torch.Tensor:
    """[Co][Ci][kh][kw] -> [Co][(ky*kw + kx)*Ci + ci]."""
    co = w.shape[0]
    return w.detach().permute(0, 2, 3, 1).reshape(co, -1).contiguous().float()


def pack_convT(wt: torch.Tensor, py: int, px: int) -> Tuple[List[Tuple[int, int]], torch.Tensor]:
    """ConvTranspose weight [Ci][Co][4][4] -> (taps, [Co][tap*Ci + ci]) for output parity (py, px)."""
    taps, cols = [], []
    for dy, ky in _CT_TAPS[py]:
        for dx, kx in _CT_TAPS[px]:
            taps.append((dy, dx))
            cols.append(wt.detach()[:, :, ky, kx].t())
    return taps, torch.cat(cols, dim=1).contiguous().float()


@dataclass
class ResPack:
    ci: int
    co: int
    g1: torch.Tensor
    be1: torch.Tensor
    w1: torch.Tensor
    b1: torch.Tensor
    g2: torch.Tensor
    be2: torch.Tensor
    w2: torch.Tensor  # conv2 (9*co) ++ residual 1x1 (ci)
    b2: torch.Tensor
    temb_off: int
    w1x6: Optional[Tuple[Optional[K.X6Weight], K.X6Weight]] = None  # bf16x6 re-packs (halo, natural order)
    w2x6: Optional[Tuple[Optional[K.X6Weight], K.X6Weight]] = None
    w1f3: Optional[K.X6Weight] = None  # f16x3 re-packs (precision 'f16x3')
    w2f3: Optional[K.X6Weight] = None
    gb1: Tuple[float, float] = (0.0, 0.0)  # (max|gamma|, max|beta|) of the GroupNorms (f16x3 bound)
    gb2: Tuple[float, float] = (0.0, 0.0)
    w1wn: Optional[K.X6Weight] = None  # Winograd F(2,3) packs (precision 'f16x3', kernels.wino_enabled())
    w2wn: Optional[K.X6Weight] = None


@dataclass
class AttnPack:
    c: int
    heads: int
    g: torch.Tensor
    be: torch.Tensor
    w_in: torch.Tensor
    b_in: torch.Tensor
    w_out: torch.Tensor
    b_out: torch.Tensor
    w_in_x6: Optional[K.X6Weight] = None
    w_out_x6: Optional[K.X6Weight] = None
    w_in_f3: Optional[K.X6Weight] = None  # f16x3 re-packs (in_proj: GN bound, out_proj: V bound)
    w_out_f3: Optional[K.X6Weight] = None
    qkv_l1: Optional[torch.Tensor] = None  # f16x3: host row-L1 norms of W_in and |b_in| (bounds)
    qkv_babs: Optional[torch.Tensor] = None
    gb: Tuple[float, float] = (0.0, 0.0)


class UnetEngine:

    def __init__(self, model):
        params = list(model.parameters())
        if not params or not params[0].is_cuda:
            raise RuntimeError('weatherconverter_amd.Unet runs on the GPU only (HIP kernels, no CPU fallback): '
                               'move the model to a ROCm device first')
        K._native.load()
        self.model = model
        self.device = params[0].device
        self.precision = getattr(model, 'conv_precision', None) or K.default_conv_precision()
        # f16x3 attention on the pre-split in-projection (WC_ATTN_PRESPLIT=0: fp32 projection + split
        # in the attention kernel, the bit-identical reference path)
        self.attn_presplit = os.environ.get('WC_ATTN_PRESPLIT', '1') != '0'
        # GroupNorm statistics from the producers' epilogue tile partials (False: a stats pass per GN)
        self.gn_partials = os.environ.get('WC_GN_PARTIALS', '1') != '0'
        self._sig = self._signature()
        self._pack()

    # ------------------------------------------------------------------ packing
    def _signature(self):
        return tuple((p.data_ptr(), p._version) for p in self.model.parameters())

    def _pack(self):
        m = self.model
        self.res_packs = []
        self.temb_rows_w, self.temb_rows_b = [], []
        self._temb_P = 0
        with torch.no_grad():
            self.downs = [self._pack_stage(blk, n_res=blk.num_layers, attn=blk.use_attn) for blk in m.downs]
            self.down_convs = []
            for blk in m.downs:
                if blk.down_sample:
                    w = pack_conv(blk.down_sample_conv.weight)
                    ci = blk.down_sample_conv.in_channels
                    self.down_convs.append((w, blk.down_sample_conv.bias.detach().float(),
                                            self._x6(w, ci, len(TAPS4S2)), self._f3n(w, ci, len(TAPS4S2)),
                                            self._f3s(w, ci)))
                else:
                    self.down_convs.append(None)
            self.mids = [self._pack_stage(blk, n_res=blk.num_layers + 1, attn=True) for blk in m.mids]
            self.ups = [self._pack_stage(blk, n_res=blk.num_layers, attn=blk.use_attn) for blk in m.ups]
            self.up_convs = []
            for blk in m.ups:
                if blk.up_sample:
                    ci = blk.up_sample_conv.in_channels
                    parts = [pack_convT(blk.up_sample_conv.weight, py, px) for py in (0, 1) for px in (0, 1)]
                    parts = [(taps, w, self._x6(w, ci, len(taps)), self._f3n(w, ci, len(taps))) for taps, w in parts]
                    self.up_convs.append((parts, blk.up_sample_conv.bias.detach().float(),
                                          self._f3t(blk.up_sample_conv.weight, ci)))
                else:
                    self.up_convs.append(None)
            self.conv_in_w = m.conv_in.weight.detach().float().contiguous()
            self.conv_in_b = m.conv_in.bias.detach().float().contiguous()
            self.norm_out = (m.norm_out.weight.detach().float(), m.norm_out.bias.detach().float())
            self.conv_out_w = pack_conv(m.conv_out.weight)
            self.conv_out_x6 = self._x6(self.conv_out_w, m.conv_out.in_channels, 9)
            self.conv_out_f3 = None
            if self.precision == 'f16x3' and m.conv_out.in_channels % 16 == 0:
                self.conv_out_f3 = K.pack_f16x3(self.conv_out_w, m.conv_out.in_channels, order='natural')
                self.norm_out_gb = (float(m.norm_out.weight.abs().max()), float(m.norm_out.bias.abs().max()))
            self.conv_out_b = m.conv_out.bias.detach().float().contiguous()
            # <= 4 output channels: the dedicated HBM-bound head kernel (an MFMA tile would waste 20x)
            self.conv_out_head = None
            if m.conv_out.out_channels <= 4 and m.conv_out.in_channels % 16 == 0:
                self.conv_out_head = K.pack_head(m.conv_out.weight)
            tp = m.t_proj
            self.tproj = [tp[0].weight.detach().float().contiguous(), tp[0].bias.detach().float().contiguous(),
                          tp[2].weight.detach().float().contiguous(), tp[2].bias.detach().float().contiguous()]
            self.temb_w = torch.cat(self.temb_rows_w, 0).contiguous()
            self.temb_b = torch.cat(self.temb_rows_b, 0).contiguous()

    def _pack_res(self, blk, i: int) -> ResPack:
        f, s, r = blk.resnet_conv_first[i], blk.resnet_conv_second[i], blk.residual_input_conv[i]
        tl = blk.t_emb_layers[i][1]
        ci, co = f[2].in_channels, f[2].out_channels
        w2 = torch.cat([pack_conv(s[2].weight), r.weight.detach().reshape(co, ci).float()], 1).contiguous()
        p = ResPack(ci=ci, co=co, g1=f[0].weight.detach().float(), be1=f[0].bias.detach().float(),
                    w1=pack_conv(f[2].weight), b1=f[2].bias.detach().float().contiguous(),
                    g2=s[0].weight.detach().float(), be2=s[0].bias.detach().float(), w2=w2,
                    b2=(s[2].bias.detach().float() + r.bias.detach().float()).contiguous(), temb_off=self._temb_P)
        if self.precision in ('bf16x6', 'f16x3') and ci % 16 == 0 and co % 16 == 0:
            # halo-order pack for the 3x3 kernel (bf16x6 mode), natural-order pack for the
            # implicit-GEMM fallback (grids the halo kernel does not tile), f16x3 pack
            f3 = self.precision == 'f16x3'
            p.w1x6 = (None if f3 else K.pack_x6(p.w1, ci), self._x6(p.w1, ci, 9))
            p.w2x6 = (None if f3 else K.pack_x6(p.w2, co, ci), self._x6(p.w2, co, 9, ci))
            if f3:
                p.w1f3 = K.pack_f16x3(p.w1, ci)
                p.w2f3 = K.pack_f16x3(p.w2, co, ci, res_f16=True)  # residual bounded by GN1's stats of X
                if K.wino_enabled():
                    p.w1wn = K.pack_wino(p.w1, ci)
                    p.w2wn = K.pack_wino(p.w2, co, ci)
                p.gb1 = (float(p.g1.abs().max()), float(p.be1.abs().max()))
                p.gb2 = (float(p.g2.abs().max()), float(p.be2.abs().max()))
        self.temb_rows_w.append(tl.weight.detach().float())
        self.temb_rows_b.append(tl.bias.detach().float())
        self._temb_P += co
        return p

    def _x6(self, w: torch.Tensor, c0: int, ntaps: int, c1: int = 0) -> Optional[K.X6Weight]:
        """bf16x6 (natural K order) re-pack for wc_conv_igemm_x6, or None in fp32 mode."""
        if self.precision == 'fp32' or c0 % 16 or c1 % 16:
            return None
        return K.pack_x6(w, c0, c1, ntaps=ntaps, order='natural')

    def _f3n(self, w: torch.Tensor, c0: int, ntaps: int) -> Optional[K.X6Weight]:
        """f16x3 (natural K order) pack for a resampling conv whose input range comes from its
        producer's per-image absmax, or None outside f16x3 mode."""
        if self.precision != 'f16x3' or c0 % 16:
            return None
        return K.pack_f16x3(w, c0, ntaps=ntaps, order='natural')

    def _f3s(self, w: torch.Tensor, c0: int) -> Optional[K.X6Weight]:
        """f16x3 space-to-depth pack of a 4x4 / stride-2 down conv for wc_conv4x4s2_f16x3 (the halo
        kernel), or None (outside f16x3 mode, N <= 64, or WC_DOWN_S2D=0: the implicit GEMM)."""
        if (self.precision != 'f16x3' or c0 % 16 or K.x6_tile(w.shape[0])[1] != 128
                or os.environ.get('WC_DOWN_S2D', '1') == '0'):
            return None
        return K.pack_f16x3_s2d(w, c0)

    def _f3t(self, wt: torch.Tensor, c0: int) -> Optional[K.X6Weight]:
        """f16x3 pack of a 4x4 / stride-2 ConvTranspose for wc_convtr4x4s2_f16x3 (all four parities in
        one launch of the halo kernel), or None (outside f16x3 mode or WC_UP_CT=0: the four
        implicit-GEMM parities)."""
        if self.precision != 'f16x3' or c0 % 16 or os.environ.get('WC_UP_CT', '1') == '0':
            return None
        return K.pack_f16x3_convT(wt.detach().float())

    def _pack_attn(self, blk, i: int) -> AttnPack:
        mha, gn = blk.attentions[i], blk.attention_norms[i]
        c = mha.embed_dim
        p = AttnPack(c=c, heads=mha.num_heads, g=gn.weight.detach().float(), be=gn.bias.detach().float(),
                     w_in=mha.in_proj_weight.detach().float().contiguous(),
                     b_in=mha.in_proj_bias.detach().float().contiguous(),
                     w_out=mha.out_proj.weight.detach().float().contiguous(),
                     b_out=mha.out_proj.bias.detach().float().contiguous())
        p.w_in_x6 = self._x6(p.w_in, c, 1)
        p.w_out_x6 = self._x6(p.w_out, c, 1)
        if self.precision == 'f16x3':
            p.w_in_f3 = K.pack_f16x3(p.w_in, c, ntaps=1, order='natural')
            p.w_out_f3 = K.pack_f16x3(p.w_out, c, ntaps=1, order='natural')
            p.qkv_l1 = p.w_in.double().abs().sum(1).cpu()
            p.qkv_babs = p.b_in.double().abs().cpu()
            p.gb = (float(p.g.abs().max()), float(p.be.abs().max()))
        return p

    def _pack_stage(self, blk, n_res: int, attn: bool):
        res = [self._pack_res(blk, i) for i in range(n_res)]
        n_attn = len(blk.attentions)
        att = [self._pack_attn(blk, i) for i in range(n_attn)] if attn else []
        return res, att

    # ------------------------------------------------------------------ building blocks
    def _new(self, B, H, W, C, gn_sw: Optional[int] = None) -> torch.Tensor:
        """Scratch activation.  With gn_sw (and a shape the partials tile) it also carries GroupNorm
        tile partials (kernels.GnPart) that its producers' epilogues fill, so that its GroupNorm
        consumers finalize from them instead of re-reading the tensor."""
        t = torch.empty((B, H, W, C), dtype=torch.float32, device=self.device)
        if gn_sw is not None and self.gn_partials and K.GnPart.eligible(t):
            K.GnPart.attach(t, gn_sw)
        return t

    @staticmethod
    def _sw(C: int) -> Optional[int]:
        """Partials sub-slot width for GroupNorm(8) over C channels (and over 2C for the skip buffers)."""
        cpg = C // 8
        for sw in (32, 16, 8, 4):
            if C % 8 == 0 and cpg % sw == 0:
                return sw
        return None

    def _gn(self, v: View, gamma, beta, bound: bool = False):
        """GroupNorm(8) affine of a view: from its tile partials when it has them, else a stats pass."""
        gp = K.GnPart.of(v)
        if gp is not None and (v.C // 8) % gp.sw == 0:
            return K.gn_affine(v, gamma, beta, bound=bound, part=gp)
        return K.gn_affine(v, gamma, beta, bound=bound)

    def _gn_fill(self, v: Optional[View], fused: bool = False):
        """Partials of a view written by a kernel that did not emit them from its epilogue."""
        gp = K.GnPart.of(v)
        if gp is not None and not fused:
            K.gn_partials(v, gp)

    def conv(self, segs, w: torch.Tensor, w6: Optional[K.X6Weight], bias, out: Optional[View], H: int, W: int,
             absmax: Optional[torch.Tensor] = None, gn_p64: int = 0, gn_defer: bool = False, **kw) -> Tuple[bool, bool]:
        """Any conv: bf16x6 implicit GEMM when packed for it, else fp32 MFMA.  Returns (the per-image
        output absmax was emitted into `absmax`, the output's GN partials came from the epilogue);
        partials not emitted are filled by a stats pass unless gn_defer."""
        gp = K.GnPart.of(out)
        fused = False
        if w6 is not None:
            fused = K.gn_conv_ok(out, gp, w6.N, H, W, 256 if w6.N <= 64 else 128)
            K.conv_igemm_x6(segs, w6, bias, out, Hm=H, Wm=W, absmax=absmax, gn=gp if fused else None, gn_p64=gn_p64,
                            **kw)
        else:
            K.conv_igemm(segs, w, bias, out, Hm=H, Wm=W, **kw)
        if not gn_defer:
            self._gn_fill(out, fused)
        return absmax is not None and w6 is not None, fused

    def resample(self, segs, pack, bias, out: View, H: int, W: int, bound: Optional[torch.Tensor], gn_p64: int = 0,
                 gn_defer: bool = False, **kw) -> bool:
        """Down-sampling conv / one transposed-conv parity: f16x3 implicit GEMM scaled per image by
        the producer's absmax when there is one (and the tiles stay within an image), else bf16x6.
        Returns whether the output's GN partials came from the epilogue."""
        w, w6, w3 = pack
        if w3 is not None and bound is not None and (H * W) % (256 if w3.N <= 64 else 128) == 0:
            gp = K.GnPart.of(out)
            fused = K.gn_conv_ok(out, gp, w3.N, H, W, 256 if w3.N <= 64 else 128)
            K.conv_igemm_f16x3(segs, w3, bias, out, Hm=H, Wm=W, a_exp=60, a_bound=bound, gn=gp if fused else None,
                               gn_p64=gn_p64, **kw)
            if not gn_defer:
                self._gn_fill(out, fused)
            return fused
        return self.conv(segs, w, w6, bias, out, H, W, gn_p64=gn_p64, gn_defer=gn_defer, **kw)[1]

    def conv3(self, segs, w: torch.Tensor, w6, w3: Optional[K.X6Weight], gb: Tuple[float, float], bias, out: View,
              H: int, W: int, a_bound: Optional[torch.Tensor] = None, absmax: Optional[torch.Tensor] = None,
              wn: Optional[K.X6Weight] = None, **kw) -> bool:
        """A ResBlock 3x3 stride-1 conv (GN+SiLU prologue): the halo-tiled kernel in f16x3 (bound
        from the GroupNorm affine gb and the group size) or bf16x6 when the grid tiles, else the
        bf16x6 implicit GEMM (or fp32 MFMA in fp32 mode).  GN partials of `out` are emitted by the
        split-precision epilogues where they can be, else filled by a stats pass.  Returns whether
        the absmax was emitted."""
        gp = K.GnPart.of(out)
        if (wn is not None and K.wino_eligible(segs, wn.N, H, W) and (len(segs) == 1 or a_bound is not None)
                and (w3 is None or K.x6_eligible(segs, w3.N, H, W))):
            # the Winograd F(2,3)-along-x form of the same f16x3 conv (1.5x fewer MFMAs)
            n_group = H * W * segs[0].view.C // 8
            fused = K.gn_conv_ok(out, gp, wn.N, H, W)
            K.conv3x3_wino(segs, wn, bias, out, Hm=H, Wm=W, a_exp=K.f16x3_a_exp(gb[0], gb[1], n_group),
                           a_bound=a_bound, absmax=absmax, gn=gp if fused else None, **kw)
            self._gn_fill(out, fused)
            return absmax is not None
        if w3 is not None and K.x6_eligible(segs, w3.N, H, W):
            n_group = H * W * segs[0].view.C // 8
            fused = K.gn_conv_ok(out, gp, w3.N, H, W)
            K.conv3x3_f16x3(segs, w3, bias, out, Hm=H, Wm=W, a_exp=K.f16x3_a_exp(gb[0], gb[1], n_group),
                            a_bound=a_bound if w3.res_f16 else None, absmax=absmax, gn=gp if fused else None, **kw)
            self._gn_fill(out, fused)
            return absmax is not None
        if w6 is not None and w6[0] is not None and K.x6_eligible(segs, w6[0].N, H, W):
            fused = K.gn_conv_ok(out, gp, w6[0].N, H, W)
            K.conv3x3_x6(segs, w6[0], bias, out, Hm=H, Wm=W, absmax=absmax, gn=gp if fused else None, **kw)
            self._gn_fill(out, fused)
            return absmax is not None
        return self.conv(segs, w, None if w6 is None else w6[1], bias, out, H, W, absmax=absmax, **kw)[0]

    def resblock(self, X: View, Y: View, p: ResPack, temb: torch.Tensor, temb_ld: int,
                 absmax: Optional[torch.Tensor] = None) -> bool:
        B, H, W = X.B, X.H, X.W
        xb = None
        if p.w2f3 is not None and p.w2f3.res_f16:
            sc1, sh1, xb = self._gn(X, p.g1, p.be1, bound=True)  # xb bounds |X| (conv2's residual input)
        else:
            sc1, sh1 = self._gn(X, p.g1, p.be1)
        h = View.full(self._new(B, H, W, p.co, gn_sw=self._sw(p.co)))
        self.conv3([Seg(X, TAPS3, scale=sc1, shift=sh1, silu=True)], p.w1, p.w1x6, p.w1f3, p.gb1, p.b1, h, H, W,
                   temb=temb[:, p.temb_off:], temb_ld=temb_ld, wn=p.w1wn)
        sc2, sh2 = self._gn(h, p.g2, p.be2)
        return self.conv3([Seg(h, TAPS3, scale=sc2, shift=sh2, silu=True),
                           Seg(X, TAPS1, kbase=9 * p.co)], p.w2, p.w2x6, p.w2f3, p.gb2, p.b2, Y, H, W, a_bound=xb,
                          absmax=absmax, wn=p.w2wn)

    def attention(self, Y: View, p: AttnPack, absmax: Optional[torch.Tensor] = None) -> bool:
        B, H, W, C = Y.B, Y.H, Y.W, Y.C
        N = H * W
        sc, sh = self._gn(Y, p.g, p.be)
        if p.w_in_f3 is not None:
            # in_proj: GN output bound; attention: q/k/v bounds; out_proj: |O| <= max|V| (convex
            # combination of V rows), so the V exponent bounds it
            a_exp = K.f16x3_a_exp(p.gb[0], p.gb[1], N * C // 8)
            exps = K.attention_exps_from_norms(p.qkv_l1, p.qkv_babs, p.gb[0], p.gb[1], N * C // 8)
            seg = Seg(Y, TAPS1, scale=sc, shift=sh, silu=False)
            if self.attn_presplit and K.qkv_presplit_ok(B, N, C, p.heads):
                # the in_proj epilogue writes Q, K, V already scaled and split (fp16 pieces, V
                # transposed in the PV key order); the attention copies K / V^T tiles by LDS-DMA
                qkv3 = torch.empty(B * 6 * C * N, dtype=torch.int16, device=self.device)
                if K.proj_pa_enabled() and K.proj_pa_ok(Y, 3 * C):
                    # GN applied and split once per element (not once per 128-column N tile), then
                    # both GEMM operands staged by LDS-DMA
                    a3 = K.split_f16x3_tiled(Y, a_exp, sc, sh)
                    K.proj_f16x3_qkv(Y, a3, p.w_in_f3, p.b_in, qkv3, a_exp=a_exp, C=C, heads=p.heads, exps=exps)
                    del a3
                else:
                    K.conv_igemm_f16x3_qkv(seg, p.w_in_f3, p.b_in, qkv3, Hm=H, Wm=W, a_exp=a_exp, C=C,
                                           heads=p.heads, exps=exps)
                if K.proj_pa_enabled() and K.proj_pa_ok(Y, C) and C % 32 == 0:
                    # the attention writes O already scaled and split in the out-projection's LDS
                    # stage order (no fp32 O round trip, no split pass); the GEMM copies it by LDS-DMA
                    a3o = K.attention_presplit_a3(qkv3, B, N, C, p.heads, exps)
                    del qkv3
                    gp = K.GnPart.of(Y)
                    fused = K.gn_conv_ok(Y, gp, p.w_out_f3.N, H, W, 256 if p.w_out_f3.N <= 64 else 128)
                    shape = View(a3o.view(torch.float32).view(B, H, W, C), 0, C)  # the operand's view shape
                    K.proj_f16x3(shape, a3o, p.w_out_f3, p.b_out, Y, a_exp=exps[2], res=Y, absmax=absmax,
                                 gn=gp if fused else None)
                    self._gn_fill(Y, fused)
                    return absmax is not None
                o = self._new(B, H, W, C)
                K.attention_presplit(qkv3, o.view(B * N, C), B, N, C, p.heads, exps)
            else:
                o = self._new(B, H, W, C)
                qkv = self._new(B, H, W, 3 * C)
                K.conv_igemm_f16x3([seg], p.w_in_f3, p.b_in, View.full(qkv), Hm=H, Wm=W, a_exp=a_exp)
                K.attention(qkv.view(B * N, 3 * C), o.view(B * N, C), B, N, C, p.heads, 'f16x3', exps)
            gp = K.GnPart.of(Y)
            fused = K.gn_conv_ok(Y, gp, p.w_out_f3.N, H, W, 256 if p.w_out_f3.N <= 64 else 128)
            K.conv_igemm_f16x3([Seg(View.full(o), TAPS1)], p.w_out_f3, p.b_out, Y, Hm=H, Wm=W, a_exp=exps[2],
                               res=Y, absmax=absmax, gn=gp if fused else None)
            self._gn_fill(Y, fused)
            return absmax is not None
        qkv = self._new(B, H, W, 3 * C)
        o = self._new(B, H, W, C)
        self.conv([Seg(Y, TAPS1, scale=sc, shift=sh, silu=False)], p.w_in, p.w_in_x6, p.b_in, View.full(qkv), H, W)
        K.attention(qkv.view(B * N, 3 * C), o.view(B * N, C), B, N, C, p.heads, self.precision)
        return self.conv([Seg(View.full(o), TAPS1)], p.w_out, p.w_out_x6, p.b_out, Y, H, W, res=Y, absmax=absmax)[0]

    # ------------------------------------------------------------------ forward
    def max_batch(self, S: int, S2: int) -> int:
        """Largest batch one pass can take: the kernels address each source tensor of the whole batch
        through one buffer descriptor (32-bit byte offsets, < 2 GiB).  Per image, the widest tensor at
        level i is the skip buffer (2*dc[i] channels), a ResBlock output (dc[i+1]) or an attention
        in-projection (3*C; 6*C fp16 pieces pre-split, the same bytes)."""
        m = self.model
        dc, mids = m.down_channels, m.mid_channels
        h, w = S, S2
        per_image = 0
        L = len(dc) - 1
        for i in range(L):
            att = m.downs[i].use_attn or m.ups[L - 1 - i].use_attn
            wide = max(2 * dc[i], dc[i + 1], 3 * max(dc[i], dc[i + 1]) if att else 0)
            per_image = max(per_image, h * w * 4 * wide)
            if m.down_sample[i]:
                h, w = h // 2, w // 2
        per_image = max(per_image, h * w * 4 * 3 * max(mids + [dc[-1]]))
        return max(1, ((1 << 31) - 1) // per_image)

    def forward(self, x: torch.Tensor, t) -> torch.Tensor:
        """Batches above max_batch run as consecutive chunks: every op is per image, and every kernel's
        reduction order is independent of the batch, so the result equals one pass bit for bit."""
        m = self.model
        if x.dim() != 4 or x.shape[1] != m.model_config.im_channels:
            raise RuntimeError(f'Unet expects (B, {m.model_config.im_channels}, H, W), got {tuple(x.shape)}')
        B = x.shape[0]
        tt = torch.as_tensor(t).long().reshape(-1).to(self.device)
        if tt.shape[0] not in (1, B):
            raise RuntimeError(f'timestep tensor has {tt.shape[0]} entries for a batch of {B}')
        cap = self.max_batch(x.shape[2], x.shape[3])
        if B <= cap:
            return self._forward(x, tt)
        outs = []
        for b0 in range(0, B, cap):
            tc = tt if tt.shape[0] == 1 else tt[b0:b0 + cap]
            outs.append(self._forward(x[b0:b0 + cap], tc))
        return torch.cat(outs)

    def _forward(self, x: torch.Tensor, tt: torch.Tensor) -> torch.Tensor:
        if self._signature() != self._sig:  # parameters changed in place: repack
            self._sig = self._signature()
            self._pack()
        m = self.model
        x = x.to(device=self.device, dtype=torch.float32).contiguous()
        B, _, S, S2 = x.shape
        nt = tt.shape[0]
        temb = K.temb(tt, *self.tproj, self.temb_w, self.temb_b)
        temb_ld = temb.shape[1] if nt > 1 else 0

        dc = m.down_channels
        L = len(dc) - 1
        sizes = [(S, S2)]
        for i in range(L):
            h, w = sizes[-1]
            sizes.append((h // 2, w // 2) if m.down_sample[i] else (h, w))
        # skip buffers: partials at the sub-slot width of the half (down-path) view, which also tiles
        # the whole (up-path, 2C-channel) view's groups
        U = [self._new(B, sizes[i][0], sizes[i][1], 2 * dc[i], gn_sw=self._sw(dc[i])) for i in range(L)]

        cur = View(U[0], dc[0], dc[0])
        self._gn_fill(cur, K.conv_in(x, self.conv_in_w, self.conv_in_b, cur, gn=K.GnPart.of(cur)))

        # per-image max |x| of each resampling conv's input, emitted by its producer's epilogue
        # (the f16x3 down / transposed convs scale by it; one row per resampling conv)
        amax = None
        if self.precision == 'f16x3':
            amax = torch.zeros((2 * L + 1, B), dtype=torch.float32, device=self.device)
        slots = iter(range(2 * L + 1))

        def bound_slot(needed: bool):
            return amax[next(slots)] if (needed and amax is not None) else None

        # ---------------- down path
        for i in range(L):
            res, att = self.downs[i]
            co = dc[i + 1]
            H, W = sizes[i]
            final = View(U[i + 1], dc[i + 1], dc[i + 1]) if i < L - 1 else View.full(
                self._new(B, sizes[i + 1][0], sizes[i + 1][1], co, gn_sw=self._sw(co)))
            bnd = None
            for li, rp in enumerate(res):
                last = li == len(res) - 1
                tgt = final if (last and self.down_convs[i] is None) else View.full(
                    self._new(B, H, W, co, gn_sw=self._sw(co)))
                slot = bound_slot(last and self.down_convs[i] is not None)
                bnd = slot if self.resblock(cur, tgt, rp, temb, temb_ld, absmax=None if att else slot) else None
                if att:
                    bnd = slot if self.attention(tgt, att[li], absmax=slot) else None
                cur = tgt
            if self.down_convs[i] is not None:
                w, b, w6, w3, w3s = self.down_convs[i]
                seg = Seg(cur, TAPS4S2, stride=2)
                Hm, Wm = sizes[i + 1]
                if w3s is not None and bnd is not None and K.conv4x4s2_f16x3_ok(seg, w3s.N, Hm, Wm):
                    gp = K.GnPart.of(final)
                    fused = K.gn_conv_ok(final, gp, w3s.N, Hm, Wm)
                    K.conv4x4s2_f16x3(seg, w3s, b, final, Hm=Hm, Wm=Wm, a_bound=bnd, gn=gp if fused else None)
                    self._gn_fill(final, fused)
                else:
                    self.resample([seg], (w, w6, w3), b, final, Hm, Wm, bnd)
                cur = final

        # ---------------- mid path
        bnd = None
        for j, (res, att) in enumerate(self.mids):
            last_mid = j == len(self.mids) - 1
            H, W = cur.H, cur.W
            for li, rp in enumerate(res):
                if last_mid and li == len(res) - 1 and self.up_convs[0] is None:
                    tgt = View(U[L - 1], 0, dc[L - 1])
                else:
                    tgt = View.full(self._new(B, H, W, rp.co, gn_sw=self._sw(rp.co)))
                has_att = li < len(att)
                slot = bound_slot(last_mid and li == len(res) - 1 and self.up_convs[0] is not None)
                bnd = slot if self.resblock(cur, tgt, rp, temb, temb_ld, absmax=None if has_att else slot) else None
                cur = tgt
                if has_att:
                    bnd = slot if self.attention(cur, att[li], absmax=slot) else None

        # ---------------- up path
        for k, (res, att) in enumerate(self.ups):
            i = L - 1 - k
            H, W = sizes[i]
            if self.up_convs[k] is not None:
                parts, b, w3t = self.up_convs[k]
                dst = View(U[i], 0, dc[i])
                seg = Seg(cur, [(0, 0)])
                if w3t is not None and bnd is not None and K.convT4x4s2_f16x3_ok(seg, w3t.N):
                    gp = K.GnPart.of(dst)
                    fused = K.gn_conv_ok(dst, gp, w3t.N, dst.H, dst.W)
                    K.convT4x4s2_f16x3(seg, w3t, b, dst, a_bound=bnd, gn=gp if fused else None)
                    self._gn_fill(dst, fused)
                else:
                    np_in = cur.H * cur.W // 64 if (cur.H * cur.W) % 64 == 0 else 0
                    fused = []
                    for par, ((py, px), (taps, w, w6, w3)) in enumerate(zip(((0, 0), (0, 1), (1, 0), (1, 1)), parts)):
                        # each parity covers a quarter of the output pixels: its own range of pixel blocks
                        fused.append(self.resample([Seg(cur, taps)], (w, w6, w3), b, dst, cur.H, cur.W, bnd,
                                                   gn_p64=par * np_in, gn_defer=True, out_map=(2, 2, py, px)))
                    self._gn_fill(dst, all(fused) and np_in > 0)
            else:
                assert cur.t is U[i] and cur.c0 == 0, 'non-upsampling level must have been written in place'
            cur = View.full(U[i])
            next_in_place = i > 0 and self.up_convs[k + 1] is None
            next_up = k + 1 < len(self.ups) and self.up_convs[k + 1] is not None
            bnd = None
            for li, rp in enumerate(res):
                last = li == len(res) - 1
                tgt = View(U[i - 1], 0, dc[i - 1]) if (last and next_in_place) else View.full(
                    self._new(B, H, W, rp.co, gn_sw=self._sw(rp.co)))
                slot = bound_slot(last and next_up)
                bnd = slot if self.resblock(cur, tgt, rp, temb, temb_ld, absmax=None if att else slot) else None
                if att:
                    bnd = slot if self.attention(tgt, att[li], absmax=slot) else None
                cur = tgt

        # ---------------- head: GN -> SiLU -> conv_out, NCHW output
        sc, sh = self._gn(cur, *self.norm_out)
        out = torch.empty((B, m.model_config.im_channels, S, S2), dtype=torch.float32, device=self.device)
        head = [Seg(cur, TAPS3, scale=sc, shift=sh, silu=True)]
        if self.conv_out_head is not None:
            K.head_conv(cur, sc, sh, self.conv_out_head, self.conv_out_b, out)
        elif self.conv_out_f3 is not None:
            K.conv_igemm_f16x3(head, self.conv_out_f3, self.conv_out_b, None, Hm=S, Wm=S2, out_nchw=out,
                               a_exp=K.f16x3_a_exp(*self.norm_out_gb, S * S2 * cur.C // 8))
        else:
            self.conv(head, self.conv_out_w, self.conv_out_x6, self.conv_out_b, None, S, S2, out_nchw=out)
        return out

"""TrainEngine: the reference ``Unet`` training step's forward (with saved activations) and its
backward, as gfx950 HIP kernels — ``loss.backward()`` of ``train_ddpm.py:106-110``.

Forward (same layout as ``UnetEngine``: NHWC fp32 activations, one skip buffer ``U[i]`` per level so
the up path's ``torch.cat`` is free) records a tape; every GroupNorm keeps both its affine
(scale, shift) and the plain normalisation (rstd, -mean*rstd) so the backward recomputes
SiLU(GN(x)) from the stored pre-norm tensor instead of keeping the activation.  Attention keeps its
pre-residual input, q/k/v, its output and the softmax log-sum-exp.

Backward, per layer type (reference modules of unet_base.py):
  Conv2d 3x3 / 1x1 / 4x4-s2, ConvTranspose2d 4x4-s2, in/out projections
      data gradient   the forward kernels on re-packed weights: a 3x3 conv's is the 3x3 conv of dY
                      with W flipped and transposed (halo kernel); a 4x4/s2 conv's is the transposed
                      conv of dY (four parity sub-convs); a transposed conv's is the 4x4/s2 conv of
                      dY with its own weight; a linear layer's is dY W.
      weight gradient wc_conv_wgrad3 (3x3: halo-tiled) or wc_conv_wgrad (GEMM over the pixels), the
                      input re-read through the forward's taps and GN prologue; split partials
                      reduced in a fixed order and scattered into the parameter's layout.
      bias            per-(b, c) pixel sums, summed over b in a fixed order.
  GroupNorm(+SiLU)    wc_gn_bwd_* (dx, dgamma, dbeta).
  attention core      wc_attention_bwd_f16x3 / _bwd6 / _bwd (dq, dk, dv from lse; no N x N matrix).
  time embedding MLP  small GEMM / SiLU kernels (B x 128).
Arithmetic (precision f16x3, the default): forward convs, projections and attention on f16x3 under
the sampler's static bounds; 3x3 and projection data gradients, the 3x3 weight gradients and the
attention backward on f16x3 under per-image range bounds of the gradients, which every kernel
writing a gradient tensor raises as it writes (_gb); the rest on bf16x6 (exact 3-piece bf16 split).
Precision bf16x6 / fp32: bf16x6 / fp32 MFMA throughout.  fp32-class gradients, checked against
PyTorch autograd of the reference restatement in float64.  Every gradient buffer is written in a
fixed order: results are deterministic run to run.
"""
import os
from typing import Dict, List, Optional, Tuple

import torch

from ... import kernels as K
from ...kernels import Seg, View
from .engine import TAPS1, TAPS3, TAPS4S2, UnetEngine, pack_conv, pack_convT

_PARITIES = ((0, 0), (0, 1), (1, 0), (1, 1))


class _Pack(dict):
    """A layer's packing record whose weight packs are built on first use: a value wrapped in
    _Pack.lazy(fn) is computed by fn() when read, then cached.  Each training step packs only the
    forms its arithmetic actually launches (e.g. the f16x3 data-gradient packs, not also the bf16x6
    ones) — the packing is host-launched torch work on every step."""

    class lazy:
        __slots__ = ('fn', )

        def __init__(self, fn):
            self.fn = fn

    def __getitem__(self, k):
        v = dict.__getitem__(self, k)
        if isinstance(v, _Pack.lazy):
            with torch.no_grad():
                v = v.fn()
            dict.__setitem__(self, k, v)
        return v

    def has(self, k) -> bool:
        """Whether form k exists for this layer, without building it (a lazy form is never None)."""
        return dict.get(self, k) is not None


class _Slot:
    """A host value of the packing pass, filled by TrainEngine._resolve."""
    __slots__ = ('value', )


class Tape:
    """Everything one training forward saved for its backward: the layer records (activations, GN
    statistics, packed weights) plus the inputs and the per-step weight packs the backward reads.  One
    per forward, owned by that forward's autograd node, consumed by exactly one backward."""
    _FIELDS = ('records', 'x', 'tt', 'U', 'P', 'head_T', 'tproj', 'temb_w', 'res_rows')

    def __init__(self, engine: 'TrainEngine'):
        self.records = engine.tape
        for f in self._FIELDS[1:]:
            setattr(self, f, getattr(engine, f))
        self.consumed = False


class TrainEngine:

    def __init__(self, model, precision: Optional[str] = None):
        params = list(model.parameters())
        if not params or not params[0].is_cuda:
            raise RuntimeError('weatherconverter_amd.Unet trains on the GPU only (HIP kernels, no CPU fallback)')
        K._native.load()
        self.model = model
        self.device = params[0].device
        p = (precision or getattr(model, 'train_precision', None) or getattr(model, 'conv_precision', None)
             or K.default_conv_precision())
        # 'f16': the 16-bit training line — the f16x3 arithmetic of mode f16x3 run on the single-piece
        # build (one fp16 piece per operand: wc_x6.hpp mfma_f16c), every kernel call routed to it
        # 'bf16': the same on the bf16 single-piece build (one bf16 piece per operand on the bf16 MFMA:
        # BASELINE config 3's bf16 training)
        self.variant = {'f16': 'single16', 'bf16': 'bf16'}.get(p, '')
        if p in ('f16', 'bf16'):
            p = 'f16x3'
        # f16x3 needs range bounds that gradients do not have: the backward runs bf16x6; the forward's
        # GroupNorm-prologue convs and projections run f16x3 under their static bounds (as inference)
        self.precision = 'fp32' if p == 'fp32' else 'bf16x6'
        self.f3 = p == 'f16x3'
        # data gradients on f16x3 under per-image absmax bounds of the incoming gradient (mode f16x3)
        self.f3d = self.f3 and K.dgrad_f16x3_enabled()
        self.tape: List[tuple] = []
        self.last_tape: Optional[Tape] = None

    # ------------------------------------------------------------------ packing (per step)
    def _pk(self, w2d: torch.Tensor, C0: int, ntaps: int, C1: int = 0):
        w2d = w2d.contiguous().float()
        x6 = None
        if self.precision == 'bf16x6' and C0 % 16 == 0 and C1 % 16 == 0:
            x6 = K.pack_x6(w2d, C0, C1, ntaps=ntaps, order='natural')
        elif C0 % 32 or C1 % 32:
            raise RuntimeError(f'fp32 implicit GEMM needs channel counts % 32 (got {C0}, {C1})')
        return (w2d, x6)

    def _conv(self, segs, pk, bias, out: Optional[View], H: int, W: int, **kw):
        w, x6 = pk
        if kw.get('absmax', 0) is None:  # no bound tracked (outside the f16x3 backward)
            del kw['absmax']
        if x6 is not None:
            K.conv_igemm_x6(segs, x6, bias, out, Hm=H, Wm=W, **kw)
        else:
            K.conv_igemm(segs, w, bias, out, Hm=H, Wm=W, **kw)

    def _pack_res(self, blk, i: int):
        f, s, r = blk.resnet_conv_first[i], blk.resnet_conv_second[i], blk.residual_input_conv[i]
        w1, w2, wr = f[2].weight.detach(), s[2].weight.detach(), r.weight.detach()
        ci, co = w1.shape[1], w1.shape[0]
        wr2 = wr.reshape(co, ci)
        f3 = self.f3 and ci % 16 == 0 and co % 16 == 0
        wino = K.wino_enabled()
        raw = all(t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() for t in (w1, w2)) \
            and 9 * (max(ci, co) + 4) * 4 <= 64 * 1024 and os.environ.get('WC_PACK_RAW', '1') != '0'
        L = _Pack.lazy
        # shared re-layouts, each built once and only if a pack that needs it is (the Winograd forms
        # usually replace the direct f16x3 ones, so those are lazy too)
        rp = _Pack(w1c=L(lambda: pack_conv(w1).float().contiguous()),
                   w2cat=L(lambda: torch.cat([pack_conv(w2), wr2], 1).float().contiguous()),
                   w1T=L(lambda: pack_conv(w1.flip([2, 3]).transpose(0, 1)).float().contiguous()),
                   w2T=L(lambda: pack_conv(w2.flip([2, 3]).transpose(0, 1)).float().contiguous()))
        rp.update(
            ci=ci, co=co, gn1=f[0], conv1=f[2], gn2=s[0], conv2=s[2], resc=r, temb=blk.t_emb_layers[i][1],
            pk1=L(lambda: self._pk(rp['w1c'], ci, 9)),
            pk2=L(lambda: self._pk(rp['w2cat'], co, 9, ci)),
            f3_1=L(lambda: K.pack_f16x3(rp['w1c'], ci)) if f3 else None,
            f3_2=L(lambda: K.pack_f16x3(rp['w2cat'], co, ci, res_f16=True)) if f3 else None,
            gb1=self._later_absmax(f[0].weight, f[0].bias),
            gb2=self._later_absmax(s[0].weight, s[0].bias),
            b2=(s[2].bias.detach() + r.bias.detach()).float().contiguous(),
            pk1T=L(lambda: self._pk(rp['w1T'], co, 9)),
            pk2T=L(lambda: self._pk(rp['w2T'], co, 9)),
            pkrT=L(lambda: self._pk(wr2.t(), co, 1)),
            # f16x3 data gradients (raw gradient operand under its per-image absmax bound)
            f3_1T=L(lambda: K.pack_f16x3(rp['w1T'], co)) if self.f3d else None,
            f3_2T=L(lambda: K.pack_f16x3(rp['w2T'], co)) if self.f3d else None,
            f3_rT=L(lambda: K.pack_f16x3(wr2.t().contiguous().float(), co, ntaps=1, order='natural'))
            if self.f3d else None,
            # the Winograd F(2,3)-along-x forms of the same f16x3 convs (forward and data gradients)
            # (from the module weights directly when they are fp32 on the device: no host re-layouts)
            wn_1=L(lambda: K.pack_wino_raw(w1) if raw else K.pack_wino(rp['w1c'], ci)) if f3 and wino else None,
            wn_2=L(lambda: K.pack_wino_raw(w2, wr2.float().contiguous()) if raw else K.pack_wino(rp['w2cat'], co, ci))
            if f3 and wino else None,
            wn_1T=L(lambda: K.pack_wino_raw(w1, transposed=True) if raw else K.pack_wino(rp['w1T'], co))
            if self.f3d and wino and ci % 16 == 0 and co % 16 == 0 else None,
            wn_2T=L(lambda: K.pack_wino_raw(w2, transposed=True) if raw else K.pack_wino(rp['w2T'], co))
            if self.f3d and wino and co % 16 == 0 else None)
        if raw:  # the raw-weight requests of the forms that exist, for _pack's one batched launch
            want = {'wn_1': (w1, None, False), 'wn_2': (w2, wr2.float().contiguous(), False),
                    'wn_1T': (w1, None, True), 'wn_2T': (w2, None, True)}
            rp['_wino_raw'] = {k: v for k, v in want.items() if rp.has(k)}
        return rp

    def _pack_attn(self, blk, i: int):
        mha, gn = blk.attentions[i], blk.attention_norms[i]
        C = mha.embed_dim
        w_in, w_out = mha.in_proj_weight.detach(), mha.out_proj.weight.detach()
        L = _Pack.lazy
        d = _Pack(C=C, heads=mha.num_heads, gn=gn, mha=mha, pk_in=L(lambda: self._pk(w_in, C, 1)),
                  pk_out=L(lambda: self._pk(w_out, C, 1)), pk_inT=L(lambda: self._pk(w_in.t(), 3 * C, 1)),
                  pk_outT=L(lambda: self._pk(w_out.t(), C, 1)), f3_in=None, f3_out=None)
        if self.f3d and C % 16 == 0:  # projection data gradients on f16x3 (per-image absmax bounds)
            d['f3_inT'] = L(lambda: K.pack_f16x3(w_in.t().contiguous().float(), 3 * C, ntaps=1, order='natural'))
            d['f3_outT'] = L(lambda: K.pack_f16x3(w_out.t().contiguous().float(), C, ntaps=1, order='natural'))
        if self.f3 and C % 16 == 0:
            d['f3_in'] = K.pack_f16x3(w_in.float(), C, ntaps=1, order='natural')
            d['f3_out'] = K.pack_f16x3(w_out.float(), C, ntaps=1, order='natural')
            d['qkv_l1'] = self._later(w_in.double().abs().sum(1), vector=True)
            d['qkv_babs'] = self._later(mha.in_proj_bias.detach().double().abs(), vector=True)
            d['gb'] = self._later_absmax(gn.weight, gn.bias)
        return d

    def _later(self, *vals, vector: bool = False):
        """A host value computed on the device now and copied to the host with every other one of
        this forward's packing bounds in ONE transfer (_resolve): one host sync per training forward
        instead of one per GroupNorm / projection bound."""
        slot = _Slot()
        self._pending.append((slot, vals, vector))
        return slot

    def _later_absmax(self, *tensors):
        """A host tuple (max|t| for t in tensors), reduced with every other such request in one
        multi-tensor launch (torch._foreach_norm, inf: exact) and copied with the rest in _resolve."""
        slot = _Slot()
        self._pending_max.append((slot, [t.detach() for t in tensors]))
        return slot

    def _resolve(self, packs):
        """Fill every slot _later / _later_absmax handed out and replace the slots inside the pack dicts."""
        parts = [v.detach().reshape(-1).double() for _, vals, _ in self._pending for v in vals]
        mx = [t for _, ts in self._pending_max for t in ts]
        if mx:
            parts.append(torch.stack(torch._foreach_norm(mx, float('inf'))).double())
        if parts:
            host = torch.cat(parts).cpu()
            i = 0
            for slot, vals, vector in self._pending:
                if vector:
                    n = vals[0].numel()
                    slot.value = host[i:i + n]
                    i += n
                else:
                    slot.value = tuple(float(host[i + j]) for j in range(len(vals)))
                    i += len(vals)
            for slot, ts in self._pending_max:
                slot.value = tuple(float(host[i + j]) for j in range(len(ts)))
                i += len(ts)
        self._pending = []
        self._pending_max = []
        for d in packs:
            for k, v in list(d.items()):
                if isinstance(v, _Slot):
                    d[k] = v.value

    def _pack(self):
        m = self.model
        self.P = 0
        self._pending = []
        self._pending_max = []

        def stage(blk, n_res):
            res = []
            for i in range(n_res):
                rp = self._pack_res(blk, i)
                rp['off'] = self.P
                self.P += rp['co']
                res.append(rp)
            att = [self._pack_attn(blk, i) for i in range(len(blk.attentions))] if blk.use_attn else []
            return res, att

        with torch.no_grad():
            self.downs = [stage(blk, blk.num_layers) for blk in m.downs]
            self.mids = [stage(blk, blk.num_layers + 1) for blk in m.mids]
            self.ups = [stage(blk, blk.num_layers) for blk in m.ups]
            self.down_pk = []
            for blk in m.downs:
                if blk.down_sample:
                    w = blk.down_sample_conv.weight.detach()
                    ci = w.shape[1]
                    L = _Pack.lazy
                    f3 = self.f3 and ci % 16 == 0 and w.shape[0] % 16 == 0 and K.x6_tile(w.shape[0])[1] == 128
                    self.down_pk.append(_Pack(
                        mod=blk.down_sample_conv, pk=L(lambda w=w, ci=ci: self._pk(pack_conv(w), ci, 16)),
                        # dgrad: ConvT of dY (in = Co), its four parity re-layouts built only if used
                        dT=L(lambda w=w: [(taps, self._pk(wp, w.shape[0], len(taps)))
                                          for taps, wp in (pack_convT(w, py, px) for py, px in _PARITIES)]),
                        # f16x3 halo forms: the forward on the space-to-depth kernel, the data gradient (the
                        # ConvT of dY with the same weight) on the one-launch ConvT kernel
                        f3=L(lambda w=w, ci=ci: K.pack_f16x3_s2d(pack_conv(w).float(), ci)) if f3 else None,
                        f3T=L(lambda w=w: K.pack_f16x3_convT(w.float())) if self.f3d and f3 else None))
                else:
                    self.down_pk.append(None)
            self.up_pk = []
            for blk in m.ups:
                if blk.up_sample:
                    wt = blk.up_sample_conv.weight.detach()  # [Cin][Cout][4][4]
                    ci = wt.shape[0]
                    L = _Pack.lazy
                    co = wt.shape[1]
                    f3 = self.f3 and ci % 16 == 0 and co % 16 == 0
                    self.up_pk.append(_Pack(
                        mod=blk.up_sample_conv,
                        fw=L(lambda wt=wt, ci=ci: [(taps, self._pk(wp, ci, len(taps)))
                                                   for taps, wp in (pack_convT(wt, py, px) for py, px in _PARITIES)]),
                        dT=L(lambda wt=wt, co=co: self._pk(pack_conv(wt), co, 16)),
                        f3=L(lambda wt=wt: K.pack_f16x3_convT(wt.float())) if f3 else None,
                        f3T=L(lambda wt=wt, co=co: K.pack_f16x3_s2d(pack_conv(wt).float(), co))
                        if self.f3d and f3 and K.x6_tile(ci)[1] == 128 else None))
                else:
                    self.up_pk.append(None)
            tp = m.t_proj
            self.tproj = [tp[0].weight.detach().float().contiguous(), tp[0].bias.detach().float().contiguous(),
                          tp[2].weight.detach().float().contiguous(), tp[2].bias.detach().float().contiguous()]
            rows = [rp for st in self.downs + self.mids + self.ups for rp in st[0]]
            # every ResBlock's Winograd packs (forward and data-gradient forms; the weights change each
            # step) in one launch instead of one each (WC_PACK_BATCH=0: built lazily one by one)
            if os.environ.get('WC_PACK_BATCH', '1') != '0':
                reqs = [(rp, k, r) for rp in rows for k, r in rp.get('_wino_raw', {}).items()]
                for (rp, k, _), pk in zip(reqs, K.pack_wino_raw_batch([r for _, _, r in reqs])):
                    dict.__setitem__(rp, k, pk)
            self._resolve(rows + [ap for st in self.downs + self.mids + self.ups for ap in st[1]])
            self.temb_w = torch.cat([rp['temb'].weight.detach().float() for rp in rows], 0).contiguous()
            self.temb_b = torch.cat([rp['temb'].bias.detach().float() for rp in rows], 0).contiguous()
            self.res_rows = rows
            co = m.conv_out.weight.detach()  # [NO][C][3][3]
            NO, C = co.shape[0], co.shape[1]
            # the 3-channel head on its fp32 VALU kernels (wc_head_conv forward, wc_head_wgrad /
            # wc_head_dgrad backward): an MFMA tile pads its 3 channels 20x (WC_TRAIN_SMALLCONV=0: the
            # generic implicit GEMMs, kept for A/B)
            self.head_small = K.smallconv_enabled() and NO == 3 and C in (32, 64)
            if self.head_small:
                self.head_wp = K.pack_head(co)
                self.head_T = None
            else:
                self.head_pk = self._pk(pack_conv(co), C, 9)
                wt = torch.zeros((C, 32, 3, 3), dtype=torch.float32, device=self.device)
                wt[:, :NO] = co.flip([2, 3]).transpose(0, 1)
                self.head_T = self._pk(pack_conv(wt), 32, 9)  # dgrad over the 32-channel padded loss gradient

    # ------------------------------------------------------------------ helpers
    def _new(self, B, H, W, C) -> torch.Tensor:
        return torch.empty((B, H, W, C), dtype=torch.float32, device=self.device)

    def _new_gn(self, B, H, W, C) -> torch.Tensor:
        """A forward activation that also carries GroupNorm tile partials (kernels.GnPart), filled by its
        producer's epilogue when that is a split-precision conv, so its GroupNorm needs no stats pass."""
        t = self._new(B, H, W, C)
        sw = UnetEngine._sw(C)
        if sw is not None and K.GnPart.eligible(t) and os.environ.get('WC_TRAIN_GN_PARTIALS', '1') != '0':
            K.GnPart.attach(t, sw)
        return t

    @staticmethod
    def _gn_out(out: View, N: int, H: int, W: int, bm: Optional[int] = None) -> Optional['K.GnPart']:
        """out's tile partials when the conv writing it can emit them from its epilogue, else None
        (bm: the implicit GEMM's M tile)."""
        gp = K.GnPart.of(out)
        return gp if K.gn_conv_ok(out, gp, N, H, W, bm) else None

    def _zrow(self, B: int) -> torch.Tensor:
        """A zeroed float32[B] on the device (a per-image bound that writers raise): rows of one pooled
        zero fill instead of a fill launch each.  A row is never handed out twice."""
        pool = getattr(self, '_zpool', None)
        if pool is None or pool.shape[1] != B or self._zi >= pool.shape[0]:
            self._zpool = pool = torch.zeros((128, B), dtype=torch.float32, device=self.device)
            self._zi = 0
        self._zi += 1
        return pool[self._zi - 1]

    def _gview(self, v: View) -> View:
        """The gradient view of a forward view, allocated on first use but NOT yet zeroed: a gradient
        tensor stays unwritten ('fresh') until its first writer overwrites it whole (_grad_w) or
        something reads or accumulates into it (_grad zeroes it then)."""
        key = id(v.t)
        if key not in self.gmap:
            self.gmap[key] = (torch.empty_like(v.t), 0)
            self.gfresh.add(id(self.gmap[key][0]))
        g, off = self.gmap[key]
        return View(g, v.c0 + off, v.C)

    def _grad(self, v: View) -> View:
        """The gradient view of a forward view, zero-initialised if nothing has written it yet."""
        gv = self._gview(v)
        if id(gv.t) in self.gfresh:
            self.gfresh.discard(id(gv.t))
            gv.t.zero_()
        return gv

    def _grad_w(self, v: View) -> Tuple[View, bool]:
        """(gradient view, overwrite) for a writer that adds into it (a conv's res=, an accumulating GN
        backward): overwrite=True when the tensor is still unwritten and the view covers it whole, so the
        writer stores its values instead of adding them to a zero fill (no fill, no read of zeros)."""
        gv = self._gview(v)
        if id(gv.t) in self.gfresh and gv.c0 == 0 and gv.C == gv.t.shape[-1] \
                and os.environ.get('WC_TRAIN_LAZY_GRAD', '1') != '0':
            self.gfresh.discard(id(gv.t))
            return gv, True
        return self._grad(v), False

    def _alias_grad(self, t: torch.Tensor, v: View):
        """The full tensor t's gradient IS the gradient of view v (t feeds v through an identity path
        and everything else adds into it afterwards in backward order)."""
        g = self._gview(v)
        self.gmap[id(t)] = (g.t, g.c0)
        self.keep.append(t)

    def _gb(self, v: View) -> Optional[torch.Tensor]:
        """The range bound of v's gradient tensor for the f16x3 backward: float32[B], raised by EVERY
        kernel that writes into that tensor to the max |value| it wrote per image (so it bounds the
        final values), zero while nothing has; None outside the f16x3 backward."""
        if not self.f3d:
            return None
        g = self._gview(v)
        t = self.gbnd.get(id(g.t))
        if t is None:
            t = self._zrow(v.B)
            self.gbnd[id(g.t)] = t
        return t

    def _bound(self, v: View, tracked: Optional[torch.Tensor]) -> torch.Tensor:
        """The per-image bound a consumer uses: the writers' tracked bound (WC_CHECK_GBOUND=1: checked
        against a fresh absmax of the view, which it must not be below)."""
        if tracked is None:
            return K.absmax_images(v)
        if os.environ.get('WC_CHECK_GBOUND', '0') == '1':
            real = K.absmax_images(v)
            if bool((real > tracked).any()):
                raise RuntimeError(f'gradient range bound below the values: {tracked.tolist()} < {real.tolist()}')
        return tracked

    def _pgrad(self, p: torch.nn.Parameter) -> torch.Tensor:
        """p's gradient: a view into one zeroed buffer holding every parameter's (one fill per backward
        instead of one per parameter)."""
        g = self.pgrads.get(id(p))
        if g is None:
            o, n = self.pflat_off[id(p)]
            g = self.pflat[o:o + n].view(p.shape)
            self.pgrads[id(p)] = g
        return g

    # ------------------------------------------------------------------ forward
    def forward(self, x: torch.Tensor, t) -> torch.Tensor:
        with K._native.variant(self.variant):
            return self._forward(x, t)

    def _forward(self, x: torch.Tensor, t) -> torch.Tensor:
        m = self.model
        mc = m.model_config
        self._pack()
        self.tape = []
        x = x.to(device=self.device, dtype=torch.float32).contiguous()
        B, _, S, S2 = x.shape
        tt = torch.as_tensor(t).long().reshape(-1).to(self.device)
        if tt.numel() == 1 and B > 1:
            tt = tt.expand(B).contiguous()
        if tt.numel() != B:
            raise RuntimeError(f'timestep tensor has {tt.numel()} entries for a batch of {B}')
        self.tt = tt
        self._raised: Dict[int, bool] = {}
        temb = K.temb(tt, *self.tproj, self.temb_w, self.temb_b)  # (B, P)
        self.x = x
        dc = m.down_channels
        L = len(dc) - 1
        sizes = [(S, S2)]
        for i in range(L):
            h, w = sizes[-1]
            sizes.append((h // 2, w // 2) if m.down_sample[i] else (h, w))
        U = [self._new(B, sizes[i][0], sizes[i][1], 2 * dc[i]) for i in range(L)]
        self.U = U
        cur = View(U[0], dc[0], dc[0])
        K.conv_in(x, m.conv_in.weight.detach().float().contiguous(), m.conv_in.bias.detach().float().contiguous(), cur)
        self.tape.append(('conv_in', cur))

        def block(X: View, tgt: View, rp, att, amx=None) -> View:
            """amx: float32[B] the final writer of tgt raises to its per-image max |value| (the bound a
            following down / up conv needs); left zero when that writer is not an f16x3 kernel."""
            if att is None:
                self._res_fwd(X, tgt, rp, temb, amx)
            else:
                ypre = View.full(self._new_gn(B, X.H, X.W, rp['co']))
                self._res_fwd(X, ypre, rp, temb)
                self._attn_fwd(ypre, tgt, att, amx)
            return tgt

        def new_amx():
            return self._zrow(B) if (self.f3 or self.f3d) else None

        def bound_of(v: View, amx):
            """The producer-raised bound when it was raised (nonzero), else a pass over v."""
            if amx is None:
                return None
            return amx if self._raised.pop(id(amx), False) else K.absmax_images(v)

        for i in range(L):
            res, att = self.downs[i]
            H, W = sizes[i]
            final = View(U[i + 1], dc[i + 1], dc[i + 1]) if i < L - 1 else View.full(
                self._new(B, sizes[i + 1][0], sizes[i + 1][1], dc[i + 1]))
            amx = new_amx() if self.down_pk[i] is not None else None
            for li, rp in enumerate(res):
                last = li == len(res) - 1
                tgt = final if (last and self.down_pk[i] is None) else View.full(self._new_gn(B, H, W, rp['co']))
                cur = block(cur, tgt, rp, att[li] if att else None, amx if last else None)
            if self.down_pk[i] is not None:
                dp = self.down_pk[i]
                seg = Seg(cur, TAPS4S2, stride=2)
                bd = dp['mod'].bias.detach().float().contiguous()
                Hm, Wm = sizes[i + 1]
                f3 = dp['f3'] is not None and K.conv4x4s2_f16x3_ok(seg, final.C, Hm, Wm)
                bcur = bound_of(cur, amx)  # the conv's A bound and the weight gradient's
                if f3:
                    K.conv4x4s2_f16x3(seg, dp['f3'], bd, final, Hm=Hm, Wm=Wm, a_bound=bcur)
                else:
                    self._conv([seg], dp['pk'], bd, final, Hm, Wm)
                self.tape.append(('down', cur, final, dp, bcur))
                cur = final

        amx = None
        for j, (res, att) in enumerate(self.mids):
            last_mid = j == len(self.mids) - 1
            H, W = cur.H, cur.W
            for li, rp in enumerate(res):
                last = last_mid and li == len(res) - 1
                if last and self.up_pk[0] is None:
                    tgt = View(U[L - 1], 0, dc[L - 1])
                else:
                    tgt = View.full(self._new_gn(B, H, W, rp['co']))
                if last and self.up_pk[0] is not None:
                    amx = new_amx()
                self._res_fwd(cur, tgt, rp, temb, amx if last and li >= len(att) else None)
                cur = tgt
                if li < len(att):
                    nxt = View.full(self._new_gn(B, H, W, rp['co']))
                    self._attn_fwd(cur, nxt, att[li], amx if last else None)
                    cur = nxt

        for k, (res, att) in enumerate(self.ups):
            i = L - 1 - k
            H, W = sizes[i]
            if self.up_pk[k] is not None:
                up = self.up_pk[k]
                dst = View(U[i], 0, dc[i])
                b = up['mod'].bias.detach().float().contiguous()
                f3 = up['f3'] is not None and K.convT4x4s2_f16x3_ok(Seg(cur, [(0, 0)]), dst.C)
                bcur = bound_of(cur, amx)
                if f3:
                    K.convT4x4s2_f16x3(Seg(cur, [(0, 0)]), up['f3'], b, dst, a_bound=bcur)
                else:
                    for (py, px), (taps, pk) in zip(_PARITIES, up['fw']):
                        self._conv([Seg(cur, taps)], pk, b, dst, cur.H, cur.W, out_map=(2, 2, py, px))
                self.tape.append(('up', cur, dst, up, bcur))
            else:
                assert cur.t is U[i] and cur.c0 == 0, 'non-upsampling level must have been written in place'
            cur = View.full(U[i])
            next_in_place = i > 0 and self.up_pk[k + 1] is None
            amx = new_amx() if k + 1 < len(self.ups) and self.up_pk[k + 1] is not None else None
            for li, rp in enumerate(res):
                last = li == len(res) - 1
                tgt = View(U[i - 1], 0, dc[i - 1]) if (last and next_in_place) else View.full(
                    self._new_gn(B, H, W, rp['co']))
                cur = block(cur, tgt, rp, att[li] if att else None, amx if last else None)

        # head: GN -> SiLU -> conv_out, NCHW output
        gn = m.norm_out
        sc, sh, a0, o0 = K.gn_stats_pair(cur, gn.weight.detach().float(), gn.bias.detach().float(),
                                         part=getattr(cur, '_wc_gn_done', None))
        out = torch.empty((B, mc.im_channels, S, S2), dtype=torch.float32, device=self.device)
        if self.head_small:
            K.head_conv(cur, sc, sh, self.head_wp, m.conv_out.bias.detach().float().contiguous(), out)
        else:
            self._conv([Seg(cur, TAPS3, scale=sc, shift=sh, silu=True)], self.head_pk,
                       m.conv_out.bias.detach().float().contiguous(), None, S, S2, out_nchw=out)
        self.tape.append(('head', cur, (sc, sh, a0, o0)))
        self.last_tape = Tape(self)
        self.tape = []
        return out

    def _res_fwd(self, X: View, Y: View, rp, temb: torch.Tensor, amx: Optional[torch.Tensor] = None):
        B, H, W = X.B, X.H, X.W
        g1, g2 = rp['gn1'], rp['gn2']
        co = rp['co']
        st1 = K.gn_stats_pair(X, g1.weight.detach().float(), g1.bias.detach().float(), bound=True,
                              part=getattr(X, '_wc_gn_done', None))
        h = View.full(self._new_gn(B, H, W, co))
        seg1 = [Seg(X, TAPS3, scale=st1[0], shift=st1[1], silu=True)]
        b1 = rp['conv1'].bias.detach().float().contiguous()
        gp1 = None  # h's GroupNorm partials, when conv1's epilogue wrote them
        if rp.has('wn_1') and K.wino_eligible(seg1, co, H, W):
            gp1 = self._gn_out(h, co, H, W)
            K.conv3x3_wino(seg1, rp['wn_1'], b1, h, Hm=H, Wm=W, a_exp=K.f16x3_a_exp(*rp['gb1'], H * W * X.C // 8),
                           temb=temb[:, rp['off']:], temb_ld=temb.shape[1], gn=gp1)
        elif rp.has('f3_1') and K.x6_eligible(seg1, co, H, W):
            gp1 = self._gn_out(h, co, H, W)
            K.conv3x3_f16x3(seg1, rp['f3_1'], b1, h, Hm=H, Wm=W,
                            a_exp=K.f16x3_a_exp(*rp['gb1'], H * W * X.C // 8), temb=temb[:, rp['off']:],
                            temb_ld=temb.shape[1], gn=gp1)
        else:
            self._conv(seg1, rp['pk1'], b1, h, H, W, temb=temb[:, rp['off']:], temb_ld=temb.shape[1])
        st2 = K.gn_stats_pair(h, g2.weight.detach().float(), g2.bias.detach().float(), part=gp1)
        seg2 = [Seg(h, TAPS3, scale=st2[0], shift=st2[1], silu=True), Seg(X, TAPS1, kbase=9 * co)]
        gp2 = None  # Y's partials (an attention block's input): the next GroupNorm's statistics
        if rp.has('wn_2') and K.wino_eligible(seg2, co, H, W):
            gp2 = self._gn_out(Y, co, H, W)
            K.conv3x3_wino(seg2, rp['wn_2'], rp['b2'], Y, Hm=H, Wm=W, a_exp=K.f16x3_a_exp(*rp['gb2'], H * W * co // 8),
                           a_bound=st1[4], absmax=amx, gn=gp2)
            if amx is not None:
                self._raised[id(amx)] = True
        elif rp.has('f3_2') and K.x6_eligible(seg2, co, H, W):
            # the residual segment (raw X) in fp16 under GN1's per-image bound of |X|
            gp2 = self._gn_out(Y, co, H, W)
            K.conv3x3_f16x3(seg2, rp['f3_2'], rp['b2'], Y, Hm=H, Wm=W, a_exp=K.f16x3_a_exp(*rp['gb2'], H * W * co // 8),
                            a_bound=st1[4], absmax=amx, gn=gp2)
            if amx is not None:
                self._raised[id(amx)] = True
        else:
            self._conv(seg2, rp['pk2'], rp['b2'], Y, H, W)
        if gp2 is not None:
            Y._wc_gn_done = gp2
        self.tape.append(('res', X, h, Y, rp, st1[:4], st2, st1[4]))

    def _attn_fwd(self, Ypre: View, Yout: View, ap, amx: Optional[torch.Tensor] = None):
        B, H, W, C = Ypre.B, Ypre.H, Ypre.W, Ypre.C
        N = H * W
        gn, mha = ap['gn'], ap['mha']
        st = K.gn_stats_pair(Ypre, gn.weight.detach().float(), gn.bias.detach().float(),
                             part=getattr(Ypre, '_wc_gn_done', None))
        qkv = self._new(B, H, W, 3 * C)
        seg = [Seg(Ypre, TAPS1, scale=st[0], shift=st[1], silu=False)]
        b_in = mha.in_proj_bias.detach().float().contiguous()
        o = self._new(B, H, W, C)
        lse = torch.empty((B, ap['heads'], N), dtype=torch.float32, device=self.device)
        b_out = mha.out_proj.bias.detach().float().contiguous()
        if ap['f3_in'] is not None:
            # in_proj under the GN bound; attention on f16x3 under the in-projection row-norm bounds
            # of Q, K, V (as the sampler); out_proj: |O| <= max|V| (a convex combination of V rows)
            ng = N * C // 8
            K.conv_igemm_f16x3(seg, ap['f3_in'], b_in, View.full(qkv), Hm=H, Wm=W, a_exp=K.f16x3_a_exp(*ap['gb'], ng))
            exps = K.attention_exps_from_norms(ap['qkv_l1'], ap['qkv_babs'], ap['gb'][0], ap['gb'][1], ng)
            K.attention_fwd_lse(qkv.view(B * N, 3 * C), o.view(B * N, C), lse, B, N, C, ap['heads'],
                                precision='f16x3', exps=exps)
            gpo = self._gn_out(Yout, C, H, W, 256 if C <= 64 else 128)
            K.conv_igemm_f16x3([Seg(View.full(o), TAPS1)], ap['f3_out'], b_out, Yout, Hm=H, Wm=W, a_exp=exps[2],
                               res=Ypre, absmax=amx, gn=gpo)
            if amx is not None:
                self._raised[id(amx)] = True
            if gpo is not None:
                Yout._wc_gn_done = gpo
        else:
            self._conv(seg, ap['pk_in'], b_in, View.full(qkv), H, W)
            K.attention_fwd_lse(qkv.view(B * N, 3 * C), o.view(B * N, C), lse, B, N, C, ap['heads'],
                                precision=self.precision)
            self._conv([Seg(View.full(o), TAPS1)], ap['pk_out'], b_out, Yout, H, W, res=Ypre)
        self.tape.append(('attn', Ypre, Yout, qkv, o, lse, st, ap))

    # ------------------------------------------------------------------ backward
    def backward(self, gout: torch.Tensor, tape: Optional[Tape] = None) -> Dict[int, torch.Tensor]:
        """Gradients of every parameter (see _backward), on this engine's library variant."""
        with K._native.variant(self.variant):
            return self._backward(gout, tape)

    def _backward(self, gout: torch.Tensor, tape: Optional[Tape] = None) -> Dict[int, torch.Tensor]:
        """Gradients of every parameter given d loss / d output (B, C, S, S) for the forward that
        recorded ``tape`` (default: the latest forward); returns {id(param): grad}.  A tape is
        consumed (its activations freed) by its backward: a second backward through it raises."""
        tape = tape if tape is not None else self.last_tape
        if tape is None or tape.consumed:
            raise RuntimeError('Unet training backward: this forward\'s saved activations were already consumed '
                               'by an earlier backward (retain_graph / a second backward is not supported)')
        for f in Tape._FIELDS[1:]:
            setattr(self, f, getattr(tape, f))
        records = tape.records
        tape.consumed = True
        tape.records = []
        if self.last_tape is tape:
            self.last_tape = None
        m = self.model
        self.gmap: Dict[int, Tuple[torch.Tensor, int]] = {}
        self.gfresh = set()  # gradient tensors allocated but not yet written (_gview)
        self.gbnd: Dict[int, torch.Tensor] = {}
        self.pgrads: Dict[int, torch.Tensor] = {}
        self.pflat_off: Dict[int, Tuple[int, int]] = {}
        tot = 0
        for prm in m.parameters():
            self.pflat_off[id(prm)] = (tot, prm.numel())
            tot += (prm.numel() + 63) // 64 * 64  # 256-byte aligned views
        self.pflat = torch.zeros(tot, dtype=torch.float32, device=self.device)
        self.keep = []
        B = gout.shape[0]
        self.dproj = torch.zeros((B, self.P), dtype=torch.float32, device=self.device)
        gout = gout.to(self.device, torch.float32).contiguous()
        K.bsum_defer()  # the ~200 per-layer dgamma / dbeta / bias sums go out in one launch at the end
        try:
            for rec in reversed(records):
                getattr(self, '_bwd_' + rec[0])(rec, gout)
            del records
            self._temb_bwd()
        finally:
            K.bsum_flush()
        self.gmap = {}
        self.gfresh = set()
        self.gbnd = {}
        self.keep = []
        for f in Tape._FIELDS[1:]:  # the tape's tensors die with it, not with the engine
            setattr(self, f, None)
        grads, self.pgrads, self.pflat = self.pgrads, {}, None
        return grads

    @staticmethod
    def _dgrad3_ok(g: View, n_out: int) -> bool:
        """The 3x3 data gradient of g (n_out output channels) fits the halo f16x3 kernel."""
        return K.x6_eligible([Seg(g, TAPS3)], n_out, g.H, g.W) and g.C % 4 == 0 and g.ldc % 4 == 0 \
            and g.ptr % 16 == 0

    def _wgrad(self, g: View, segs, dw0, s0, f3=None, **kw):
        """Weight gradient on bf16x6 (precision bf16x6) or fp32 MFMA; f3 = (x_exp, per-image max |g|):
        the 3x3 halo kernel on f16x3 (mode f16x3)."""
        K.conv_wgrad(g, segs, dw0, s0, x6=self.precision == 'bf16x6', f3=f3 if self.f3d else None, **kw)

    def _bias_grad(self, g: View, *params):
        sums = K.channel_sums(g)
        for p in params:
            K.bsum(sums, 0, self._pgrad(p), accumulate=True)
        return sums

    def _bwd_head(self, rec, gout):
        m = self.model
        _, cur, (sc, sh, a0, o0) = rec
        B, NO, S, S2 = gout.shape
        C = cur.C
        if self.head_small:
            g = gout.contiguous().float()
            K.head_wgrad(cur, sc, sh, g, self._pgrad(m.conv_out.weight))
            self._pgrad(m.conv_out.bias).copy_(g.sum((0, 2, 3)))
            dz = View.full(self._new(B, S, S2, C))
            K.head_dgrad(g, m.conv_out.weight, dz)
            gn = m.norm_out
            gcur, ow = self._grad_w(cur)
            K.gn_backward(dz, cur, a0, o0, gn.weight.detach().float(), gn.bias.detach().float(), True, gcur,
                          dgamma=self._pgrad(gn.weight), dbeta=self._pgrad(gn.bias), accumulate=not ow,
                          absmax=self._gb(cur))
            return
        g32 = K.nchw_to_nhwc(gout, 32)
        g4 = View(g32, 0, 4)
        wtmp = torch.zeros((4, C, 3, 3), dtype=torch.float32, device=self.device)
        self._wgrad(g4, [Seg(cur, TAPS3, scale=sc, shift=sh, silu=True)], wtmp, (C * 9, 9, 1))
        self._pgrad(m.conv_out.weight).copy_(wtmp[:NO])
        btmp = torch.zeros(4, dtype=torch.float32, device=self.device)
        K.bsum(K.channel_sums(g4), 0, btmp, now=True)  # read by the copy below
        self._pgrad(m.conv_out.bias).copy_(btmp[:NO])
        dz = View.full(self._new(B, S, S2, C))
        self._conv([Seg(View.full(g32), TAPS3)], self.head_T, None, dz, S, S2)
        gn = m.norm_out
        gcur, ow = self._grad_w(cur)
        K.gn_backward(dz, cur, a0, o0, gn.weight.detach().float(), gn.bias.detach().float(), True, gcur,
                      dgamma=self._pgrad(gn.weight), dbeta=self._pgrad(gn.bias), accumulate=not ow,
                      absmax=self._gb(cur))

    def _bwd_res(self, rec, gout):
        _, X, h, Y, rp, st1, st2, bXf = rec  # bXf: GN1's per-image bound of |X| (the forward's)
        B, H, W = X.B, X.H, X.W
        ci, co = rp['ci'], rp['co']
        gY = self._grad(Y)
        gX = self._gview(X)  # written first by the residual conv's data gradient below
        self._bias_grad(gY, rp['conv2'].bias, rp['resc'].bias)
        # per-image max |gY|: the range bound of the f16x3 data gradients and weight gradient
        f3Y = rp.has('f3_2T') and self._dgrad3_ok(gY, co)
        bY = self._bound(gY, self._gb(Y)) if f3Y else None
        bX = self._gb(X)
        self._wgrad(gY, [Seg(h, TAPS3, scale=st2[0], shift=st2[1], silu=True), Seg(X, TAPS1, kbase=9 * co)],
                    self._pgrad(rp['conv2'].weight), (co * 9, 9, 1), dw1=self._pgrad(rp['resc'].weight), s1=ci,
                    f3=K.F3Bounds(bY, K.f16x3_a_exp(*rp['gb2'], H * W * co // 8), None, bXf) if f3Y else None)
        dz2 = View.full(self._new(B, H, W, co))
        g2 = rp['gn2']
        ga2, be2 = g2.weight.detach().float(), g2.bias.detach().float()
        # dh's per-(image, channel) sums (conv1's bias / time-embedding gradients) in closed form from the
        # GN backward's own sums (WC_TRAIN_DH_SUMS=0: a channel_sums pass over dh)
        dh_sums = os.environ.get('WC_TRAIN_DH_SUMS', '1') != '0'
        pre2 = None
        if f3Y:
            if rp.has('wn_2T') and K.wino_eligible([Seg(gY, TAPS3)], co, H, W):
                # GN2's backward sums of dz2 formed in the data-gradient conv's epilogue (no pass over dz2)
                if K.gnb_epilogue_enabled():
                    pre2 = K.GnbSums.make(h, st2[2], st2[3], ga2, be2, True, dx_sums=dh_sums)
                K.conv3x3_wino([Seg(gY, TAPS3)], rp['wn_2T'], None, dz2, Hm=H, Wm=W, a_exp=60, a_bound=bY, gnb=pre2)
            else:
                K.conv3x3_f16x3([Seg(gY, TAPS3)], rp['f3_2T'], None, dz2, Hm=H, Wm=W, a_exp=60, a_bound=bY)
            gX, ow = self._grad_w(X)
            rX = None if ow else gX
            if (H * W) % (256 if ci <= 64 else 128) == 0 and co % 16 == 0:  # one-image M tiles (per-image bound)
                K.conv_igemm_f16x3([Seg(gY, TAPS1)], rp['f3_rT'], None, gX, Hm=H, Wm=W, a_exp=60, a_bound=bY, res=rX,
                                   absmax=bX)
            else:
                self._conv([Seg(gY, TAPS1)], rp['pkrT'], None, gX, H, W, res=rX, absmax=bX)
        else:
            self._conv([Seg(gY, TAPS3)], rp['pk2T'], None, dz2, H, W)
            gX, ow = self._grad_w(X)
            self._conv([Seg(gY, TAPS1)], rp['pkrT'], None, gX, H, W, res=None if ow else gX, absmax=bX)
        dh = View.full(self._new(B, H, W, co))
        bdh = self._zrow(B) if self.f3d else None
        sums = K.gn_backward(dz2, h, st2[2], st2[3], ga2, be2, True, dh, dgamma=self._pgrad(g2.weight),
                             dbeta=self._pgrad(g2.bias), accumulate=False, absmax=bdh, dx_sums=dh_sums, pre=pre2)
        if sums is None:
            sums = K.channel_sums(dh)
        K.bsum(sums, 0, self._pgrad(rp['conv1'].bias), accumulate=True)
        self.dproj[:, rp['off']:rp['off'] + co].copy_(sums[:, :, 0])
        f3h = rp.has('f3_1T') and self._dgrad3_ok(dh, ci)
        bh = self._bound(dh, bdh) if f3h else None
        self._wgrad(dh, [Seg(X, TAPS3, scale=st1[0], shift=st1[1], silu=True)], self._pgrad(rp['conv1'].weight),
                    (ci * 9, 9, 1), f3=K.F3Bounds(bh, K.f16x3_a_exp(*rp['gb1'], H * W * ci // 8)) if f3h else None)
        dz1 = View.full(self._new(B, H, W, ci))
        g1 = rp['gn1']
        ga1, be1 = g1.weight.detach().float(), g1.bias.detach().float()
        pre1 = None
        if f3h:
            if rp.has('wn_1T') and K.wino_eligible([Seg(dh, TAPS3)], ci, H, W):
                if K.gnb_epilogue_enabled():
                    pre1 = K.GnbSums.make(X, st1[2], st1[3], ga1, be1, True)
                K.conv3x3_wino([Seg(dh, TAPS3)], rp['wn_1T'], None, dz1, Hm=H, Wm=W, a_exp=60, a_bound=bh, gnb=pre1)
            else:
                K.conv3x3_f16x3([Seg(dh, TAPS3)], rp['f3_1T'], None, dz1, Hm=H, Wm=W, a_exp=60, a_bound=bh)
        else:
            self._conv([Seg(dh, TAPS3)], rp['pk1T'], None, dz1, H, W)
        K.gn_backward(dz1, X, st1[2], st1[3], ga1, be1, True, gX, dgamma=self._pgrad(g1.weight),
                      dbeta=self._pgrad(g1.bias), accumulate=True, absmax=bX, pre=pre1)

    def _bwd_attn(self, rec, gout):
        _, Ypre, Yout, qkv, o, lse, st, ap = rec
        B, H, W, C = Ypre.B, Ypre.H, Ypre.W, Ypre.C
        N = H * W
        mha, gn = ap['mha'], ap['gn']
        gY = self._grad(Yout)
        self._bias_grad(gY, mha.out_proj.bias)
        f3a = self.f3d and ap['f3_in'] is not None
        # the forward's Q / K / V exponents (|O| <= max|V|: O shares V's)
        exps = K.attention_exps_from_norms(ap['qkv_l1'], ap['qkv_babs'], ap['gb'][0], ap['gb'][1], N * C // 8) \
            if f3a else None
        bgY = self._bound(gY, self._gb(Yout)) if self.f3d else None
        self._wgrad(gY, [Seg(View.full(o), TAPS1)], self._pgrad(mha.out_proj.weight), (C, 1, 0),
                    f3=K.F3Bounds(bgY, exps[2]) if f3a else None)
        do = self._new(B, H, W, C)
        bdo = self._zrow(B) if self.f3d else None
        f3p = 'f3_outT' in ap and (H * W) % (256 if C <= 64 else 128) == 0
        if f3p:
            K.conv_igemm_f16x3([Seg(gY, TAPS1)], ap['f3_outT'], None, View.full(do), Hm=H, Wm=W, a_exp=60,
                               a_bound=bgY, absmax=bdo)
        else:
            self._conv([Seg(gY, TAPS1)], ap['pk_outT'], None, View.full(do), H, W, absmax=bdo)
        dqkv = self._new(B, H, W, 3 * C)
        bgq = None
        if f3a:
            # f16x3 under the forward's Q / K / V exponents and the per-image max |dO|; the kernels raise
            # the per-image max |dqkv| as they write it (head dims 32 / 64 / 128)
            bgq = self._zrow(B)
            if not K.attention_bwd(qkv.view(B * N, 3 * C), o.view(B * N, C), do.view(B * N, C), lse,
                                   dqkv.view(B * N, 3 * C), B, N, C, ap['heads'], precision='f16x3', exps=exps,
                                   dout_bound=self._bound(View.full(do), bdo), dqkv_absmax=bgq):
                bgq = None
        else:
            K.attention_bwd(qkv.view(B * N, 3 * C), o.view(B * N, C), do.view(B * N, C), lse, dqkv.view(B * N, 3 * C),
                            B, N, C, ap['heads'], precision=self.precision)
        gq = View.full(dqkv)
        self._bias_grad(gq, mha.in_proj_bias)
        if f3a or f3p:
            bgq = self._bound(gq, bgq) if bgq is not None else K.absmax_images(gq)
        self._wgrad(gq, [Seg(Ypre, TAPS1, scale=st[0], shift=st[1], silu=False)], self._pgrad(mha.in_proj_weight),
                    (C, 1, 0), f3=K.F3Bounds(bgq, K.f16x3_a_exp(*ap['gb'], N * C // 8)) if f3a else None)
        da = View.full(self._new(B, H, W, C))
        if f3p:
            K.conv_igemm_f16x3([Seg(gq, TAPS1)], ap['f3_inT'], None, da, Hm=H, Wm=W, a_exp=60, a_bound=bgq)
        else:
            self._conv([Seg(gq, TAPS1)], ap['pk_inT'], None, da, H, W)
        # Yout = Ypre + out_proj(...): Ypre's gradient is Yout's plus the GroupNorm path
        self._alias_grad(Ypre.t, Yout)
        K.gn_backward(da, Ypre, st[2], st[3], gn.weight.detach().float(), gn.bias.detach().float(), False,
                      self._grad(Ypre), dgamma=self._pgrad(gn.weight), dbeta=self._pgrad(gn.bias), accumulate=True,
                      absmax=self._gb(Ypre))

    def _bwd_down(self, rec, gout):
        _, cur, final, dp, bcur = rec  # bcur: the forward's per-image max |cur|
        gF = self._grad(final)
        w = dp['mod'].weight
        self._bias_grad(gF, dp['mod'].bias)
        bgF = self._bound(gF, self._gb(final)) if self.f3d else None
        self._wgrad(gF, [Seg(cur, TAPS4S2, stride=2)], self._pgrad(w), (w.shape[1] * 16, 16, 1),
                    f3=K.F3Bounds(bgF, 60, bcur) if bgF is not None and bcur is not None else None)
        gc, ow = self._grad_w(cur)  # the four output parities together cover every pixel
        rc = None if ow else gc
        if dp['f3T'] is not None and K.convT4x4s2_f16x3_ok(Seg(gF, [(0, 0)]), gc.C) and gF.ptr % 16 == 0:
            # the ConvT of dY (same weight) in one launch on f16x3 under dY's tracked bound
            K.convT4x4s2_f16x3(Seg(gF, [(0, 0)]), dp['f3T'], None, gc, a_bound=bgF, res=rc, absmax=self._gb(cur))
            return
        for (py, px), (taps, pk) in zip(_PARITIES, dp['dT']):
            self._conv([Seg(gF, taps)], pk, None, gc, gF.H, gF.W, out_map=(2, 2, py, px), res=rc, absmax=self._gb(cur))

    def _bwd_up(self, rec, gout):
        _, cur, dst, up, bcur = rec
        gD = self._grad(dst)
        wt = up['mod'].weight  # [Cin][Cout][4][4]
        self._bias_grad(gD, up['mod'].bias)
        # dW[ci][co][ky][kx] = sum_pixels x[ci] * dY[co] at (2y - 1 + ky, 2x - 1 + kx): the 4x4/s2 tap
        # grid over dY with x in the gradient role
        bgD = self._bound(gD, self._gb(dst)) if self.f3d else None
        self._wgrad(cur, [Seg(gD, TAPS4S2, stride=2)], self._pgrad(wt), (wt.shape[1] * 16, 16, 1),
                    f3=K.F3Bounds(bcur, 60, bgD) if bgD is not None and bcur is not None else None)
        seg = Seg(gD, TAPS4S2, stride=2)
        gc, ow = self._grad_w(cur)
        rc = None if ow else gc
        if up['f3T'] is not None and K.conv4x4s2_f16x3_ok(seg, gc.C, cur.H, cur.W) and gD.ptr % 16 == 0:
            # the 4x4/s2 conv of dY on the space-to-depth halo kernel, f16x3 under dY's tracked bound
            K.conv4x4s2_f16x3(seg, up['f3T'], None, gc, Hm=cur.H, Wm=cur.W, a_bound=bgD, res=rc, absmax=self._gb(cur))
            return
        self._conv([seg], up['dT'], None, gc, cur.H, cur.W, res=rc, absmax=self._gb(cur))

    def _bwd_conv_in(self, rec, gout):
        m = self.model
        _, cur = rec
        g = self._grad(cur)
        self._bias_grad(g, m.conv_in.bias)
        w = m.conv_in.weight
        if K.smallconv_enabled() and w.shape[1] == 3 and g.C in (32, 64) and self.x.is_contiguous():
            K.stem_wgrad(self.x, g, self._pgrad(w))  # fp32 VALU, the 3 input channels unpadded
            return
        xn = K.nchw_to_nhwc(self.x, 4)
        self._wgrad(g, [Seg(View.full(xn), TAPS3)], self._pgrad(w), (w.shape[1] * 9, 9, 1), Cw=w.shape[1])

    def _temb_bwd(self):
        """t_proj (Linear, SiLU, Linear) and the t_emb_layers (SiLU, Linear) backward (B x 128)."""
        m = self.model
        w1, b1, w2, b2 = self.tproj
        D = w1.shape[0]
        B, P = self.dproj.shape
        e = K.time_embedding(self.tt, D)
        a1 = b1.expand(B, D).contiguous()
        K.gemm_small(B, D, D, e, (D, 1), w1, (1, D), a1, D, beta=1.0)
        h1 = K.silu_map(a1)
        a2 = b2.expand(B, D).contiguous()
        K.gemm_small(B, D, D, h1, (D, 1), w2, (1, D), a2, D, beta=1.0)
        s = K.silu_map(a2)
        dp = self.dproj
        for rp in self.res_rows:
            off, co = rp['off'], rp['co']
            lin = rp['temb']
            K.gemm_small(co, D, B, dp, (1, P), s, (D, 1), self._pgrad(lin.weight), D, offs=(off, 0, 0))
            K.colsum(dp, self._pgrad(lin.bias), col0=off, ncol=co)
        ds = torch.empty((B, D), dtype=torch.float32, device=self.device)
        K.gemm_small(B, D, P, dp, (P, 1), self.temb_w, (D, 1), ds, D)
        da2 = K.silu_map(a2, ds)
        tp = m.t_proj
        K.gemm_small(D, D, B, da2, (1, D), h1, (D, 1), self._pgrad(tp[2].weight), D)
        K.colsum(da2, self._pgrad(tp[2].bias))
        dh1 = torch.empty((B, D), dtype=torch.float32, device=self.device)
        K.gemm_small(B, D, D, da2, (D, 1), w2, (D, 1), dh1, D)
        da1 = K.silu_map(a1, dh1)
        K.gemm_small(D, D, B, da1, (1, D), e, (D, 1), self._pgrad(tp[0].weight), D)
        K.colsum(da1, self._pgrad(tp[0].bias))


class UnetTrainFunction(torch.autograd.Function):
    """Unet.forward in training mode: the HIP forward records its tape, and autograd's backward runs
    TrainEngine.backward, returning one gradient per parameter (so the reference's own
    ``loss.backward(); optimizer.step()`` loop works unchanged)."""

    @staticmethod
    def forward(ctx, engine: TrainEngine, x: torch.Tensor, t, *params):
        if x.requires_grad:
            raise RuntimeError('Unet training forward: the gradient w.r.t. the input image is not computed; '
                               'pass a tensor that does not require grad (x.detach())')
        with torch.no_grad():
            out = engine.forward(x, t)
        ctx.engine = engine
        ctx.tape = engine.last_tape  # this forward's own saved state (gradient accumulation safe)
        engine.last_tape = None
        ctx.param_ids = [id(p) for p in engine.model.parameters()]
        # the backward builds its data-gradient weight packs lazily from the live parameters: saving
        # them makes autograd's version check raise if one is modified in place (an optimizer / EMA
        # step) between this forward and its backward, instead of mixing old and new weights
        ctx.save_for_backward(*params)
        return out

    @staticmethod
    def backward(ctx, gout):
        ctx.saved_tensors  # noqa: B018  (raises if a parameter changed in place since the forward)
        grads = ctx.engine.backward(gout, ctx.tape)
        ctx.tape = None
        # hand autograd the only references, so it can take each gradient as param.grad instead of
        # copying it
        out = tuple(grads.pop(i, None) for i in ctx.param_ids)
        del grads
        return (None, None, None) + out

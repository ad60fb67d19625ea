"""ORACLE (test infrastructure only) — functional PyTorch-CPU restatement of the reference DDPM UNet.

Follows ``/root/reference/diffusion_model/models/unet_base.py`` op for op, reading parameters by
their state_dict key:
  get_time_embedding      unet_base.py:7-30
  ResBlock                unet_base.py:146-150 (Down), 242-246/262-266 (Mid), 353-357 (Up)
  attention block         unet_base.py:153-161 / 250-259 / 359-367  (nn.MultiheadAttention math)
  Unet.__init__ layout    unet_base.py:378-449 (attention placement rule :404-405, :434-435)
  Unet.forward            unet_base.py:451-488
Pinned against the reference import by tests/golden (tests/test_oracle_golden.py).
"""
from typing import Dict, List

import torch
import torch.nn.functional as F

EPS = 1e-5


def time_embedding(t: torch.Tensor, dim: int) -> torch.Tensor:  # unet_base.py:7-30
    half = dim // 2
    factor = 10000**(torch.arange(0, half, dtype=torch.float32) / half)
    arg = t.reshape(-1)[:, None].repeat(1, half) / factor
    return torch.cat([torch.sin(arg), torch.cos(arg)], dim=-1)


def _resblock(sd: Dict[str, torch.Tensor], pfx: str, i: int, x: torch.Tensor, temb: torch.Tensor) -> torch.Tensor:
    g = lambda name: sd[f'{pfx}.{name}']  # noqa: E731
    h = F.group_norm(x, 8, g(f'resnet_conv_first.{i}.0.weight'), g(f'resnet_conv_first.{i}.0.bias'), EPS)
    h = F.conv2d(F.silu(h), g(f'resnet_conv_first.{i}.2.weight'), g(f'resnet_conv_first.{i}.2.bias'), padding=1)
    te = F.linear(F.silu(temb), g(f't_emb_layers.{i}.1.weight'), g(f't_emb_layers.{i}.1.bias'))
    h = h + te[:, :, None, None]
    h2 = F.group_norm(h, 8, g(f'resnet_conv_second.{i}.0.weight'), g(f'resnet_conv_second.{i}.0.bias'), EPS)
    h2 = F.conv2d(F.silu(h2), g(f'resnet_conv_second.{i}.2.weight'), g(f'resnet_conv_second.{i}.2.bias'), padding=1)
    return h2 + F.conv2d(x, g(f'residual_input_conv.{i}.weight'), g(f'residual_input_conv.{i}.bias'))


def mha(a: torch.Tensor, w_in, b_in, w_out, b_out, heads: int) -> torch.Tensor:
    """softmax(Q K^T / sqrt(d)) V with packed in_proj (nn.MultiheadAttention, batch_first, eval).

    fp32 without autograd: the reference module in eval under no_grad takes PyTorch's fused
    self-attention fast path (nn.MultiheadAttention.forward -> torch._native_multi_head_attention),
    so the oracle calls that same op and is bitwise-equal to the reference import.  Otherwise
    (float64 / autograd, the training tests' reference) the same math written out."""
    B, N, C = a.shape
    if a.dtype == torch.float32 and not torch.is_grad_enabled() and not a.requires_grad:
        # need_weights=True, average_attn_weights=True: the reference's own call (self.attentions[i](x, x, x),
        # nn.MultiheadAttention's defaults), so the same native kernel path; the weights are discarded as
        # the reference discards them (unet_base.py:158)
        return torch._native_multi_head_attention(a, a, a, C, heads, w_in, b_in, w_out, b_out, None, True, True,
                                                  None)[0]
    d = C // heads
    qkv = F.linear(a, w_in, b_in)
    q, k, v = qkv.split(C, dim=-1)
    q = q.reshape(B, N, heads, d).transpose(1, 2)
    k = k.reshape(B, N, heads, d).transpose(1, 2)
    v = v.reshape(B, N, heads, d).transpose(1, 2)
    att = torch.softmax((q * (d**-0.5)) @ k.transpose(-1, -2), dim=-1)
    o = (att @ v).transpose(1, 2).reshape(B, N, C)
    return F.linear(o, w_out, b_out)


def _attn(sd, pfx: str, i: int, x: torch.Tensor, heads: int) -> torch.Tensor:
    B, C, H, W = x.shape
    a = x.reshape(B, C, H * W)
    a = F.group_norm(a, 8, sd[f'{pfx}.attention_norms.{i}.weight'], sd[f'{pfx}.attention_norms.{i}.bias'], EPS)
    a = a.transpose(1, 2)
    o = mha(a, sd[f'{pfx}.attentions.{i}.in_proj_weight'], sd[f'{pfx}.attentions.{i}.in_proj_bias'],
            sd[f'{pfx}.attentions.{i}.out_proj.weight'], sd[f'{pfx}.attentions.{i}.out_proj.bias'], heads)
    return x + o.transpose(1, 2).reshape(B, C, H, W)


def level_has_attn(mc, i: int) -> bool:  # unet_base.py:404-405,434-435
    return (mc.im_size // (2**i)) in mc.attn_resolutions


def unet_forward(sd: Dict[str, torch.Tensor], mc, x: torch.Tensor, t) -> torch.Tensor:
    """Reference Unet.forward (unet_base.py:451-488) on CPU fp32 (float64 when x is float64: the
    autograd reference of the training-backward tests)."""
    x = x if x.dtype == torch.float64 else x.float()
    dc: List[int] = list(mc.down_channels)
    L = len(dc) - 1
    heads = mc.num_heads
    out = F.conv2d(x, sd['conv_in.weight'], sd['conv_in.bias'], padding=1)
    temb = time_embedding(torch.as_tensor(t).long(), mc.time_emb_dim).to(x.dtype)
    temb = F.linear(F.silu(F.linear(temb, sd['t_proj.0.weight'], sd['t_proj.0.bias'])), sd['t_proj.2.weight'],
                    sd['t_proj.2.bias'])
    skips = []
    for i in range(L):
        skips.append(out)
        pfx = f'downs.{i}'
        for l in range(mc.num_down_layers):
            out = _resblock(sd, pfx, l, out, temb)
            if level_has_attn(mc, i):
                out = _attn(sd, pfx, l, out, heads)
        if mc.down_sample[i]:
            out = F.conv2d(out, sd[f'{pfx}.down_sample_conv.weight'], sd[f'{pfx}.down_sample_conv.bias'], stride=2,
                           padding=1)
    for j in range(len(mc.mid_channels) - 1):
        pfx = f'mids.{j}'
        out = _resblock(sd, pfx, 0, out, temb)
        for l in range(mc.num_mid_layers):
            out = _attn(sd, pfx, l, out, heads)
            out = _resblock(sd, pfx, l + 1, out, temb)
    for k in range(L):
        i = L - 1 - k
        pfx = f'ups.{k}'
        if mc.down_sample[i]:
            out = F.conv_transpose2d(out, sd[f'{pfx}.up_sample_conv.weight'], sd[f'{pfx}.up_sample_conv.bias'],
                                     stride=2, padding=1)
        out = torch.cat([out, skips.pop()], dim=1)
        for l in range(mc.num_up_layers):
            out = _resblock(sd, pfx, l, out, temb)
            if level_has_attn(mc, i):
                out = _attn(sd, pfx, l, out, heads)
    out = F.silu(F.group_norm(out, 8, sd['norm_out.weight'], sd['norm_out.bias'], EPS))
    return F.conv2d(out, sd['conv_out.weight'], sd['conv_out.bias'], padding=1)


def unet_state_dict_keys(mc) -> Dict[str, tuple]:
    """Key -> shape map of the reference Unet built from ``mc`` (unet_base.py:378-449)."""
    shapes = {}
    d = mc.time_emb_dim
    shapes['t_proj.0.weight'] = (d, d)
    shapes['t_proj.0.bias'] = (d, )
    shapes['t_proj.2.weight'] = (d, d)
    shapes['t_proj.2.bias'] = (d, )
    dc = list(mc.down_channels)
    shapes['conv_in.weight'] = (dc[0], mc.im_channels, 3, 3)
    shapes['conv_in.bias'] = (dc[0], )

    def stage(pfx, cin, cout, n_res, n_attn, attn):
        for i in range(n_res):
            ci = cin if i == 0 else cout
            shapes[f'{pfx}.resnet_conv_first.{i}.0.weight'] = (ci, )
            shapes[f'{pfx}.resnet_conv_first.{i}.0.bias'] = (ci, )
            shapes[f'{pfx}.resnet_conv_first.{i}.2.weight'] = (cout, ci, 3, 3)
            shapes[f'{pfx}.resnet_conv_first.{i}.2.bias'] = (cout, )
        for i in range(n_res):
            shapes[f'{pfx}.t_emb_layers.{i}.1.weight'] = (cout, d)
            shapes[f'{pfx}.t_emb_layers.{i}.1.bias'] = (cout, )
        for i in range(n_res):
            shapes[f'{pfx}.resnet_conv_second.{i}.0.weight'] = (cout, )
            shapes[f'{pfx}.resnet_conv_second.{i}.0.bias'] = (cout, )
            shapes[f'{pfx}.resnet_conv_second.{i}.2.weight'] = (cout, cout, 3, 3)
            shapes[f'{pfx}.resnet_conv_second.{i}.2.bias'] = (cout, )
        if attn:
            for i in range(n_attn):
                shapes[f'{pfx}.attention_norms.{i}.weight'] = (cout, )
                shapes[f'{pfx}.attention_norms.{i}.bias'] = (cout, )
            for i in range(n_attn):
                shapes[f'{pfx}.attentions.{i}.in_proj_weight'] = (3 * cout, cout)
                shapes[f'{pfx}.attentions.{i}.in_proj_bias'] = (3 * cout, )
                shapes[f'{pfx}.attentions.{i}.out_proj.weight'] = (cout, cout)
                shapes[f'{pfx}.attentions.{i}.out_proj.bias'] = (cout, )
        for i in range(n_res):
            ci = cin if i == 0 else cout
            shapes[f'{pfx}.residual_input_conv.{i}.weight'] = (cout, ci, 1, 1)
            shapes[f'{pfx}.residual_input_conv.{i}.bias'] = (cout, )

    L = len(dc) - 1
    for i in range(L):
        stage(f'downs.{i}', dc[i], dc[i + 1], mc.num_down_layers, mc.num_down_layers, level_has_attn(mc, i))
        if mc.down_sample[i]:
            shapes[f'downs.{i}.down_sample_conv.weight'] = (dc[i + 1], dc[i + 1], 4, 4)
            shapes[f'downs.{i}.down_sample_conv.bias'] = (dc[i + 1], )
    mcn = list(mc.mid_channels)
    for j in range(len(mcn) - 1):
        stage(f'mids.{j}', mcn[j], mcn[j + 1], mc.num_mid_layers + 1, mc.num_mid_layers, True)
    for k in range(L):
        i = L - 1 - k
        cin = dc[i] * 2
        cout = dc[i - 1] if i != 0 else dc[0]
        stage(f'ups.{k}', cin, cout, mc.num_up_layers, mc.num_up_layers, level_has_attn(mc, i))
        if mc.down_sample[i]:
            shapes[f'ups.{k}.up_sample_conv.weight'] = (cin // 2, cin // 2, 4, 4)
            shapes[f'ups.{k}.up_sample_conv.bias'] = (cin // 2, )
    shapes['norm_out.weight'] = (dc[0], )
    shapes['norm_out.bias'] = (dc[0], )
    shapes['conv_out.weight'] = (mc.im_channels, dc[0], 3, 3)
    shapes['conv_out.bias'] = (mc.im_channels, )
    return shapes

"""Batch-sharded DDPM sampling over the GPUs of one node (BASELINE config 5).

One process per GPU (``torch.distributed``, backend ``nccl`` = RCCL over xGMI).  Every sample's
reverse trajectory is independent (GroupNorm and attention are per sample, the scheduler is
elementwise, t is shared), so rank r of W owns the contiguous global sample range
``shard_range(B, W, r)`` and runs the whole T-step loop with NO intra-step collective.  Noise is keyed
by the GLOBAL sample index (Philox(seed, sample, step) on the device, or the reference's CPU stream
sliced to the rank's rows), so the gathered result is identical for any W.  The only collective is
one all-gather of x0 at the end (config 5: 128 x 3 x 256^2 fp32 = 100.7 MB, ≈0.6 ms on xGMI against
minutes of compute).
"""
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist


def shard_range(total: int, world: int, rank: int) -> Tuple[int, int]:
    """(first global sample, count) of ``rank``: contiguous, sizes differ by at most one."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError('bad world/rank')
    base, extra = divmod(total, world)
    count = base + (1 if rank < extra else 0)
    start = rank * base + min(rank, extra)
    return start, count


def gather_samples(x_local: torch.Tensor, total: int, group=None) -> torch.Tensor:
    """All-gather the per-rank sample blocks into the full (total, ...) batch on every rank.

    RCCL (backend ``nccl``) gathers device tensors in place over xGMI.  gloo cannot gather device
    tensors, so under gloo (CPU tests, or several ranks sharing one GPU) the blocks are staged through
    host memory and the result is copied back to ``x_local``'s device.
    """
    world = dist.get_world_size(group)
    counts = [shard_range(total, world, r)[1] for r in range(world)]
    if x_local.shape[0] != counts[dist.get_rank(group)]:
        raise ValueError(f'gather_samples: rank holds {x_local.shape[0]} samples, shard_range says '
                         f'{counts[dist.get_rank(group)]}')
    dev = x_local.device
    staged = dist.get_backend(group) == 'gloo' and dev.type != 'cpu'
    xs = x_local.detach().to('cpu') if staged else x_local
    if all(c == counts[0] for c in counts):
        out = torch.empty((total, ) + tuple(xs.shape[1:]), dtype=xs.dtype, device=xs.device)
        if dist.get_backend(group) == 'gloo':
            parts = list(out.split(counts[0]))
            dist.all_gather(parts, xs.contiguous(), group=group)
        else:
            dist.all_gather_into_tensor(out, xs.contiguous(), group=group)
    else:
        cmax = max(counts)
        pad = torch.zeros((cmax, ) + tuple(xs.shape[1:]), dtype=xs.dtype, device=xs.device)
        pad[:xs.shape[0]] = xs
        parts: List[torch.Tensor] = [torch.empty_like(pad) for _ in range(world)]
        dist.all_gather(parts, pad, group=group)
        out = torch.cat([p[:c] for p, c in zip(parts, counts)], dim=0)
    return out.to(dev) if staged else out


@torch.no_grad()
def sample_sharded(model, scheduler, total_batch: int, im_channels: int, im_size: int, *, noise: str = 'philox',
                   seed: int = 0, graph: bool = False, group=None, gather: bool = True) -> torch.Tensor:
    """Reference sample loop (sample_ddpm.py:35-44) for ``total_batch`` images split over the group."""
    from .sample_ddpm import sample_tensor
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    start, count = shard_range(total_batch, world, rank)
    if count == 0:  # more ranks than images: this rank launches nothing and only joins the gather
        dev = next(model.parameters()).device
        x = torch.empty((0, im_channels, im_size, im_size), dtype=torch.float32, device=dev)
        return gather_samples(x, total_batch, group) if gather else x
    x = sample_tensor(model, scheduler, count, im_channels, im_size, noise=noise, seed=seed, sample0=start,
                      total_batch=total_batch, graph=graph)
    if world == 1 or not gather:
        return x
    return gather_samples(x, total_batch, group)

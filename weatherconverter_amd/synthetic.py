"""Name-keyed deterministic synthetic weights and inputs.

No checkpoints ship with the reference, so every parity fixture and every benchmark
uses weights generated from the state_dict KEY: ``rng = numpy.random.default_rng(crc32(f"{seed}:{key}"))``.
The same recipe runs here (to make golden vectors from the reference import) and on the GPU box
(to rebuild the exact same weights), so fixtures store inputs/outputs + a weight digest, never the
110 M parameters.

Recipe per tensor (float64 draw, cast to the parameter dtype):
  * >=2-D weights (conv / linear / in_proj): U(-1/sqrt(fan_in), 1/sqrt(fan_in)), fan_in = prod(shape[1:])
  * 1-D "*weight" (GroupNorm / LayerNorm / BatchNorm gamma): 1 + 0.1 N(0, 1)
  * 1-D "*bias": 0.1 U(-1, 1)
  * BatchNorm running_mean: 0.1 N(0, 1); running_var: 1 + 0.2 |N(0, 1)|; num_batches_tracked: 0
"""
import hashlib
import zlib
from typing import Dict

import numpy as np
import torch


def _rng(seed: int, key: str) -> np.random.Generator:
    return np.random.default_rng(zlib.crc32(f'{seed}:{key}'.encode()))


def synth_tensor(key: str, shape, dtype=torch.float32, seed: int = 0) -> torch.Tensor:
    rng = _rng(seed, key)
    shape = tuple(shape)
    if key.endswith('num_batches_tracked'):
        return torch.zeros(shape, dtype=dtype)
    if key.endswith('running_mean'):
        a = 0.1 * rng.standard_normal(shape)
    elif key.endswith('running_var'):
        a = 1.0 + 0.2 * np.abs(rng.standard_normal(shape))
    elif len(shape) >= 2:
        fan_in = int(np.prod(shape[1:]))
        bound = 1.0 / np.sqrt(max(fan_in, 1))
        a = rng.uniform(-bound, bound, size=shape)
    elif key.endswith('weight'):
        a = 1.0 + 0.1 * rng.standard_normal(shape)
    else:
        a = 0.1 * rng.uniform(-1.0, 1.0, size=shape)
    return torch.from_numpy(np.ascontiguousarray(a)).to(dtype)


def synthetic_state_dict(template: Dict[str, torch.Tensor], seed: int = 0) -> Dict[str, torch.Tensor]:
    """Synthetic values for every key of ``template`` (a state_dict or {key: tensor-like with .shape})."""
    return {k: synth_tensor(k, v.shape, v.dtype, seed) for k, v in template.items()}


def init_synthetic_(model: torch.nn.Module, seed: int = 0) -> torch.nn.Module:
    """Overwrite every parameter/buffer of ``model`` with the keyed recipe (in place)."""
    sd = model.state_dict()
    with torch.no_grad():
        for k, v in sd.items():
            v.copy_(synth_tensor(k, v.shape, v.dtype, seed))
    return model


def state_dict_digest(sd: Dict[str, torch.Tensor]) -> str:
    """SHA-256 over (key, shape, float32 bytes) in sorted key order."""
    h = hashlib.sha256()
    for k in sorted(sd):
        v = sd[k].detach().cpu()
        h.update(k.encode())
        h.update(str(tuple(v.shape)).encode())
        h.update(v.contiguous().numpy().tobytes())
    return h.hexdigest()


def synthetic_images(shape, seed: int = 3455) -> torch.Tensor:
    """x_T ~ N(0,1) from the torch CPU generator (reference sampling draws on the CPU, §3.1)."""
    g = torch.Generator().manual_seed(seed)
    return torch.randn(shape, generator=g)

"""GPU: bench.py's N-rank branch end to end (the code the driver's 8-GPU SCALE run executes).

``python bench.py --gpus 2 --backend gloo`` self-launches torch.distributed.run with two ranks that
share cuda:0, runs the timed sharded loop (reference sample_ddpm.py:35-44 per rank), gathers x0
(host-staged under gloo), reduces the per-rank timings and prints one JSON line on rank 0.  The
RCCL branch differs only in the two collectives (``bench._gather_x0`` / ``bench._gather_times``).
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_gloo_one_gpu():
    cmd = [sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', '2', '--backend', 'gloo', '--size', '64',
           '--batch', '2', '--steps', '3', '--warmup', '1', '--timesteps', '50', '--no-roofline',
           '--no-cpu-baseline']
    env = dict(os.environ, MASTER_ADDR='127.0.0.1')
    env.pop('WORLD_SIZE', None)
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, r.stdout[-2000:]
    res = json.loads(lines[0])
    assert res['n_gpus'] == 2
    assert res['steps'] == 3 and res['warmup'] == 1
    assert len(res['per_rank_ms_per_step']) == 2
    assert all(v > 0 for v in res['per_rank_ms_per_step'])
    assert res['all_gather_ms'] is not None and len(res['all_gather_ms']) == 2
    assert res['config']['global_batch'] == 4
    assert res['config']['x_finite'] is True
    assert res['config']['backend'] == 'gloo'
    assert res['ms_per_step'] == pytest.approx(max(res['per_rank_ms_per_step']), rel=1e-3)
    assert res['cpu_baseline'] is None

"""CPU: bench.py's launch contract (no GPU needed): --gpus N>1 without WORLD_SIZE re-launches itself
under torch.distributed.run with one rank per GPU on a loopback rendezvous; under a launcher the
world size must equal --gpus; the CPU-share probe reports what the baseline leg may use."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_launch_cmd_one_rank_per_gpu_loopback():
    cmd = bench._launch_cmd(8, ['--gpus', '8', '--steps', '5'], 29500)
    assert cmd[1:3] == ['-m', 'torch.distributed.run']
    assert '--nproc-per-node=8' in cmd and '--nnodes=1' in cmd
    assert cmd[cmd.index('--master-addr') + 1] == '127.0.0.1'
    assert cmd[cmd.index('--master-port') + 1] == '29500'
    assert cmd[-4:] == ['--gpus', '8', '--steps', '5'] and cmd[-5].endswith('bench.py')


def test_world_size_must_match_gpus(monkeypatch):
    monkeypatch.setenv('WORLD_SIZE', '2')
    assert bench._world(bench.parse(['--gpus', '2'])) == 2
    assert bench._world(bench.parse([])) == 2
    with pytest.raises(SystemExit):
        bench._world(bench.parse(['--gpus', '4']))
    monkeypatch.delenv('WORLD_SIZE')
    assert bench._world(bench.parse([])) == 1


def test_cpu_share_probe():
    share = bench._cpu_share()
    assert 1 <= share['usable_cpus'] <= share['host_cpus']
    assert share['usable_cpus'] <= share['affinity_cpus']


def _bench_gather_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        x = torch.full((2, 3, 4, 4), float(rank))
        g = bench._gather_x0(x, world, 'gloo')
        t = bench._gather_times([0.5 + rank, 0.01 * rank], world, 'gloo', None)
        q.put((rank, g.numpy().copy(), t.numpy().copy()))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 4])
def test_bench_gloo_collectives(world):
    """bench.py's gloo branch of the x0 all-gather and of the per-rank timing reduction."""
    import socket

    import numpy as np
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_bench_gather_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    for _, g, t in res:
        assert g.shape == (2 * world, 3, 4, 4)
        for r in range(world):
            assert np.all(g[2 * r:2 * r + 2] == r)
        assert t.shape == (world, 2)
        assert np.allclose(t[:, 0], 0.5 + np.arange(world))


def test_self_launch_refused_under_profiler(monkeypatch):
    monkeypatch.setenv('LD_PRELOAD', '/opt/rocm/lib/rocprofiler-sdk/librocprofiler-sdk-tool.so')
    assert bench._profiler_preloaded()
    with pytest.raises(SystemExit):
        bench._self_launch(bench.parse(['--gpus', '2']))


def test_hbm_leg_bytes_from_nbytes_or_flops_field():
    """hbm_leg reads a launch's stated nbytes (wino_vsplit) and falls back to the 'flops' field, where the
    GroupNorm / split wrappers state their bytes."""
    hbm = {'wino_vsplit_kernel': [2, 0.0, 2e-4, 1.6e9, 0.0], 'split_tiled_kernel': [1, 4e8, 1e-4, 0.0, 0.0]}
    out = bench.hbm_leg(hbm)
    assert out['wino_vsplit_kernel']['gbytes'] == 1.6 and out['wino_vsplit_kernel']['achieved'] == 8000.0
    assert out['split_tiled_kernel']['gbytes'] == 0.4 and out['split_tiled_kernel']['frac'] == 0.5

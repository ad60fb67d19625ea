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

"""bench.py's launch contract on CPU: ``--gpus N`` without torchrun starts N
ranks (torch.distributed.run as a child process), every rank sees
WORLD_SIZE = N, and rank 0 alone prints the line with n_gpus = N."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args):
    env = dict(os.environ)
    env.pop('WORLD_SIZE', None)
    res = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py')] + list(args),
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env,
                         timeout=240)
    assert res.returncode == 0, res.stderr[-2000:]
    lines = [json.loads(line) for line in res.stdout.splitlines() if line.startswith('{')]
    return lines


def test_gpus_2_spawns_two_ranks():
    lines = _run('--gpus', '2', '--dry-run', '--steps', '3', '--warmup', '1')
    assert len(lines) == 1                      # rank 0 only
    line = lines[0]
    assert line['n_gpus'] == 2 and line['world_size_env'] == '2'
    assert line['steps'] == 3 and line['warmup'] == 1


def test_default_is_one_rank():
    (line,) = _run('--dry-run', '--steps', '2', '--warmup', '0')
    assert line['n_gpus'] == 1 and line['world_size_env'] is None


def test_parse_defaults():
    sys.path.insert(0, ROOT)
    import bench
    args = bench.parse([])
    assert args.gpus == 1 and args.envs == 4096 and args.workload == 'optimize'
    assert bench.parse(['--workload', 'multi']).envs == 1024


def test_run_length_defaults():
    """The microsecond-step workloads default to 20,000 warmup + 20,000 timed
    steps (the chip's clock ramp); a given --steps /
    --warmup (either spelling) wins; the other workloads keep theirs."""
    sys.path.insert(0, ROOT)
    import bench
    a = bench.parse([])
    assert (a.steps, a.warmup) == (20000, 20000)
    a = bench.parse(['--steps', '20', '--warmup', '5'])
    assert (a.steps, a.warmup) == (20, 5)
    a = bench.parse(['--workload', 'multi', '--steps=7'])
    assert (a.steps, a.warmup) == (7, 20000)
    a = bench.parse(['--workload', 'mlp'])
    assert (a.steps, a.warmup) == (2000, 200)


"""Env-sharded multi-rank path on CPU (gloo, world_size 2).

Each rank runs its contiguous shard of a 5-env batch (uneven: 3 + 2) and
all-gathers the packed outputs every step.  The gathered global arrays must
equal a 1-rank run bit for bit.  The shard engine here is the oracle (the
test's stand-in for the HIP engine, which needs a GPU); the sharding, the
seeds = global index rule, the packed layout and the collective are the
product code (custom_envs_amd/distributed.py).
"""
import os
import socket

import numpy as np
import pytest
import torch

from custom_envs_amd.distributed import PackedLayout, ShardedEnvs, shard_range


class OracleShardEngine:
    """The engine interface ShardedEnvs drives, backed by oracle envs."""

    obs_dim, act_dim = 41, 20

    def __init__(self, features, targets, num_envs):
        from oracle.optimize import Optimize
        self.num_envs = num_envs
        self.envs = [Optimize(features, targets) for _ in range(num_envs)]

    def output_fields(self):
        from custom_envs_amd.engine import OptimizeEngine
        return OptimizeEngine.output_fields(self)

    def seed(self, seeds):
        for env, s in zip(self.envs, seeds):
            env.seed(s)
        return seeds

    def reset_device(self, out):
        for i, env in enumerate(self.envs):
            out['obs'][i] = torch.from_numpy(env.reset().astype(np.float32))

    def step_device(self, actions, out):
        for i, env in enumerate(self.envs):
            obs, reward, done, info = env.step(actions[i].numpy())
            out['episode_len'][i] = info['episode']['l']
            if done:
                obs = env.reset()
            out['obs'][i] = torch.from_numpy(obs.astype(np.float32))
            out['reward'][i] = reward
            out['done'][i] = int(done)
            out['objective'][i] = info['objective']
            out['accuracy'][i] = info['accuracy']


def _rollout(features, targets, num_envs, rank, world, steps=44):
    lo, hi = shard_range(num_envs, world, rank)
    shard = ShardedEnvs(OracleShardEngine(features, targets, hi - lo), num_envs, rank, world,
                        device='cpu')
    shard.seed(100)
    shard.reset()
    rec = [{k: v.clone() for k, v in shard.gather().items()}]
    acts = torch.from_numpy(np.random.RandomState(3).normal(
        0, 0.01, (steps, num_envs, 20)).astype(np.float32))
    for t in range(steps):
        shard.step(acts[t, lo:hi].contiguous())
        rec.append({k: v.clone() for k, v in shard.gather().items()})
    return rec


def _worker(rank, world, port, features, targets, expected):
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        got = _rollout(features, targets, 5, rank, world)
        assert len(got) == len(expected)
        for t, (g, e) in enumerate(zip(got, expected)):
            for key in e:
                assert torch.equal(g[key], e[key]), (rank, t, key)
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def test_shard_ranges_cover_and_balance():
    for n in (1, 5, 4096, 32768, 32771):
        for world in (1, 2, 3, 8):
            spans = [shard_range(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_range(4, 2, 2)


def test_packed_layout_segments_are_aligned_and_disjoint():
    fields = [('obs', torch.float32, 4, (15,)), ('done', torch.uint8, 4, ()),
              ('info', torch.float32, 1, (14,)), ('episode_len', torch.int32, 1, ())]
    lay = PackedLayout(fields, capacity=7)
    buf = torch.zeros(lay.nbytes, dtype=torch.uint8)
    views = lay.views(buf, 5)
    assert views['obs'].shape == (20, 15) and views['info'].shape == (5, 14)
    for i, (name, *_) in enumerate(fields):
        assert lay.offsets[name] % 256 == 0
        views[name].fill_(i + 1)
    for i, (name, *_) in enumerate(fields):          # no segment overlaps another
        assert bool((views[name] == i + 1).all()), name
    # two shards unpack in rank order with their own counts
    b2 = torch.zeros(lay.nbytes, dtype=torch.uint8)
    v2 = lay.views(b2, 2)
    v2['episode_len'][:] = torch.tensor([7, 8], dtype=torch.int32)
    views['episode_len'][:] = torch.arange(5, dtype=torch.int32)
    glob = lay.unpack(torch.cat([buf, b2]), [5, 2])
    assert glob['episode_len'].tolist() == [0, 1, 2, 3, 4, 7, 8]
    assert glob['obs'].shape == (28, 15)


@pytest.mark.parametrize('world', [2, 3])
def test_gloo_world2_gather_equals_single_rank(lr_dataset, world):
    """5 envs over 2 ranks (3 + 2) and 3 ranks (2 + 2 + 1)."""
    import torch.multiprocessing as mp
    features, targets = lr_dataset
    expected = _rollout(features, targets, 5, 0, 1)
    mp.spawn(_worker, args=(world, _free_port(), features, targets, expected), nprocs=world,
             join=True)

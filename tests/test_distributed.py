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
    """The engine interface ShardedEnvs drives, backed by oracle envs; with
    ``supports_compact`` it writes the compact record as the HIP two-class
    kernel does (obs_tail = obs[P:], no done)."""

    obs_dim, act_dim, max_steps = 41, 20, 40

    def __init__(self, features, targets, num_envs, supports_compact=False):
        from oracle.optimize import Optimize
        self.num_envs = num_envs
        self.envs = [Optimize(features, targets) for _ in range(num_envs)]
        self.compact = False
        if supports_compact:
            self.set_compact_outputs = self._set_compact

    def _set_compact(self, on=True):
        self.compact = bool(on)

    def output_fields(self):
        from custom_envs_amd.engine import OptimizeEngine
        return OptimizeEngine.output_fields(self)

    def derived_fields(self):
        from custom_envs_amd.engine import OptimizeEngine
        return OptimizeEngine.derived_fields(self)

    def _put_obs(self, out, i, obs):
        if self.compact:
            assert np.all(obs[:self.act_dim] == 0)
            out['obs_tail'][i] = torch.from_numpy(obs[self.act_dim:].astype(np.float32))
        else:
            out['obs'][i] = torch.from_numpy(obs.astype(np.float32))

    def seed(self, seeds):
        for env, s in zip(self.envs, seeds):
            env.seed(s)
        return seeds

    def reset_device(self, out):
        for i, env in enumerate(self.envs):
            self._put_obs(out, i, env.reset())

    def step_device(self, actions, out):
        for i, env in enumerate(self.envs):
            obs, reward, done, info = env.step(actions[i].numpy())
            out['episode_len'][i] = info['episode']['l']
            if done:
                obs = env.reset()
            self._put_obs(out, i, obs)
            if not self.compact:
                out['reward'][i] = reward
                out['done'][i] = int(done)
            else:             # the compact record derives reward = -objective (B = N)
                assert np.float32(reward) == -np.float32(info['objective'])
            out['objective'][i] = info['objective']
            out['accuracy'][i] = info['accuracy']


    def rollout_device(self, k, actions, fields, record_bytes):
        """k steps, step t's outputs into record t (the HIP engine's
        ce_step_many_strided contract)."""
        for t in range(k):
            self.step_device(actions[t], {n: v[t] for n, v in fields.items()})


def _chunk_rollout(features, targets, num_envs, rank, world, chunk, steps=44, compact=True):
    """The chunk schedule: K-step rollouts into alternating slots, one
    gather per chunk (the tail chunk shorter), every step's global outputs
    snapshotted in order."""
    lo, hi = shard_range(num_envs, world, rank)
    shard = ShardedEnvs(OracleShardEngine(features, targets, hi - lo, compact), num_envs, rank,
                        world, device='cpu', compact=compact, slots=2, chunk=chunk,
                        collective=world > 1)
    shard.seed(100)
    shard.reset()
    rec = [shard.gather().snapshot()]
    acts = torch.from_numpy(np.random.RandomState(3).normal(
        0, 0.01, (steps, num_envs, 20)).astype(np.float32))
    t = c = 0
    while t < steps:
        k = min(chunk, steps - t)
        slot = c % 2
        shard.rollout(acts[t:t + k, lo:hi].contiguous(), slot, k)
        rec += [g.snapshot() for g in shard.gather_chunk(slot, k=k)]
        t += k
        c += 1
    return rec


def _chunk_worker(rank, world, port, features, targets, expected, chunk):
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        got = _chunk_rollout(features, targets, 5, rank, world, chunk)
        assert len(got) == len(expected)
        for t, (g, e) in enumerate(zip(got, expected)):
            for key in e:
                assert torch.equal(g[key], e[key]), (rank, t, key, chunk)
    finally:
        dist.destroy_process_group()


def _rollout(features, targets, num_envs, rank, world, steps=44, compact=False):
    lo, hi = shard_range(num_envs, world, rank)
    shard = ShardedEnvs(OracleShardEngine(features, targets, hi - lo, compact), num_envs, rank,
                        world, device='cpu', compact=compact)
    assert shard.compact == compact
    shard.seed(100)
    shard.reset()
    rec = [{k: v.clone() for k, v in shard.gather().items()}]
    acts = torch.from_numpy(np.random.RandomState(3).normal(
        0, 0.01, (steps, num_envs, 20)).astype(np.float32))
    for t in range(steps):
        shard.step(acts[t, lo:hi].contiguous())
        rec.append({k: v.clone() for k, v in shard.gather().items()})
    return rec


def _worker(rank, world, port, features, targets, expected, compact=False):
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        got = _rollout(features, targets, 5, rank, world, compact=compact)
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


@pytest.mark.parametrize('compact', [False, True])
@pytest.mark.parametrize('world', [2, 3])
def test_gloo_world2_gather_equals_single_rank(lr_dataset, world, compact):
    """5 envs over 2 ranks (3 + 2) and 3 ranks (2 + 2 + 1), with the full
    record and with the compact one (the zero weight block of obs and done
    rebuilt on the receiving side): the same global arrays as a 1-rank run of
    the full record, bit for bit."""
    import torch.multiprocessing as mp
    features, targets = lr_dataset
    expected = _rollout(features, targets, 5, 0, 1)
    mp.spawn(_worker, args=(world, _free_port(), features, targets, expected, compact),
             nprocs=world, join=True)


def test_compact_record_is_smaller_and_rebuilds_full_fields(lr_dataset):
    """The compact record drops ~47 % of the bytes per env (P = 20: 96 B
    against 181 B) and the gathered view rebuilds obs, done and reward
    exactly."""
    features, targets = lr_dataset
    full = ShardedEnvs(OracleShardEngine(features, targets, 4), 4, device='cpu', compact=False)
    comp = ShardedEnvs(OracleShardEngine(features, targets, 4, True), 4, device='cpu',
                       compact=True)
    per_env = {}
    for name, sh in (('full', full), ('compact', comp)):
        per_env[name] = sum(PackedLayout._nbytes(d, r, t, 1) for _, d, r, t in sh.layout.fields)
    assert per_env == {'full': 181, 'compact': 96}
    for sh in (full, comp):
        sh.seed(3)
        sh.reset()
    acts = torch.from_numpy(np.random.RandomState(1).normal(0, 0.01, (41, 4, 20)).astype(np.float32))
    for t in range(41):
        a, b = full.step(acts[t]), comp.step(acts[t])
        ga, gb = full.gather(), comp.gather()
        assert set(ga) == set(gb) - {'obs_tail'}
        for key in ga:
            assert torch.equal(ga[key], gb[key]), (t, key)


def test_gathered_outputs_snapshot_survives_the_next_gather(lr_dataset):
    """A GatheredOutputs reads its slot's buffer: a field first read after the
    next gather into that slot sees the newer step; snapshot() does not."""
    features, targets = lr_dataset
    sh = ShardedEnvs(OracleShardEngine(features, targets, 3), 3, device='cpu')
    sh.seed(0)
    sh.reset()
    acts = torch.from_numpy(np.random.RandomState(2).normal(0, 0.01, (2, 3, 20)).astype(np.float32))
    sh.step(acts[0])
    first = sh.gather()
    snap = first.snapshot()
    obs0 = first['obs'].clone()
    sh.step(acts[1])
    later = sh.gather()
    assert torch.equal(snap['obs'], obs0)
    assert not torch.equal(later['obs'], obs0)
    assert torch.equal(first['reward'], later['reward'])   # unread until now: the newer step


# ---------------------------------------------------------------------------
# Config 5: MultiOptLRs-v0 behind OptVecEnv, sharded (run_multiagent_exp_single.py:
# 37,78-86).  The stand-in writes the MultiOptEngine output fields from oracle
# OptEnvRunners; the gathered arrays of 2 and 3 ranks equal a 1-rank run.

class OracleMultiShardEngine:
    n_params, max_history = 4, 5

    def __init__(self, num_envs, max_batches=30):
        from oracle.multioptlrs import MultiOptLRs, OptEnvRunner
        self.num_envs = num_envs
        self.runners = [OptEnvRunner(MultiOptLRs(self.n_params, max_batches=max_batches,
                                                 max_history=self.max_history))
                        for _ in range(num_envs)]

    def output_fields(self):
        from custom_envs_amd.multi_engine import MultiOptEngine
        return MultiOptEngine.output_fields(self)

    def seed(self, seeds):
        return seeds

    def reset_device(self, out):
        P = self.n_params
        for e, r in enumerate(self.runners):
            out['obs'][e * P:(e + 1) * P] = torch.from_numpy(np.stack(r.reset()).astype(np.float32))

    def step_device(self, actions, out):
        from custom_envs_amd._native import MULTI_INFO_KEYS
        P = self.n_params
        for e, r in enumerate(self.runners):
            states, rewards, dones, infos = r.step(list(actions[e * P:(e + 1) * P].numpy().reshape(P, 1)))
            out['episode_len'][e] = infos[0]['episode']['l']
            if dones[0]:
                states = r.reset()
            rows = slice(e * P, (e + 1) * P)
            out['obs'][rows] = torch.from_numpy(np.stack(states).astype(np.float32))
            out['reward'][rows] = float(rewards[0])
            out['done'][rows] = int(dones[0])
            out['info'][e] = torch.tensor([np.nan if infos[0][k] is None else float(infos[0][k])
                                           for k in MULTI_INFO_KEYS], dtype=torch.float32)


def _multi_rollout(num_envs, rank, world, steps=36):
    lo, hi = shard_range(num_envs, world, rank)
    shard = ShardedEnvs(OracleMultiShardEngine(hi - lo), num_envs, rank, world, device='cpu')
    shard.reset()
    rec = [shard.gather().snapshot()]
    rs = np.random.RandomState(5)
    lows = rs.uniform(-1.0, 1.5, num_envs)
    P = OracleMultiShardEngine.n_params
    acts = np.stack([rs.uniform(lows[e], lows[e] + 1.5, (steps, P)) for e in range(num_envs)], 1)
    acts = torch.from_numpy(acts.astype(np.float32).reshape(steps, num_envs * P))
    for t in range(steps):
        shard.step(acts[t, lo * P:hi * P].contiguous())
        rec.append(shard.gather().snapshot())
    return rec


def _multi_worker(rank, world, port, expected):
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        got = _multi_rollout(5, rank, world)
        assert len(got) == len(expected)
        for t, (g, e) in enumerate(zip(got, expected)):
            for key in e:
                assert torch.equal(g[key], e[key]) or (
                    g[key].dtype.is_floating_point and
                    torch.equal(torch.nan_to_num(g[key], 7.0), torch.nan_to_num(e[key], 7.0))), \
                    (rank, t, key)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 3])
def test_gloo_multiagent_gather_equals_single_rank(world):
    """Config 5's layout (per-agent obs/reward/done rows, per-env info and
    episode length) over 2 and 3 ranks, divergent and stable envs mixed,
    across max_batches episode ends."""
    import torch.multiprocessing as mp
    expected = _multi_rollout(5, 0, 1)
    assert any(bool(r['done'].any()) for r in expected)
    mp.spawn(_multi_worker, args=(world, _free_port(), expected), nprocs=world, join=True)


@pytest.mark.parametrize('chunk', [1, 7, 20])
@pytest.mark.parametrize('world', [2, 3])
def test_gloo_chunk_schedule_equals_single_rank(lr_dataset, world, chunk):
    """The chunk schedule (one K-step rollout and ONE all-gather of its K
    compact records per chunk, two alternating slots, a shorter tail chunk
    gathered out of place): 5 envs over 2 and 3 ranks give, step for step,
    the same global arrays as a 1-rank run of per-step gathers of the full
    record, bit for bit (concurrentvecenv.py:99-104,200-227 reassembly)."""
    import torch.multiprocessing as mp
    features, targets = lr_dataset
    expected = [{k: v.clone() for k, v in r.items()} for r in _rollout(features, targets, 5, 0, 1)]
    one = _chunk_rollout(features, targets, 5, 0, 1, chunk)
    for t, (g, e) in enumerate(zip(one, expected)):
        for key in e:
            assert torch.equal(g[key], e[key]), (t, key)
    mp.spawn(_chunk_worker, args=(world, _free_port(), features, targets, expected, chunk),
             nprocs=world, join=True)

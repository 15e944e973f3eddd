"""The env-sharded multi-GPU path over the real HIP engine (config 4), on
one GPU: the engine writes every output straight into ShardedEnvs' packed
buffers (PackedLayout views, 256-B-aligned segments), the RCCL all-gather
runs as a real collective (world 1 on the nccl backend), and the gathered
global arrays match the CPU oracle: done / episode length bit for bit, obs
within 1e-6 (float64 engine rounded to float32, as test_gpu_parity.py).
The 2-rank protocol itself runs on gloo in tests/test_distributed.py."""
import os
import socket

import numpy as np
import pytest

from oracle.optimize import Optimize as OracleEnv

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def nccl_world1():
    import torch
    import torch.distributed as dist
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need a ROCm device (run under gpurun)')
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ['MASTER_PORT'] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group('nccl', rank=0, world_size=1,
                            device_id=torch.device('cuda', 0))
    yield dist
    dist.destroy_process_group()


def _oracle_rows(features, targets, seeds, acts):
    rows = []
    envs = []
    for s in seeds:
        env = OracleEnv(features, targets)
        env.seed(s)
        env.reset()
        envs.append(env)
    for t in range(acts.shape[0]):
        rec = {'obs': [], 'done': [], 'len': [], 'reward': []}
        for i, env in enumerate(envs):
            obs, rew, done, info = env.step(acts[t, i])
            rec['len'].append(info['episode']['l'])
            if done:
                obs = env.reset()
            rec['obs'].append(obs)
            rec['done'].append(done)
            rec['reward'].append(rew)
        rows.append({k: np.array(v) for k, v in rec.items()})
    return rows


@pytest.mark.parametrize('pipelined', [False, True])
def test_sharded_engine_gather_matches_oracle(nccl_world1, lr_dataset, pipelined):
    import torch
    from custom_envs_amd.distributed import ShardedEnvs
    from custom_envs_amd.engine import OptimizeEngine
    features, targets = lr_dataset
    E, steps, base = 37, 44, 500
    eng = OptimizeEngine(features, targets, num_envs=E)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    eng.set_stream(stream.cuda_stream)
    shard = ShardedEnvs(eng, E, 0, 1, slots=2, collective=True)
    # packed segments: every field 256-B aligned, obs rows [E][41]
    assert all(off % 256 == 0 for off in shard.layout.offsets.values())
    assert shard.outs[0]['obs'].shape == (E, 41)
    assert shard.outs[0]['obs'].data_ptr() == shard.buffers[0].data_ptr() + \
        shard.layout.offsets['obs']
    shard.seed(base)
    shard.reset(0)
    acts = np.random.RandomState(8).normal(0, 0.02, (steps, E, 20)).astype(np.float32)
    dacts = torch.from_numpy(acts).cuda()
    expected = _oracle_rows(features, targets, [base + i for i in range(E)], acts)
    got, pending = {}, [None, None]
    keys = ('obs', 'done', 'episode_len', 'reward')

    def collect(entry):
        work, res, t = entry
        work.wait()              # the current stream waits for the collective
        assert res.rank_major['obs'].shape == (1, E, 41)   # zero-copy view
        got[t] = {k: res[k].cpu().numpy() for k in keys}

    for t in range(steps):
        slot = t & 1 if pipelined else 0
        if pending[slot] is not None:    # read slot's last gather before reusing it
            collect(pending[slot])
            pending[slot] = None
        shard.step(dacts[t], slot)
        res, work = shard.gather(slot, async_op=True)
        pending[slot] = (work, res, t)
        if not pipelined:
            collect(pending[slot])
            pending[slot] = None
    for slot in (0, 1):
        if pending[slot] is not None:
            collect(pending[slot])
    torch.cuda.synchronize()
    assert sorted(got) == list(range(steps))
    for t in range(steps):
        g, e = got[t], expected[t]
        assert np.array_equal(g['done'].astype(bool), e['done']), t
        assert np.array_equal(g['episode_len'], e['len']), t
        np.testing.assert_allclose(g['obs'], e['obs'], rtol=1e-6, atol=1e-9)
        np.testing.assert_allclose(g['reward'], e['reward'], rtol=1e-6)
    eng.close()
    torch.cuda.set_stream(torch.cuda.default_stream())

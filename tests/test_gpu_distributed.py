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


@pytest.mark.parametrize('compact', [True, False])
@pytest.mark.parametrize('pipelined', [False, True])
def test_sharded_engine_gather_matches_oracle(nccl_world1, lr_dataset, pipelined, compact):
    """compact (the default when the collective runs): the engine writes
    obs[P:] and no done; the gathered view rebuilds both."""
    import torch
    from custom_envs_amd.distributed import ShardedEnvs
    from custom_envs_amd.engine import OptimizeEngine
    features, targets = lr_dataset
    E, steps, base = 37, 44, 500
    eng = OptimizeEngine(features, targets, num_envs=E)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    eng.set_stream(stream.cuda_stream)
    shard = ShardedEnvs(eng, E, 0, 1, slots=2, collective=True, compact=compact)
    assert shard.compact == compact and eng.compact == compact
    # packed segments: every field 256-B aligned, obs rows [E][41] (compact: [E][21])
    obs_key, width = ('obs_tail', 21) if compact else ('obs', 41)
    assert all(off % 256 == 0 for off in shard.layout.offsets.values())
    assert shard.outs[0][obs_key].shape == (E, width)
    assert shard.outs[0][obs_key].data_ptr() == shard.buffers[0].data_ptr() + \
        shard.layout.offsets[obs_key]
    assert ('done' in shard.outs[0]) != compact
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
        assert res.rank_major[obs_key].shape == (1, E, width)   # zero-copy view
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


def test_compact_outputs_need_the_two_class_kernel(lr_dataset):
    """Only the two-class full-batch float64 kernel writes the compact form."""
    from custom_envs_amd import NativeEngineError
    from custom_envs_amd.engine import OptimizeEngine
    features, targets = lr_dataset
    eng = OptimizeEngine(features, targets, num_envs=4, batch_size=32)
    with pytest.raises(NativeEngineError, match='compact'):
        eng.set_compact_outputs(True)
    eng.close()


def test_sharded_multiagent_gather_matches_oracle(nccl_world1):
    """Config 5 (run_multiagent_exp_single.py:37,78-86): MultiOptEngine
    (4 agents, 4-D Rosenbrock pairs, H = 5) driven through ShardedEnvs with a
    real RCCL all-gather at world 1, against oracle OptEnvRunners: done and
    episode length exact, obs rows and reward within float32 rounding,
    info within 1e-5 (tolerances of test_gpu_multi.py)."""
    import torch
    from custom_envs_amd._native import MULTI_INFO_KEYS
    from custom_envs_amd.distributed import ShardedEnvs
    from custom_envs_amd.multi_engine import MultiOptEngine
    from oracle.multioptlrs import MultiOptLRs as OracleMulti, OptEnvRunner
    E, P, H, MB, T = 13, 4, 5, 30, 45
    rs = np.random.RandomState(12)
    lows = rs.uniform(-1.5, 1.5, E)
    acts = np.stack([rs.uniform(lows[e], lows[e] + 1.5, (T, P)) for e in range(E)], 1)
    acts = acts.astype(np.float32).reshape(T, E * P)
    eng = MultiOptEngine(E, 'func4', max_batches=MB, max_history=H)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    eng.set_stream(stream.cuda_stream)
    shard = ShardedEnvs(eng, E, 0, 1, collective=True)
    refs = [OptEnvRunner(OracleMulti(P, max_batches=MB, max_history=H)) for _ in range(E)]
    dacts = torch.from_numpy(acts).cuda()
    try:
        shard.reset()
        first = shard.gather()['obs'].cpu().numpy()
        assert np.array_equal(first, np.concatenate([np.stack(r.reset()) for r in refs]))
        for t in range(T):
            shard.step(dacts[t])
            g = shard.gather().snapshot()
            torch.cuda.synchronize()
            g = {k: v.cpu().numpy() for k, v in g.items()}
            for e, runner in enumerate(refs):
                states, rewards, dones, infos = runner.step(list(acts[t, e * P:(e + 1) * P].reshape(P, 1)))
                if dones[0]:
                    states = runner.reset()
                rows = slice(e * P, (e + 1) * P)
                assert np.all(g['done'][rows] == dones[0]), (t, e)
                assert int(g['episode_len'][e]) == infos[0]['episode']['l'], (t, e)
                ref = np.stack(states).astype(np.float64)
                scale = np.maximum(np.abs(ref).max(axis=-1), 1.0)
                assert np.all(np.abs(g['obs'][rows] - ref).max(axis=-1) / scale <= 1e-6), (t, e)
                assert abs(g['reward'][e * P] - rewards[0]) <= 1e-6 * max(1.0, abs(rewards[0]))
                ref_info = np.array([np.nan if infos[0][k] is None else float(infos[0][k])
                                     for k in MULTI_INFO_KEYS])
                fin = np.isfinite(ref_info) & (np.arange(len(ref_info)) != 8) & \
                    (np.arange(len(ref_info)) != 9)     # signed gradient sums: test_gpu_multi.py
                assert np.array_equal(np.isnan(g['info'][e]), np.isnan(ref_info)), (t, e)
                err = np.abs(g['info'][e][fin] - ref_info[fin]) / np.maximum(np.abs(ref_info[fin]), 1e-6)
                assert np.all(err <= 1e-5), (t, e, err.max())
    finally:
        eng.close()
        torch.cuda.set_stream(torch.cuda.default_stream())


@pytest.mark.parametrize('world,compact,pipelined,problem', [
    (2, True, False, 'optimize'), (3, True, True, 'optimize'), (2, False, True, 'optimize'),
    (2, False, False, 'multi'), (3, False, True, 'multi')])
def test_world_n_on_one_gpu_matches_world_1(tmp_path, world, compact, pipelined, problem):
    """N > 1 data movement with real HIP engine shards: `world` rank
    processes on this one GPU (tests/gpu_dist_worker.py), each stepping its
    contiguous shard of 37 envs (uneven splits) and all-gathering the packed
    record every step through the product's ShardedEnvs (gloo carries the
    collective between processes on one device); the gathered global arrays
    of every step must equal a 1-rank run bit for bit (seeds = global index,
    so the sharding is invisible in the results); `multi`: config 5's
    multi-agent engine, 13 envs x 4 agents."""
    import subprocess
    import sys
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'gpu_dist_worker.py')

    def run(n, out):
        with socket.socket() as s:
            s.bind(('127.0.0.1', 0))
            port = s.getsockname()[1]
        procs = []
        for r in range(n):
            env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), MASTER_ADDR='127.0.0.1',
                       MASTER_PORT=str(port), LOCAL_RANK='0')
            procs.append(subprocess.Popen([sys.executable, worker, str(out), str(int(compact)),
                                           str(int(pipelined)), problem], env=env))
        codes = []
        for p in procs:
            try:
                codes.append(p.wait(timeout=150))
            except subprocess.TimeoutExpired:
                for q in procs:
                    q.kill()
                raise
        assert codes == [0] * n, codes
        return np.load(out)

    one = run(1, tmp_path / 'w1.npz')
    many = run(world, tmp_path / 'wn.npz')
    for k in one.files:
        assert np.array_equal(one[k], many[k], equal_nan=True), k
    if problem == 'multi':
        assert one['obs'].shape == (46, 52, 15) and one['done'].any()
    else:
        assert one['obs'].shape == (44, 37, 41) and one['done'].any()


@pytest.mark.parametrize('world,compact,pipelined', [(2, True, True), (3, True, False), (3, False, True)])
def test_chunk_schedule_world_n_on_one_gpu_matches_per_step(tmp_path, world, compact, pipelined):
    """The chunk schedule with real HIP engine shards: `world`
    rank processes on this one GPU, each running its shard of 37 envs as
    persistent 7-step launches into a slot's records and all-gathering each
    slot with ONE collective (the 2-step tail out of place); every step's
    gathered global arrays must equal a 1-rank run stepping ONE launch and
    ONE gather per step, bit for bit -- the persistent kernel, the strided
    records and the chunk gather together are invisible in the results."""
    import subprocess
    import sys
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'gpu_dist_worker.py')

    def run(n, out, mode, pipe):
        with socket.socket() as s:
            s.bind(('127.0.0.1', 0))
            port = s.getsockname()[1]
        procs = []
        for r in range(n):
            env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), MASTER_ADDR='127.0.0.1',
                       MASTER_PORT=str(port), LOCAL_RANK='0')
            procs.append(subprocess.Popen([sys.executable, worker, str(out), str(int(compact)),
                                           str(int(pipe)), mode], env=env))
        codes = []
        for p in procs:
            try:
                codes.append(p.wait(timeout=150))
            except subprocess.TimeoutExpired:
                for q in procs:
                    q.kill()
                raise
        assert codes == [0] * n, codes
        return np.load(out)

    one = run(1, tmp_path / 'w1.npz', 'optimize', False)
    many = run(world, tmp_path / 'wn.npz', 'chunk', pipelined)
    for k in one.files:
        assert np.array_equal(one[k], many[k], equal_nan=True), k
    assert one['obs'].shape == (44, 37, 41) and one['done'].any()


def test_bench_n_ranks_rehearsal_on_one_gpu():
    """bench.py's N-rank path end to end on a 1-GPU box (--one-gpu-rehearsal:
    2 ranks on cuda:0, the collectives on gloo, so the gathers run eager):
    launcher, shards, the chunk schedule (persistent 4-step launches, one
    gather per chunk, a shorter tail chunk) as `value`, the per-step gathers
    in both schedules beside it, max-over-ranks timing and rank 0's one JSON
    line, marked as a rehearsal."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(root, 'bench.py'), '--gpus', '2', '--one-gpu-rehearsal',
           '--steps', '10', '--warmup', '2', '--chunk-steps', '4', '--no-cpu-baseline',
           '--no-measure-traffic', '--envs', '512']
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=root)
    assert res.returncode == 0, res.stderr[-2000:]
    lines = [json.loads(l) for l in res.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, res.stdout[-2000:]
    line = lines[0]
    assert line['n_gpus'] == 2 and 'rehearsal' in line
    assert line['config']['global_envs'] == 1024
    assert line['value_gather_serial_per_step'] > 0 and line['value_gather_pipelined_per_step'] > 0
    assert line['gather_mode'] == 'chunk_pipelined' and line['gather_chunk_steps'] == 4
    assert line['value_gather_chunk_serial'] > 0
    assert line['value'] == line['value_gather_chunk_pipelined']
    assert line['gather_record'] == 'compact'

"""One rank of the world-N rehearsal on ONE GPU
(tests/test_gpu_distributed.py::test_world_n_on_one_gpu_matches_world_1): the
product's ShardedEnvs over a real HIP engine shard on cuda:0, the per-step
all-gather of the packed (compact) record as a real collective between the
rank processes (gloo: RCCL does not put two ranks on one device), serial or
pipelined over two buffers as bench.py runs it.  Rank 0 writes the gathered
global arrays of every step to OUT.

    RANK=r WORLD_SIZE=n MASTER_ADDR=127.0.0.1 MASTER_PORT=p \\
        python tests/gpu_dist_worker.py OUT COMPACT(0|1) PIPELINED(0|1) [multi]

``multi``: config 5's MultiOptEngine (13 envs x 4 agents, func4, H = 5,
max_batches = 30) instead of Optimize-v0.  ``chunk``: the chunk schedule
(ShardedEnvs(chunk=7): one persistent K-step launch per chunk into a slot of
7 records, then ONE all-gather of the slot; the last chunk of 2 steps
gathers out of place), pipelined over the two slots or serial.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

E, STEPS, BASE = 37, 44, 500


def main():
    out_path, compact, pipelined = sys.argv[1], sys.argv[2] == '1', sys.argv[3] == '1'
    if len(sys.argv) > 4 and sys.argv[4] == 'multi':
        return main_multi(out_path, pipelined)
    if len(sys.argv) > 4 and sys.argv[4] == 'chunk':
        return main_chunk(out_path, compact, pipelined)
    rank, world = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
    import torch
    import torch.distributed as dist
    from custom_envs_amd.distributed import ShardedEnvs, shard_range
    from custom_envs_amd.engine import OptimizeEngine
    dist.init_process_group('gloo', rank=rank, world_size=world)
    torch.cuda.set_device(0)
    d = np.load(os.path.join(HERE, 'golden', 'lr_256x10.npz'))
    lo, hi = shard_range(E, world, rank)
    eng = OptimizeEngine(d['features'], d['targets'], num_envs=hi - lo)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    eng.set_stream(stream.cuda_stream)
    shard = ShardedEnvs(eng, E, rank, world, slots=2, collective=True, compact=compact)
    assert (shard.lo, shard.hi) == (lo, hi)
    shard.seed(BASE)
    shard.reset(0)
    acts = np.random.RandomState(8).normal(0, 0.02, (STEPS, E, 20)).astype(np.float32)
    dacts = torch.from_numpy(np.ascontiguousarray(acts[:, lo:hi])).cuda()
    keys = ('obs', 'done', 'episode_len', 'reward', 'objective', 'accuracy')
    got, pending = {}, [None, None]

    def collect(entry):
        work, res, t = entry
        work.wait()
        got[t] = {k: res[k].cpu().numpy() for k in keys}

    for t in range(STEPS):
        slot = t & 1 if pipelined else 0
        if pending[slot] is not None:
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
    if rank == 0:
        np.savez(out_path, **{k: np.stack([got[t][k] for t in range(STEPS)]) for k in keys})
    eng.close()
    dist.destroy_process_group()
    return 0


def main_chunk(out_path, compact, pipelined, chunk=7):
    rank, world = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
    import torch
    import torch.distributed as dist
    from custom_envs_amd.distributed import ShardedEnvs, shard_range
    from custom_envs_amd.engine import OptimizeEngine
    dist.init_process_group('gloo', rank=rank, world_size=world)
    torch.cuda.set_device(0)
    d = np.load(os.path.join(HERE, 'golden', 'lr_256x10.npz'))
    lo, hi = shard_range(E, world, rank)
    eng = OptimizeEngine(d['features'], d['targets'], num_envs=hi - lo)
    assert eng.persistent, eng.many_kernel
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    eng.set_stream(stream.cuda_stream)
    shard = ShardedEnvs(eng, E, rank, world, slots=2, collective=True, compact=compact, chunk=chunk)
    shard.seed(BASE)
    shard.reset(0)
    acts = np.random.RandomState(8).normal(0, 0.02, (STEPS, E, 20)).astype(np.float32)
    dacts = torch.from_numpy(np.ascontiguousarray(acts[:, lo:hi])).cuda()
    keys = ('obs', 'done', 'episode_len', 'reward', 'objective', 'accuracy')
    got, pending = {}, [None, None]

    def collect(entry):
        work, steps, t0 = entry
        work.wait()
        for i, res in enumerate(steps):
            got[t0 + i] = {k: res[k].cpu().numpy() for k in keys}

    t0, c = 0, 0
    while t0 < STEPS:
        k = min(chunk, STEPS - t0)
        slot = c & 1 if pipelined else 0
        if pending[slot] is not None:
            collect(pending[slot])
            pending[slot] = None
        shard.rollout(dacts[t0:t0 + k], slot, k)
        steps, work = shard.gather_chunk(slot, async_op=True, k=k)
        pending[slot] = (work, steps, t0)
        if not pipelined:
            collect(pending[slot])
            pending[slot] = None
        t0 += k
        c += 1
    for slot in (0, 1):
        if pending[slot] is not None:
            collect(pending[slot])
    torch.cuda.synchronize()
    if rank == 0:
        np.savez(out_path, **{k: np.stack([got[t][k] for t in range(STEPS)]) for k in keys})
    eng.close()
    dist.destroy_process_group()
    return 0


def main_multi(out_path, pipelined):
    rank, world = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
    import torch
    import torch.distributed as dist
    from custom_envs_amd.distributed import ShardedEnvs, shard_range
    from custom_envs_amd.multi_engine import MultiOptEngine
    dist.init_process_group('gloo', rank=rank, world_size=world)
    torch.cuda.set_device(0)
    En, P, H, MB, T = 13, 4, 5, 30, 45
    lo, hi = shard_range(En, world, rank)
    eng = MultiOptEngine(hi - lo, 'func4', max_batches=MB, max_history=H)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    eng.set_stream(stream.cuda_stream)
    shard = ShardedEnvs(eng, En, rank, world, slots=2, collective=True)
    rs = np.random.RandomState(12)
    lows = rs.uniform(-1.5, 1.5, En)
    acts = np.stack([rs.uniform(lows[e], lows[e] + 1.5, (T, P)) for e in range(En)], 1)
    acts = acts.astype(np.float32).reshape(T, En * P)
    dacts = torch.from_numpy(np.ascontiguousarray(acts[:, lo * P:hi * P])).cuda()
    keys = ('obs', 'done', 'episode_len', 'reward', 'info')
    shard.reset(0)
    got = {-1: {k: v.cpu().numpy() for k, v in shard.gather(0).snapshot().items() if k in keys}}
    for t in range(T):
        slot = t & 1 if pipelined else 0
        shard.step(dacts[t], slot)
        g = shard.gather(slot).snapshot()
        torch.cuda.synchronize()
        got[t] = {k: g[k].cpu().numpy() for k in keys}
    if rank == 0:
        np.savez(out_path, **{k: np.stack([got[t][k] for t in range(-1, T)]) for k in keys})
    eng.close()
    dist.destroy_process_group()
    return 0


if __name__ == '__main__':
    sys.exit(main())

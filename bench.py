"""Benchmark: vectorised Optimize-v0 env-steps/s on MI355X (BASELINE.json metric).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--envs E] [--precision f64|f32]

One "step" = one VecEnv.step of every env: the fused HIP kernel advances
E = 4096 envs per GPU (weak scaling: N GPUs own N*4096 envs, contiguous
shards, seed = global env index) of the 256x10 softmax-regression problem by
one Optimize-v0 step, auto-reset included.  Actions are device-resident
([S][E][P] float32 in HBM, a different action block per step) and the
outputs (obs/reward/done/info) are written to HBM every step.  Steps are
replayed as hipGraphs of S consecutive launches (ce_step_many).  Envs are
independent, so there is no data-path collective; ``--gather`` adds the
optional RCCL all-gather of the packed outputs per step (reported apart).

Rank 0 prints ONE JSON line.  With N>1 run under
``python -m torch.distributed.run --nproc-per-node N bench.py --gpus N``.
"""
import argparse
import json
import os
import resource
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = 'vectorised env-steps/sec, Optimize-v0 @4096 envs, 1/2/4/8 MI355X vs host CPU'
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md chip table (spec)
F64_VALU_PEAK_TFLOPS = 78.6


def algorithmic_bytes_per_env_step(n_params, precision):
    """Bytes one env-step must move given the state it carries.

    action read 4P; W read+write and G read+write at sizeof(T) each; loss
    scalar (f64) read+write 16; step counter read+write 8; obs write
    4(2P+1); reward/objective/accuracy/episode_len 16; done 1.
    The dataset (20 KB, L2-resident, shared by all envs) and W0 (reset
    only) are excluded.
    """
    t = 8 if precision == 'f64' else 4
    return 4 * n_params + 4 * t * n_params + 16 + 8 + 4 * (2 * n_params + 1) + 16 + 1


def parse():
    p = argparse.ArgumentParser()
    p.add_argument('--gpus', type=int, default=1)
    p.add_argument('--steps', type=int, default=2000)
    p.add_argument('--warmup', type=int, default=200)
    p.add_argument('--envs', type=int, default=4096, help='envs per GPU')
    p.add_argument('--precision', default='f64', choices=['f64', 'f32'])
    p.add_argument('--graph-steps', type=int, default=250, help='steps per hipGraph replay')
    p.add_argument('--gather', action='store_true', help='all-gather outputs every step')
    p.add_argument('--cpu-seconds', type=float, default=15.0, help='CPU baseline budget')
    p.add_argument('--no-cpu-baseline', action='store_true')
    p.add_argument('--profile-only', action='store_true',
                   help='run the timed steps only (for rocprofv3)')
    return p.parse_args()


def lr_dataset():
    from custom_envs_amd.data import load_data
    seq = load_data('gaussians_256x10', batch_size=None)
    return seq.features, seq.targets


def cpu_baseline(features, targets, envs, budget_s):
    """The reference's NumPy path restated: oracle envs under ThreadVecEnv."""
    from oracle.optimize import Optimize as OracleEnv
    from oracle.vectorize import ThreadVecEnv
    soft, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
    want = 4 * envs + 256
    if soft < want and (hard == resource.RLIM_INFINITY or hard >= want):
        resource.setrlimit(resource.RLIMIT_NOFILE, (want, hard))
        soft = want
    n = min(envs, max(1, (soft - 256) // 4))

    def factory(seed):
        def make():
            env = OracleEnv(features, targets)
            env.seed(seed)
            return env
        return make

    venv = ThreadVecEnv([factory(i) for i in range(n)])
    venv.reset()
    rs = np.random.RandomState(0)
    acts = rs.normal(0, 0.01, (n, 20)).astype(np.float32)
    venv.step(acts)                                   # warm-up
    steps = 0
    wall0, cpu0 = time.perf_counter(), time.process_time()
    while True:
        venv.step(acts)
        steps += 1
        wall = time.perf_counter() - wall0
        if wall >= budget_s or steps >= 1000:
            break
    cpu = time.process_time() - cpu0
    venv.close()
    return {'value': n * steps / wall, 'unit': 'env-steps/s',
            'cores': max(1, int(round(cpu / wall))), 'kind': 'port',
            'sample': '%d envs x %d steps of ThreadVecEnv (1 thread + mp.Pipe per env, '
                      'pickled step msgs, np.stack) over the float64 numpy oracle '
                      'Optimize env; %.1f s wall, %.1f s CPU; os.cpu_count()=%d'
                      % (n, steps, wall, cpu, os.cpu_count())}


def main():
    args = parse()
    import torch
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local_rank = int(os.environ.get('LOCAL_RANK', '0'))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group('nccl', device_id=torch.device('cuda', local_rank))
    else:
        torch.cuda.set_device(0)
    device = torch.cuda.current_device()

    from custom_envs_amd.engine import OptimizeEngine
    features, targets = lr_dataset()
    E = args.envs
    eng = OptimizeEngine(features, targets, num_envs=E, precision=args.precision,
                         device=device)
    P = eng.act_dim
    eng.seed([rank * E + i for i in range(E)])
    stream = torch.cuda.Stream()          # a real stream: graphs cannot capture the null stream
    torch.cuda.set_stream(stream)
    eng.set_stream(stream.cuda_stream)
    out = eng.alloc_device_outputs()
    S = max(1, min(args.graph_steps, args.steps))
    gen = torch.Generator(device='cuda').manual_seed(1234 + rank)
    actions = torch.randn((S, E, P), generator=gen, device='cuda') * 0.01
    eng.reset_device(out)

    packed = gathered = None
    if args.gather and dist is not None:
        rec = 2 * P + 1 + 5
        packed = torch.empty((E, rec), device='cuda')
        gathered = torch.empty((world * E, rec), device='cuda')

    def run(k):
        done = 0
        while done < k:
            n = min(S, k - done)
            if packed is None:
                eng.step_many_device(n, actions, out)
            else:
                for s in range(n):
                    eng.step_device(actions[s], out)
                    packed[:, :2 * P + 1] = out['obs']
                    packed[:, 2 * P + 1] = out['reward']
                    packed[:, 2 * P + 2] = out['done']
                    packed[:, 2 * P + 3] = out['objective']
                    packed[:, 2 * P + 4] = out['accuracy']
                    packed[:, 2 * P + 5] = out['episode_len']
                    dist.all_gather_into_tensor(gathered, packed)
            done += n

    run(args.warmup)
    torch.cuda.synchronize()
    if args.profile_only:
        run(args.steps)
        torch.cuda.synchronize()
        return

    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(args.steps)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device='cuda')
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # live kernel duration: HIP events around individual launches on the
    # engine's stream (= torch's current stream)
    n_ev = 200
    eng.step_many_device(S, actions, out)   # backlog: events then time the kernels, not the host
    starts = [torch.cuda.Event(enable_timing=True) for _ in range(n_ev)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(n_ev)]
    for i in range(n_ev):
        starts[i].record(stream)
        eng.step_device(actions[i % S], out)
        ends[i].record(stream)
    torch.cuda.synchronize()
    kernel_ms = float(np.median([s.elapsed_time(e) for s, e in zip(starts, ends)]))
    kernel_ms_mean = float(np.mean([s.elapsed_time(e) for s, e in zip(starts, ends)]))

    # host-loop rate (numpy actions in, numpy outputs out: PCIe-inclusive)
    host_rate = None
    if rank == 0 and world == 1:
        heng = OptimizeEngine(features, targets, num_envs=E, precision=args.precision,
                              device=device)
        heng.seed(list(range(E)))
        heng.reset()
        hact = np.random.RandomState(5).normal(0, 0.01, (E, P)).astype(np.float32)
        for _ in range(20):
            heng.step(hact)
        h0 = time.perf_counter()
        hn = 300
        for _ in range(hn):
            o = heng.step(hact)
            o['obs'].copy()
        host_rate = E * hn / (time.perf_counter() - h0)
        heng.close()

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(features, targets, E, args.cpu_seconds)

    if rank == 0:
        env_steps = world * E * args.steps
        bpe = algorithmic_bytes_per_env_step(P, args.precision)
        achieved_gbs = bpe * E / (kernel_ms * 1e-3) / 1e9
        traffic = None
        pmc_path = os.path.join(ROOT, 'profiles', 'pmc_latest.json')
        if os.path.exists(pmc_path):
            with open(pmc_path) as fh:
                pmc = json.load(fh)
            if pmc.get('envs') == E and pmc.get('precision') == args.precision:
                traffic = pmc.get('hbm_bytes_per_launch')
        line = {
            'metric': METRIC,
            'value': env_steps / elapsed,
            'unit': 'env-steps/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': elapsed / args.steps * 1e3,
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': None,
            'dtype': args.precision,
            'data': 'synthetic: make_classification(256 x 10, random_state=0) one-hot(2); '
                    'actions N(0, 0.01) float32 generated on device',
            'config': {
                'workload': 'Optimize-v0 softmax-regression 256x10 (P=20, obs 41), '
                            '%d envs per GPU, B=N=256, 40-step episodes with in-kernel '
                            'auto-reset, device-resident actions/outputs' % E,
                'envs_per_gpu': E, 'global_envs': world * E, 'n_rows': 256,
                'n_features': 10, 'n_classes': 2, 'batch_size': 256,
                'graph_steps': S, 'parallelism': 'env-sharded x%d (no collective)' % world
                if packed is None else 'env-sharded x%d + all-gather/step' % world,
            },
            'roofline': {
                'bound': 'hbm', 'achieved': achieved_gbs, 'peak': HBM_PEAK_GBS,
                'unit': 'GB/s', 'frac': achieved_gbs / HBM_PEAK_GBS,
                'traffic': traffic,
                'bytes_per_env_step': bpe, 'kernel_ms_median': kernel_ms,
                'kernel_ms_mean': kernel_ms_mean,
                'kernel': 'ce::optimize_step_kernel<%s,10,2>' % (
                    'double' if args.precision == 'f64' else 'float'),
                # the limiter is the f64/f32 VALU, not HBM:
                # algorithmic FLOPs 2NFK (logits) + 2NFK (X^T(P-Y)) + 5NK
                'flops_per_env_step': 4 * 256 * P + 5 * 256 * 2,
                'valu_tflops': (4 * 256 * P + 5 * 256 * 2) * E / (kernel_ms * 1e-3) / 1e12,
                'valu_peak_tflops': F64_VALU_PEAK_TFLOPS if args.precision == 'f64' else 157.3,
            },
            'cpu_baseline': cpu,
            'host_loop_env_steps_per_s': host_rate,
        }
        print(json.dumps(line))
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()

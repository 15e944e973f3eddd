"""Benchmark: vectorised Optimize-v0 env-steps/s on MI355X (BASELINE.json metric).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--envs E] [--precision f64|f32]
                  [--workload optimize|multi] [--gather]

One "step" = one VecEnv.step of every env: the fused HIP kernel advances
E = 4096 envs per GPU (weak scaling: N GPUs own N*4096 envs, contiguous
shards, seed = global env index) of the 256x10 softmax-regression problem by
one Optimize-v0 step, auto-reset included.  Actions are device-resident
([S][E][P] float32 in HBM, a different action block per step) and the
outputs (obs/reward/done/info) are written to HBM every step.  Steps are
replayed as hipGraphs of S consecutive launches (ce_step_many).  Envs are
independent, so there is no data-path collective; ``--gather`` adds the
north star's RCCL all-gather of the packed outputs every step (config 4,
custom_envs_amd/distributed.py), reported as its own line.

``--workload multi`` measures config 5 instead: MultiOptLRs-v0 (4 agents,
4-D Rosenbrock pairs, H=5, max_batches=400) behind OptVecEnv, 1024 envs per
GPU, actions uniform(1, 3) as in SURVEY 8d.  ``--workload mlp`` measures
config 3: Optimize-v0 over the 784 -> 64 -> 10 MLP on 1024 MNIST-sized
synthetic rows, B = 32, 4096 envs, float32 on MFMA (roofline bound "mfma").

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
METRIC_MULTI = ('vectorised env-steps/sec, MultiOptLRs-v0 (4 agents) via OptVecEnv, '
                'config 5, MI355X vs host CPU')
METRIC_MLP = ('vectorised env-steps/sec, Optimize-v0 over the 784-64-10 MLP @4096 envs, '
              'config 3, MI355X vs host CPU')
METRIC_NN = ('vectorised env-steps/sec, MultiOptLRs-v0 over the OptimizeNN (256, 256) network '
             'via OptVecEnv, one agent per parameter, 1/2/4/8 MI355X vs host CPU')
MFMA_F32_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md chip table (spec)
F64_VALU_PEAK_TFLOPS = 78.6


def algorithmic_bytes_per_env_step(n_params, precision):
    """Bytes one Optimize env-step must move given the state it carries.

    action read 4P; W read+write and G read+write at sizeof(T) each; loss
    scalar (f64) read+write 16; step counter read+write 8; obs write
    4(2P+1); reward/objective/accuracy/episode_len 16; done 1.
    The dataset (20 KB, L2-resident, shared by all envs) and W0 (reset
    only) are excluded.
    """
    t = 8 if precision == 'f64' else 4
    return 4 * n_params + 4 * t * n_params + 16 + 8 + 4 * (2 * n_params + 1) + 16 + 1


def multi_bytes_per_env_step(P, H, raw=5):
    """Bytes one MultiOptLRs env-step moves: actions 4P;
    theta and gradient r/w 16P; raw history: newest loss/grad/weight written
    (4 + 8P), the previous weights read (4P), all `raw` losses and gradients
    read for the info means (raw*(4 + 4P)); adjusted history (float64): one
    entry written (8 + 16P), H entries read for the observation (H*(8 + 16P));
    step r/w 8; outputs: obs 4*3H*P, reward 4P, done P, info 56, length 4."""
    return (4 * P + 16 * P + (4 + 8 * P) + 4 * P + raw * (4 + 4 * P) + (8 + 16 * P)
            + H * (8 + 16 * P) + 8 + 12 * H * P + 4 * P + P + 56 + 4)


def mlp_flops(F=784, H=64, K=10, B=32, N=1024):
    """Algorithmic FLOPs of one config-3 env-step: minibatch forward
    2B(FH + HK), backward 2BFH + 4BHK, full-data info forward 2N(FH + HK)."""
    train = 2 * B * (F * H + H * K) + 2 * B * F * H + 4 * B * H * K
    info = 2 * N * (F * H + H * K)
    return train, info


def mlp_train_bytes(P):
    """HBM bytes of the train kernel per env-step: action 4P, W r/w 8P, G (float64)
    r/w 16P, obs 4(2P+1), L r/w 16, step r/w 8, reward/done/length 9."""
    return 4 * P + 8 * P + 16 * P + 4 * (2 * P + 1) + 16 + 8 + 9


def nn_bytes_per_env_step(P, H=5):
    """Algorithmic HBM bytes per env-step of MultiOptLRs over the network
    (the job's own traffic, not the engine's): theta read and
    theta' written 8P, actions 4P, the previous gradient read and the new
    one written 8P, the adjusted w~/g~ rings read 8(H-1)P and written 8P,
    obs rows 4*3H*P, reward 4P and done P."""
    return 8 * P + 4 * P + 8 * P + 8 * (H - 1) * P + 8 * P + 12 * H * P + 5 * P


def nn_flops_per_env_step(dims):
    """MFMA/VALU FLOPs of two forward+backward passes on a 32-row batch:
    forward 2B sum(d_l d_l+1), dW 2B sum(d_l d_l+1), dH 2B sum_{l>0}(d_l d_l+1)."""
    pairs = [a * b for a, b in zip(dims[:-1], dims[1:])]
    one = 2 * 32 * (2 * sum(pairs) + sum(pairs[1:]))
    return 2 * one


def parse():
    p = argparse.ArgumentParser()
    p.add_argument('--gpus', type=int, default=1)
    p.add_argument('--steps', type=int, default=2000)
    p.add_argument('--warmup', type=int, default=200)
    p.add_argument('--envs', type=int, default=None,
                   help='envs per GPU (default 4096 optimize, 1024 multi)')
    p.add_argument('--workload', default='optimize', choices=['optimize', 'multi', 'mlp', 'nn'])
    p.add_argument('--precision', default='f64', choices=['f64', 'f32'])
    p.add_argument('--graph-steps', type=int, default=250, help='steps per hipGraph replay')
    p.add_argument('--gather', action='store_true', help='all-gather outputs every step')
    p.add_argument('--cpu-seconds', type=float, default=15.0, help='CPU baseline budget')
    p.add_argument('--no-cpu-baseline', action='store_true')
    p.add_argument('--profile-only', action='store_true',
                   help='run the timed steps only (for rocprofv3)')
    args = p.parse_args()
    if args.envs is None:
        args.envs = {'multi': 1024, 'nn': 1024}.get(args.workload, 4096)
    return args


def lr_dataset():
    from custom_envs_amd.data import load_data
    seq = load_data('gaussians_256x10', batch_size=None)
    return seq.features, seq.targets


def _raise_fd_limit(envs):
    soft, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
    want = 4 * envs + 256
    if soft < want and (hard == resource.RLIM_INFINITY or hard >= want):
        resource.setrlimit(resource.RLIMIT_NOFILE, (want, hard))
        soft = want
    return min(envs, max(1, (soft - 256) // 4))


def _time_cpu(venv, acts, budget_s):
    venv.step(acts)                                   # warm-up
    steps = 0
    wall0, cpu0 = time.perf_counter(), time.process_time()
    while True:
        venv.step(acts)
        steps += 1
        wall = time.perf_counter() - wall0
        if wall >= budget_s or steps >= 1000:
            break
    return steps, wall, time.process_time() - cpu0


def cpu_baseline(features, targets, envs, budget_s):
    """The reference's NumPy path restated: oracle envs under ThreadVecEnv."""
    from oracle.optimize import Optimize as OracleEnv
    from oracle.vectorize import ThreadVecEnv
    n = _raise_fd_limit(envs)

    def factory(seed):
        def make():
            env = OracleEnv(features, targets)
            env.seed(seed)
            return env
        return make

    venv = ThreadVecEnv([factory(i) for i in range(n)])
    venv.reset()
    acts = np.random.RandomState(0).normal(0, 0.01, (n, 20)).astype(np.float32)
    steps, wall, cpu = _time_cpu(venv, acts, budget_s)
    venv.close()
    return {'value': n * steps / wall, 'unit': 'env-steps/s',
            'cores': max(1, int(round(cpu / wall))), 'kind': 'port',
            'sample': '%d envs x %d steps of ThreadVecEnv (1 thread + mp.Pipe per env, '
                      'pickled step msgs, np.stack) over the float64 numpy oracle '
                      'Optimize env; %.1f s wall, %.1f s CPU; os.cpu_count()=%d'
                      % (n, steps, wall, cpu, os.cpu_count())}


def cpu_baseline_multi(envs, budget_s):
    """OptVecEnv restated (ThreadVecEnv of OptEnvRunner over MultiOptLRs)."""
    from oracle.multioptlrs import MultiOptLRs, OptVecEnv
    n = _raise_fd_limit(envs)
    venv = OptVecEnv([lambda: MultiOptLRs(4, max_batches=400, max_history=5)] * n)
    venv.reset()
    acts = np.random.RandomState(7).uniform(1, 3, (4 * n, 1)).astype(np.float32)
    steps, wall, cpu = _time_cpu(venv, acts, budget_s)
    venv.close()
    return {'value': n * steps / wall, 'unit': 'env-steps/s',
            'cores': max(1, int(round(cpu / wall))), 'kind': 'port',
            'sample': '%d envs x 4 agents x %d steps of OptVecEnv over ThreadVecEnv '
                      '(1 thread + mp.Pipe per env) around the numpy oracle MultiOptLRs; '
                      '%.1f s wall, %.1f s CPU; os.cpu_count()=%d'
                      % (n, steps, wall, cpu, os.cpu_count())}


def build_optimize(args, torch, device, rank, world):
    from custom_envs_amd.engine import OptimizeEngine
    features, targets = lr_dataset()
    E = args.envs
    eng = OptimizeEngine(features, targets, num_envs=E, precision=args.precision,
                         device=device)
    eng.seed([rank * E + i for i in range(E)])
    gen = torch.Generator(device='cuda').manual_seed(1234 + rank)
    S = max(1, min(args.graph_steps, args.steps))
    actions = torch.randn((S, E, eng.act_dim), generator=gen, device='cuda') * 0.01
    return eng, actions, S


def mlp_dataset():
    from custom_envs_amd.data import load_data
    seq = load_data('mnist_synthetic', batch_size=32)
    return seq.features, seq.targets


def build_mlp(args, torch, device, rank, world, phases=None):
    from custom_envs_amd.engine import OptimizeEngine
    features, targets = mlp_dataset()
    E = args.envs
    if phases:
        os.environ['CE_MLP_PHASES'] = phases
    try:
        eng = OptimizeEngine(features, targets, num_envs=E, batch_size=32, model='mlp',
                             device=device)
    finally:
        os.environ.pop('CE_MLP_PHASES', None)
    eng.seed([rank * E + i for i in range(E)])
    gen = torch.Generator(device='cuda').manual_seed(4321 + rank)
    S = 2                                  # two action blocks of [E][P] (833 MB each)
    actions = torch.randn((S, E, eng.act_dim), generator=gen, device='cuda') * 1e-3
    return eng, actions, S


def cpu_baseline_mlp(envs, budget_s):
    """Oracle float32 MLP Optimize envs under the restated ThreadVecEnv."""
    from oracle.optimize import Optimize as OracleEnv
    from oracle.vectorize import ThreadVecEnv
    features, targets = mlp_dataset()
    n = min(_raise_fd_limit(envs), 64)

    def factory(seed):
        def make():
            env = OracleEnv(features, targets, batch_size=32, model='mlp')
            env.seed(seed)
            return env
        return make

    venv = ThreadVecEnv([factory(i) for i in range(n)])
    venv.reset()
    acts = np.random.RandomState(0).normal(0, 1e-3, (n, 50890)).astype(np.float32)
    steps, wall, cpu = _time_cpu(venv, acts, budget_s)
    venv.close()
    return {'value': n * steps / wall, 'unit': 'env-steps/s',
            'cores': max(1, int(round(cpu / wall))), 'kind': 'port',
            'sample': '%d envs x %d steps of ThreadVecEnv over the numpy oracle Optimize env '
                      'with the float32 784-64-10 MLP (BLAS sgemm); %.1f s wall, %.1f s CPU; '
                      'os.cpu_count()=%d' % (n, steps, wall, cpu, os.cpu_count())}


def build_multi(args, torch, device, rank, world):
    from custom_envs_amd.multi_engine import MultiOptEngine
    E = args.envs
    eng = MultiOptEngine(E, 'func4', max_batches=400, max_history=5, device=device)
    gen = torch.Generator(device='cuda').manual_seed(7 + rank)
    S = max(1, min(args.graph_steps, args.steps))
    actions = torch.rand((S, E * eng.n_params), generator=gen, device='cuda') * 2.0 + 1.0
    return eng, actions, S


def build_nn(args, torch, device, rank, world):
    from custom_envs_amd.multi_engine import NNMultiEngine
    E = args.envs
    eng = NNMultiEngine(E, max_batches=400, max_history=5, device=device,
                        seeds=[rank * E + i for i in range(E)])
    gen = torch.Generator(device='cuda').manual_seed(11 + rank)
    S = 2                                 # two action blocks of [E*P] rows
    actions = torch.rand((S, E * eng.n_params), generator=gen, device='cuda') * 1.5 + 1.0
    return eng, actions, S


def cpu_baseline_nn(budget_s):
    """The reference's path restated: OptVecEnv (ThreadVecEnv of OptEnvRunner)
    over the numpy oracle MultiOptLRs with the OptimizeNN (256, 256) problem."""
    from custom_envs_amd.data import load_data
    from oracle.multioptlrs import OptVecEnv
    from oracle.multinn import MultiOptLRsNN
    ds = load_data('iris_synthetic', batch_size=32)
    n = 2

    def make(seed):
        def build():
            env = MultiOptLRsNN(ds.features, ds.targets, hidden=(256, 256), max_batches=400)
            env.seed(seed)
            return env
        return build
    venv = OptVecEnv([make(i) for i in range(n)])
    venv.reset()
    acts = np.random.RandomState(11).uniform(1, 2.5, (venv.num_envs, 1)).astype(np.float32)
    steps, wall, cpu = _time_cpu(venv, acts, budget_s)
    venv.close()
    return {'value': n * steps / wall, 'unit': 'env-steps/s',
            'cores': max(1, int(round(cpu / wall))), 'kind': 'port',
            'sample': '%d envs x 67843 agents x %d steps of OptVecEnv over ThreadVecEnv around '
                      'the numpy oracle MultiOptLRs(problem=nn); %.1f s wall, %.1f s CPU; '
                      'os.cpu_count()=%d' % (n, steps, wall, cpu, os.cpu_count())}


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
    multi = args.workload == 'multi'
    mlp = args.workload == 'mlp'
    nn = args.workload == 'nn'
    builder = {'optimize': build_optimize, 'multi': build_multi, 'mlp': build_mlp,
               'nn': build_nn}[args.workload]
    eng, actions, S = builder(args, torch, device, rank, world)
    E = args.envs
    stream = torch.cuda.Stream()          # a real stream: graphs cannot capture the null stream
    torch.cuda.set_stream(stream)
    eng.set_stream(stream.cuda_stream)
    shard = None
    if args.gather and dist is not None:
        from custom_envs_amd.distributed import ShardedEnvs
        shard = ShardedEnvs(eng, world * E, rank, world)
        out = shard.out                   # the engine writes straight into the packed buffer
    else:
        out = eng.alloc_device_outputs()
    eng.reset_device(out)

    def run(k):
        done = 0
        while done < k:
            n = min(S, k - done)
            if shard is None:
                eng.step_many_device(n, actions, out)
            else:
                for s in range(n):
                    eng.step_device(actions[s], out)
                    shard.gather()
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

    # live kernel duration: HIP events on the engine's stream (= torch's
    # current stream) around graph replays of S back-to-back step launches,
    # divided by S: the per-launch time on the stream, i.e. the kernel plus
    # its share of the inter-kernel boundary (rocprofv3's kernel-only average
    # is the same minus that gap; profiles/ holds both)
    n_ev = 8
    eng.step_many_device(S, actions, out)   # backlog: events then time the kernels, not the host
    starts = [torch.cuda.Event(enable_timing=True) for _ in range(n_ev)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(n_ev)]
    for i in range(n_ev):
        starts[i].record(stream)
        eng.step_many_device(S, actions, out)
        ends[i].record(stream)
    torch.cuda.synchronize()
    times = [s.elapsed_time(e) / S for s, e in zip(starts, ends)]
    kernel_ms, kernel_ms_mean = float(np.median(times)), float(np.mean(times))
    phase_ms = {}
    if mlp and rank == 0:
        # each MLP kernel alone (CE_MLP_PHASES engines), same events method
        for phase in ('train', 'info'):
            peng, pact, _ = build_mlp(args, torch, device, rank, world, phases=phase)
            peng.set_stream(stream.cuda_stream)
            pout = peng.alloc_device_outputs()
            peng.reset_device(pout)
            for i in range(3):
                peng.step_device(pact[i % 2], pout)
            n_ph = 20
            st = [torch.cuda.Event(enable_timing=True) for _ in range(n_ph)]
            en = [torch.cuda.Event(enable_timing=True) for _ in range(n_ph)]
            for i in range(n_ph):
                st[i].record(stream)
                peng.step_device(pact[i % 2], pout)
                en[i].record(stream)
            torch.cuda.synchronize()
            phase_ms[phase] = float(np.median([a.elapsed_time(b) for a, b in zip(st, en)]))
            peng.close()
            del pact, pout

    host_rate = None
    if rank == 0 and world == 1 and args.workload == 'optimize':
        host_rate = host_loop_rate(args, device, E)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        if nn:
            cpu = cpu_baseline_nn(args.cpu_seconds)
        elif multi:
            cpu = cpu_baseline_multi(E, args.cpu_seconds)
        elif mlp:
            cpu = cpu_baseline_mlp(E, args.cpu_seconds)
        else:
            cpu = cpu_baseline(*lr_dataset(), E, args.cpu_seconds)

    if rank == 0:
        if mlp:
            line = mlp_line(args, eng, world, E, S, elapsed, kernel_ms, kernel_ms_mean, shard,
                            phase_ms)
        elif nn:
            line = nn_line(args, eng, world, E, S, elapsed, kernel_ms, kernel_ms_mean, shard)
        else:
            line = (multi_line if multi else optimize_line)(args, eng, world, E, S, elapsed,
                                                            kernel_ms, kernel_ms_mean, shard)
        line['cpu_baseline'] = cpu
        if host_rate is not None:
            line['host_loop_env_steps_per_s'] = host_rate
        print(json.dumps(line))
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


def host_loop_rate(args, device, E):
    """numpy actions in, numpy outputs out: the PCIe-inclusive VecEnv rate."""
    from custom_envs_amd.engine import OptimizeEngine
    features, targets = lr_dataset()
    heng = OptimizeEngine(features, targets, num_envs=E, precision=args.precision,
                          device=device)
    heng.seed(list(range(E)))
    heng.reset()
    hact = np.random.RandomState(5).normal(0, 0.01, (E, heng.act_dim)).astype(np.float32)
    for _ in range(20):
        heng.step(hact)
    h0 = time.perf_counter()
    hn = 300
    for _ in range(hn):
        o = heng.step(hact)
        o['obs'].copy()
    rate = E * hn / (time.perf_counter() - h0)
    heng.close()
    return rate


def _common(args, world, E, S, elapsed, shard):
    return {
        'value': world * E * args.steps / elapsed,
        'unit': 'env-steps/s',
        'n_gpus': world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': elapsed / args.steps * 1e3,
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': None,
    }


def _pmc_traffic(E, precision, kernel):
    pmc_path = os.path.join(ROOT, 'profiles', 'pmc_latest.json')
    if not os.path.exists(pmc_path):
        return None
    with open(pmc_path) as fh:
        pmc = json.load(fh)
    entry = pmc.get(kernel) if isinstance(pmc.get(kernel), dict) else (
        pmc if kernel == 'optimize' else {})
    if entry.get('envs') == E and entry.get('precision') == precision:
        return entry.get('hbm_bytes_per_launch')
    return None


def optimize_line(args, eng, world, E, S, elapsed, kernel_ms, kernel_ms_mean, shard):
    P = eng.act_dim
    bpe = algorithmic_bytes_per_env_step(P, args.precision)
    achieved_gbs = bpe * E / (kernel_ms * 1e-3) / 1e9
    flops = 4 * 256 * P + 5 * 256 * 2
    line = {'metric': METRIC}
    line.update(_common(args, world, E, S, elapsed, shard))
    line.update({
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
            if shard is None else 'env-sharded x%d + all-gather/step' % world,
        },
        'roofline': {
            'bound': 'hbm', 'achieved': achieved_gbs, 'peak': HBM_PEAK_GBS,
            'unit': 'GB/s', 'frac': achieved_gbs / HBM_PEAK_GBS,
            'traffic': _pmc_traffic(E, args.precision, 'optimize'),
            'bytes_per_env_step': bpe, 'kernel_ms_median': kernel_ms,
            'kernel_ms_mean': kernel_ms_mean,
            'kernel': 'ce::' + eng.step_kernel,
            # the limiter is the f64/f32 VALU, not HBM:
            # algorithmic FLOPs 2NFK (logits) + 2NFK (X^T(P-Y)) + 5NK
            'flops_per_env_step': flops,
            'valu_tflops': flops * E / (kernel_ms * 1e-3) / 1e12,
            'valu_peak_tflops': F64_VALU_PEAK_TFLOPS if args.precision == 'f64' else 157.3,
        },
    })
    return line


def multi_line(args, eng, world, E, S, elapsed, kernel_ms, kernel_ms_mean, shard):
    P, H = eng.n_params, eng.max_history
    bpe = multi_bytes_per_env_step(P, H)
    achieved_gbs = bpe * E / (kernel_ms * 1e-3) / 1e9
    line = {'metric': METRIC_MULTI}
    line.update(_common(args, world, E, S, elapsed, shard))
    line.update({
        'agent_steps_per_s': P * world * E * args.steps / elapsed,
        'dtype': 'f32',
        'data': 'synthetic: 4-D Rosenbrock pairs from [-1.9, 2, -1.9, 2]; actions '
                'uniform(1, 3) float32 generated on device (lr 1e-3..1e-1)',
        'config': {
            'workload': 'MultiOptLRs-v0 x OptVecEnv, P=4 agents, H=5, max_batches=400, '
                        '%d envs (%d agent rows) per GPU, in-kernel auto-reset, '
                        'device-resident actions/outputs' % (E, E * P),
            'envs_per_gpu': E, 'global_envs': world * E, 'agents': P, 'max_history': H,
            'graph_steps': S, 'parallelism': 'env-sharded x%d (no collective)' % world
            if shard is None else 'env-sharded x%d + all-gather/step' % world,
        },
        'roofline': {
            'bound': 'hbm', 'achieved': achieved_gbs, 'peak': HBM_PEAK_GBS,
            'unit': 'GB/s', 'frac': achieved_gbs / HBM_PEAK_GBS,
            'traffic': _pmc_traffic(E, 'f32', 'multi'),
            'bytes_per_env_step': bpe, 'kernel_ms_median': kernel_ms,
            'kernel_ms_mean': kernel_ms_mean,
            'kernel': 'ce::multi_step_kernel<4>',
        },
    })
    return line


def nn_line(args, eng, world, E, S, elapsed, kernel_ms, kernel_ms_mean, shard):
    P, H = eng.n_params, eng.max_history
    bpe = nn_bytes_per_env_step(P, H)
    flops = nn_flops_per_env_step(eng.dims)
    achieved = bpe * E / (kernel_ms * 1e-3) / 1e9
    line = {'metric': METRIC_NN}
    line.update(_common(args, world, E, S, elapsed, shard))
    line.update({
        'agent_steps_per_s': P * world * E * args.steps / elapsed,
        'dtype': 'f32',
        'data': 'synthetic: iris-shaped 150 x 4, 3 classes (load_data default stand-in), '
                'batches of 32; glorot-uniform init per env seed; actions uniform(1, 2.5) '
                'float32 generated on device (lr 1e-3..3e-2)',
        'config': {
            'workload': 'MultiOptLRs-v0(problem=nn) x OptVecEnv: network 4-256-256-3 '
                        '(P=%d agents per env), H=5, max_batches=400, %d envs per GPU, '
                        'minibatch cycling with on-device reshuffle, in-kernel auto-reset, '
                        'device-resident actions/outputs' % (P, E),
            'envs_per_gpu': E, 'global_envs': world * E, 'agents': P, 'hidden': list(eng.hidden),
            'parallelism': 'env-sharded x%d (no collective)' % world,
        },
        'roofline': {
            'bound': 'hbm', 'achieved': achieved, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
            'frac': achieved / HBM_PEAK_GBS, 'traffic': None,
            'kernel': 'one step = ce::nn_grad_kernel, nn_update_kernel, nn_step_kernel, '
                      'nn_agent_kernel (dominant), nn_finalize_kernel',
            'bytes_per_env_step': bpe,
            'step_ms_median': kernel_ms, 'step_ms_mean': kernel_ms_mean,
            'flops_per_env_step': flops,
            'mfma_tflops': flops * E / (kernel_ms * 1e-3) / 1e12,
            'mfma_peak_tflops': MFMA_F32_PEAK_TFLOPS,
        },
    })
    return line


def mlp_line(args, eng, world, E, S, elapsed, kernel_ms, kernel_ms_mean, shard, phase_ms):
    P = eng.act_dim
    train_f, info_f = mlp_flops()
    info_ms = phase_ms.get('info') or kernel_ms
    train_ms = phase_ms.get('train')
    achieved = info_f * E / (info_ms * 1e-3) / 1e12
    line = {'metric': METRIC_MLP}
    line.update(_common(args, world, E, S, elapsed, shard))
    line.update({
        'dtype': 'f32',
        'data': 'synthetic: RandomState(0).rand(1024, 784), labels argmax(X T), '
                'T = RandomState(1).normal(784, 10); glorot-uniform init per env seed; '
                'actions N(0, 1e-3) float32 generated on device',
        'config': {
            'workload': 'Optimize-v0 over the 784-64-10 relu MLP (P=50890, obs 101781), '
                        '%d envs per GPU, B=32 of N=1024, full-data info pass every step, '
                        'in-kernel auto-reset, device-resident actions/outputs' % E,
            'envs_per_gpu': E, 'global_envs': world * E, 'n_rows': 1024, 'n_features': 784,
            'n_hidden': 64, 'n_classes': 10, 'batch_size': 32,
            'parallelism': 'env-sharded x%d (no collective)' % world,
        },
        'roofline': {
            'bound': 'mfma', 'achieved': achieved, 'peak': MFMA_F32_PEAK_TFLOPS,
            'unit': 'TFLOP/s', 'frac': achieved / MFMA_F32_PEAK_TFLOPS, 'traffic': None,
            'kernel': 'ce::mlp_info_kernel (full-data forward, 94% of the FLOPs)',
            'flops_per_env_step': train_f + info_f, 'info_flops_per_env_step': info_f,
            'info_kernel_ms': info_ms, 'train_kernel_ms': train_ms,
            'step_ms_median': kernel_ms, 'step_ms_mean': kernel_ms_mean,
            'step_tflops': (train_f + info_f) * E / (kernel_ms * 1e-3) / 1e12,
            'train_kernel_hbm_bytes_per_env_step': mlp_train_bytes(P),
            'train_kernel_gbs': (mlp_train_bytes(P) * E / (train_ms * 1e-3) / 1e9
                                 if train_ms else None),
        },
    })
    return line


if __name__ == '__main__':
    main()

"""Benchmark: vectorised Optimize-v0 env-steps/s on MI355X (BASELINE.json metric).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--envs E] [--precision f64|f32]
                  [--workload optimize|multi|mlp|nn] [--no-gather]

One "step" = one VecEnv.step of every env: the fused HIP kernel advances
E = 4096 envs per GPU (weak scaling: N GPUs own N*4096 envs, contiguous
shards, seed = global env index) of the 256x10 softmax-regression problem by
one Optimize-v0 step, auto-reset included.  Actions are device-resident
([S][E][P] float32 in HBM, a different action block per step) and the
outputs (obs/reward/done/info) are written to HBM every step.

Launch.  ``--gpus N`` with N > 1 and no WORLD_SIZE in the environment starts
``torch.distributed.run`` with N ranks (one process per GPU, RCCL) as a
child process before anything touches a GPU; under torchrun (the driver's
launch) the ranks come from RANK/WORLD_SIZE.

Multi-GPU (config 4).  Every step all-gathers the packed outputs of every
rank (custom_envs_amd/distributed.py: ONE all_gather_into_tensor of the
compact per-env record [obs without its identically-zero weight block |
objective | accuracy | episode_len], 96 B at P = 20, in 256-B-aligned
segments, RCCL over xGMI; done is episode_len >= 40, reward is -objective
(B = N) and the full obs rows are rebuilt lazily on the consumer).  ``value`` is the SERIAL schedule: the
step kernel, then the collective, every step -- what a closed-loop learner
consumes.  The line also carries ``value_gather_pipelined`` (two output
buffers, the collective of step t on RCCL's stream while step t+1's kernel
writes the other buffer: an open-loop consumer one step behind) and
``value_no_gather`` (the env kernels alone, hipGraph replay).  At N = 1
(without --force-gather) there is no collective and ``value`` is the
hipGraph replay of S steps.

``--workload multi`` measures config 5 instead: MultiOptLRs-v0 (4 agents,
4-D Rosenbrock pairs, H=5, max_batches=400) behind OptVecEnv, 1024 envs per
GPU, actions uniform(1, 3) as in SURVEY 8d.  ``--workload mlp`` measures
config 3: Optimize-v0 over the 784 -> 64 -> 10 MLP on 1024 MNIST-sized
synthetic rows, B = 32, 4096 envs, float32 on MFMA (roofline bound "mfma").

Rank 0 prints ONE JSON line.  ``--dry-run`` exercises the launcher and the
rank protocol on CPU (gloo, no engine) for the tests.
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
HBM_COPY_GBS = 6290.0         # MI355X_MICROARCH.md: measured device-to-device copy rate
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


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument('--gpus', type=int, default=1)
    p.add_argument('--steps', type=int, default=2000,
                   help='timed steps (optimize / multi: 20000 unless given)')
    p.add_argument('--warmup', type=int, default=200,
                   help='untimed steps first (optimize / multi: 20000 unless given)')
    p.add_argument('--envs', type=int, default=None,
                   help='envs per GPU (default 4096 optimize, 1024 multi)')
    p.add_argument('--workload', default='optimize',
                   choices=['optimize', 'multi', 'mlp', 'nn', 'mnist'])
    p.add_argument('--precision', default='f64', choices=['f64', 'f32'])
    p.add_argument('--hidden', default='64',
                   help='mlp workload: hidden widths, e.g. 256,256 (create_neural_net default)')
    p.add_argument('--batch-size', type=int, default=32, help='mlp workload: minibatch rows')
    p.add_argument('--graph-steps', type=int, default=250,
                   help='steps per launch (persistent kernel) or per hipGraph replay')
    p.add_argument('--chunk-steps', type=int, default=10,
                   help='N > 1, optimize: steps per rollout launch and per all-gather in the '
                        'chunk schedule')
    p.add_argument('--no-gather', action='store_true',
                   help='N > 1: no per-step all-gather in the headline value')
    p.add_argument('--gather', action='store_true',
                   help='all-gather every step also for the multi workload')
    p.add_argument('--cpu-seconds', type=float, default=12.0, help='CPU baseline budget per leg')
    p.add_argument('--no-cpu-baseline', action='store_true')
    p.add_argument('--cpu-baseline-only', action='store_true', help=argparse.SUPPRESS)
    p.add_argument('--force-gather', action='store_true',
                   help='run the gather modes at world 1 too (a real 1-rank RCCL collective)')
    p.add_argument('--dry-run', action='store_true',
                   help='launcher + rank protocol only (gloo on CPU, no engine)')
    p.add_argument('--one-gpu-rehearsal', action='store_true',
                   help='N > 1 on a 1-GPU box: every rank on cuda:0, the collectives on gloo '
                        '(RCCL puts no two ranks on one device); the whole N-rank path runs, '
                        'the line says "rehearsal" and its rates are not N-GPU rates')
    p.add_argument('--profile-only', action='store_true',
                   help='run the timed steps only (for rocprofv3)')
    p.add_argument('--measure-traffic', action='store_true', default=None,
                   help='rank 0 at N = 1: measure roofline.traffic in this run (two rocprofv3 '
                        '--pmc passes of this workload as child processes, scripts/traffic.py); '
                        'the default when rocprofv3 is on PATH')
    p.add_argument('--timed-events', action='store_true',
                   help='diagnostic: HIP events around every launch INSIDE the timed region '
                        '(roofline.kernel_ms_timed_region); adds two event records per launch '
                        'to the timed host path')
    p.add_argument('--repeat-timed', type=int, default=0,
                   help='diagnostic: after the timed region, time the same K steps R more '
                        'times (same bracket) and list them as timed_repeats_ms; value stays '
                        'the first measurement')
    p.add_argument('--no-measure-traffic', dest='measure_traffic', action='store_false',
                   help='take roofline.traffic from the committed '
                        'profiles/<round>_traffic_<workload>.json instead')
    args = p.parse_args(argv)
    args.hidden = tuple(int(h) for h in str(args.hidden).split(',') if h)
    if args.measure_traffic is None:
        import shutil
        args.measure_traffic = shutil.which('rocprofv3') is not None and not args.profile_only
    if args.workload == 'mnist' and '--steps' not in (argv or sys.argv):
        args.steps, args.warmup = 30, 3      # ~13 ms per step at 4096 envs
    if args.workload in ('optimize', 'multi'):
        # microsecond steps: 20,000 untimed steps bring the chip to its
        # steady clock first (the timed region's kernel ran 2.53 us per step
        # after 200, 2.26 after 20,000: profiles/r05z_*), then 20,000 timed
        # (~50 ms); the driver's short form passes its own --steps / --warmup
        given = argv or sys.argv

        def has(flag):
            return any(a == flag or a.startswith(flag + '=') for a in given)
        if not has('--steps'):
            args.steps = 20000
        if not has('--warmup'):
            args.warmup = 20000
    if args.envs is None:
        args.envs = {'multi': 1024, 'nn': 1024}.get(args.workload, 4096)
    return args


def _free_port():
    import socket
    with socket.socket() as sock:
        sock.bind(('127.0.0.1', 0))
        return sock.getsockname()[1]


def launch_ranks(args):
    """``--gpus N`` without a torchrun environment: run this script under
    ``torch.distributed.run`` with N ranks as a CHILD process (this process
    has not touched a GPU and never execs) and return its exit code."""
    import subprocess
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
           '--nproc-per-node', str(args.gpus), '--master-addr', '127.0.0.1',
           '--master-port', str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
    return subprocess.call(cmd, env=env)


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
        if wall >= budget_s or steps >= 100000:
            break
    return steps, wall, time.process_time() - cpu0


def host_info():
    """What the CPU numbers ran on: model, cores, BLAS threads."""
    model = None
    try:
        with open('/proc/cpuinfo') as fh:
            for line in fh:
                if line.startswith('model name'):
                    model = line.split(':', 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count()
    return {'cpu_model': model, 'os_cpu_count': os.cpu_count(), 'affinity_cpus': affinity,
            'blas_threads': {k: os.environ.get(k) for k in
                             ('OMP_NUM_THREADS', 'OPENBLAS_NUM_THREADS', 'MKL_NUM_THREADS')},
            'ulimit_n': resource.getrlimit(resource.RLIMIT_NOFILE)[0],
            'numpy': np.__version__}


def affinity_cpus():
    """CPUs this process may run on (os.cpu_count() is the whole machine)."""
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_share():
    """The per-GPU CPU share of the GPU boxes (16 CPUs per GPU there): the
    second SubprocVecEnv leg, kept beside the full-affinity leg."""
    return max(1, min(affinity_cpus(), 16))


def _children_cpu():
    ru = resource.getrusage(resource.RUSAGE_CHILDREN)
    return ru.ru_utime + ru.ru_stime


def _optimize_factory(features, targets, seed):
    def make():
        from oracle.optimize import Optimize as OracleEnv
        env = OracleEnv(features, targets)
        env.seed(seed)
        return env
    return make


def cpu_baseline(features, targets, envs, budget_s):
    """The reference's NumPy path restated: oracle envs under the restated
    custom_envs.vectorize (concurrentvecenv.py:64-268, 230-248), three legs:
    ThreadVecEnv at the GPU's env count (one thread + mp.Pipe per env, the
    reference's configuration), SubprocVecEnv with one process per CPU of the
    affinity mask and SubprocVecEnv at the 16-CPU per-GPU share.
    Each leg reports the cores it used (its CPU time over its wall time).
    ``value`` is the fastest leg."""
    from oracle.vectorize import SubprocVecEnv, ThreadVecEnv
    n = _raise_fd_limit(envs)
    venv = ThreadVecEnv([_optimize_factory(features, targets, i) for i in range(n)])
    venv.reset()
    acts = np.random.RandomState(0).normal(0, 0.01, (n, 20)).astype(np.float32)
    steps, wall, cpu = _time_cpu(venv, acts, budget_s)
    venv.close()
    thread = {'value': n * steps / wall, 'envs': n, 'steps': steps, 'wall_s': wall,
              'cpu_s': cpu, 'cores': max(1, int(round(cpu / wall)))}

    def subproc(p):
        # workers' CPU time from RUSAGE_CHILDREN once they are joined: the
        # cores the leg actually used, not the ones it was offered
        c0 = _children_cpu()
        venv = SubprocVecEnv([_optimize_factory(features, targets, i) for i in range(p)], 'fork')
        venv.reset()
        acts = np.random.RandomState(0).normal(0, 0.01, (p, 20)).astype(np.float32)
        steps, wall, cpu = _time_cpu(venv, acts, budget_s)
        venv.close()
        used = _children_cpu() - c0 + cpu
        return {'value': p * steps / wall, 'envs': p, 'steps': steps, 'wall_s': wall,
                'cpu_s': used, 'cores': max(1, int(round(used / wall))), 'processes': p}

    # SubprocVecEnv at one process per CPU of the host's affinity
    # mask; the 16-process per-GPU share leg stays beside it
    full_p = _raise_fd_limit(affinity_cpus())
    full = subproc(full_p)
    share_p = cpu_share()
    share = subproc(share_p) if share_p != full_p else dict(full)
    legs = {'ThreadVecEnv': thread, 'SubprocVecEnv_affinity': full, 'SubprocVecEnv_gpu_share': share}
    best = max(legs.items(), key=lambda x: x[1]['value'])
    return {'value': best[1]['value'], 'unit': 'env-steps/s', 'cores': best[1]['cores'],
            'kind': 'port',
            'sample': ('%s leg (the fastest of three): ThreadVecEnv %d envs x %d steps '
                       '(1 thread + mp.Pipe per env, pickled step msgs, np.stack; %.1f s wall, '
                       '%d cores used) = %.3g env-steps/s; SubprocVecEnv at the full affinity '
                       'mask, %d processes x %d steps (%.1f s wall, %d cores used) = %.3g '
                       'env-steps/s; SubprocVecEnv at the 16-CPU per-GPU share, %d processes x '
                       '%d steps (%.1f s wall, %d cores used) = %.3g env-steps/s; all over the '
                       'float64 numpy oracle Optimize env, 256x10, B=N' % (
                           best[0], thread['envs'], thread['steps'], thread['wall_s'], thread['cores'],
                           thread['value'], full['envs'], full['steps'], full['wall_s'], full['cores'],
                           full['value'], share['envs'], share['steps'], share['wall_s'],
                           share['cores'], share['value'])),
            'legs': legs,
            'host': host_info()}


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


def mnist_dataset():
    from custom_envs_amd.data import load_data
    seq = load_data('mnist7x7_synthetic', batch_size=None)
    return seq.features, seq.targets


def build_mnist(args, torch, device, rank, world):
    """Optimize-v0 at the reference's default data shape (load_data('mnist'):
    60,000 rows, 7x7 = 49 features, 10 classes; batch_size=None = all rows,
    optimize.py:40), float64 on the MFMA kernel."""
    from custom_envs_amd.engine import OptimizeEngine
    features, targets = mnist_dataset()
    E = args.envs
    eng = OptimizeEngine(features, targets, num_envs=E, device=device)
    eng.seed([rank * E + i for i in range(E)])
    gen = torch.Generator(device='cuda').manual_seed(99 + rank)
    S = max(1, min(args.graph_steps, args.steps, 4))
    actions = torch.randn((S, E, eng.act_dim), generator=gen, device='cuda') * 0.01
    return eng, actions, S


def cpu_baseline_mnist(budget_s):
    """The reference's path restated (oracle Optimize envs, float64 numpy,
    under the restated SubprocVecEnv) on the same 60,000 x 49 x 10 set."""
    from oracle.vectorize import SubprocVecEnv
    features, targets = mnist_dataset()
    p = cpu_share()
    venv = SubprocVecEnv([_optimize_factory(features, targets, i) for i in range(p)], 'fork')
    venv.reset()
    acts = np.random.RandomState(0).normal(0, 0.01, (p, 490)).astype(np.float32)
    steps, wall, _ = _time_cpu(venv, acts, budget_s)
    venv.close()
    return {'value': p * steps / wall, 'unit': 'env-steps/s', 'cores': p, 'kind': 'port',
            'sample': 'SubprocVecEnv %d processes x %d steps (%.1f s wall) of the float64 '
                      'numpy oracle Optimize env on the 60000 x 49 x 10 set, B = N'
                      % (p, steps, wall)}


def build_mlp(args, torch, device, rank, world, phases=None):
    from custom_envs_amd.engine import OptimizeEngine
    features, targets = mlp_dataset()
    E = args.envs
    if phases:
        os.environ['CE_MLP_PHASES'] = phases
    try:
        eng = OptimizeEngine(features, targets, num_envs=E, batch_size=args.batch_size,
                             model='mlp', hidden=args.hidden, device=device)
    finally:
        os.environ.pop('CE_MLP_PHASES', None)
    eng.seed([rank * E + i for i in range(E)])
    gen = torch.Generator(device='cuda').manual_seed(4321 + rank)
    S = 2                                  # two action blocks of [E][P] (833 MB each)
    actions = torch.randn((S, E, eng.act_dim), generator=gen, device='cuda') * 1e-3
    return eng, actions, S


def cpu_baseline_mlp(envs, budget_s, hidden=(64,), batch_size=32):
    """Oracle float32 MLP Optimize envs under the restated ThreadVecEnv."""
    from oracle.optimize import Optimize as OracleEnv
    from oracle.vectorize import ThreadVecEnv
    features, targets = mlp_dataset()
    n = min(_raise_fd_limit(envs), 64)

    def factory(seed):
        def make():
            env = OracleEnv(features, targets, batch_size=batch_size, model='mlp', hidden=hidden)
            env.seed(seed)
            return env
        return make

    venv = ThreadVecEnv([factory(i) for i in range(n)])
    venv.reset()
    n_params = venv.get_attr('obs_size')[0] // 2
    acts = np.random.RandomState(0).normal(0, 1e-3, (n, n_params)).astype(np.float32)
    steps, wall, cpu = _time_cpu(venv, acts, budget_s)
    venv.close()
    dims = '-'.join(map(str, (784,) + tuple(hidden) + (10,)))
    return {'value': n * steps / wall, 'unit': 'env-steps/s',
            'cores': max(1, int(round(cpu / wall))), 'kind': 'port',
            'sample': '%d envs x %d steps of ThreadVecEnv over the numpy oracle Optimize env '
                      'with the float32 %s network, B=%d (BLAS sgemm); %.1f s wall, %.1f s CPU; '
                      'os.cpu_count()=%d' % (n, steps, dims, batch_size, wall, cpu,
                                              os.cpu_count())}


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


def run_cpu_baseline_child(args):
    """The CPU legs in a child process started before this process touches
    the GPU (SubprocVecEnv forks workers; nothing forks from a GPU process)."""
    import subprocess
    cmd = [sys.executable, os.path.abspath(__file__), '--cpu-baseline-only',
           '--workload', args.workload, '--envs', str(args.envs),
           '--cpu-seconds', str(args.cpu_seconds),
           '--hidden', ','.join(map(str, args.hidden)), '--batch-size', str(args.batch_size)]
    res = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    for line in reversed(res.stdout.splitlines()):
        if line.startswith('{'):
            return json.loads(line)
    return {'value': None, 'error': 'cpu baseline child failed rc=%d: %s'
            % (res.returncode, res.stderr[-500:])}


def cpu_baseline_only(args):
    if args.workload == 'mnist':
        cpu = cpu_baseline_mnist(args.cpu_seconds)
    elif args.workload == 'nn':
        cpu = cpu_baseline_nn(args.cpu_seconds)
    elif args.workload == 'multi':
        cpu = cpu_baseline_multi(args.envs, args.cpu_seconds)
    elif args.workload == 'mlp':
        cpu = cpu_baseline_mlp(args.envs, args.cpu_seconds, args.hidden, args.batch_size)
    else:
        cpu = cpu_baseline(*lr_dataset(), args.envs, args.cpu_seconds)
    cpu.setdefault('host', host_info())
    print(json.dumps(cpu))


def dry_run(args, world, rank):
    """The rank protocol without an engine: gloo, barrier + max-over-ranks
    timing of K no-op steps; rank 0 prints the line with n_gpus = world."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group('gloo')
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pass
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({'metric': METRIC, 'value': None, 'n_gpus': world, 'steps': args.steps,
                          'warmup': args.warmup, 'dry_run': True, 'elapsed_s': elapsed,
                          'world_size_env': os.environ.get('WORLD_SIZE')}))


def _timed(torch, dist, fn, steps):
    """barrier + synchronize on both sides of exactly `steps` steps; the max
    over ranks."""
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn(steps)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device='cuda')
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def main():
    args = parse()
    if args.cpu_baseline_only:
        cpu_baseline_only(args)
        return 0
    if 'WORLD_SIZE' not in os.environ and args.gpus > 1:
        return launch_ranks(args)
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local_rank = int(os.environ.get('LOCAL_RANK', '0'))
    if world != args.gpus:
        print('bench: --gpus %d but WORLD_SIZE=%d; measuring %d ranks'
              % (args.gpus, world, world), file=sys.stderr)
    if args.dry_run:
        dry_run(args, world, rank)
        return 0
    cpu = None
    if rank == 0 and not args.no_cpu_baseline and not args.profile_only:
        # every N: the reference path on the same box's host cores, in the
        # same run (north_star); a child process started before this rank
        # touches the GPU, while the other ranks wait in the rendezvous
        cpu = run_cpu_baseline_child(args)

    import torch
    dist = None
    if world > 1 or args.force_gather:
        import torch.distributed as dist
        dev_index = 0 if args.one_gpu_rehearsal else local_rank
        torch.cuda.set_device(dev_index)
        if world == 1:
            os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
            os.environ.setdefault('MASTER_PORT', str(_free_port()))
            os.environ.setdefault('RANK', '0')
            os.environ.setdefault('WORLD_SIZE', '1')
        if args.one_gpu_rehearsal:
            dist.init_process_group('gloo')
        else:
            dist.init_process_group('nccl', device_id=torch.device('cuda', local_rank))
    else:
        torch.cuda.set_device(0)
    device = torch.cuda.current_device()
    multi = args.workload == 'multi'
    mlp = args.workload == 'mlp'
    nn = args.workload == 'nn'
    mnist = args.workload == 'mnist'
    builder = {'optimize': build_optimize, 'multi': build_multi, 'mlp': build_mlp,
               'nn': build_nn, 'mnist': build_mnist}[args.workload]
    eng, actions, S = builder(args, torch, device, rank, world)
    E = args.envs
    stream = torch.cuda.Stream()          # a real stream: graphs cannot capture the null stream
    torch.cuda.set_stream(stream)
    eng.set_stream(stream.cuda_stream)
    gather_modes = (world > 1 or args.force_gather) and not args.no_gather and (
        args.workload == 'optimize' or (multi and args.gather))
    shard = None
    if gather_modes:
        from custom_envs_amd.distributed import ShardedEnvs
        # two packed buffers: the engine writes straight into them (no packing kernels)
        # the chunk schedule where the engine runs K steps per launch: each
        # slot holds K step records, gathered by ONE collective
        # (at most S: the action tensor holds S step blocks)
        chunk = (max(1, min(args.chunk_steps, args.steps, S))
                 if args.workload == 'optimize' and getattr(eng, 'persistent', False) else 1)
        shard = ShardedEnvs(eng, world * E, rank, world, slots=2, collective=True, chunk=chunk)
        out = shard.outs[0]
    else:
        out = eng.alloc_device_outputs()
    # the optimize workload without a collective keeps every step's outputs:
    # a [S] slab of output records (the device-resident rollout a learner
    # consumes), written by ONE persistent launch per S steps where the
    # engine has the K-step kernel (ce_step_many_strided)
    slab = None
    if args.workload in ('optimize', 'multi') and shard is None and getattr(eng, 'persistent', False):
        slab = eng.alloc_rollout(S)
        out = {k: v[0] for k, v in slab[0].items() if k != '_buffer'}
    eng.reset_device(out)

    def chunks(k):
        sizes = [S] * (k // S) + ([k % S] if k % S else [])
        return sizes

    runners = {}

    def runner(n):
        # the engines with a pre-bound form skip the per-call argument checks
        if slab is not None:
            return eng.rollout_runner(n, actions, slab[0], slab[1])
        if hasattr(eng, 'many_runner'):
            return eng.many_runner(n, actions, out)
        return lambda: eng.step_many_device(n, actions, out)

    timed_events = []               # --timed-events: (start, end, steps) per launch

    def run_graph(k):
        for n in chunks(k):
            if n not in runners:
                runners[n] = runner(n)
            if record_events[0]:
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True), n)
                ev[0].record(stream)
                runners[n]()
                ev[1].record(stream)
                timed_events.append(ev)
            else:
                runners[n]()
    record_events = [False]

    pending = [None, None]
    counter = [0]

    def run_gather_pipelined(k):
        # step t writes slot t % 2; its all-gather runs on RCCL's stream while
        # step t+1 writes the other slot; before a slot is rewritten, the
        # engine stream waits for the collective that read it
        for _ in range(k):
            t = counter[0]
            slot = t & 1
            if pending[slot] is not None:
                pending[slot].wait()
            eng.step_device(actions[t % S], shard.outs[slot])
            _, pending[slot] = shard.gather(slot, async_op=True)
            counter[0] += 1
        for slot in (0, 1):
            if pending[slot] is not None:
                pending[slot].wait()
                pending[slot] = None

    def run_gather_serial(k):
        for _ in range(k):
            t = counter[0]
            eng.step_device(actions[t % S], shard.outs[0])
            shard.gather(0)
            counter[0] += 1

    # the chunk schedule: ONE persistent launch of C steps into
    # a C-record slot, then ONE all-gather of the slot; pipelined, chunk c's
    # gather runs on RCCL's stream while chunk c + 1's launch writes the
    # other slot (the engine stream waits for the gather that read a slot
    # before rewriting it)
    chunk_runners = {}
    C = shard.chunk if shard is not None else 1

    def cchunks(k):
        return [C] * (k // C) + ([k % C] if k % C else [])

    def chunk_launch(slot, n):
        if (slot, n) not in chunk_runners:
            chunk_runners[slot, n] = shard.rollout_runner(actions[:n], slot, n)
        chunk_runners[slot, n]()

    def run_chunk_pipelined(k):
        for n in cchunks(k):
            slot = counter[0] & 1
            if pending[slot] is not None:
                pending[slot].wait()
            chunk_launch(slot, n)
            _, pending[slot] = shard.gather_chunk(slot, async_op=True, k=n)
            counter[0] += 1
        for slot in (0, 1):
            if pending[slot] is not None:
                pending[slot].wait()
                pending[slot] = None

    def run_chunk_serial(k):
        for n in cchunks(k):
            chunk_launch(0, n)
            shard.gather_chunk(0, k=n)

    # hipGraphs for every chunk size the graph mode replays, built before any timing
    for n in sorted(set(chunks(args.warmup) + chunks(args.steps))):
        if slab is None:
            eng.prepare_many_device(n, actions, out)
        runners[n] = runner(n)
    if args.profile_only:
        run_graph(args.warmup)
        torch.cuda.synchronize()
        run_graph(args.steps)
        torch.cuda.synchronize()
        return 0

    modes = {}
    gather_graph = None
    if gather_modes:
        # both gather modes also as hipGraphs (torch.cuda.graph capturing the
        # engine's launches and RCCL's collectives, one replay per chunk):
        # eager, each step costs a ctypes launch plus a torch collective call
        # on the host, which is more than the kernel
        gg_chunk = max(1, min(args.graph_steps, 50))

        def gchunks(k):
            return [gg_chunk] * (k // gg_chunk) + ([k % gg_chunk] if k % gg_chunk else [])

        run_gather_pipelined(max(args.warmup, 4))     # communicators up before capture
        run_gather_serial(2)
        kinds = [('pipelined', run_gather_pipelined), ('serial', run_gather_serial)]
        if C > 1:
            run_chunk_pipelined(2 * C + 1)
            run_chunk_serial(C + 1)
            kinds += [('chunk_pipelined', run_chunk_pipelined), ('chunk_serial', run_chunk_serial)]
        torch.cuda.synchronize()
        graphs = {}
        try:
            if dist.get_backend() != 'nccl':     # gloo (--one-gpu-rehearsal) cannot be captured
                raise RuntimeError('backend %s has no graph capture' % dist.get_backend())
            for kind, fn in kinds:
                for n in sorted(set(gchunks(args.warmup) + gchunks(args.steps))):
                    g = torch.cuda.CUDAGraph()
                    counter[0] = 0
                    with torch.cuda.graph(g, stream=stream):
                        fn(n)
                    graphs[kind, n] = g
            torch.cuda.synchronize()
            gather_graph = True
        except Exception as exc:          # fall back to eager replays, say so
            gather_graph = 'eager (capture failed: %s)' % str(exc)[:200]
            graphs = {}
            pending[0] = pending[1] = None       # handles from inside the failed capture
            counter[0] = 0
            chunk_runners.clear()
            torch.cuda.synchronize()
            # a stream whose capture was invalidated keeps failing launches:
            # the eager replays run on a fresh one
            stream = torch.cuda.Stream()
            torch.cuda.set_stream(stream)
            eng.set_stream(stream.cuda_stream)
            print('bench: gather capture failed, eager gathers: %s' % str(exc)[:200],
                  file=sys.stderr)

        def replayer(kind, eager):
            if not graphs:
                return eager

            def run(k):
                for n in gchunks(k):
                    graphs[kind, n].replay()
            return run

        for kind, fn in kinds:
            run = replayer(kind, fn)
            run(args.warmup)
            modes[kind] = _timed(torch, dist, run, args.steps)
        run_graph(args.warmup)
        modes['no_gather'] = _timed(torch, dist, run_graph, args.steps)
        # every schedule runs every step AND the all-gather of its outputs
        # inside the timed region.  `value`: the chunk schedule where the
        # engine has the K-step launch (the actions of a chunk are device-
        # resident before it starts -- the open-loop rollout a persistent
        # launch serves; the gather of chunk c overlaps chunk c + 1), else
        # the per-step serial schedule (a closed-loop learner acting on step
        # t's outputs before step t + 1), which rides along either way
        gather_mode = 'chunk_pipelined' if C > 1 else 'serial'
        elapsed = modes[gather_mode]
    else:
        primary = run_graph
        # the W warmup steps as waited launches -- four of one step, then
        # the rest: the first launch-and-wait cycles of a process carry a
        # one-time cost (5-16 us, profiles/r05n_bench20_repeats_*.json,
        # r05k_launch_floor.json) that the warmup is there to absorb (two
        # waited halves: 3.52-3.57 us per driver-form step, this: 3.48-3.54,
        # r05ac_*); still exactly W steps
        w1 = min(args.warmup, 4)
        warm_sizes = [1] * w1 + ([args.warmup - w1] if args.warmup > w1 else [])
        for n in warm_sizes:
            if n:
                for c in chunks(n):                         # launch sizes up to S
                    if c not in runners:
                        if slab is None:
                            eng.prepare_many_device(c, actions, out)
                        runners[c] = runner(c)
                primary(n)
                torch.cuda.synchronize()
        # HIP events around every launch of the timed region itself when its
        # launches queue back to back (4 or more: the host's two event
        # records per launch run ahead of the GPU), or when asked
        record_events[0] = args.timed_events or len(chunks(args.steps)) >= 4
        elapsed = _timed(torch, dist, primary, args.steps)
        record_events[0] = False
        if timed_events:
            per = [a.elapsed_time(b) / n for a, b, n in timed_events]
            modes['timed_region_kernel_ms'] = float(np.median(per))
            modes['timed_region_kernel_ms_mean'] = float(np.mean(per))
        if args.repeat_timed > 0:
            modes['timed_repeats'] = [_timed(torch, dist, primary, args.steps)
                                      for _ in range(args.repeat_timed)]
        if slab is not None:
            # the same steps as one launch per step (the one-step kernel,
            # what a closed-loop caller gets), timed the same way: the A/B
            # beside `value`
            eng.set_persistent(False)
            runners.clear()
            run_graph(args.warmup)
            torch.cuda.synchronize()
            modes['per_step_launch'] = _timed(torch, dist, run_graph, args.steps)
            ev = launch_events(torch, stream, lambda: run_graph(S), S)
            modes['per_step_launch_kernel_ms'] = ev[0]
            eng.set_persistent(True)
            runners.clear()
            run_graph(args.warmup)
            torch.cuda.synchronize()

    # live kernel duration: HIP events on the engine's stream (= torch's
    # current stream) around graph replays of S back-to-back step launches,
    # divided by S: the per-launch time on the stream, i.e. the kernel plus
    # its share of the inter-kernel boundary (rocprofv3's kernel-only average
    # is the same minus that gap; profiles/ holds both)
    if slab is not None:
        kernel_ms, kernel_ms_mean = launch_events(torch, stream, lambda: run_graph(S), S)
    else:
        kernel_ms, kernel_ms_mean = launch_events(torch, stream,
                                                  lambda: eng.step_many_device(S, actions, out), S)
    # the roofline's kernel time: the timed region's own launches where they
    # were timed (the same kernels rocprofv3 traces in that run), else the
    # loop above, which runs after the timed region on a warmer chip
    warm_loop_ms = kernel_ms
    if 'timed_region_kernel_ms' in modes:
        kernel_ms, kernel_ms_mean = modes['timed_region_kernel_ms'], modes['timed_region_kernel_ms_mean']
    phase_ms = {}
    if mlp and rank == 0 and not eng.step_kernel.startswith('net<'):
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

    if rank == 0:
        if mlp and eng.step_kernel.startswith('net<'):
            line = net_line(args, eng, world, E, S, elapsed, kernel_ms, kernel_ms_mean, shard)
        elif mlp:
            line = mlp_line(args, eng, world, E, S, elapsed, kernel_ms, kernel_ms_mean, shard,
                            phase_ms)
        elif nn:
            line = nn_line(args, eng, world, E, S, elapsed, kernel_ms, kernel_ms_mean, shard)
        elif mnist:
            line = mnist_line(args, eng, world, E, S, elapsed, kernel_ms, kernel_ms_mean)
        else:
            line = (multi_line if multi else optimize_line)(args, eng, world, E, S, elapsed,
                                                            kernel_ms, kernel_ms_mean, shard)
        if 'timed_region_kernel_ms' in modes:
            line['roofline']['kernel_ms_source'] = ('HIP events around every launch of the timed '
                                                    'region (median / mean per step)')
            line['roofline']['kernel_ms_warm_loop'] = warm_loop_ms
        else:
            line['roofline']['kernel_ms_source'] = ('HIP events around a loop of the same launches '
                                                    'after the timed region (one launch timed: '
                                                    'events inside it would sit on its host path)')
        if 'timed_repeats' in modes:
            line['timed_repeats_ms'] = [round(t * 1e3, 5) for t in modes['timed_repeats']]
        if 'per_step_launch' in modes:
            line['value_per_step_launch'] = world * E * args.steps / modes['per_step_launch']
            line['ms_per_step_per_step_launch'] = modes['per_step_launch'] / args.steps * 1e3
            line['roofline']['per_step_launch_kernel_ms'] = modes['per_step_launch_kernel_ms']
        elif 'serial' in modes:                      # the gather schedules (N > 1 / --force-gather)
            units = world * E * args.steps
            line['value_gather_serial_per_step'] = units / modes['serial']
            line['value_gather_pipelined_per_step'] = units / modes['pipelined']
            for kind in ('chunk_pipelined', 'chunk_serial'):
                if kind in modes:
                    line['value_gather_' + kind] = units / modes[kind]
            line['value_no_gather'] = units / modes['no_gather']
            line['gather_chunk_steps'] = C
            line['ms_per_step_modes'] = {k: v / args.steps * 1e3 for k, v in modes.items()}
            line['gather_bytes_per_rank'] = shard.layout.nbytes
            line['gather_record'] = 'compact' if shard.compact else 'full'
            line['gather_mode'] = gather_mode
            line['gather_graph'] = gather_graph
        # the traffic is compared with what the launch form must move
        # (persistent: the state once per launch), else the per-step count
        r = line['roofline']
        bpe = r.get('bytes_per_env_step_moved', r.get('hbm', {}).get('bytes_per_env_step_moved',
                    r.get('bytes_per_env_step', r.get('hbm', {}).get('bytes_per_env_step'))))
        line['roofline'].update(traffic_fields(args, eng, E, bpe if isinstance(bpe, (int, float)) else None))
        line['cpu_baseline'] = cpu
        if host_rate is not None:
            line['host_loop_env_steps_per_s'] = host_rate
        if args.one_gpu_rehearsal:
            line['rehearsal'] = '%d ranks on one GPU, collectives on gloo: not an N-GPU rate' % world
        print(json.dumps(line))
    eng.close()
    if dist is not None:
        dist.destroy_process_group()
    return 0


def launch_events(torch, stream, fn, steps, n_ev=8):
    """(median, mean) ms per step of `fn` (which issues `steps` steps on
    `stream`) by HIP events on that stream: one warm call queued first so the
    events time the GPU, not the host."""
    fn()
    starts = [torch.cuda.Event(enable_timing=True) for _ in range(n_ev)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(n_ev)]
    for i in range(n_ev):
        starts[i].record(stream)
        fn()
        ends[i].record(stream)
    torch.cuda.synchronize()
    times = [a.elapsed_time(b) / steps for a, b in zip(starts, ends)]
    return float(np.median(times)), float(np.mean(times))


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


# roofline.traffic: HBM bytes per step from rocprofv3 counters
# (scripts/traffic.py).  The committed summaries of this round are named here
# and reported in roofline.traffic_source; --measure-traffic takes them in
# the run instead.
TRAFFIC_ROUND = 'r06'
TRAFFIC_FALLBACK_ROUNDS = ('r06', 'r05')     # committed summaries, newest first
TRAFFIC_MARKER = {'optimize': 'optimize_lr_', 'multi': 'multi_',
                  'mlp': 'mlp_step_kernel', 'net': 'net_finish_kernel',
                  'nn': 'nn_finalize_kernel', 'mnist': 'optimize_'}


def _traffic_name(args, eng):
    if args.workload == 'mlp':
        return 'net' if eng.step_kernel.startswith('net<') else 'mlp'
    return args.workload


def _traffic_steps(args):
    """Steps per counted dispatch: the bench's launch size for the persistent
    K-step kernel (every dispatch the same S steps), else 1."""
    if args.workload in ('optimize', 'multi') and int(os.environ.get('CE_PERSIST', '1')) != 0:
        return max(1, min(args.graph_steps, args.steps))
    return 1


def _traffic_bench_args(args):
    k = _traffic_steps(args)
    out = ['--workload', args.workload, '--envs', str(args.envs), '--profile-only',
           '--steps', str(max(k, 6)), '--warmup', str(k), '--graph-steps', str(args.graph_steps),
           '--precision', args.precision]
    if args.workload == 'mlp':            # the nn workload's network and batch are fixed
        out += ['--batch-size', str(args.batch_size), '--hidden', ','.join(map(str, args.hidden))]
    return out


def traffic_fields(args, eng, E, bpe=None):
    """{'traffic': bytes per step, 'traffic_source': where it came from}."""
    name = _traffic_name(args, eng)
    sys.path.insert(0, os.path.join(ROOT, 'scripts'))
    import traffic as tr
    if args.measure_traffic and int(os.environ.get('WORLD_SIZE', '1')) == 1:
        try:
            run_dir = os.path.join(ROOT, 'gpurun_out', 'traffic', name)
            f, w = tr.collect(TRAFFIC_ROUND, name, _traffic_bench_args(args), run_dir)
            out, path = tr.summarize(f, w, TRAFFIC_MARKER[name], E, name, TRAFFIC_ROUND, bpe,
                                     {'bench_args': ' '.join(_traffic_bench_args(args))},
                                     out_dir=run_dir, steps_per_dispatch=_traffic_steps(args))
            return {'traffic': out['hbm_bytes_per_step'],
                    'traffic_source': 'measured in this run: %s' % os.path.relpath(path, ROOT)}
        except Exception as exc:      # the committed file, and say why
            why = 'in-run measurement failed (%s); ' % str(exc)[:160]
    else:
        why = ''
    for rnd in TRAFFIC_FALLBACK_ROUNDS:
        path = os.path.join(ROOT, 'profiles', '%s_traffic_%s.json' % (rnd, name))
        if os.path.exists(path):
            break
    if not os.path.exists(path):
        return {'traffic': None, 'traffic_source': why + 'no %s' % os.path.relpath(path, ROOT)}
    with open(path) as fh:
        rec = json.load(fh)
    if rec.get('envs') != E:
        return {'traffic': None, 'traffic_source': why + '%s is for %s envs' % (
            os.path.relpath(path, ROOT), rec.get('envs'))}
    return {'traffic': rec['hbm_bytes_per_step'],
            'traffic_source': why + '%s (round %s, %s)' % (os.path.relpath(path, ROOT), rec['round'],
                                                          rec['bench_args'])}


def optimize_line(args, eng, world, E, S, elapsed, kernel_ms, kernel_ms_mean, shard):
    """The headline line.  The dominant kernel is f64 work (MFMA for the two
    GEMMs, VALU for the softmax: on gfx950 both issue at the same 78.6 TF/s
    f64 rate and share the SIMD), so the roofline is the f64
    pipe over the step's algorithmic FLOPs (2NFK + 2NFK + 5NK);
    the HBM fraction of SURVEY 8d's byte count rides beside it."""
    P = eng.act_dim
    bpe = algorithmic_bytes_per_env_step(P, args.precision)
    achieved_gbs = bpe * E / (kernel_ms * 1e-3) / 1e9
    flops = 4 * 256 * P + 5 * 256 * 2
    achieved_tf = flops * E / (kernel_ms * 1e-3) / 1e12
    peak_tf = F64_VALU_PEAK_TFLOPS if args.precision == 'f64' else 157.3
    kernel = getattr(eng, 'many_kernel', eng.step_kernel)
    persistent = kernel.startswith('optimize_lr_persist')
    # bytes a persistent launch of S steps moves per env-step: actions 4P and
    # the outputs 4(2P+1) + 17 every step, the state (W, W0, G read; W, G
    # written, f64; L, step r/w) once per launch
    moved = 4 * P + 4 * (2 * P + 1) + 17 + (40 * P + 24) / S if persistent else bpe
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
            'steps_per_launch': S if persistent else 1,
            'outputs': ('every step kept: a [%d]-record slab per launch' % S
                        if persistent and shard is None else
                        'every step kept: [%d]-record slots, all-gathered' % shard.chunk
                        if shard is not None and shard.chunk > 1 else
                        'every step into the same output buffers'),
            # say which stepping contract `value` measures
            'stepping': ('open-loop rollout: the actions of all %d steps of a launch are '
                         'on the device before it starts (ce_step_many_strided); a '
                         'closed-loop caller (step t+1 chosen from step t\'s obs) gets '
                         'value_per_step_launch' % (S if persistent else 1)
                         if persistent else
                         'one launch per step (the closed-loop contract of VecEnv.step)'),
            'parallelism': 'env-sharded x%d (no collective)' % world
            if shard is None else
            ('env-sharded x%d; chunks of %d steps: one persistent launch, then ONE RCCL '
             'all-gather of the %d compact records, pipelined over 2 slots' % (
                 world, shard.chunk, shard.chunk) if shard.chunk > 1 else
             'env-sharded x%d + one RCCL all-gather of the packed outputs per step' % world),
        },
        'roofline': {
            'bound': 'mfma', 'pipe': 'f64 (MFMA + VALU, one 78.6 TF/s rate on gfx950)',
            'achieved': achieved_tf, 'peak': peak_tf, 'unit': 'TFLOP/s',
            'frac': achieved_tf / peak_tf, 'traffic': None,
            'flops_per_env_step': flops,
            'kernel': 'ce::' + kernel, 'steps_per_launch': S if persistent else 1,
            'kernel_ms_median': kernel_ms, 'kernel_ms_mean': kernel_ms_mean,
            'kernel_ms_note': 'per step: HIP events around launches of S steps on the engine '
                              'stream, divided by S',
            'hbm': {'bytes_per_env_step': bpe, 'achieved': achieved_gbs, 'peak': HBM_PEAK_GBS,
                    'unit': 'GB/s', 'frac': achieved_gbs / HBM_PEAK_GBS,
                    'bytes_per_env_step_moved': moved,
                    'note': 'bytes_per_env_step is SURVEY 8d\'s count (state read+written every '
                            'step, f64); bytes_per_env_step_moved is what the launch form moves'},
        },
    })
    return line


def multi_line(args, eng, world, E, S, elapsed, kernel_ms, kernel_ms_mean, shard):
    P, H = eng.n_params, eng.max_history
    bpe = multi_bytes_per_env_step(P, H)
    achieved_gbs = bpe * E / (kernel_ms * 1e-3) / 1e9
    kernel = getattr(eng, 'many_kernel', 'multi_step_kernel<4>')
    persistent = kernel.startswith('multi_persist')
    # a persistent launch of S steps moves per env-step the actions 4P and
    # the outputs (obs 12HP, reward 4P, done P, info 56, length 4); the state
    # (theta, g, the raw ring 5(1 + 2P), the adjusted ring H(1 + 2P) floats +
    # HP doubles, step) is read and written once per launch
    state = 4 * (2 * P + 5 * (1 + 2 * P) + H * (1 + 2 * P)) + 8 * H * P + 4
    moved = (4 * P + 12 * H * P + 4 * P + P + 56 + 4 + 2 * state / S) if persistent else bpe
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
            'steps_per_launch': S if persistent else 1,
            'graph_steps': S, 'parallelism': 'env-sharded x%d (no collective)' % world
            if shard is None else 'env-sharded x%d + one RCCL all-gather of the packed '
            'outputs per step, pipelined over 2 buffers' % world,
        },
        'roofline': {
            'bound': 'hbm', 'achieved': achieved_gbs, 'peak': HBM_PEAK_GBS,
            'unit': 'GB/s', 'frac': achieved_gbs / HBM_PEAK_GBS,
            'traffic': None,
            'bytes_per_env_step': bpe, 'kernel_ms_median': kernel_ms,
            'kernel_ms_mean': kernel_ms_mean, 'bytes_per_env_step_moved': moved,
            'kernel': 'ce::' + kernel, 'steps_per_launch': S if persistent else 1,
            'note': 'bytes_per_env_step: the state read and written every step (DESIGN 3.6); '
                    'bytes_per_env_step_moved: what the launch form moves',
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
                      'nn_agent_rows_kernel (dominant), nn_finalize_kernel',
            'bytes_per_env_step': bpe,
            'step_ms_median': kernel_ms, 'step_ms_mean': kernel_ms_mean,
            'flops_per_env_step': flops,
            'mfma_tflops': flops * E / (kernel_ms * 1e-3) / 1e12,
            'mfma_peak_tflops': MFMA_F32_PEAK_TFLOPS,
        },
    })
    return line


METRIC_MNIST = ('vectorised env-steps/sec, Optimize-v0 at the reference default data shape '
                '(mnist 7x7: 60000 x 49, 10 classes, B = N) @4096 envs, MI355X vs host CPU')
MFMA_F64_PEAK_TFLOPS = 78.6    # MI355X spec, f64 matrix (16x16x4 f64 measured at ~32 ns per wave instruction: profiles/r03_mfma_valu_mix.jsonl)


def mnist_line(args, eng, world, E, S, elapsed, kernel_ms, kernel_ms_mean):
    N, F, K = eng.n_rows, eng.n_features, eng.n_classes
    flops = 4 * N * F * K            # X W (2NFK) and X^T (P - Y) (2NFK) per env-step
    achieved = flops * E / (kernel_ms * 1e-3) / 1e12
    line = {'metric': METRIC_MNIST}
    line.update(_common(args, world, E, S, elapsed, None))
    line.update({
        'dtype': 'f64',
        'data': 'synthetic mnist7x7_synthetic: 60000 28x28 uint8 blob digits sampled at the '
                'PIL NEAREST 28->7 pixels, normalised, 10 classes; actions N(0, 0.01) float32 '
                'generated on device',
        'config': {'workload': 'Optimize-v0 softmax regression 49 x 10 (P=490, obs 981) over '
                               'N=60000 rows, B=N, %d envs per GPU, in-kernel auto-reset, '
                               'device-resident actions/outputs' % E,
                   'envs_per_gpu': E, 'global_envs': world * E, 'n_rows': N, 'n_features': F,
                   'n_classes': K, 'batch_size': eng.batch_size,
                   'parallelism': 'env-sharded x%d (no collective)' % world},
        'roofline': {'bound': 'mfma', 'achieved': achieved, 'peak': MFMA_F64_PEAK_TFLOPS,
                     'unit': 'TFLOP/s', 'frac': achieved / MFMA_F64_PEAK_TFLOPS,
                     'traffic': None, 'kernel': 'ce::' + eng.step_kernel,
                     'flops_per_env_step': flops, 'kernel_ms_median': kernel_ms,
                     'kernel_ms_mean': kernel_ms_mean,
                     'note': ('algorithmic GEMM flops; the class-concatenated kernel puts the '
                              '8 envs x 10 classes of a workgroup on 5 MFMA tiles of 16 (no class '
                              'padding) and the 49th feature on the VALU'
                              if 'cat' in eng.step_kernel else
                              'algorithmic GEMM flops; the kernel pads K 10 -> 16 and F 49 -> '
                              '52 (forward) / 64 (gradient) on 16x16x4 MFMA tiles')},
    })
    return line


def net_flops(dims, B, N):
    """Algorithmic FLOPs of one Optimize-v0 step over the network dims (F,
    hidden..., K): minibatch forward 2B sum(d_l d_l+1), backward dW 2B
    sum(d_l d_l+1) and dH 2B sum_{l>0}(d_l d_l+1); the full-data info forward
    2N sum(d_l d_l+1) when B < N (B == N reuses the minibatch pass)."""
    pairs = [a * b for a, b in zip(dims[:-1], dims[1:])]
    train = 2 * B * (2 * sum(pairs) + sum(pairs[1:]))
    info = 2 * N * sum(pairs) if B < N else 0
    return train, info


def net_line(args, eng, world, E, S, elapsed, kernel_ms, kernel_ms_mean, shard):
    """The layered network path on the hand-written MFMA kernels of
    csrc/net_kernels.h; the roofline is the MFMA rate over the step's
    algorithmic FLOPs (the reference's: minibatch forward + backward + the
    full-data info forward)."""
    dims = (784,) + tuple(args.hidden) + (10,)
    P = eng.act_dim
    train_f, info_f = net_flops(dims, args.batch_size, 1024)
    achieved = (train_f + info_f) * E / (kernel_ms * 1e-3) / 1e12
    line = {'metric': METRIC_MLP.replace('784-64-10 MLP @4096 envs',
                                         '%s network @%d envs' % ('-'.join(map(str, dims)), E))}
    line.update(_common(args, world, E, S, elapsed, shard))
    line.update({
        'dtype': 'f32',
        'data': 'synthetic: RandomState(0).rand(1024, 784), labels argmax(X T), '
                'T = RandomState(1).normal(784, 10); glorot-uniform init per env seed; '
                'actions N(0, 1e-3) float32 generated on device',
        'config': {
            'workload': 'Optimize-v0 over the %s relu network (P=%d, obs %d), %d envs per GPU, '
                        'B=%d of N=1024, full-data info pass every step, auto-reset, '
                        'device-resident actions/outputs' % ('-'.join(map(str, dims)), P,
                                                             2 * P + 1, E, args.batch_size),
            'envs_per_gpu': E, 'global_envs': world * E, 'n_rows': 1024, 'n_features': 784,
            'hidden': list(args.hidden), 'n_classes': 10, 'batch_size': args.batch_size,
            'parallelism': 'env-sharded x%d (no collective)' % world,
        },
        'roofline': {
            'bound': 'mfma', 'achieved': achieved, 'peak': MFMA_F32_PEAK_TFLOPS,
            'unit': 'TFLOP/s', 'frac': achieved / MFMA_F32_PEAK_TFLOPS, 'traffic': None,
            'kernel': 'one step = %s: net_fwd FUSED (W - a into the weight image by producer '
                      'waves + the minibatch forward in 16x16x4 f32 MFMA accumulators), then '
                      'concurrently net_fwd (every row, weights by LDS-DMA) on the main stream '
                      'and net_bwd + net_grad ([dW; db] on 32x32x2 MFMA with the float64 G/obs '
                      'epilogue from the accumulators) on a side stream, then net_finish; '
                      'no BLAS library' % eng.step_kernel,
            'flops_per_env_step': train_f + info_f, 'info_flops_per_env_step': info_f,
            'step_ms_median': kernel_ms, 'step_ms_mean': kernel_ms_mean,
        },
    })
    return line


def mlp_line(args, eng, world, E, S, elapsed, kernel_ms, kernel_ms_mean, shard, phase_ms):
    """The fused mlp_step_kernel is the step (one launch); its MFMA rate over
    the step's FLOPs is the roofline.  The split kernels, timed alone, give the
    two floors the fused kernel overlaps: the train phase's HBM streaming and
    the info phase's MFMA work."""
    P = eng.act_dim
    train_f, info_f = mlp_flops()
    info_ms = phase_ms.get('info')
    train_ms = phase_ms.get('train')
    achieved = (train_f + info_f) * E / (kernel_ms * 1e-3) / 1e12
    train_floor_ms = mlp_train_bytes(P) * E / (HBM_COPY_GBS * 1e9) * 1e3
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
            'kernel': 'ce::%s (train + full-data info pass, one launch per step)'
                      % eng.step_kernel,
            'flops_per_env_step': train_f + info_f, 'info_flops_per_env_step': info_f,
            'step_ms_median': kernel_ms, 'step_ms_mean': kernel_ms_mean,
            'split_info_kernel_ms': info_ms, 'split_train_kernel_ms': train_ms,
            'train_hbm_floor_ms': train_floor_ms,
            'overlap_floor_ms': max(train_floor_ms, info_ms) if info_ms else None,
            'train_kernel_hbm_bytes_per_env_step': mlp_train_bytes(P),
            'split_train_kernel_gbs': (mlp_train_bytes(P) * E / (train_ms * 1e-3) / 1e9
                                       if train_ms else None),
        },
    })
    return line


if __name__ == '__main__':
    sys.exit(main())

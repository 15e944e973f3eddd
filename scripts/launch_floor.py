"""Decompose the driver-form time of the persistent K-step launch.

    python scripts/launch_floor.py [--envs 4096] [--k 1 2 5 10 20 40]

For each K: the wall time of ONE rollout launch of K steps, bracketed by
torch.cuda.synchronize() as bench.py's timed region is, median over
--repeat launches; once right after a 5-step warmup (the driver's form), the same after
0.3 s of idle, and once after 2000 steps of back-to-back launches (the chip at its busy
clock).  A least-squares line through t(K) gives the per-step slope and the
fixed cost of one launch (host submission + dispatch + prologue + drain +
completion signal).  Also the same bracket around a 1-element torch kernel:
the host/GPU round-trip floor with no work.  One JSON line.
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--envs', type=int, default=4096)
    p.add_argument('--k', type=int, nargs='+', default=[1, 2, 5, 10, 20, 40])
    p.add_argument('--repeat', type=int, default=30)
    p.add_argument('--torch-stream', action='store_true',
                   help="run the engine on a torch.cuda.Stream() as bench.py does "
                        "(default: the engine's own non-blocking stream)")
    args = p.parse_args()
    import numpy as np
    import torch
    from custom_envs_amd.data import load_data
    from custom_envs_amd.engine import OptimizeEngine
    E = args.envs
    seq = load_data('gaussians_256x10', batch_size=None)
    eng = OptimizeEngine(seq.features, seq.targets, num_envs=E)
    eng.seed(list(range(E)))
    if args.torch_stream:
        stream = torch.cuda.Stream()
        torch.cuda.set_stream(stream)
        eng.set_stream(stream.cuda_stream)
    kmax = max(args.k)
    acts = torch.randn((kmax, E, eng.act_dim), device='cuda') * 0.01
    fields, rb = eng.alloc_rollout(kmax)
    eng.reset_device({n: v[0] for n, v in fields.items() if n != '_buffer'})
    runners = {k: eng.rollout_runner(k, acts, fields, rb) for k in args.k}

    def once(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e6

    res = {'kernel': eng.many_kernel, 'envs': E, 'torch_stream': args.torch_stream}
    x = torch.zeros(1, device='cuda')
    res['empty_torch_kernel_us'] = statistics.median(once(lambda: x.add_(1)) for _ in range(args.repeat))

    # the host side alone: the submission call (no wait), and a wait with
    # nothing pending
    def host_only(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        return (t1 - t0) * 1e6

    def idle_sync():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e6
    k0 = min(args.k)
    res['submit_call_us'] = statistics.median(host_only(runners[k0]) for _ in range(args.repeat))
    res['idle_sync_us'] = statistics.median(idle_sync() for _ in range(args.repeat))
    first = {}
    for state in ('after_warmup5', 'after_idle', 'busy'):
        t = {}
        for k in args.k:
            vals = []
            for _ in range(args.repeat):
                if state == 'after_idle':
                    torch.cuda.synchronize()
                    time.sleep(0.3)                      # long idle, then the 5-step warmup
                    runners[5 if 5 in runners else min(args.k)]()
                elif state == 'busy':
                    for _ in range(2000 // kmax):
                        runners[kmax]()
                else:
                    torch.cuda.synchronize()
                    time.sleep(0.002)                    # the chip idles, as between bench phases
                    runners[5 if 5 in runners else min(args.k)]()   # the driver's 5-step warmup
                vals.append(once(runners[k]))
            t[k] = statistics.median(vals)
            first[state, k] = vals[0]
        ks = np.array(sorted(t), float)
        ts = np.array([t[int(k)] for k in ks])
        slope, icept = np.polyfit(ks, ts, 1)
        res[state] = {'t_us': {int(k): round(t[int(k)], 2) for k in ks},
                      'per_step_us': round(float(slope), 3), 'fixed_us': round(float(icept), 2),
                      'us_per_step_at_20': round(t.get(20, float('nan')) / 20, 3),
                      'first_sample_us': {int(k): round(first[state, int(k)], 2) for k in ks}}
    print(json.dumps(res))
    eng.close()


if __name__ == '__main__':
    main()

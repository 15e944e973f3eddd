"""Host-loop (numpy in / numpy out, PCIe-inclusive) VecEnv rate at 4096
envs, with the time split into the parts of one step:
    python scripts/host_loop.py [--steps 300]"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--steps', type=int, default=300)
    p.add_argument('--envs', type=int, default=4096)
    args = p.parse_args()
    import torch  # noqa: F401  (the same process state as bench.py)
    from bench import lr_dataset
    from custom_envs_amd.engine import OptimizeEngine
    features, targets = lr_dataset()
    E = args.envs
    eng = OptimizeEngine(features, targets, num_envs=E)
    eng.seed(list(range(E)))
    eng.reset()
    act = np.random.RandomState(5).normal(0, 0.01, (E, eng.act_dim)).astype(np.float32)
    for _ in range(20):
        eng.step(act)
    res = {}
    t0 = time.perf_counter()
    for _ in range(args.steps):
        o = eng.step(act)
        o['obs'].copy()
    res['step_plus_obs_copy_us'] = (time.perf_counter() - t0) / args.steps * 1e6
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.step(act)
    res['step_us'] = (time.perf_counter() - t0) / args.steps * 1e6
    t0 = time.perf_counter()
    for _ in range(args.steps):
        o['obs'].copy()
    res['obs_copy_us'] = (time.perf_counter() - t0) / args.steps * 1e6
    buf = np.empty_like(act)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        np.copyto(buf, act)
    res['act_memcpy_us'] = (time.perf_counter() - t0) / args.steps * 1e6
    res['env_steps_per_s'] = E / (res['step_plus_obs_copy_us'] * 1e-6)
    res['h2d_direct'] = os.environ.get('CE_H2D_DIRECT', '0')
    print(res)
    eng.close()


if __name__ == '__main__':
    main()

"""Median step time of the config-3 MLP engine (4096 envs) on the current
CE_LIB build: HIP events around single device steps, no correctness checks
(experiment builds may skip work)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from bench import mlp_dataset
    from custom_envs_amd.engine import OptimizeEngine
    E = int(os.environ.get('MLP_ENVS', 4096))
    features, targets = mlp_dataset()
    eng = OptimizeEngine(features, targets, num_envs=E, batch_size=32, model='mlp')
    eng.seed(list(range(E)))
    stream = torch.cuda.Stream()
    eng.set_stream(stream.cuda_stream)
    out = eng.alloc_device_outputs()
    acts = torch.randn((2, E, eng.act_dim), device='cuda') * 1e-3
    torch.cuda.synchronize()
    eng.reset_device(out)
    for i in range(3):
        eng.step_device(acts[i % 2], out)
    n = 15
    st = [torch.cuda.Event(enable_timing=True) for _ in range(n)]
    en = [torch.cuda.Event(enable_timing=True) for _ in range(n)]
    for i in range(n):
        st[i].record(stream)
        eng.step_device(acts[i % 2], out)
        en[i].record(stream)
    torch.cuda.synchronize()
    ms = [a.elapsed_time(b) for a, b in zip(st, en)]
    print('%s %s step_ms median %.4f min %.4f' % (os.environ.get('CE_LIB', 'default'),
                                                   eng.step_kernel, float(np.median(ms)), min(ms)))
    eng.close()


if __name__ == '__main__':
    main()

"""Phase breakdown of the fused step kernel from the CE_DIAG stamp build.

    CE_LIB=diag python scripts/diag_phases.py [--envs 4096] [--precision f64]

Stamps (s_memtime, shader clock ticks) per wave:
  0 entry  1 after LDS staging barrier  2 after state loads + W broadcast
  3 after minibatch row loop  4 after wave reduction (+ info pass)
  5 after epilogue stores drained
Reports medians of each phase, the spread of wave start times and the
whole-kernel span.  Timing numbers from this build are shares, not speeds.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--envs', type=int, default=4096)
    p.add_argument('--precision', default='f64')
    p.add_argument('--steps', type=int, default=20)
    p.add_argument('--workload', default='optimize', choices=['optimize', 'mlp', 'mnist'])
    args = p.parse_args()
    assert os.environ.get('CE_LIB', '').startswith('diag'), 'run with CE_LIB=diag*'
    import torch
    from custom_envs_amd import _native
    from custom_envs_amd.data import load_data
    from custom_envs_amd.engine import OptimizeEngine
    lib = _native.load()
    lib.ce_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    E = args.envs
    if args.workload == 'mlp':
        from bench import mlp_dataset
        features, targets = mlp_dataset()
        eng = OptimizeEngine(features, targets, num_envs=E, batch_size=32, model='mlp')
    elif args.workload == 'mnist':
        from bench import mnist_dataset
        features, targets = mnist_dataset()
        eng = OptimizeEngine(features, targets, num_envs=E, precision='f64')
    else:
        seq = load_data('gaussians_256x10', batch_size=None)
        eng = OptimizeEngine(seq.features, seq.targets, num_envs=E, precision=args.precision)
    eng.seed(list(range(E)))
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    eng.set_stream(stream.cuda_stream)
    out = eng.alloc_device_outputs()
    acts = torch.randn((2, E, eng.act_dim), device='cuda') * 0.01
    eng.reset_device(out)
    for s in range(args.steps):
        eng.step_device(acts[s % 2], out)
    torch.cuda.synchronize()
    st = np.zeros((E, 8), np.uint64)
    _native.check(lib.ce_diag_stamps(eng._h, st.ctypes.data), 'diag')
    st = st.astype(np.int64)
    res = {'envs': E, 'precision': args.precision}
    names = ['stage+barrier', 'state loads+bcast', 'row loop', 'reduce+info', 'epilogue']
    if 'lr_mfma' in eng.step_kernel:
        # optimize_lr_mfma_kernel: one row per wave (16 envs x 8 waves per workgroup)
        st = st[st[:, 0] != 0]                      # rows = workgroups x waves (4, 8 or 16)
        names = ['W + first tile loads', 'row tiles', 'partials meet', 'scalar epilogue',
                 'param epilogue + drain']
    if 'optimize_cat_kernel' in eng.step_kernel:
        # class-concatenated kernel: slots 0-5 = per-phase sums over the
        # 64-row blocks, 6 / 7 = the wave's start / end s_memtime
        names = ['top wait (LDS-DMA + barrier 1)', 'forward', 'barrier 2', 'softmax', 'barrier 3',
                 'gradient issue']
        res['kernel'] = eng.step_kernel
        total = st[:, 7] - st[:, 6]
        res['wave_total_median'] = float(np.median(total))
        for k, name in enumerate(names):
            res[name] = {'median': float(np.median(st[:, k])),
                         'share': float(np.median(st[:, k] / total))}
        print(json.dumps(res))
        return
    if 'mlp' in eng.step_kernel:
        # mlp_step_kernel: train half stamps 0-3, info half 4-6 of the same env
        names = ['forward', 'softmax + small grads', 'dW1 + G/obs', 'train end -> info start',
                 'info passes', 'info epilogue + drain']
        res['kernel'] = eng.step_kernel
        for k, name in enumerate(names):
            d = st[:, k + 1] - st[:, k]
            res[name] = {'median': float(np.median(d)), 'p90': float(np.percentile(d, 90))}
        res['train_median'] = float(np.median(st[:, 3] - st[:, 0]))
        res['info_median'] = float(np.median(st[:, 6] - st[:, 4]))
        print(json.dumps(res))
        return
    res['kernel'] = eng.step_kernel
    for k, name in enumerate(names):
        d = st[:, k + 1] - st[:, k]
        res[name] = {'median': float(np.median(d)), 'p90': float(np.percentile(d, 90))}
    res['wave_total_median'] = float(np.median(st[:, 5] - st[:, 0]))
    # s_memrealtime (100 MHz, chip-wide): wave start/end relative to the first start
    rt0 = st[:, 6].min()
    starts_us = (st[:, 6] - rt0) / 100.0
    ends_us = (st[:, 7] - rt0) / 100.0
    res['start_us'] = {'p50': float(np.median(starts_us)), 'p90': float(np.percentile(starts_us, 90)),
                       'max': float(starts_us.max())}
    res['end_us'] = {'p10': float(np.percentile(ends_us, 10)), 'p50': float(np.median(ends_us)),
                     'max': float(ends_us.max())}
    res['life_us_p50'] = float(np.median(ends_us - starts_us))
    print(json.dumps(res))


if __name__ == '__main__':
    main()

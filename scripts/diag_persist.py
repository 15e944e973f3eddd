"""Phase breakdown of the persistent K-step kernel (CE_DIAG stamp build).

    CE_LIB=diag python scripts/diag_persist.py [--envs 4096] [--k 20 250]

Stamps (s_memrealtime, 100 MHz chip-wide, per wave): 0 entry, 1 prologue
loaded (state + row tiles + first actions, vmcnt(0)), 2 / 3 steps 0 / 1
done (after their barrier), 4 step K-1's barrier, 5 loop exit, 6 final
stores drained; ws form: 7 step 1's row work done (row waves) and, for the
epilogue waves, 2 = step 1's barrier passed, 7 = step 1's epilogue
drained.  One JSON line per K: medians over waves in microseconds, the
spread of wave starts and the launch span (first start to last drain).
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
    p.add_argument('--k', type=int, nargs='+', default=[20, 250])
    p.add_argument('--repeat', type=int, default=5)
    args = p.parse_args()
    assert os.environ.get('CE_LIB', '').startswith('diag'), 'run with CE_LIB=diag'
    import torch
    from custom_envs_amd import _native
    from custom_envs_amd.data import load_data
    from custom_envs_amd.engine import OptimizeEngine
    lib = _native.load()
    lib.ce_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    E = args.envs
    seq = load_data('gaussians_256x10', batch_size=None)
    eng = OptimizeEngine(seq.features, seq.targets, num_envs=E)
    eng.seed(list(range(E)))
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    eng.set_stream(stream.cuda_stream)
    kmax = max(args.k)
    acts = torch.randn((kmax, E, eng.act_dim), device='cuda') * 0.01
    fields, rb = eng.alloc_rollout(kmax)
    eng.reset_device({n: v[0] for n, v in fields.items() if n != '_buffer'})
    for k in args.k:
        rows, epi = [], []
        for _ in range(args.repeat):
            eng.rollout_device(k, acts, fields, rb)
            torch.cuda.synchronize()
            st = np.zeros((E, 8), np.uint64)
            _native.check(lib.ce_diag_stamps(eng._h, st.ctypes.data), 'diag')
            st = st.astype(np.int64)
            epi.append(st[(st[:, 0] != 0) & (st[:, 1] == 0)])   # ws form: the epilogue waves
            st = st[(st[:, 0] != 0) & (st[:, 1] != 0)]    # row waves (ws form: not the epilogue waves)
            rows.append(st)
        st = np.concatenate(rows)
        us = lambda d: float(np.median(d)) / 100.0     # 10 ns ticks
        res = {'kernel': eng.many_kernel, 'envs': E, 'k': k, 'waves_sampled': int(len(st)),
               'prologue_us': us(st[:, 1] - st[:, 0]),
               'step0_us': us(st[:, 2] - st[:, 1]),
               'step1_us': us(st[:, 3] - st[:, 2]),
               'steady_step_us': us((st[:, 4] - st[:, 3]) / max(1, k - 2)),
               'last_epilogue_us': us(st[:, 5] - st[:, 4]),
               'final_flush_drain_us': us(st[:, 6] - st[:, 5]),
               'wave_life_us': us(st[:, 6] - st[:, 0])}
        if st[:, 7].any():      # ws form: step 1's row work and the barrier wait after it
            res['step1_row_work_us'] = us(st[:, 7] - st[:, 2])
            res['step1_barrier_wait_us'] = us(st[:, 3] - st[:, 7])
        ep = np.concatenate(epi)
        if len(ep) and ep[:, 7].any():
            res['epilogue_waves_sampled'] = int(len(ep))
            res['step1_epilogue_work_us'] = us(ep[:, 7] - ep[:, 2])
        last = rows[-1]
        t0 = last[:, 0].min()
        res['start_spread_us'] = float(np.percentile(last[:, 0] - t0, 99)) / 100.0
        res['span_us'] = float(last[:, 6].max() - t0) / 100.0
        print(json.dumps(res))
    eng.close()


if __name__ == '__main__':
    main()

"""Phase breakdown of the NN eval kernels (nn_grad_kernel, nn_step_kernel)
from the CE_DIAG stamp build.

    CE_LIB=diag python scripts/diag_nn.py [--envs 1024]

Stamps (s_memtime, thread 0 of each workgroup): 0 entry, 1 batch staged,
2 first hidden layer (+ output-kernel staging), 3 remaining hidden layers,
4 logits + softmax, 5 output-layer backward, 6 hidden backward down to layer
1, 7 layer-0 backward; 8/9 s_memrealtime (100 MHz) at entry/exit.
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
    p.add_argument('--envs', type=int, default=1024)
    p.add_argument('--steps', type=int, default=4)
    args = p.parse_args()
    assert os.environ.get('CE_LIB', '').startswith('diag'), 'run with CE_LIB=diag*'
    import torch
    from custom_envs_amd import _native
    from custom_envs_amd.multi_engine import NNMultiEngine
    lib = _native.load()
    lib.ce_nn_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    E = args.envs
    eng = NNMultiEngine(E)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    eng.set_stream(stream.cuda_stream)
    out = eng.alloc_device_outputs()
    acts = torch.rand((args.steps, E * eng.n_params), device='cuda') * 1.5 + 1.0
    eng.reset_device(out)
    for s in range(args.steps):
        eng.step_device(acts[s], out)
    torch.cuda.synchronize()
    st = np.zeros((2, E, 10), np.uint64)
    _native.check(lib.ce_nn_diag_stamps(eng._h, st.ctypes.data), 'diag')
    st = st.astype(np.int64)
    names = ['stage', 'fwd layer0 + Wout stage', 'fwd hidden', 'logits+softmax', 'bwd output',
             'bwd hidden', 'bwd layer0']
    res = {'envs': E}
    for kk, kern in enumerate(('grad', 'step')):
        r = {}
        for k, name in enumerate(names):
            d = st[kk, :, k + 1] - st[kk, :, k]
            r[name] = float(np.median(d))
        r['total'] = float(np.median(st[kk, :, 7] - st[kk, :, 0]))
        t0 = st[kk, :, 8].min()
        r['life_us_p50'] = float(np.median(st[kk, :, 9] - st[kk, :, 8])) / 100.0
        r['span_us'] = float(st[kk, :, 9].max() - t0) / 100.0
        r['start_us_p90'] = float(np.percentile(st[kk, :, 8] - t0, 90)) / 100.0
        res[kern] = r
    print(json.dumps(res))
    eng.close()


if __name__ == '__main__':
    main()

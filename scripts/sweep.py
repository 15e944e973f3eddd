"""Per-step time of the fused step kernel across precisions and env counts.

    python scripts/sweep.py [--envs 1024,4096,16384] [--precisions f64,f32]

Device-resident actions, hipGraph replay of S steps, wall time per step and
the derived env-steps/s; one JSON line per configuration.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--envs', default='1024,4096,16384,65536')
    p.add_argument('--precisions', default='f64,f32')
    p.add_argument('--steps', type=int, default=1000)
    p.add_argument('--batch-size', type=int, default=0)
    args = p.parse_args()
    import torch
    from custom_envs_amd.data import load_data
    from custom_envs_amd.engine import OptimizeEngine
    seq = load_data('gaussians_256x10', batch_size=None)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    for prec in args.precisions.split(','):
        for E in [int(v) for v in args.envs.split(',')]:
            eng = OptimizeEngine(seq.features, seq.targets, num_envs=E, precision=prec,
                                 batch_size=args.batch_size or None)
            eng.seed(list(range(E)))
            eng.set_stream(stream.cuda_stream)
            out = eng.alloc_device_outputs()
            S = 250
            acts = torch.randn((S, E, eng.act_dim), device='cuda') * 0.01
            eng.reset_device(out)
            eng.step_many_device(S, acts, out)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps // S):
                eng.step_many_device(S, acts, out)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / (args.steps // S * S)
            print(json.dumps({'precision': prec, 'envs': E, 'us_per_step': dt * 1e6,
                              'env_steps_per_s': E / dt}), flush=True)
            eng.close()


if __name__ == '__main__':
    main()

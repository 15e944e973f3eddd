"""Experiment: the benchmark's envs split into S engines on S HIP streams
(each engine a hipGraph chain of its own steps), against one engine.  Envs
are independent, so the chains need no cross-stream sync; the question is
whether one chain's kernel boundary hides under another chain's work.

  python scripts/stream_shards.py [--envs 4096] [--shards 1,2,4] [--steps 2000]
Prints one JSON line per shard count.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--envs', type=int, default=4096)
    p.add_argument('--shards', default='1,2,4')
    p.add_argument('--steps', type=int, default=2000)
    p.add_argument('--chunk', type=int, default=250)
    args = p.parse_args()
    import torch
    from bench import lr_dataset
    from custom_envs_amd.engine import OptimizeEngine
    features, targets = lr_dataset()
    for S in [int(s) for s in args.shards.split(',')]:
        n = args.envs // S
        engs, outs, acts, streams = [], [], [], []
        for i in range(S):
            st = torch.cuda.Stream()
            eng = OptimizeEngine(features, targets, num_envs=n, device=0)
            eng.seed([i * n + j for j in range(n)])
            eng.set_stream(st.cuda_stream)
            gen = torch.Generator(device='cuda').manual_seed(1234 + i)
            a = torch.randn((args.chunk, n, eng.act_dim), generator=gen, device='cuda') * 0.01
            o = eng.alloc_device_outputs()
            eng.reset_device(o)
            eng.prepare_many_device(args.chunk, a, o)
            engs.append(eng), outs.append(o), acts.append(a), streams.append(st)
        torch.cuda.synchronize()

        def run(k):
            for _ in range(k // args.chunk):
                for eng, a, o in zip(engs, acts, outs):
                    eng.step_many_device(args.chunk, a, o)

        run(2 * args.chunk)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(args.steps)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({'shards': S, 'envs': args.envs, 'kernel': engs[0].step_kernel,
                          'us_per_step': dt / args.steps * 1e6,
                          'env_steps_per_s': args.envs * args.steps / dt}), flush=True)
        for eng in engs:
            eng.close()
        del outs, acts
        torch.cuda.synchronize()
    return 0


if __name__ == '__main__':
    sys.exit(main())

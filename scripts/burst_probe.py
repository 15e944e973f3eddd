"""Where the driver's 20-step form spends its time: host wall time of the
timed region (synchronize, K steps through the bench's pre-bound runner,
synchronize) against the GPU time between HIP events recorded on the engine
stream right before the first and after the last step, and each kernel's
own duration (events around every launch).  4096 envs, f64.

    python scripts/burst_probe.py [--steps 20] [--reps 5] [--preheat-ms 0]

--preheat-ms X: before each rep, X ms of back-to-back steps and then an idle
gap of --gap-ms (is a burst's per-kernel time a clock / power state that a
busy GPU leaves behind?).
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
    p.add_argument('--steps', type=int, default=20)
    p.add_argument('--reps', type=int, default=5)
    p.add_argument('--warmup', type=int, default=5)
    p.add_argument('--preheat-ms', type=float, default=0.0)
    p.add_argument('--gap-ms', type=float, default=0.0)
    args = p.parse_args()
    import torch
    from bench import lr_dataset
    from custom_envs_amd.engine import OptimizeEngine
    features, targets = lr_dataset()
    E, K = 4096, args.steps
    eng = OptimizeEngine(features, targets, num_envs=E, device=0)
    eng.seed(list(range(E)))
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    eng.set_stream(stream.cuda_stream)
    out = eng.alloc_device_outputs()
    acts = torch.randn((K, E, eng.act_dim), device='cuda') * 0.01
    eng.reset_device(out)
    run_k = eng.many_runner(K, acts, out)
    run_w = eng.many_runner(args.warmup, acts, out) if args.warmup else None
    torch.cuda.synchronize()
    run_heat = eng.many_runner(250, torch.randn((250, E, eng.act_dim), device='cuda') * 0.01, out)
    for rep in range(args.reps):
        if args.preheat_ms > 0:
            t_h = time.perf_counter()
            while (time.perf_counter() - t_h) * 1e3 < args.preheat_ms:
                run_heat()
                torch.cuda.synchronize()
        if args.gap_ms > 0:
            time.sleep(args.gap_ms / 1e3)
        if run_w:
            run_w()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(stream)
        run_k()
        e1.record(stream)
        t_issue = time.perf_counter()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        gpu_us = e0.elapsed_time(e1) * 1e3
        print(json.dumps({'rep': rep, 'steps': K, 'preheat_ms': args.preheat_ms, 'gap_ms': args.gap_ms, 'wall_us': (t1 - t0) * 1e6,
                          'issue_us': (t_issue - t0) * 1e6, 'gpu_events_us': gpu_us,
                          'wall_us_per_step': (t1 - t0) * 1e6 / K,
                          'gpu_us_per_step': gpu_us / K}), flush=True)
    eng.close()
    return 0


if __name__ == '__main__':
    sys.exit(main())

"""Does the gloo backend all-gather CUDA tensors (all_gather_into_tensor,
in place) between two processes on one GPU?  Run as
    python scripts/gloo_cuda_probe.py   (spawns its two ranks as children)"""
import os
import subprocess
import sys


def rank_main(rank):
    import torch
    import torch.distributed as dist
    dist.init_process_group('gloo', rank=rank, world_size=2)
    torch.cuda.set_device(0)
    n = 8
    out = torch.zeros(2 * n, device='cuda')
    out[rank * n:(rank + 1) * n] = rank + 1
    dist.all_gather_into_tensor(out, out[rank * n:(rank + 1) * n])
    torch.cuda.synchronize()
    print('rank', rank, out.cpu().tolist(), flush=True)
    dist.destroy_process_group()


if __name__ == '__main__':
    if len(sys.argv) > 1:
        rank_main(int(sys.argv[1]))
        sys.exit(0)
    env = dict(os.environ, MASTER_ADDR='127.0.0.1', MASTER_PORT='29611')
    procs = [subprocess.Popen([sys.executable, __file__, str(r)], env=env) for r in range(2)]
    sys.exit(max(p.wait(timeout=120) for p in procs))

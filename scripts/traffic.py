"""HBM traffic of one bench step from rocprofv3 counters (committed evidence).

    python scripts/traffic.py collect --round r04 --name optimize -- <bench.py args>
    python scripts/traffic.py summarize --round r04 --name optimize --src DIR --steps K \
        --envs E --step-kernel SUBSTR [--bytes-per-env-step B]

``collect`` runs bench.py twice under ``rocprofv3 --pmc`` as CHILD processes
(FETCH_SIZE and WRITE_SIZE need separate passes on gfx950: 3 + 2 of the 4 TCC
slots), each under its own hard time limit, then summarises.  ``summarize``
averages each counter over the dispatches of every engine kernel (name
contains ``ce::``), applies the gfx950 corrections of MI355X_MICROARCH.md
(HBM section: both counters are KiB; FETCH_SIZE reports half the bytes of
a wide coalesced read, so it is doubled -- narrower accesses are
uncalibrated, and the doubling then overstates them) and sums the kernels
of one step: bytes per step = sum over kernels of mean bytes per dispatch x
dispatches per step, dispatches per step = dispatches / the step kernel's
dispatches, divided by ``steps_per_dispatch`` when the step kernel runs
several steps per launch (the persistent K-step kernel).  The CLI writes
profiles/<round>_traffic_<name>.json (the committed evidence); bench.py's
in-run measurement writes under gpurun_out/traffic/ and names that file in
``roofline.traffic_source``.
"""
import argparse
import collections
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _counters(src, counter):
    per = collections.defaultdict(list)
    for path in sorted(glob.glob(os.path.join(src, '**', '*counter_collection.csv'), recursive=True)):
        for row in csv.DictReader(open(path)):
            # a step's kernels: the engine's (ce::), not the one-off resets
            # before the timed steps (an auto-reset runs inside the step)
            if row['Counter_Name'] == counter and 'ce::' in row['Kernel_Name'] \
                    and 'reset' not in row['Kernel_Name']:
                per[row['Kernel_Name']].append(float(row['Counter_Value']))
    return per


def _short(name):
    name = name.split('(')[0]
    return name.replace('void ', '')


def summarize(src_fetch, src_write, step_kernel, envs, name, rnd, bpe=None, extra=None,
              out_dir=None, steps_per_dispatch=1):
    """Bytes per step from the two counter passes.  Raises ValueError when
    no dispatch of `step_kernel` was counted (a caller catching Exception
    keeps going); writes <out_dir>/<rnd>_traffic_<name>.json (default: the
    CE_TRAFFIC_OUT directory, else profiles/)."""
    fetch = _counters(src_fetch, 'FETCH_SIZE')
    write = _counters(src_write, 'WRITE_SIZE')
    marker = [k for k in fetch if step_kernel in k]
    if not marker:
        raise ValueError('no dispatch of %r in the FETCH_SIZE pass' % step_kernel)
    steps = len(fetch[marker[0]]) * steps_per_dispatch
    wsteps = sum(len(v) for k, v in write.items() if step_kernel in k)
    kernels = {}
    total_r = total_w = 0.0
    for k in sorted(set(fetch) | set(write)):
        rd = fetch.get(k, [])
        wr = write.get(k, [])
        r_mean = 2.0 * 1024 * sum(rd) / len(rd) if rd else 0.0
        w_mean = 1024 * sum(wr) / len(wr) if wr else 0.0
        per_step = (len(rd) / steps if rd else
                    (len(wr) / (wsteps * steps_per_dispatch) if wsteps else 0.0))
        kernels[_short(k)] = {'read_bytes_per_dispatch': r_mean, 'write_bytes_per_dispatch': w_mean,
                              'dispatches_per_step': per_step}
        total_r += r_mean * per_step
        total_w += w_mean * per_step
    out = {'round': rnd, 'name': name, 'envs': envs, 'step_kernel': step_kernel,
           'steps_profiled': steps, 'steps_per_dispatch': steps_per_dispatch, 'hbm_read_bytes_per_step': total_r,
           'hbm_write_bytes_per_step': total_w, 'hbm_bytes_per_step': total_r + total_w,
           'kernels': kernels,
           'method': 'rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate runs; '
                     'KiB x 1024, FETCH_SIZE doubled (gfx950, MI355X_MICROARCH HBM section); '
                     'summed over the step\'s kernels'}
    if bpe:
        out['algorithmic_bytes_per_step'] = bpe * envs
        out['traffic_over_algorithmic'] = (total_r + total_w) / (bpe * envs)
    if extra:
        out.update(extra)
    # CE_TRAFFIC_OUT: where to write (a GPU box returns only gpurun_out/;
    # the committed copies live in profiles/)
    out_dir = out_dir or os.environ.get('CE_TRAFFIC_OUT', os.path.join(ROOT, 'profiles'))
    os.makedirs(out_dir, exist_ok=True)
    path = os.path.join(out_dir, '%s_traffic_%s.json' % (rnd, name))
    with open(path, 'w') as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    return out, path


def collect(rnd, name, bench_args, out_dir, limit=150):
    """Two counter passes of bench.py as child processes (never exec'd from a
    process that touched the GPU), each killed at `limit` seconds."""
    dirs = {}
    os.makedirs(out_dir, exist_ok=True)
    for counter in ('FETCH_SIZE', 'WRITE_SIZE'):
        d = os.path.join(out_dir, counter.lower())
        cmd = ['timeout', '-s', 'KILL', str(limit), 'rocprofv3', '--pmc', counter, '-d', d, '-o', 'run',
               '--output-format', 'csv', '--', sys.executable, os.path.join(ROOT, 'bench.py')] + bench_args
        with open(d + '.log', 'w') as log:
            rc = subprocess.call(cmd, cwd=ROOT, stdout=log, stderr=subprocess.STDOUT,
                                 env=dict(os.environ, TMPDIR=os.environ.get('TMPDIR', '/tmp')))
        if rc != 0:
            raise RuntimeError('rocprofv3 --pmc %s exited %d (log %s.log)' % (counter, rc, d))
        dirs[counter] = d
    return dirs['FETCH_SIZE'], dirs['WRITE_SIZE']


def main():
    p = argparse.ArgumentParser()
    p.add_argument('mode', choices=['collect', 'summarize'])
    p.add_argument('--round', required=True)
    p.add_argument('--name', required=True)
    p.add_argument('--step-kernel', required=True, help='substring of the once-per-step kernel')
    p.add_argument('--envs', type=int, required=True)
    p.add_argument('--bytes-per-env-step', type=float, default=None)
    p.add_argument('--steps-per-dispatch', type=int, default=1)
    p.add_argument('--src', default=None, help='summarize: directory with fetch_size/ write_size/')
    p.add_argument('--out', default=os.path.join(ROOT, 'gpurun_out', 'traffic'))
    p.add_argument('bench_args', nargs=argparse.REMAINDER)
    args = p.parse_args()
    bench_args = [a for a in args.bench_args if a != '--']
    if args.mode == 'collect':
        os.makedirs(args.out, exist_ok=True)
        f, w = collect(args.round, args.name, bench_args, os.path.join(args.out, args.name))
    else:
        src = args.src or os.path.join(args.out, args.name)
        f, w = os.path.join(src, 'fetch_size'), os.path.join(src, 'write_size')
    try:
        out, path = summarize(f, w, args.step_kernel, args.envs, args.name, args.round,
                              args.bytes_per_env_step, {'bench_args': ' '.join(bench_args)},
                              steps_per_dispatch=args.steps_per_dispatch)
    except ValueError as exc:
        raise SystemExit(str(exc))
    print(path)
    print(json.dumps({k: v for k, v in out.items() if k != 'kernels'}, indent=1, sort_keys=True))


if __name__ == '__main__':
    main()

"""Summarise rocprofv3 outputs into profiles/ (committed evidence).

    python scripts/pmc_summary.py --round r01 [--envs 4096 --precision f64]

Reads gpurun_out/prof/run_kernel_stats.csv (kernel trace --stats) and the
--pmc passes under gpurun_out/pmc/p*/run_counter_collection.csv, averages
each counter over the step-kernel dispatches, and applies the gfx950
corrections of MI355X_MICROARCH.md (HBM section): FETCH_SIZE and
WRITE_SIZE are KiB; FETCH_SIZE reports half the bytes of a wide coalesced
read, so it is doubled.  Writes profiles/<round>_kernel_stats.csv,
profiles/<round>_pmc.json.  (bench.py's roofline.traffic comes from
scripts/traffic.py's named per-round summaries, not from this file.)
"""
import argparse
import collections
import csv
import glob
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = ('optimize_lr_mfma_kernel', 'optimize_pair_kernel', 'optimize_step_kernel')   # the engine's step kernels


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--round', required=True)
    p.add_argument('--envs', type=int, default=4096)
    p.add_argument('--precision', default='f64')
    p.add_argument('--bytes-per-env-step', type=int, default=925)
    p.add_argument('--tag', default='', help='suffix of the summary file name')
    p.add_argument('--src', default='gpurun_out', help='directory holding prof/ and pmc/')
    args = p.parse_args()
    out_dir = os.path.join(ROOT, 'profiles')
    os.makedirs(out_dir, exist_ok=True)
    stats = os.path.join(ROOT, args.src, 'prof', 'run_kernel_stats.csv')
    summary = {'round': args.round, 'envs': args.envs, 'precision': args.precision}
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(out_dir, '%s_kernel_stats%s.csv' % (args.round, args.tag)))
        for row in csv.DictReader(open(stats)):
            if any(k in row['Name'] for k in KERNELS):
                summary['kernel'] = row['Name']
                summary['kernel_avg_ns'] = float(row['AverageNs'])
                summary['kernel_calls'] = int(row['Calls'])
    counters = collections.defaultdict(list)
    for path in sorted(glob.glob(os.path.join(ROOT, args.src, 'pmc', 'p*',
                                              'run_counter_collection.csv'))):
        for row in csv.DictReader(open(path)):
            if any(k in row['Kernel_Name'] for k in KERNELS):
                counters[row['Counter_Name']].append(float(row['Counter_Value']))
    means = {k: sum(v) / len(v) for k, v in counters.items()}
    summary['pmc_mean_per_dispatch'] = means
    if 'FETCH_SIZE' in means and 'WRITE_SIZE' in means:
        read_b = 2.0 * means['FETCH_SIZE'] * 1024      # gfx950: FETCH_SIZE = half
        write_b = means['WRITE_SIZE'] * 1024
        summary['hbm_read_bytes_per_launch'] = read_b
        summary['hbm_write_bytes_per_launch'] = write_b
        summary['hbm_bytes_per_launch'] = read_b + write_b
        summary['algorithmic_bytes_per_launch'] = args.bytes_per_env_step * args.envs
    if 'SQ_WAVES' in means:
        waves = means['SQ_WAVES']
        for key in ('SQ_INSTS_VALU', 'SQ_INSTS_SALU', 'SQ_INSTS_LDS', 'SQ_INSTS_VMEM'):
            if key in means:
                summary[key.lower() + '_per_wave'] = means[key] / waves
        for key in ('SQ_WAVE_CYCLES', 'SQ_WAIT_ANY', 'SQ_WAIT_INST_ANY', 'SQ_ACTIVE_INST_ANY',
                    'SQ_ACTIVE_INST_VALU'):
            if key in means:   # quad-cycles per the microarch guide
                summary[key.lower() + '_cycles_per_wave'] = 4 * means[key] / waves
    with open(os.path.join(out_dir, '%s_pmc%s.json' % (args.round, args.tag)), 'w') as fh:
        json.dump(summary, fh, indent=1, sort_keys=True)
    print(json.dumps(summary, indent=1, sort_keys=True))


if __name__ == '__main__':
    main()

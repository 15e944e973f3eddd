"""Per-kernel means of the NN PMC passes (gpurun_out/pmc_nn/p*/): counters
averaged over each kernel's dispatches; FETCH_SIZE / WRITE_SIZE are KiB and
FETCH_SIZE is doubled on gfx950 (MI355X_MICROARCH.md, HBM section)."""
import collections
import csv
import glob
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in glob.glob(os.path.join(ROOT, 'gpurun_out', 'pmc_nn', 'p*', '**',
                                       '*counter_collection.csv'), recursive=True):
        for row in csv.DictReader(open(path)):
            name = row.get('Kernel_Name', '')
            short = name.split('(')[0].replace('ce::', '')
            acc[short][row['Counter_Name']].append(float(row['Counter_Value']))
    out = {}
    for k, ctrs in acc.items():
        d = {c: sum(v) / len(v) for c, v in ctrs.items()}
        if 'FETCH_SIZE' in d:
            d['hbm_read_bytes'] = d['FETCH_SIZE'] * 1024 * 2
        if 'WRITE_SIZE' in d:
            d['hbm_write_bytes'] = d['WRITE_SIZE'] * 1024
        out[k] = d
    print(json.dumps(out, indent=1, sort_keys=True))
    with open(os.path.join(ROOT, 'gpurun_out', 'pmc_nn', 'summary.json'), 'w') as fh:
        json.dump(out, fh, indent=1, sort_keys=True)


if __name__ == '__main__':
    main()

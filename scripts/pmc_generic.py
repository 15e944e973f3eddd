"""Mean of every --pmc counter over the dispatches of one kernel.

    python scripts/pmc_generic.py <rocprofv3 output dir> <kernel-name substring> [out.json]

Reads <dir>/p*/run_counter_collection.csv (one rocprofv3 --pmc pass per
p* directory) and prints / writes {counter: mean per dispatch}."""
import collections
import csv
import glob
import json
import os
import sys


def main():
    root, name = sys.argv[1], sys.argv[2]
    counters = collections.defaultdict(list)
    for path in sorted(glob.glob(os.path.join(root, 'p*', '**', '*counter_collection.csv'),
                                 recursive=True)):
        for row in csv.DictReader(open(path)):
            if name in row['Kernel_Name']:
                counters[row['Counter_Name']].append(float(row['Counter_Value']))
    means = {k: sum(v) / len(v) for k, v in sorted(counters.items())}
    means['_dispatches'] = {k: len(v) for k, v in counters.items()}
    text = json.dumps(means, indent=1)
    print(text)
    if len(sys.argv) > 3:
        with open(sys.argv[3], 'w') as fh:
            fh.write(text + '\n')


if __name__ == '__main__':
    main()

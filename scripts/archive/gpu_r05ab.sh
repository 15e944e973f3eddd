#!/bin/bash
# Round 5 diagnosis of the three-wave config-5 kernel: timing-only builds
# (incomplete outputs) with the state wave's exp10 replaced by a multiply
# (mpnoexp), the info wave's reductions skipped (mpnoinfo), the rows wave's
# copy-out skipped (mpnocopy).
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r05ab
mkdir -p $OUT
for i in 1 2; do
  for lib in default mpnoexp mpnoinfo mpnocopy; do
    if [ $lib = default ]; then L=""; else L=$lib; fi
    CE_LIB=$L timeout -k 10 300 python -u bench.py --workload multi --no-cpu-baseline --no-measure-traffic \
        > $OUT/bench_${lib}_$i.json 2>> $OUT/bench.err || exit $?
  done
done
python -c "
import json,sys
for f in sys.argv[1:]:
    d=json.loads([l for l in open(f).read().splitlines() if l.startswith('{')][-1]); print(f, '%.4g'%d['value'], round(d['ms_per_step']*1e3,4))" $OUT/bench_*.json

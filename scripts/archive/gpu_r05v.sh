#!/bin/bash
# Round 5 diagnosis: which half of config 5's two-wave K-step kernel bounds
# the step -- timing-only builds whose output wave skips its info reductions
# (CE_LIB=mpnoinfo) or its observation copy-out (CE_LIB=mpnocopy); their
# outputs are incomplete by design.
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r05v
mkdir -p $OUT
for i in 1 2; do
  for lib in default mpnoinfo mpnocopy; do
    if [ $lib = default ]; then L=""; else L=$lib; fi
    CE_LIB=$L timeout -k 10 300 python -u bench.py --workload multi --no-cpu-baseline --no-measure-traffic \
        > $OUT/bench_${lib}_$i.json 2>> $OUT/bench.err || exit $?
  done
done
python -c "
import json,sys
for f in sys.argv[1:]:
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d['value'], d['ms_per_step']*1e3)" $OUT/bench_*.json

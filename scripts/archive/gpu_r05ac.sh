#!/bin/bash
# Round 5 A/B: the driver form's warmup as two waited launches (shipped) vs
# four single-step waited launches and the rest (CE_BENCH_WARM=single4, an
# A/B switch of that experiment build; the shipped bench now does the latter).
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r05ac
mkdir -p $OUT
for i in 1 2 3 4; do
  for m in split2 single4; do
    CE_BENCH_WARM=$m timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline \
        --no-measure-traffic > $OUT/bench20_${m}_$i.json 2>> $OUT/bench.err || exit $?
  done
done
python -c "
import json,sys
for f in sys.argv[1:]:
    d=json.loads([l for l in open(f).read().splitlines() if l.startswith('{')][-1]); print(f, '%.4g'%d['value'], round(d['ms_per_step']*1e3,4))" $OUT/bench20_*.json

#!/bin/bash
# Round 5 experiment: touching the slab and actions before the timed region.
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r05p
mkdir -p $OUT
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-measure-traffic \
      --repeat-timed 5 > $OUT/bench20_plain_$i.json 2> $OUT/bench20.err || exit $?
  CE_BENCH_TOUCH=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline \
      --no-measure-traffic --repeat-timed 5 > $OUT/bench20_touch_$i.json 2> $OUT/bench20.err || exit $?
done
python -c "
import json,sys
for f in sys.argv[1:]:
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d['value'], d['ms_per_step']*1e3, d['timed_repeats_ms'])" $OUT/bench20_*.json

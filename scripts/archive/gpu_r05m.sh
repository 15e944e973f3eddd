#!/bin/bash
# Round 5: host wait mode -- HSA_ENABLE_INTERRUPT=0 (polling signal waits)
# against the default, for one launch's round trip and the driver form.
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r05m
mkdir -p $OUT
for i in 1 2; do
  timeout -k 10 240 python -u scripts/launch_floor.py --k 1 5 20 > $OUT/floor_default_$i.json 2> $OUT/floor.err || exit $?
  HSA_ENABLE_INTERRUPT=0 timeout -k 10 240 python -u scripts/launch_floor.py --k 1 5 20 > $OUT/floor_poll_$i.json 2>> $OUT/floor.err || exit $?
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-measure-traffic \
      > $OUT/bench20_default_$i.json 2> $OUT/bench20.err || exit $?
  HSA_ENABLE_INTERRUPT=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline \
      --no-measure-traffic > $OUT/bench20_poll_$i.json 2>> $OUT/bench20.err || exit $?
done
cat $OUT/floor_*.json
python -c "
import json,sys
for f in sys.argv[1:]:
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d['value'], d['ms_per_step']*1e3)" $OUT/bench20_*.json

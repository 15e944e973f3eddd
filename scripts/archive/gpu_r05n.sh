#!/bin/bash
# Round 5: is the driver form's single timed sample a first-launch outlier?
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r05n
mkdir -p $OUT
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-measure-traffic \
      --repeat-timed 10 > $OUT/bench20_$i.json 2> $OUT/bench20.err || exit $?
done
timeout -k 10 240 python -u scripts/launch_floor.py --k 5 20 --torch-stream > $OUT/floor.json 2> $OUT/floor.err || exit $?
cat $OUT/floor.json
python -c "
import json,sys
for f in sys.argv[1:]:
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d['ms_per_step']*1e3, d['timed_repeats_ms'])" $OUT/bench20_*.json

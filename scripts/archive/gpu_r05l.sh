#!/bin/bash
# Round 5: the driver form's fixed cost, bench vs launch_floor on one box,
# engine stream own vs torch.
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r05l
mkdir -p $OUT
for i in 1 2; do
  timeout -k 10 240 python -u scripts/launch_floor.py --k 1 5 20 > $OUT/floor_own_$i.json 2> $OUT/floor.err || exit $?
  timeout -k 10 240 python -u scripts/launch_floor.py --k 1 5 20 --torch-stream > $OUT/floor_torch_$i.json 2>> $OUT/floor.err || exit $?
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-measure-traffic \
      > $OUT/bench20_$i.json 2> $OUT/bench20_$i.err || exit $?
done
cat $OUT/floor_*.json
python -c "
import json,sys
for f in sys.argv[1:]:
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d['value'], d['ms_per_step']*1e3)" $OUT/bench20_*.json

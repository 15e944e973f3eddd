#!/bin/bash
# Round 5: is the timed region's kernel slower than the post-run events loop
# because the chip is still ramping?  --timed-events at warmup 200 (default)
# and 4000, interleaved.
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r05y
mkdir -p $OUT
for i in 1 2; do
  for w in 200 4000; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-measure-traffic --timed-events --warmup $w \
        > $OUT/bench_w${w}_$i.json 2>> $OUT/bench.err || exit $?
  done
done
python -c "
import json,sys
for f in sys.argv[1:]:
    d=json.loads([l for l in open(f).read().splitlines() if l.startswith('{')][-1]); r=d['roofline']; print(f, round(d['ms_per_step']*1e3,4), round(r['kernel_ms_median']*1e3,4), r.get('kernel_ms_timed_region'))" $OUT/bench*.json

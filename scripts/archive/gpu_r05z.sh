#!/bin/bash
# Round 5: warmup and run length for the default headline line (the chip's
# clock ramp), with the roofline's kernel time from the timed region itself.
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r05z
mkdir -p $OUT
for i in 1 2; do
  for wk in "200 2000" "4000 2000" "20000 20000"; do
    set -- $wk
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-measure-traffic --warmup $1 --steps $2 \
        > $OUT/bench_w$1_k$2_$i.json 2>> $OUT/bench.err || exit $?
  done
done
timeout -k 10 300 python -u bench.py --workload multi --no-cpu-baseline --no-measure-traffic --warmup 20000 --steps 20000 \
    > $OUT/bench_multi_w20000_k20000.json 2>> $OUT/bench.err || exit $?
python -c "
import json,sys
for f in sys.argv[1:]:
    d=json.loads([l for l in open(f).read().splitlines() if l.startswith('{')][-1]); r=d['roofline']; print(f, '%.4g'%d['value'], round(d['ms_per_step']*1e3,4), r.get('kernel_ms_median'), r.get('kernel_ms_warm_loop'), r.get('frac'))" $OUT/bench*.json

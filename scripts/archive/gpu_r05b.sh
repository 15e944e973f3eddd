#!/bin/bash
# Round 5: persistent kernel phase stamps and the 4- vs 8-wave A/B.
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r05b
mkdir -p $OUT
for w in 4 8; do
  CE_LIB=diag CE_LP_WAVES=$w timeout -k 10 120 python -u scripts/diag_persist.py --k 20 250 > $OUT/diag_w$w.jsonl 2> $OUT/diag_w$w.err || exit $?
  cat $OUT/diag_w$w.jsonl
done
for rep in 1 2; do
for w in 4 8; do
  CE_LP_WAVES=$w timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-measure-traffic > $OUT/b20_w$w.$rep.json 2>> $OUT/bench.err || exit $?
  CE_LP_WAVES=$w timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-measure-traffic > $OUT/b_w$w.$rep.json 2>> $OUT/bench.err || exit $?
  python - $OUT/b20_w$w.$rep.json $OUT/b_w$w.$rep.json <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.load(open(f))
    print(f, d['roofline']['kernel'], 'value %.4g' % d['value'], 'us/step %.3f' % (d['ms_per_step'] * 1e3),
          'kernel us/step %.3f' % (d['roofline']['kernel_ms_median'] * 1e3),
          'per-step-launch %.4g' % d.get('value_per_step_launch', 0))
PY
done
done

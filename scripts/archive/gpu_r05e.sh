#!/bin/bash
# Round 5: parity of the persistent kernels (Optimize-v0 and MultiOptLRs),
# the bench-size tests, the NN checks; then the phase stamps, the 4- vs
# 8-wave A/B and the multi bench line.
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r05e
mkdir -p $OUT
for w in 4 8; do
  CE_LIB=diag CE_LP_WAVES=$w timeout -k 10 120 python -u scripts/diag_persist.py --k 20 250 > $OUT/diag_w$w.jsonl 2> $OUT/diag_w$w.err || exit $?
  cat $OUT/diag_w$w.jsonl
done
for w in 4 8; do
  CE_LP_WAVES=$w timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-measure-traffic > $OUT/b20_w$w.json 2>> $OUT/bench.err || exit $?
  CE_LP_WAVES=$w timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-measure-traffic > $OUT/b_w$w.json 2>> $OUT/bench.err || exit $?
done
timeout -k 10 200 python -u bench.py --workload multi --steps 20 --warmup 5 --no-cpu-baseline --no-measure-traffic > $OUT/bm20.json 2>> $OUT/bench.err || exit $?
timeout -k 10 200 python -u bench.py --workload multi --no-cpu-baseline --no-measure-traffic > $OUT/bm.json 2>> $OUT/bench.err || exit $?
python - $OUT/b20_w4.json $OUT/b_w4.json $OUT/b20_w8.json $OUT/b_w8.json $OUT/bm20.json $OUT/bm.json <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.load(open(f))
    print(f, d['roofline']['kernel'], 'value %.4g' % d['value'], 'us/step %.3f' % (d['ms_per_step'] * 1e3),
          'kernel us/step %.3f' % (d['roofline']['kernel_ms_median'] * 1e3),
          'per-step-launch %.4g' % d.get('value_per_step_launch', 0))
PY

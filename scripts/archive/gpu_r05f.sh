#!/bin/bash
# Round 5: the wave-specialised persistent kernel -- parity, stamps, A/B.
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r05g
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_persist.py tests/test_gpu_parity.py > $OUT/tests.log 2>&1
rc=$?
tail -5 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
for form in ws plain; do
  CE_LIB=diag CE_LP_FORM=$form timeout -k 10 120 python -u scripts/diag_persist.py --k 20 250 > $OUT/diag_$form.jsonl 2> $OUT/diag_$form.err || exit $?
  cat $OUT/diag_$form.jsonl
done
for rep in 1 2; do
for form in ws plain; do
  CE_LP_FORM=$form timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-measure-traffic > $OUT/b20_$form.$rep.json 2>> $OUT/bench.err || exit $?
  CE_LP_FORM=$form timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-measure-traffic > $OUT/b_$form.$rep.json 2>> $OUT/bench.err || exit $?
done
done
python - $OUT/b20_*.json $OUT/b_*.json <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.load(open(f))
    print(f, d['roofline']['kernel'], 'value %.4g' % d['value'], 'us/step %.3f' % (d['ms_per_step'] * 1e3),
          'kernel us/step %.3f' % (d['roofline']['kernel_ms_median'] * 1e3))
PY

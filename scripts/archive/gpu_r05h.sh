#!/bin/bash
# Round 5: the two-wave persistent MultiOptLRs kernel -- parity and A/B.
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r05h
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_multi.py > $OUT/tests.log 2>&1
rc=$?
tail -5 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for form in two one; do
  CE_MULTI_FORM=$form timeout -k 10 200 python -u bench.py --workload multi --steps 20 --warmup 5 --no-cpu-baseline --no-measure-traffic > $OUT/bm20_$form.$rep.json 2>> $OUT/bench.err || exit $?
  CE_MULTI_FORM=$form timeout -k 10 200 python -u bench.py --workload multi --no-cpu-baseline --no-measure-traffic > $OUT/bm_$form.$rep.json 2>> $OUT/bench.err || exit $?
done
done
python - $OUT/bm*.json <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.load(open(f))
    print(f, d['roofline']['kernel'], 'value %.4g' % d['value'], 'us/step %.3f' % (d['ms_per_step'] * 1e3),
          'kernel us/step %.3f' % (d['roofline']['kernel_ms_median'] * 1e3), 'per-step %.4g' % d.get('value_per_step_launch', 0))
PY

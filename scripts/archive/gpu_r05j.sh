#!/bin/bash
# Round 5: the table exponential (CE_LR_TEXP) -- LR parity tests, then an
# A/B of the headline bench against the polynomial build (CE_LIB=noexp),
# long-run and driver form, interleaved.
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r05j
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_persist.py tests/test_gpu_parity.py tests/test_gpu_mfma.py tests/test_gpu_ref_pins.py > $OUT/tests.log 2>&1
rc=$?
tail -5 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for lib in default noexp; do
    if [ $lib = default ]; then L=""; else L=$lib; fi
    CE_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-measure-traffic \
        > $OUT/bench_${lib}_$rep.json 2> $OUT/bench_${lib}_$rep.err || exit $?
    CE_LIB=$L timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline \
        --no-measure-traffic > $OUT/bench20_${lib}_$rep.json 2> $OUT/bench20_${lib}_$rep.err || exit $?
    echo "$lib $rep"; python -c "
import json,sys
for f in sys.argv[1:]:
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d['value'], d['ms_per_step'], d.get('value_per_step_launch'))" \
        $OUT/bench_${lib}_$rep.json $OUT/bench20_${lib}_$rep.json
  done
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
    python -u bench.py --profile-only --steps 20 --warmup 5 > $OUT/prof.log 2>&1 || exit $?
find $OUT/prof -name '*kernel_stats.csv' -exec cat {} \;

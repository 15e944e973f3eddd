#!/bin/bash
# Round 5: config 5's two-wave K-step kernel with the learning rate's exp10
# a step ahead (off the dependent state chain) -- parity tests, then an
# interleaved A/B against the previous build (CE_LIB=mpold).
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r05u
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_multi.py tests/test_gpu_ref_pins.py > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for lib in default mpold; do
    if [ $lib = default ]; then L=""; else L=$lib; fi
    CE_LIB=$L timeout -k 10 300 python -u bench.py --workload multi --no-cpu-baseline --no-measure-traffic \
        > $OUT/bench_${lib}_$i.json 2>> $OUT/bench.err || exit $?
    CE_LIB=$L timeout -k 10 300 python -u bench.py --workload multi --steps 20 --warmup 5 --no-cpu-baseline \
        --no-measure-traffic --repeat-timed 5 > $OUT/bench20_${lib}_$i.json 2>> $OUT/bench.err || exit $?
  done
done
python -c "
import json,sys
for f in sys.argv[1:]:
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d['value'], d['ms_per_step']*1e3, d.get('timed_repeats_ms'))" $OUT/bench*_*.json

#!/bin/bash
# Round 5: the 2048-entry exp table (degree-3 polynomial, one workgroup copy
# in LDS) -- the two-class parity tests, then an interleaved A/B of the
# headline bench against the 256-entry build (CE_LIB=prev), long run and
# driver form.
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r05ag
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_persist.py tests/test_gpu_parity.py tests/test_gpu_mfma.py tests/test_gpu_ref_pins.py \
    tests/test_gpu_bench_sizes.py > $OUT/tests.log 2>&1
rc=$?
tail -5 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for lib in default prev; do
    if [ $lib = default ]; then L=""; else L=$lib; fi
    CE_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-measure-traffic \
        > $OUT/bench_${lib}_$rep.json 2>> $OUT/bench.err || exit $?
    CE_LIB=$L timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline \
        --no-measure-traffic > $OUT/bench20_${lib}_$rep.json 2>> $OUT/bench.err || exit $?
  done
done
python -c "
import json,sys
for f in sys.argv[1:]:
    d=json.loads([l for l in open(f).read().splitlines() if l.startswith('{')][-1]); print(f, '%.4g'%d['value'], round(d['ms_per_step']*1e3,4), d['roofline'].get('kernel_ms'), d.get('value_per_step_launch'))" $OUT/bench_*.json $OUT/bench20_*.json

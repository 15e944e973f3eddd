#!/bin/bash
# Round 5: the table exponential in the image-shape kernel (CE_CAT_TEXP) --
# its parity tests, then an interleaved A/B of the mnist bench line against
# the polynomial build (CE_LIB=catpoly).
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r05s
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_mfma.py tests/test_gpu_bench_sizes.py tests/test_gpu_persist.py > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for lib in default catpoly; do
    if [ $lib = default ]; then L=""; else L=$lib; fi
    CE_LIB=$L timeout -k 10 300 python -u bench.py --workload mnist --no-cpu-baseline --no-measure-traffic \
        > $OUT/bench_mnist_${lib}_$i.json 2>> $OUT/bench.err || exit $?
  done
done
python -c "
import json,sys
for f in sys.argv[1:]:
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d['value'], d['ms_per_step'], d['roofline'].get('kernel_ms_median'))" $OUT/bench_mnist_*.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
    python -u bench.py --workload mnist --profile-only --steps 10 --warmup 2 > $OUT/prof.log 2>&1 || exit $?
grep cat_kernel $OUT/prof/*/run_kernel_stats.csv $OUT/prof/run_kernel_stats.csv 2>/dev/null | cut -c1-200

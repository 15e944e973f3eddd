#!/bin/bash
# Round 5, first GPU pass: the persistent K-step kernel's parity tests, the
# driver-form bench line (with the in-run traffic passes) and its kernel trace.
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r05a
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_persist.py tests/test_gpu_parity.py > $OUT/tests.log 2>&1
rc=$?
tail -5 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench20.json 2> $OUT/bench20.err || exit $?
cat $OUT/bench20.json
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-measure-traffic > $OUT/bench.json 2> $OUT/bench.err || exit $?
cat $OUT/bench.json
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
    python -u bench.py --profile-only --steps 20 --warmup 5 > $OUT/prof.log 2>&1 || exit $?
find $OUT/prof -name '*kernel_stats.csv' -exec cat {} \;

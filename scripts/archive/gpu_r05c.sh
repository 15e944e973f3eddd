#!/bin/bash
# Round 5: the bench-size parity tests, the tightened NN checks, then the
# persistent kernel's phase stamps and 4- vs 8-wave A/B.
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r05c
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
    tests/test_gpu_persist.py tests/test_gpu_distributed.py tests/test_gpu_bench_sizes.py tests/test_gpu_multinn.py > $OUT/tests.log 2>&1
rc=$?
tail -15 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r05b.sh

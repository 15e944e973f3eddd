#!/bin/bash
# GPU tests (+ smoke) in one call; OUT names the result directory.
# Usage: OUT=gpurun_out/r3a scripts/gpu_tests.sh [pytest args...]
set -u
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/tests}
mkdir -p $OUT
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
ARGS=${*:-tests -m gpu}
timeout -k 10 900 python -u -m pytest $ARGS -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log; fatal $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 $OUT/smoke.log; fatal $rc
echo ALL_OK

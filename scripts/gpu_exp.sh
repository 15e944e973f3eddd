#!/bin/bash
# Experiment session: GPU parity tests, bench, a sweep (staged and unstaged
# dataset) and the phase stamps at 4096 envs.  Each GPU step has its own time
# limit; a hard failure ends the script.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log; fatal $rc
timeout -k 10 400 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 $OUT/bench.log; fatal $rc
timeout -k 10 300 python scripts/sweep.py --envs 1024,4096,16384 > $OUT/sweep.log 2>&1; rc=$?
grep envs $OUT/sweep.log; fatal $rc
CE_NO_STAGE=1 timeout -k 10 300 python scripts/sweep.py --envs 4096 > $OUT/sweep_nostage.log 2>&1; rc=$?
grep envs $OUT/sweep_nostage.log; fatal $rc
CE_LIB=diag timeout -k 10 120 python scripts/diag_phases.py --envs 4096 --precision f64 > $OUT/diag.log 2>&1; rc=$?
grep envs $OUT/diag.log; fatal $rc
exit 0

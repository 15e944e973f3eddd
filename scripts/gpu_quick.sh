#!/bin/bash
# Quick check: GPU tests, per-path sweep at 1024/4096/16384 envs, phase stamps.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $OUT/pytest_gpu.log; fatal $rc
for U in ${PAIRS:-0 1 2}; do
  CE_PAIR_U=$U timeout -k 10 120 python scripts/sweep.py --envs 1024,4096,16384 > $OUT/sweep_u$U.txt 2>&1; rc=$?
  echo "== CE_PAIR_U=$U"; grep envs $OUT/sweep_u$U.txt; fatal $rc
done
CE_LIB=diag timeout -k 10 120 python scripts/diag_phases.py --envs 4096 --precision f64 > $OUT/diag.txt 2>&1; rc=$?; grep envs $OUT/diag.txt; fatal $rc

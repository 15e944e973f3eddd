#!/bin/bash
# GPU tests, then 4096/16384-env step time of every pair-kernel variant
# (CE_PAIR_U x CE_PAIR_R) and the one-env-per-wave kernel.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $OUT/pytest_gpu.log; fatal $rc
for V in "0 1" "1 1" "2 1" "1 2" "2 2"; do
  set -- $V
  CE_PAIR_U=$1 CE_PAIR_R=$2 timeout -k 10 120 python scripts/sweep.py --envs 4096,16384 > $OUT/sweep_u$1_r$2.txt 2>&1; rc=$?
  echo "== U=$1 R=$2: $(grep envs $OUT/sweep_u$1_r$2.txt | python3 -c 'import sys,json; print(" | ".join("%s %d: %.2f us" % (d["precision"], d["envs"], d["us_per_step"]) for d in map(json.loads, sys.stdin)))')"; fatal $rc
done

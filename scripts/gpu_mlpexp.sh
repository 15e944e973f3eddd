#!/bin/bash
# MLP step kernel experiment builds, one step-time line each (CE_LIB selects the build).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/mlpexp
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
for V in ${MLP_VARIANTS:-default}; do
  unset CE_LIB CE_MLP_PERSIST
  case $V in default) ;; persist) export CE_MLP_PERSIST=1;; *) export CE_LIB=$V;; esac
  timeout -k 10 300 python scripts/mlp_time.py > $OUT/time_$V.log 2>&1; rc=$?
  echo "$V rc=$rc $(tail -1 $OUT/time_$V.log)"; fatal $rc
done
echo ALL_OK

#!/bin/bash
# Config-3 step-time A/B of experiment builds (VARIANTS, CE_LIB; "main" = the
# product library), interleaved twice: scripts/mlp_time.py (HIP events, 4096
# envs).  Every GPU step has its own time limit; any failure stops the script.
set -u
cd "$(dirname "$0")/../.."
OUT=${OUT:-gpurun_out/mlp_ab}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
for rep in 1 2; do
  for V in ${VARIANTS:-main}; do
    if [ $V = main ]; then L=""; else L=$V; fi
    CE_LIB=$L timeout -k 10 120 python scripts/mlp_time.py > $OUT/t_$V.txt 2>&1; rc=$?
    echo "== $V rep $rep: $(tail -1 $OUT/t_$V.txt)"; fatal $rc
  done
done
echo ALL_OK

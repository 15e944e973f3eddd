#!/bin/bash
# A/B step-time comparison of experiment builds (CE_LIB variants), 4096 envs,
# interleaved runs to expose run-to-run noise.
set -u
cd "$(dirname "$0")/../.."
OUT=${OUT:-gpurun_out}
mkdir -p $OUT
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
for rep in 1 2; do
  for V in ${VARIANTS:-main}; do
    if [ $V = main ]; then L=""; else L=$V; fi
    CE_LIB=$L timeout -k 10 120 python scripts/sweep.py --envs ${ENVS:-4096} --precisions ${PRECS:-f64} > $OUT/ab_$V.txt 2>&1; rc=$?
    echo "== $V rep $rep: $(grep envs $OUT/ab_$V.txt | python3 -c 'import sys,json; print(" ".join("%s %d: %.3f us" % (d["precision"], d["envs"], d["us_per_step"]) for d in map(json.loads, sys.stdin)))')"; fatal $rc
  done
done

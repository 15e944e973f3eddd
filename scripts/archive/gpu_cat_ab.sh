#!/bin/bash
# mnist image-shape (class-concatenated kernel) A/B of experiment builds (VARIANTS, CE_LIB; "main" =
# the product library), interleaved twice, 4096 envs.
set -u
cd "$(dirname "$0")/../.."
OUT=${OUT:-gpurun_out/cat_ab}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
for rep in 1 2; do
  for V in ${VARIANTS:-main}; do
    if [ $V = main ]; then L=""; else L=$V; fi
    CE_LIB=$L timeout -k 10 300 python bench.py --workload mnist --steps 30 --warmup 3 --no-cpu-baseline > $OUT/b_$V.log 2>&1; rc=$?
    echo "== $V rep $rep: $(tail -1 $OUT/b_$V.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("%.4g env-steps/s, %.3f ms/step" % (d["value"], d["ms_per_step"]))')"; fatal $rc
  done
done
echo ALL_OK

#!/bin/bash
# Interleaved A/B of network-path experiment builds (CE_LIB variants; "main" =
# the product library): the 1024-env (256, 256) bench, REPS rounds, each
# variant once per round so drift hits every arm alike.
set -u
cd "$(dirname "$0")/../.."
OUT=${OUT:-gpurun_out/net_ab}
mkdir -p $OUT
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
for rep in $(seq ${REPS:-3}); do
  for V in ${VARIANTS:-main}; do
    if [ $V = main ]; then L=""; else L=$V; fi
    CE_LIB=$L timeout -k 10 200 python bench.py --workload mlp --hidden 256,256 --batch-size 32 --envs 1024 --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline > $OUT/b_${V}_$rep.log 2>&1; rc=$?
    echo "== $V rep $rep: $(tail -1 $OUT/b_${V}_$rep.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("%.3f ms" % d["ms_per_step"])')"; fatal $rc
  done
done
echo ALL_OK

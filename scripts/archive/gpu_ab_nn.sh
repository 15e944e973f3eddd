#!/bin/bash
# A/B of experiment builds (CE_LIB variants) on the NN multi-agent bench,
# interleaved to expose run-to-run noise.
set -u
cd "$(dirname "$0")/../.."
OUT=gpurun_out
mkdir -p $OUT
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
for rep in 1 2; do
  for V in ${VARIANTS:-main}; do
    if [ $V = main ]; then L=""; else L=$V; fi
    CE_LIB=$L timeout -k 10 200 python bench.py --workload nn --envs ${NN_ENVS:-1024} --steps 10 --warmup 2 --no-cpu-baseline > $OUT/abnn_$V.json 2>$OUT/abnn_$V.err; rc=$?
    echo "== $V rep $rep: $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print("%.3f ms/step (events %.3f)" % (d["ms_per_step"], d["roofline"]["step_ms_median"]))' $OUT/abnn_$V.json)"; fatal $rc
  done
done

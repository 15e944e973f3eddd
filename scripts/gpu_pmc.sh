#!/bin/bash
# PMC passes over the bench's timed steps (no sys/runtime trace with --pmc).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/pmc
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--profile-only --steps 500 --warmup 50 ${BENCH_ARGS:-}"
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
i=0
for CTRS in "${@}"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $CTRS -d $OUT/p$i -o run --output-format csv -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1; rc=$?
  echo "pass $i ($CTRS) rc=$rc"
  case $rc in 0) ;; *) tail -5 $OUT/p$i.log; exit $rc;; esac
done

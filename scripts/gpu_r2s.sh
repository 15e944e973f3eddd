#!/bin/bash
# Headline kernel anatomy (round 2 re-measure): launch floor of empty
# kernels, phase stamps of the default two-class MFMA kernel, and the
# CE_LR_EXP builds (1 = no row work, 2 = no epilogue, 3 = neither).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2s
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
timeout -k 10 60 scripts/bin/launch_floor > $OUT/launch_floor.jsonl 2>&1; rc=$?; cat $OUT/launch_floor.jsonl; fatal $rc
CE_LIB=diag timeout -k 10 200 python scripts/diag_phases.py --steps 30 > $OUT/diag_lr.json 2>&1; rc=$?
cat $OUT/diag_lr.json; fatal $rc
for V in "" lrexp1 lrexp2 lrexp3; do
  CE_LIB=$V timeout -k 10 200 python bench.py --no-cpu-baseline --steps 2000 --warmup 200 > $OUT/bench_$V.log 2>&1; rc=$?
  fatal $rc
  python - "$V" <<'PY'
import json, sys
d = json.loads([l for l in open('gpurun_out/r2s/bench_%s.log' % sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[1] or 'full', 'ms/step %.5f kernel %.5f ms' % (d['ms_per_step'], d['roofline']['kernel_ms_median']))
PY
done
echo ALL_OK

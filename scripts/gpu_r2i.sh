#!/bin/bash
# Short timed regions (the driver's --steps 20 --warmup 5): graph replay vs
# plain launches for ce_step_many.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2i
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
for MODE in 0 100000 0 100000; do
  for ST in "20 5" "100 10" "2000 200"; do
    set -- $ST
    CE_MANY_DIRECT=$MODE timeout -k 10 120 python bench.py --steps $1 --warmup $2 --no-cpu-baseline > $OUT/b_${MODE}_$1.log 2>&1; rc=$?
    fatal $rc
    python3 -c "import json,sys; d=json.loads([l for l in open('$OUT/b_${MODE}_$1.log') if l.startswith('{')][-1]); print('direct<=$MODE steps $1', round(d['ms_per_step']*1e3,3), 'us/step; kernel', round(d['roofline']['kernel_ms_median']*1e3,3))"
  done
done
timeout -k 10 60 scripts/bin/launch_floor > $OUT/launch_floor.jsonl 2>&1; rc=$?; cat $OUT/launch_floor.jsonl; fatal $rc
CE_LIB=diag timeout -k 10 200 python scripts/diag_phases.py --steps 30 > $OUT/diag_pair.json 2>&1; rc=$?; tail -1 $OUT/diag_pair.json; fatal $rc
CE_LR_MFMA=1 CE_LIB=diag timeout -k 10 200 python scripts/diag_phases.py --steps 30 > $OUT/diag_lr.json 2>&1; rc=$?; tail -1 $OUT/diag_lr.json; fatal $rc
CE_LR_MFMA=1 timeout -k 10 120 python bench.py --steps 2000 --warmup 200 --no-cpu-baseline > $OUT/b_lr.log 2>&1; rc=$?; fatal $rc
python3 -c "import json; d=json.loads([l for l in open('$OUT/b_lr.log') if l.startswith('{')][-1]); print('LR MFMA', round(d['ms_per_step']*1e3,3), 'us/step; kernel', round(d['roofline']['kernel_ms_median']*1e3,3), d['roofline']['kernel'])"
echo ALL_OK

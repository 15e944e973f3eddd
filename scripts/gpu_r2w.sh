#!/bin/bash
# Two-class MFMA kernel: SIMD-partner arbitration experiments (s_setprio
# for waves 4-7, one-tile-at-a-time stagger for waves 4-7, both).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2w
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --steps 2000 --warmup 200 --no-cpu-baseline > $OUT/b_$name.log 2>&1; rc=$?; fatal $rc
  python3 -c "import json; d=json.loads([l for l in open('$OUT/b_$name.log') if l.startswith('{')][-1]); print('$name', '%.4g' % d['value'], round(d['ms_per_step']*1e3,3), 'us/step; kernel', round(d['roofline']['kernel_ms_median']*1e3,3))"
}
for rep in 1 2; do
  run base_$rep
  run prio_$rep CE_LIB=prio
  run stag_$rep CE_LIB=stag
  run prst_$rep CE_LIB=prst
done
echo ALL_OK

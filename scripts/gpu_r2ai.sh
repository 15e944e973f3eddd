#!/bin/bash
# Where do 16 waves lose?  Full / no-rows (lrexp1) / no-rows-no-epilogue
# (lrexp3) builds at 4 and 16 waves per workgroup.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2ai
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --steps 2000 --warmup 200 --no-cpu-baseline > $OUT/b_$name.log 2>&1; rc=$?; fatal $rc
  python3 -c "import json; d=json.loads([l for l in open('$OUT/b_$name.log') if l.startswith('{')][-1]); print('$name', round(d['roofline']['kernel_ms_median']*1e3,3), 'us')"
}
for W in 4 16 8; do
  run full_w$W CE_LR_WAVES=$W
  run norows_w$W CE_LR_WAVES=$W CE_LIB=lrexp1
  run bare_w$W CE_LR_WAVES=$W CE_LIB=lrexp3
done
echo ALL_OK

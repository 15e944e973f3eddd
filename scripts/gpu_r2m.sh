#!/bin/bash
# Floor of the LR MFMA kernel: experiment builds without row work (1),
# without epilogue (2), without both (3), against the full kernel.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2m
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --steps 2000 --warmup 200 --no-cpu-baseline > $OUT/b_$name.log 2>&1; rc=$?; fatal $rc
  python3 -c "import json; d=json.loads([l for l in open('$OUT/b_$name.log') if l.startswith('{')][-1]); print('$name', round(d['ms_per_step']*1e3,3), 'us/step; kernel', round(d['roofline']['kernel_ms_median']*1e3,3), d['roofline']['kernel'])"
}
run full CE_LR_MFMA=1
run norows CE_LR_MFMA=1 CE_LIB=lrexp1
run noepi CE_LR_MFMA=1 CE_LIB=lrexp2
run neither CE_LR_MFMA=1 CE_LIB=lrexp3
run mode1 CE_LR_MFMA=1 CE_LR_MODE=1
echo ALL_OK

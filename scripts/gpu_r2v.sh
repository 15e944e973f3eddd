#!/bin/bash
# Where does the two-class MFMA kernel's time go?  Experiment builds
# (CE_LR_EXP): 1 = no row work, 2 = no epilogue, 3 = neither; plus the
# launch floor of empty kernels in a hipGraph.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2v
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
for V in ""; do
  CE_LIB=$V timeout -k 10 200 python bench.py --no-cpu-baseline --steps 2000 --warmup 200 > $OUT/bench_$V.log 2>&1; rc=$?
  fatal $rc
  python - "$V" <<'PY'
import json, sys
d = json.loads([l for l in open('gpurun_out/r2v/bench_%s.log' % sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[1] or 'full', 'ms/step %.5f kernel %.5f ms' % (d['ms_per_step'], d['roofline']['kernel_ms_median']))
PY
done
echo ALL_OK

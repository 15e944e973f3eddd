#!/bin/bash
# Config 2 as BASELINE.json words it (1024 envs, fp32) next to the f64 engine
# at 1024 envs and every wave count, and the f32 engine at 4096.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2ak
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
run() {  # name, args, env...
  local name=$1 args=$2; shift 2
  env "$@" timeout -k 10 120 python bench.py $args --steps 2000 --warmup 200 --no-cpu-baseline > $OUT/b_$name.log 2>&1; rc=$?; fatal $rc
  python3 -c "import json; d=json.loads([l for l in open('$OUT/b_$name.log') if l.startswith('{')][-1]); print('$name', '%.4g' % d['value'], round(d['ms_per_step']*1e3,3), 'us/step; kernel', round(d['roofline']['kernel_ms_median']*1e3,3), d['roofline']['kernel'])"
}
for W in 4 8 16; do run e1024_f64_w$W "--envs 1024" CE_LR_WAVES=$W; done
run e1024_f64_default "--envs 1024"
run e1024_f32 "--envs 1024 --precision f32"
run e4096_f32 "--precision f32"
run e16384_f64 "--envs 16384"
echo ALL_OK

#!/bin/bash
# The driver's 20-step form: plain launches (default) vs one hipGraph
# (CE_MANY_DIRECT=0); and the pipelined all-gather path of config 4 at
# world 1 (--force-gather, nccl) on the 4096-env shard.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2ae
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
run() {  # name, args, env...
  local name=$1 args=$2; shift 2
  env "$@" timeout -k 10 120 python bench.py $args --no-cpu-baseline > $OUT/b_$name.log 2>&1; rc=$?; fatal $rc
  python3 -c "import json; d=json.loads([l for l in open('$OUT/b_$name.log') if l.startswith('{')][-1]); print('$name', '%.4g' % d['value'], round(d['ms_per_step']*1e3,3), 'us/step', {k: d[k] for k in d if k.startswith('value_') or k=='ms_per_step_modes'})"
}
for rep in 1 2 3; do
  run direct20_$rep "--steps 20 --warmup 5"
  run graph20_$rep "--steps 20 --warmup 5" CE_MANY_DIRECT=0
done
run gather "--steps 2000 --warmup 200 --force-gather"
echo ALL_OK

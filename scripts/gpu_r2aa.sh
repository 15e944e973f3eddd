#!/bin/bash
# NN problem: row-order agent kernel (default) vs agent order; parity,
# bench and kernel trace.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2aa
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_multinn.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAIL|Error" $OUT/pytest.log | head -5; tail -1 $OUT/pytest.log; fatal $rc
for V in rows agent; do
  CE_NN_AGENT=$V timeout -k 10 300 python bench.py --workload nn --steps 40 --warmup 4 --no-cpu-baseline > $OUT/b_$V.log 2>&1; rc=$?; fatal $rc
  python3 -c "import json; d=json.loads([l for l in open('$OUT/b_$V.log') if l.startswith('{')][-1]); print('$V', '%.4g' % d['value'], round(d['ms_per_step'],4), 'ms/step')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_nn -o nn --output-format csv -- python3 bench.py --workload nn --profile-only --steps 10 --warmup 2 > $OUT/prof_nn.log 2>&1; rc=$?
echo "rocprof nn rc=$rc"; fatal $rc
head -4 $OUT/prof_nn/nn_kernel_stats.csv | cut -c1-120
echo ALL_OK

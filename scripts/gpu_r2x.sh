#!/bin/bash
# Full GPU suite + smoke + default bench + kernel trace + PMC passes of the
# default step kernel (round-2 evidence after the LR kernel rework).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2x
mkdir -p $OUT/pmc
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAIL|Error" $OUT/pytest_gpu.log | head; tail -2 $OUT/pytest_gpu.log; fatal $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 $OUT/smoke.log; fatal $rc
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 $OUT/bench.log | cut -c1-400; fatal $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --profile-only --steps 2000 --warmup 100 > $OUT/prof.log 2>&1; rc=$?
echo "rocprof rc=$rc"; fatal $rc
i=0
for CTRS in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CTRS -d $OUT/pmc/p$i -o run --output-format csv -- python3 bench.py --profile-only --steps 500 --warmup 50 > $OUT/pmc/p$i.log 2>&1; rc=$?
  echo "pmc pass $i rc=$rc"; fatal $rc
done
echo ALL_OK

#!/bin/bash
# Config-5 (MultiOptLRs under OptVecEnv) session (OUT names the result
# directory): the multi-agent GPU tests, an interleaved bench A/B of
# experiment builds (VARIANTS, CE_LIB; "main" = the product library) and the
# product kernel's trace.  Every GPU step has its own time limit; any
# failure stops the script.
set -u
cd "$(dirname "$0")/../.."
OUT=${OUT:-gpurun_out/multi}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_multi.py tests/test_gpu_ref_pins.py tests/test_gpu_distributed.py} -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; fatal $rc
for rep in 1 2; do
  for V in ${VARIANTS:-main}; do
    if [ $V = main ]; then L=""; else L=$V; fi
    CE_LIB=$L timeout -k 10 200 python bench.py --workload multi --no-cpu-baseline > $OUT/bench_$V.log 2>&1; rc=$?
    echo "== $V rep $rep: $(tail -1 $OUT/bench_$V.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("%.4g env-steps/s, %.3f us/step, kernel %.3f us" % (d["value"], d["ms_per_step"]*1e3, d["roofline"]["kernel_ms_median"]*1e3))')"; fatal $rc
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --workload multi --profile-only --steps 2000 --warmup 100 > $OUT/prof.log 2>&1; rc=$?
echo "rocprof rc=$rc"; fatal $rc
echo ALL_OK

#!/bin/bash
# Round-6 evidence (OUT names the result directory).
#  PART=a: GPU tests, smoke, the default bench (with the CPU baseline and the
#          in-run counter traffic), the driver's 20-step form with 10 repeats
#          of its timed region, the headline kernel's rocprofv3 traces (long
#          and 20-step) and the launch-floor decomposition.
#  PART=b: config 5 (default and driver form), config 3, the network, the NN
#          problem and the image shape, each with its in-run counter traffic
#          and kernel trace; the world-1 chunk-schedule gather line.
# Every GPU step has its own time limit; any failure stops the script.
set -u
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/ev6}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
summ() { python3 -c "import json,sys; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); r=d.get('roofline',{}); print('$2', '%.4g' % d['value'], '%.4g ms' % d['ms_per_step'], 'frac %.3g' % r.get('frac',0), 'traffic', r.get('traffic'), (d.get('cpu_baseline') or {}).get('value'))"; }
if [ "${PART:-a}" = a ]; then
  nproc > $OUT/host.txt; lscpu | grep "Model name" >> $OUT/host.txt
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -1 $OUT/pytest_gpu.log; fatal $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
  echo "smoke rc=$rc"; tail -3 $OUT/smoke.log; fatal $rc
  echo PART_A_TESTS_OK
elif [ "${PART}" = a2 ]; then
  timeout -k 10 500 python bench.py --measure-traffic > $OUT/bench.log 2>&1; rc=$?
  echo "bench rc=$rc"; summ $OUT/bench.log optimize; fatal $rc
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --repeat-timed 10 > $OUT/bench20.log 2>&1; rc=$?
  echo "bench20 rc=$rc"; summ $OUT/bench20.log optimize20; fatal $rc
  # the default command itself under the tracer (its traffic passes and CPU
  # baseline off: no nested profiler, no child processes)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-measure-traffic --no-cpu-baseline > $OUT/prof.log 2>&1; rc=$?
  echo "rocprof rc=$rc"; fatal $rc
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof20 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-measure-traffic --no-cpu-baseline > $OUT/prof20.log 2>&1; rc=$?
  echo "rocprof20 rc=$rc"; fatal $rc
  timeout -k 10 300 python -u scripts/launch_floor.py --k 1 5 20 40 --repeat 20 > $OUT/launch_floor.json 2> $OUT/launch_floor.err; rc=$?
  echo "floor rc=$rc"; cat $OUT/launch_floor.json; fatal $rc
  # the headline kernel's issue counters (two --pmc passes, 250-step dispatches)
  OUT=$OUT/pmc_persist timeout -k 10 400 scripts/gpu_pmc_persist.sh > $OUT/pmc_persist.log 2>&1; rc=$?
  echo "pmc rc=$rc"; tail -14 $OUT/pmc_persist.log; fatal $rc
  echo PART_A2_OK
else
  for W in "multi:--workload multi" "multi20:--workload multi --steps 20 --warmup 5" \
           "mlp:--workload mlp --steps 20 --warmup 4" \
           "net:--workload mlp --hidden 256,256 --batch-size 32 --envs 1024 --steps 10 --warmup 2" \
           "nn:--workload nn --steps 40 --warmup 4" "mnist:--workload mnist"; do
    name=${W%%:*}; args=${W#*:}
    # ONLY: a space-separated subset of the workload names to run
    if [ -n "${ONLY:-}" ] && ! echo " $ONLY " | grep -q " $name "; then continue; fi
    timeout -k 10 500 python bench.py $args --cpu-seconds 10 --measure-traffic > $OUT/bench_$name.log 2>&1; rc=$?
    echo "bench $name rc=$rc"; summ $OUT/bench_$name.log $name; fatal $rc
    [ "$name" = multi20 ] && continue
    pargs=$(echo "$args" | sed 's/--steps [0-9]*//; s/--warmup [0-9]*//')
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_$name -o run --output-format csv -- python3 bench.py $pargs --profile-only --steps 10 --warmup 2 > $OUT/prof_$name.log 2>&1; rc=$?
    echo "rocprof $name rc=$rc"; fatal $rc
  done
  if [ -n "${ONLY:-}" ]; then echo PART_B_OK; exit 0; fi
  # config 4's global batch on one GPU: the open-loop value and the
  # closed-loop (one launch per step) rate at 32,768 envs
  timeout -k 10 300 python bench.py --envs 32768 --steps 2000 --warmup 200 --no-cpu-baseline --no-measure-traffic > $OUT/bench_e32768.log 2>&1; rc=$?
  echo "bench e32768 rc=$rc"; summ $OUT/bench_e32768.log e32768; fatal $rc
  timeout -k 10 300 python bench.py --force-gather --no-cpu-baseline --steps 2000 --warmup 200 > $OUT/bench_gather.log 2>&1; rc=$?
  echo "bench gather rc=$rc"; summ $OUT/bench_gather.log gather; fatal $rc
  timeout -k 10 300 python bench.py --force-gather --no-cpu-baseline --steps 20 --warmup 5 > $OUT/bench_gather20.log 2>&1; rc=$?
  echo "bench gather20 rc=$rc"; summ $OUT/bench_gather20.log gather20; fatal $rc
  echo PART_B_OK
fi

#!/bin/bash
# Round-4 evidence (OUT names the result directory).  PART=a: GPU tests, smoke,
# the default bench (with the CPU baseline and the in-run counter traffic)
# and the driver's 20-step form, the headline kernel's rocprofv3 trace and
# PMC passes.  PART=b: the config-3 / network / config-5 / NN / image-shape
# workloads, each bench line with its in-run counter traffic, and their
# kernel traces; the world-1 gather line.  Every GPU step has its own time
# limit; any failure stops the script.
set -u
cd "$(dirname "$0")/../.."
OUT=${OUT:-gpurun_out/ev4}
mkdir -p $OUT/pmc
export TMPDIR=/tmp CE_TRAFFIC_OUT=$PWD/${OUT}/traffic
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
summ() { python3 -c "import json,sys; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); r=d.get('roofline',{}); print('$2', '%.4g' % d['value'], '%.4g ms' % d['ms_per_step'], 'frac %.3g' % r.get('frac',0), 'traffic', r.get('traffic'), (d.get('cpu_baseline') or {}).get('value'))"; }
if [ "${PART:-a}" = a ]; then
  nproc > $OUT/host.txt; lscpu | grep "Model name" >> $OUT/host.txt
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -1 $OUT/pytest_gpu.log; fatal $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
  echo "smoke rc=$rc"; tail -3 $OUT/smoke.log; fatal $rc
  timeout -k 10 500 python bench.py --measure-traffic > $OUT/bench.log 2>&1; rc=$?
  echo "bench rc=$rc"; summ $OUT/bench.log optimize; fatal $rc
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench20.log 2>&1; rc=$?
  echo "bench20 rc=$rc"; summ $OUT/bench20.log optimize20; fatal $rc
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --profile-only --steps 2000 --warmup 100 > $OUT/prof.log 2>&1; rc=$?
  echo "rocprof rc=$rc"; fatal $rc
  i=0
  for CTRS in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_SALU"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $CTRS -d $OUT/pmc/p$i -o run --output-format csv -- python3 bench.py --profile-only --steps 500 --warmup 50 > $OUT/pmc/p$i.log 2>&1; rc=$?
    echo "pmc pass $i rc=$rc"; fatal $rc
  done
  echo PART_A_OK
else
  for W in "multi:--workload multi" "mlp:--workload mlp --steps 20 --warmup 4" \
           "net:--workload mlp --hidden 256,256 --batch-size 32 --envs 1024 --steps 10 --warmup 2" \
           "nn:--workload nn --steps 40 --warmup 4" "mnist:--workload mnist"; do
    name=${W%%:*}; args=${W#*:}
    timeout -k 10 500 python bench.py $args --cpu-seconds 10 --measure-traffic > $OUT/bench_$name.log 2>&1; rc=$?
    echo "bench $name rc=$rc"; summ $OUT/bench_$name.log $name; fatal $rc
    pargs=$(echo "$args" | sed 's/--steps [0-9]*//; s/--warmup [0-9]*//')
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_$name -o run --output-format csv -- python3 bench.py $pargs --profile-only --steps 10 --warmup 2 > $OUT/prof_$name.log 2>&1; rc=$?
    echo "rocprof $name rc=$rc"; fatal $rc
  done
  timeout -k 10 300 python bench.py --force-gather --no-cpu-baseline --steps 2000 --warmup 200 > $OUT/bench_gather.log 2>&1; rc=$?
  echo "bench gather rc=$rc"; summ $OUT/bench_gather.log gather; fatal $rc
  echo PART_B_OK
fi

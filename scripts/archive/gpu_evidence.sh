#!/bin/bash
# Round evidence in one call (OUT names the result directory): GPU tests, smoke, the default bench (with the
# CPU baseline) and the driver's 20-step form, rocprofv3 kernel trace + PMC
# passes of the benchmark kernel, and the config-3 / config-5 / NN / image-
# shape workloads with their kernel traces.  Every GPU step has its own time
# limit; any failure stops the script.
set -u
cd "$(dirname "$0")/../.."
OUT=${OUT:-gpurun_out/evidence}
mkdir -p $OUT/pmc
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
nproc > $OUT/host.txt; lscpu | grep "Model name" >> $OUT/host.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 $OUT/pytest_gpu.log; fatal $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 $OUT/smoke.log; fatal $rc
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 $OUT/bench.log | cut -c1-300; fatal $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench20.log 2>&1; rc=$?
echo "bench20 rc=$rc"; tail -1 $OUT/bench20.log | cut -c1-300; fatal $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --profile-only --steps 2000 --warmup 100 > $OUT/prof.log 2>&1; rc=$?
echo "rocprof rc=$rc"; fatal $rc
i=0
for CTRS in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CTRS -d $OUT/pmc/p$i -o run --output-format csv -- python3 bench.py --profile-only --steps 500 --warmup 50 > $OUT/pmc/p$i.log 2>&1; rc=$?
  echo "pmc pass $i rc=$rc"; fatal $rc
done
timeout -k 10 300 python bench.py --workload multi > $OUT/bench_multi.log 2>&1; rc=$?
echo "bench multi rc=$rc"; fatal $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_multi -o run --output-format csv -- python3 bench.py --workload multi --profile-only --steps 2000 --warmup 100 > $OUT/prof_multi.log 2>&1; rc=$?
echo "rocprof multi rc=$rc"; fatal $rc
timeout -k 10 400 python bench.py --workload mlp --steps 20 --warmup 4 --cpu-seconds 10 > $OUT/bench_mlp.log 2>&1; rc=$?
echo "bench mlp rc=$rc"; fatal $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_mlp -o run --output-format csv -- python3 bench.py --workload mlp --profile-only --steps 10 --warmup 2 > $OUT/prof_mlp.log 2>&1; rc=$?
echo "rocprof mlp rc=$rc"; fatal $rc
timeout -k 10 300 python bench.py --workload nn --steps 40 --warmup 4 --cpu-seconds 20 > $OUT/bench_nn.log 2>&1; rc=$?
echo "bench nn rc=$rc"; fatal $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_nn -o run --output-format csv -- python3 bench.py --workload nn --profile-only --steps 10 --warmup 2 > $OUT/prof_nn.log 2>&1; rc=$?
echo "rocprof nn rc=$rc"; fatal $rc
timeout -k 10 400 python bench.py --workload mnist --cpu-seconds 10 > $OUT/bench_mnist.log 2>&1; rc=$?
echo "bench mnist rc=$rc"; fatal $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_mnist -o run --output-format csv -- python3 bench.py --workload mnist --profile-only --steps 10 --warmup 2 > $OUT/prof_mnist.log 2>&1; rc=$?
echo "rocprof mnist rc=$rc"; fatal $rc
timeout -k 10 600 python bench.py --workload mlp --hidden 256,256 --batch-size 32 --envs 1024 --steps 10 --warmup 2 --cpu-seconds 10 > $OUT/bench_net.log 2>&1; rc=$?
echo "bench net rc=$rc"; fatal $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_net -o run --output-format csv -- python3 bench.py --workload mlp --hidden 256,256 --batch-size 32 --envs 1024 --profile-only --steps 5 --warmup 1 > $OUT/prof_net.log 2>&1; rc=$?
echo "rocprof net rc=$rc"; fatal $rc
timeout -k 10 300 python bench.py --force-gather --no-cpu-baseline --steps 2000 --warmup 200 > $OUT/bench_gather.log 2>&1; rc=$?
echo "bench gather rc=$rc"; fatal $rc
for w in multi mlp nn mnist net gather; do python3 -c "import json; d=json.loads([l for l in open('$OUT/bench_$w.log') if l.startswith('{')][-1]); print('$w', '%.4g' % d['value'], d['ms_per_step'], (d.get('cpu_baseline') or {}).get('value'))"; done
echo ALL_OK

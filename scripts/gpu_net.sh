#!/bin/bash
# Layered network path + two-class kernel A/B session (OUT names the result
# directory): the affected GPU tests, the A/B of experiment builds
# (VARIANTS, CE_LIB), the network bench with and without the hipBLASLt relu
# epilogue, and its kernel trace.  Every GPU step has its own time limit;
# any failure stops the script.
set -u
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/net}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
timeout -k 10 500 python -u -m pytest ${TESTS:-tests/test_gpu_mlp.py tests/test_gpu_parity.py tests/test_gpu_mfma.py tests/test_gpu_ref_pins.py} -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; fatal $rc
OUT=$OUT VARIANTS="${VARIANTS:-main}" bash scripts/gpu_ab.sh; fatal $?
timeout -k 10 400 python bench.py --workload mlp --hidden 256,256 --batch-size 32 --envs 1024 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_net.log 2>&1; rc=$?
tail -1 $OUT/bench_net.log | cut -c1-300; fatal $rc
CE_NET_LT=0 timeout -k 10 400 python bench.py --workload mlp --hidden 256,256 --batch-size 32 --envs 1024 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_net_relu.log 2>&1; rc=$?
tail -1 $OUT/bench_net_relu.log | cut -c1-300; fatal $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_net -o run --output-format csv -- python3 bench.py --workload mlp --hidden 256,256 --batch-size 32 --envs 1024 --profile-only --steps 5 --warmup 1 > $OUT/prof_net.log 2>&1; rc=$?
echo "prof rc=$rc"; fatal $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench20.log 2>&1; rc=$?
tail -1 $OUT/bench20.log | cut -c1-200; fatal $rc
echo ALL_OK

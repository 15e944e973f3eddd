#!/bin/bash
# Round-4 network-path session (OUT names the result directory): the
# network GPU tests, then the 1024-env (256, 256) bench and its kernel trace.
# Every GPU step has its own time limit; any failure stops the script.
set -u
cd "$(dirname "$0")/../.."
OUT=${OUT:-gpurun_out/net4}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_mlp.py} -x -v --timeout 150 --timeout-method thread ${K:+-k "$K"} > $OUT/pytest.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" $OUT/pytest.log | tail -25; fatal $rc
[ -n "${NOBENCH:-}" ] && { echo ALL_OK; exit 0; }
timeout -k 10 300 python bench.py --workload mlp --hidden 256,256 --batch-size 32 --envs 1024 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_net.log 2>&1; rc=$?
tail -1 $OUT/bench_net.log | cut -c1-400; fatal $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_net -o run --output-format csv -- python3 bench.py --workload mlp --hidden 256,256 --batch-size 32 --envs 1024 --profile-only --steps 5 --warmup 1 > $OUT/prof_net.log 2>&1; rc=$?
echo "prof rc=$rc"; fatal $rc
find $OUT/prof_net -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-200 | head -20
for V in ${NETVARIANTS:-}; do
  CE_LIB=$V timeout -k 10 300 python bench.py --workload mlp --hidden 256,256 --batch-size 32 --envs 1024 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_net_$V.log 2>&1; rc=$?
  echo "variant $V: $(tail -1 $OUT/bench_net_$V.log | cut -c1-160)"; fatal $rc
done
[ -n "${PMC:-}" ] && { OUT=$OUT/pmc bash scripts/gpu_pmc_net.sh || exit $?; }
echo ALL_OK

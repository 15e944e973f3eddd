set -u
OUT=gpurun_out/prel; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_mfma.py tests/test_gpu_distributed.py > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc = 0 ] || exit $rc
VARIANTS="main noprel r3c" OUT=$OUT bash scripts/gpu_ab.sh || exit 1
VARIANTS="main noprel r3c" OUT=$OUT bash scripts/gpu_ab.sh || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 2000 --warmup 100 --profile-only > $OUT/prof.log 2>&1 || exit 1
CE_LIB=r3c timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_r3c -o run -- python3 bench.py --steps 2000 --warmup 100 --profile-only > $OUT/prof_r3c.log 2>&1 || exit 1
for d in prof prof_r3c; do echo $d; grep lr_mfma $OUT/$d/run_kernel_stats.csv | cut -d, -f2-7; done

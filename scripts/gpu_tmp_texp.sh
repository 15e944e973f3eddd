set -u
OUT=gpurun_out/texp; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_mfma.py > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc = 0 ] || exit $rc
OUT=$OUT VARIANTS="main notexp" bash scripts/gpu_ab.sh || exit 1
VARIANTS="main notexp" OUT=$OUT bash scripts/gpu_ab.sh || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --steps 2000 --warmup 100 --profile-only > $OUT/prof.log 2>&1 || exit 1
CE_LIB=notexp timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/prof_old -o run -- python3 bench.py --steps 2000 --warmup 100 --profile-only > $OUT/prof_old.log 2>&1 || exit 1
find $OUT -name '*kernel_stats.csv' | while read f; do echo $f; grep lr_mfma $f | cut -d, -f2-7; done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_multi.py > $OUT/pytest_multi.log 2>&1; rc=$?; tail -2 $OUT/pytest_multi.log; [ $rc = 0 ] || exit $rc
for rep in 1 2; do for V in main multinowt; do
  L=$V; [ $V = main ] && L=""
  CE_LIB=$L timeout -k 10 120 python bench.py --workload multi --steps 2000 --warmup 200 --no-cpu-baseline > $OUT/multi_$V.json 2>$OUT/multi_$V.err || exit 1
  echo "multi $V rep $rep: $(tail -1 $OUT/multi_$V.json | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("%.3f us/step" % (d["ms_per_step"]*1e3), d["roofline"].get("kernel_ms_median"))')"
done; done

set -u
OUT=gpurun_out/multi; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_multi.py tests/test_gpu_distributed.py tests/test_gpu_dropin.py > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc = 0 ] || exit $rc
for rep in 1 2 3; do for V in main r3d; do
  L=$V; [ $V = main ] && L=""
  CE_LIB=$L timeout -k 10 120 python bench.py --workload multi --steps 2000 --warmup 200 --no-cpu-baseline > $OUT/multi_$V.json 2>$OUT/multi_$V.err || exit 1
  echo "multi $V rep $rep: $(tail -1 $OUT/multi_$V.json | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("%.3f us/step kernel %.3f" % (d["ms_per_step"]*1e3, d["roofline"].get("kernel_ms_median")*1e3))')"
done; done

set -u
OUT=gpurun_out/wt; mkdir -p $OUT
VARIANTS="main wtout nowt" OUT=$OUT bash scripts/gpu_ab.sh || exit 1
VARIANTS="main wtout nowt" OUT=$OUT bash scripts/gpu_ab.sh || exit 1
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k device_path > $OUT/pytest.log 2>&1; rc=$?; tail -1 $OUT/pytest.log; [ $rc = 0 ] || exit $rc
for rep in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/b20.json 2>/dev/null || exit 1
  echo "20-step runner rep $rep: $(tail -1 $OUT/b20.json | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("%.3e %.3f us kernel %.3f" % (d["value"], d["ms_per_step"]*1e3, d["roofline"]["kernel_ms_median"]*1e3))')"
done

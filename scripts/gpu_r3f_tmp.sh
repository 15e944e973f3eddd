set -u
OUT=gpurun_out/r3f
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_mlp.py tests/test_gpu_distributed.py -v --maxfail 8 --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; grep -E "^FAILED|^E  " $OUT/pytest.log | head -20
[ $rc = 0 ] || [ $rc = 1 ] || exit $rc
timeout -k 10 300 python bench.py --force-gather --no-cpu-baseline --steps 2000 --warmup 200 > $OUT/bench_gather.json 2> $OUT/bench_gather.err; echo "gather rc=$?"; tail -1 $OUT/bench_gather.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ('value','ms_per_step_modes','gather_bytes_per_rank','gather_record')})"
timeout -k 10 300 python bench.py --workload mnist --no-cpu-baseline > $OUT/bench_mnist.json 2> $OUT/bench_mnist.err; echo "mnist rc=$?"; tail -1 $OUT/bench_mnist.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel'], r['kernel_ms_median'], r['frac'])"
CE_GEN_CAT=0 timeout -k 10 300 python bench.py --workload mnist --no-cpu-baseline > $OUT/bench_mnist_gen.json 2> $OUT/bench_mnist_gen.err; echo "mnist gen rc=$?"; tail -1 $OUT/bench_mnist_gen.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel'], r['kernel_ms_median'], r['frac'])"
exit $rc

set -u
OUT=gpurun_out/r3e
mkdir -p $OUT
OUT=$OUT VARIANTS="main agpr r2" bash scripts/gpu_ab.sh
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail 8 --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; grep -E "^FAILED|^E  .*err" $OUT/pytest.log | head -20
timeout -k 10 300 python bench.py --force-gather --no-cpu-baseline --steps 2000 --warmup 200 > $OUT/bench_gather.json 2> $OUT/bench_gather.err; echo "gather rc=$?"; python3 -c "
import json; d=json.load(open('$OUT/bench_gather.json')); print({k: d.get(k) for k in ('value','ms_per_step_modes','gather_bytes_per_rank','gather_record','value_no_gather','value_gather_pipelined')})"
timeout -k 10 600 python bench.py --workload mlp --hidden 256,256 --batch-size 32 --envs 1024 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_net.json 2> $OUT/bench_net.err; echo "net rc=$?"; tail -c 700 $OUT/bench_net.json
exit $rc

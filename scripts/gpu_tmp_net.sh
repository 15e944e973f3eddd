set -u
OUT=gpurun_out/net; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_mlp.py -k "network" > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload mlp --hidden 256,256 --batch-size 32 --envs 1024 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_net.json 2>$OUT/bench_net.err || exit 1
tail -1 $OUT/bench_net.json | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("net %.3f ms/step frac %.3f" % (d["ms_per_step"], d["roofline"]["frac"]))'
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --workload mlp --hidden 256,256 --batch-size 32 --envs 1024 --steps 6 --warmup 2 --profile-only > $OUT/prof.log 2>&1 || exit 1
find $OUT/prof -name '*kernel_stats.csv' | head -1 | xargs -I{} python3 -c "
import csv,sys
for x in csv.DictReader(open('{}')): print(x['Name'][:60], x['Calls'], round(float(x['AverageNs'])/1e3,1))"
for rep in 1 2 3; do for md in 32 0; do
  CE_MANY_DIRECT=$md timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/b20_$md.json 2>/dev/null || exit 1
  echo "20-step many_direct=$md rep $rep: $(tail -1 $OUT/b20_$md.json | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("%.3e %.3f us kernel %.3f" % (d["value"], d["ms_per_step"]*1e3, d["roofline"]["kernel_ms_median"]*1e3))')"
done; done
mkdir -p /tmp/xb && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 scripts/xcd_map.hip -o /tmp/xb/xcd_map 2>/dev/null && timeout -k 10 60 /tmp/xb/xcd_map > $OUT/xcd_map.txt 2>&1; cat $OUT/xcd_map.txt

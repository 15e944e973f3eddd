#!/bin/bash
# NN path: update fused into nn_grad_kernel's tail (default) vs the separate
# nn_update_kernel (CE_NN_FUSE_UPDATE=0): parity both ways, bench A/B, rocprof
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r2am
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_multinn.py > gpurun_out/r2am/test_fused.log 2>&1
tail -1 gpurun_out/r2am/test_fused.log
CE_NN_FUSE_UPDATE=0 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_multinn.py > gpurun_out/r2am/test_sep.log 2>&1
tail -1 gpurun_out/r2am/test_sep.log
for rep in 1 2; do
for f in 1 0; do
  CE_NN_FUSE_UPDATE=$f timeout -k 10 180 python bench.py --workload nn > gpurun_out/r2am/bench_f${f}_$rep.json 2> gpurun_out/r2am/bench_f${f}_$rep.err
  echo "fuse=$f rep=$rep $(python -c "import json;d=json.load(open('gpurun_out/r2am/bench_f${f}_$rep.json'));print(d['value'],d['ms_per_step'])")"
done
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r2am/prof -o nn --output-format csv -- python3 bench.py --workload nn --profile-only --steps 12 --warmup 2 > gpurun_out/r2am/prof.log 2>&1
find gpurun_out/r2am/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/r2am/nn_fused_kernel_stats.csv
head -8 gpurun_out/r2am/nn_fused_kernel_stats.csv | cut -c1-120

#!/bin/bash
# MLP step: info-first stagger A/B (CE_MLP_STAGGER 0..3) + parity with stagger on
set -e
mkdir -p gpurun_out/r2al
for s in 1 2; do
  CE_MLP_STAGGER=$s timeout -k 10 240 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mlp.py > gpurun_out/r2al/test_s$s.log 2>&1
done
for rep in 1 2; do
for s in 0 1 2 3; do
  CE_MLP_STAGGER=$s timeout -k 10 120 python bench.py --workload mlp --steps 20 --warmup 3 > gpurun_out/r2al/bench_s${s}_$rep.json 2> gpurun_out/r2al/bench_s${s}_$rep.err
  echo "s=$s rep=$rep $(python -c "import json;d=json.load(open('gpurun_out/r2al/bench_s${s}_$rep.json'));print(d['value'],d['ms_per_step'])")"
done
done

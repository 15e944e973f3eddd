#!/bin/bash
# MLP step: operand-pipeline depth variants (experiment builds selected by CE_LIB)
set -e
mkdir -p gpurun_out/r2an
for rep in 1 2; do
for v in default mi_d2 mt_d2 mt_d8; do
  if [ $v = default ]; then L=""; else L=$v; fi
  CE_LIB=$L timeout -k 10 120 python bench.py --workload mlp --steps 20 --warmup 3 > gpurun_out/r2an/bench_${v}_$rep.json 2> gpurun_out/r2an/bench_${v}_$rep.err
  echo "$v rep=$rep $(python -c "import json;d=json.load(open('gpurun_out/r2an/bench_${v}_$rep.json'));print(d['value'],d['ms_per_step'])")"
done
done

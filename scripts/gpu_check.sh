#!/bin/bash
# Round-end check: the driver's three GPU tiers in one call (tests, smoke, bench)
set -e
mkdir -p gpurun_out/check
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/check/pytest_gpu.log 2>&1
tail -3 gpurun_out/check/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/check/smoke.log 2>&1
tail -1 gpurun_out/check/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/check/bench.json 2> gpurun_out/check/bench.err
cat gpurun_out/check/bench.json

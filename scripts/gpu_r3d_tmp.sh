set -u
mkdir -p gpurun_out/r3d
OUT=gpurun_out/r3d VARIANTS="main r2 lazy0 rcp2 clamp" bash scripts/gpu_ab.sh
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail 8 --timeout 300 --timeout-method thread > gpurun_out/r3d/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r3d/pytest.log; grep -E "^FAILED|^E  .*err" gpurun_out/r3d/pytest.log | head -20; exit $rc

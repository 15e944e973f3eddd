set -u
mkdir -p gpurun_out/r3d
hipcc --offload-arch=gfx950 -O3 -Wno-unused-value scripts/mfma_valu_mix.hip -o /tmp/mvm && timeout -k 5 60 /tmp/mvm > gpurun_out/r3d/mfma_valu_mix.jsonl; cat gpurun_out/r3d/mfma_valu_mix.jsonl
timeout -k 10 400 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3d/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r3d/pytest.log; [ $rc = 0 ] || exit $rc
OUT=gpurun_out/r3d VARIANTS="main r2 lazy0 rcp2 clamp" bash scripts/gpu_ab.sh

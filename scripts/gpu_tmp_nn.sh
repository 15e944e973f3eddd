set -u
OUT=gpurun_out/nnab; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_multinn.py > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc = 0 ] || exit $rc
VARIANTS="main nnfin" bash scripts/gpu_ab_nn.sh

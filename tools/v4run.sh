set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
MAECLIP_GEMM_VARIANT=8 timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q -m gpu > gpurun_out/v4_pytest.log 2>&1 || { tail -30 gpurun_out/v4_pytest.log; exit 1; }
tail -1 gpurun_out/v4_pytest.log
AB="${AB:-MAECLIP_GEMM_VARIANT=0 MAECLIP_GEMM_VARIANT=8}" bash tools/ab_bench.sh

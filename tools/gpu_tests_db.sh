set -o pipefail
mkdir -p gpurun_out/db1
timeout -k 10 300 python -u -m pytest tests/test_delta_bytes.py tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/db1/pytest.log 2>&1
rc=$?; tail -25 gpurun_out/db1/pytest.log; exit $rc

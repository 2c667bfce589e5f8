set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_ipc.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/sharded_tests.log 2>&1
rc=$?; tail -15 gpurun_out/sharded_tests.log; exit $rc

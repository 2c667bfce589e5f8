# Round 6: the host-read-free sharded kinds through the C ABI -- multi-process
# (world 2, 3: XGMI + fixed + the RCCL kind) and world-1 graph capture.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06r}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded_capture.py tests/test_gpu_sharded_c.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed|Error|assert" gpurun_out/$T/tests.log | head -30
exit $rc

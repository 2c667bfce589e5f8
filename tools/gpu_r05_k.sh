# Round 5, batch K: the one-wave-per-SIMD TN dW kernel (DR_CROSSNET_DW_KERNEL
# =w4) -- its parity test, the interleaved forward (variant 16) parity, then
# the dW probe with and without it.  Tag $1.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r05k}
mkdir -p gpurun_out/$T
DR_CROSSNET_DW_KERNEL=w4 timeout -k 10 300 python -u -m pytest tests/test_gpu_dcn.py -k "dw" -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -2 gpurun_out/$T/tests.log; grep -E "^FAILED|^ERROR|Error" gpurun_out/$T/tests.log | head -10
[ $rc -ne 0 ] && exit $rc
DR_CROSSNET_VARIANT=16 timeout -k 10 300 python -u -m pytest tests/test_gpu_dcn.py -k "forward or dx or repeatable" -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/$T/tests_v16.log 2>&1
rc=$?; tail -2 gpurun_out/$T/tests_v16.log; grep -E "^FAILED|^ERROR|Error" gpurun_out/$T/tests_v16.log | head -10
[ $rc -ne 0 ] && exit $rc
DR_CROSSNET_DW_KERNEL=w4 timeout -k 10 200 python -u tools/cross_dw_probe.py > gpurun_out/$T/probe_w4.log 2>&1 || { tail -5 gpurun_out/$T/probe_w4.log; exit 1; }
grep -E "crossnet_dw|matmul|mm\(" gpurun_out/$T/probe_w4.log
timeout -k 10 200 python -u tools/cross_dw_probe.py > gpurun_out/$T/probe_8ph.log 2>&1 || { tail -5 gpurun_out/$T/probe_8ph.log; exit 1; }
grep -E "crossnet_dw" gpurun_out/$T/probe_8ph.log

# Round 5, batch J: every lookup kernel and every long-run walker through
# the parity tests (per-call DR_LOOKUP_KERNEL / DR_GRAD_SERIAL_PLAIN), then
# the headline parity at full size.  Tag $1.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r05j}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_rows_grad.py tests/test_gpu_headline.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -2 gpurun_out/$T/tests.log; grep -E "^FAILED|^ERROR" gpurun_out/$T/tests.log | head -20
exit $rc

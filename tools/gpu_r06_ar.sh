# Round 6: DIN item-gradient order pinned against the oracle (rows-grad tests).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06ar}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_rows_grad.py > gpurun_out/$T/tests.log 2>&1; rc=$?
tail -3 gpurun_out/$T/tests.log; grep -E "^E |Error" gpurun_out/$T/tests.log | head -10; exit $rc

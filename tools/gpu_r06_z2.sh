# Round 6: rounds walk with plain adds for the failing segment: rows tests, DIN A/B, stats.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06z2}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_rows_grad.py > gpurun_out/$T/tests.log 2>&1 || { tail -20 gpurun_out/$T/tests.log; exit 1; }
tail -1 gpurun_out/$T/tests.log
bash tools/gpu_r06_z.sh $T

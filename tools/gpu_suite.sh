# Whole -m gpu suite + smoke (tag $1).
set -o pipefail
T=${1:-suite}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1
rc=$?; tail -8 gpurun_out/$T/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/$T/smoke.log; exit $rc

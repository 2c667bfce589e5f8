# Round 6: xgmi serve without per-table mirror copies: sharded tests + native legs.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06ac}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded_capture.py tests/test_gpu_sharded_c.py tests/test_gpu_sharded.py tests/test_gpu_ev_concurrency.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$T/tests.log; grep -E "^FAILED|^ERROR" gpurun_out/$T/tests.log | head -10
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/sharded_c_check.py > gpurun_out/$T/c_check.log 2>&1 || { tail -5 gpurun_out/$T/c_check.log; exit 1; }
tail -2 gpurun_out/$T/c_check.log
timeout -k 10 600 python3 -u bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-criteo --no-dcn --no-hybrid --no-deepfm --model-steps 0 --train-steps 0 --din-steps 0 --native-steps 20 > gpurun_out/$T/bench.log 2>&1 || { tail -5 gpurun_out/$T/bench.log; exit 1; }
grep "native engine" gpurun_out/$T/bench.log | cut -c1-220
